// Input-side kernels: the graph operator of every knot and the backward-Hermite coefficients,
// written straight into the engine's interval-major HBM layout (include/gncde.h) — no reference-layout
// [B, T-1, n, n, 2] x 4 intermediate.
//
//   gncde_graph_operator       misc.py:58-113 get_graph_operator: norm_lap (default), norm_adj, kipf (zipf
//                              smoothing), normalized_plus (misc.py:36-57)
//   gncde_hermite_coefficients diffrax.backward_hermite_coefficients (dataset_configs.py:170;
//                              tgb_graph_neural_cde.py:130 rebuilds the data spline inside every forward)
#include "gncde_internal.h"

namespace gncde {
namespace {

// Degrees: dout[i] = sum_k M[i][k], din[k] = sum_i M[i][k] with M = A (+ I).  One block per graph.
__global__ void __launch_bounds__(256) k_degrees(int n, int self_loops, const float* __restrict__ A,
                                                 float* __restrict__ dout, float* __restrict__ din) {
  const int g = blockIdx.x;
  const float* Ag = A + (size_t)g * n * n;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int k = tid; k < n; k += blockDim.x) {  // column sums: threads along the row, coalesced
    float s = self_loops ? 1.f : 0.f;
    for (int i = 0; i < n; ++i) s += Ag[(size_t)i * n + k];
    din[(size_t)g * n + k] = s;
  }
  for (int i = w; i < n; i += (int)(blockDim.x >> 6)) {  // row sums: one wave per row
    float s = 0.f;
    for (int k = lane; k < n; k += 64) s += Ag[(size_t)i * n + k];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) dout[(size_t)g * n + i] = s + (self_loops ? 1.f : 0.f);
  }
}

// out = [I -] diag(so) (A + I) diag(si), so/si = deg^-1/2 (0 where the degree is 0 for normalized_plus)
__global__ void k_operator(int n, int kind, const float* __restrict__ A, const float* __restrict__ dout,
                           const float* __restrict__ din, float* __restrict__ out) {
  const int g = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nn = (size_t)n * n;
  if (e >= nn) return;
  const int i = (int)(e / n), k = (int)(e % n);
  const float doi = dout[(size_t)g * n + i], dik = din[(size_t)g * n + k];
  float so, si;
  if (kind == GNCDE_OP_NORMALIZED_PLUS) {
    so = doi != 0.f ? 1.0f / sqrtf(doi) : 0.f;
    si = dik != 0.f ? 1.0f / sqrtf(dik) : 0.f;
  } else {
    so = 1.0f / sqrtf(doi);
    si = 1.0f / sqrtf(dik);
  }
  const float aik = A[(size_t)g * nn + e] + (i == k ? 1.f : 0.f);
  const float v = so * aik * si;
  out[(size_t)g * nn + e] = kind == GNCDE_OP_NORM_LAP ? (i == k ? 1.f : 0.f) - v : v;
}

// Backward Hermite coefficients of X [B, T, C] over knots ts [B, T]; out[b, i, q, c] for q < ncoef in
// (d, c, b, a) order (ncoef = 4; 3 drops a).  Interval 0 uses the forward difference as its left derivative.
__global__ void k_hermite(int T, int C, int ncoef, const float* __restrict__ ts, const float* __restrict__ X,
                          float* __restrict__ out) {
  const int b = blockIdx.z, i = blockIdx.y;  // interval i in [0, T-1)
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float* tb = ts + (size_t)b * T;
  const float* xb = X + (size_t)b * T * C;
  const float dt = tb[i + 1] - tb[i];
  const float y0 = xb[(size_t)i * C + c], y1 = xb[(size_t)(i + 1) * C + c];
  const float slope = (y1 - y0) / dt;
  float deriv = slope;
  if (i > 0) deriv = (y0 - xb[(size_t)(i - 1) * C + c]) / (tb[i] - tb[i - 1]);
  const float dd = slope - deriv;
  float* o = out + ((size_t)b * (T - 1) + i) * ncoef * C + c;
  const float q[4] = {-dd / (dt * dt), 2.0f * dd / dt, deriv, y0};
  for (int j = 0; j < ncoef; ++j) o[(size_t)j * C] = q[j];
}

// Reverse of k_hermite.  With s_i the slope of interval i, r_i its left derivative (r_0 = s_0, r_i = s_{i-1}) and
// e_i = s_i - r_i:  d = -e/dt^2, c = 2e/dt, b = r, a = y_i.  Cotangents: ge_i = -gd_i/dt_i^2 + 2 gc_i/dt_i,
// gr_i = gb_i - ge_i, and the slope s_i collects ge_i + gr_{i+1} (+ gr_0 for i = 0).  Gathered per knot j:
// gy_j = ga_j + gs_{j-1}/dt_{j-1} - gs_j/dt_j, so each thread writes one output and nothing is accumulated.
__global__ void k_hermite_vjp(int T, int C, int ncoef, const float* __restrict__ ts, const float* __restrict__ g,
                              float* __restrict__ gX) {
  const int b = blockIdx.z, j = blockIdx.y;  // knot j in [0, T)
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float* tb = ts + (size_t)b * T;
  const float* gb = g + (size_t)b * (T - 1) * ncoef * C + c;
  auto gq = [&](int i, int q) { return gb[((size_t)i * ncoef + q) * C]; };
  auto ge = [&](int i) {
    const float dt = tb[i + 1] - tb[i];
    return -gq(i, 0) / (dt * dt) + 2.0f * gq(i, 1) / dt;
  };
  auto gr = [&](int i) { return gq(i, 2) - ge(i); };
  auto gs = [&](int i) {  // i in [0, T-2]
    float v = ge(i);
    if (i + 1 <= T - 2) v += gr(i + 1);
    if (i == 0) v += gr(0);
    return v;
  };
  float out = 0.f;
  if (j <= T - 2 && ncoef == 4) out += gq(j, 3);
  if (j >= 1) out += gs(j - 1) / (tb[j] - tb[j - 1]);
  if (j <= T - 2) out -= gs(j) / (tb[j + 1] - tb[j]);
  gX[((size_t)b * T + j) * C + c] = out;
}

}  // namespace
}  // namespace gncde

extern "C" {

int gncde_graph_operator(int32_t kind, int32_t graphs, int32_t n, const float* A, float* out, float* workspace,
                         void* stream) {
  using namespace gncde;
  if (graphs < 0 || n <= 0) return GNCDE_ERR_SHAPE;
  if (kind != GNCDE_OP_NORM_LAP && kind != GNCDE_OP_NORM_ADJ && kind != GNCDE_OP_KIPF &&
      kind != GNCDE_OP_NORMALIZED_PLUS)
    return GNCDE_ERR_ARG;
  if (graphs == 0) return GNCDE_OK;
  if (!A || !out || !workspace) return GNCDE_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* dout = workspace;
  float* din = workspace + (size_t)graphs * n;
  const int loops = kind == GNCDE_OP_NORMALIZED_PLUS ? 0 : 1;
  hipLaunchKernelGGL(k_degrees, dim3(graphs), dim3(256), 0, st, n, loops, A, dout, din);
  const size_t nn = (size_t)n * n;
  hipLaunchKernelGGL(k_operator, dim3((unsigned)((nn + 255) / 256), graphs), dim3(256), 0, st, n, kind, A, dout, din,
                     out);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

int gncde_hermite_coefficients(int32_t B, int32_t T, int32_t C, int32_t ncoef, const float* ts, const float* X,
                               float* out, void* stream) {
  using namespace gncde;
  if (B < 0 || T < 2 || C <= 0 || (ncoef != 3 && ncoef != 4)) return GNCDE_ERR_SHAPE;
  if (B == 0) return GNCDE_OK;
  if (!ts || !X || !out) return GNCDE_ERR_ARG;
  hipLaunchKernelGGL(k_hermite, dim3((unsigned)((C + 255) / 256), T - 1, B), dim3(256), 0,
                     static_cast<hipStream_t>(stream), T, C, ncoef, ts, X, out);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

int gncde_hermite_coefficients_vjp(int32_t B, int32_t T, int32_t C, int32_t ncoef, const float* ts,
                                   const float* gout, float* gX, void* stream) {
  using namespace gncde;
  if (B < 0 || T < 2 || C <= 0 || (ncoef != 3 && ncoef != 4)) return GNCDE_ERR_SHAPE;
  if (B == 0) return GNCDE_OK;
  if (!ts || !gout || !gX) return GNCDE_ERR_ARG;
  hipLaunchKernelGGL(k_hermite_vjp, dim3((unsigned)((C + 255) / 256), T, B), dim3(256), 0,
                     static_cast<hipStream_t>(stream), T, C, ncoef, ts, gout, gX);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

}  // extern "C"
