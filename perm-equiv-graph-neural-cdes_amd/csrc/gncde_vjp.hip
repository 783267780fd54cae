// Reverse-mode (discrete adjoint) of the fixed-grid solve — SURVEY §8(a) row a9.
//
// Reference: value_and_grad through diffrax.diffeqsolve with the default RecursiveCheckpointAdjoint
// (trainer.py:315, graph_neural_cde.py:94-104) = the exact gradient of the discrete RK solve.  Here:
// the forward solve's per-step states are the checkpoints; every step is recomputed from its
// checkpoint (stage inputs u_i), then the RK combination is reversed stage by stage; each stage's
// vector-field VJP recomputes the layer activations at u_i and back-propagates through
//   F(u) = tg * Z_L,  Z_l = act((I + Abar_l) m_l),  m_l = Linear(RMSNorm(Z_{l-1}))
// accumulating per-sample parameter and fusion-table gradients, which are reduced over the batch at
// the end (fixed order: deterministic, no atomics).
//
// Generic multi-kernel path (any n, widths, fusion kind, CDE wrapper).
#include "gncde_internal.h"

#include <initializer_list>
#include <utility>

namespace gncde {
namespace {

constexpr int kRedStride = 8;  // same reduction layout as gncde_generic.hip

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// ---- forward pieces (with activations kept) --------------------------------------------------------
__global__ void v_spline(int n, int T, const float* __restrict__ ts, const float* __restrict__ coef,
                         const float* __restrict__ tcoef, const float* __restrict__ t, float* __restrict__ A,
                         float* __restrict__ dA, float* __restrict__ tg) {
  const int b = blockIdx.y;
  const size_t nn = (size_t)n * n;
  const float tb = t[b];
  const float* tsb = ts + (size_t)b * T;
  const int idx = interval_index(tsb, T, tb);
  const float f = tb - tsb[idx];
  const float* cb = coef + ((size_t)b * (T - 1) + idx) * 4 * nn;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nn) {
    const float d = cb[e], c = cb[nn + e], bb = cb[2 * nn + e], a = cb[3 * nn + e];
    A[(size_t)b * nn + e] = fmaf(f, fmaf(f, fmaf(f, d, c), bb), a);
    dA[(size_t)b * nn + e] = fmaf(f, fmaf(3.0f * f, d, 2.0f * c), bb);
  }
  if (e < (size_t)n) {
    const float* tc = tcoef + ((size_t)b * (T - 1) + idx) * 3 * n;
    tg[(size_t)b * n + e] = fmaf(f, fmaf(3.0f * f, tc[e], 2.0f * tc[n + e]), tc[2 * n + e]);
  }
}

__global__ void v_reduce(int n, const float* __restrict__ A, const float* __restrict__ dA, float* __restrict__ red) {
  const int b = blockIdx.x;
  const size_t nn = (size_t)n * n;
  const float* Ab = A + b * nn;
  const float* dAb = dA + b * nn;
  float* rb = red + (size_t)b * kRedStride * n;
  __shared__ float part[2][256];
  float ps = 0.f, psd = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float r = 0.f, rd = 0.f, c = 0.f, cd = 0.f;
    for (int k = 0; k < n; ++k) {
      r += Ab[(size_t)i * n + k];
      rd += dAb[(size_t)i * n + k];
      c += Ab[(size_t)k * n + i];
      cd += dAb[(size_t)k * n + i];
    }
    rb[i] = r;
    rb[n + i] = rd;
    rb[2 * n + i] = c;
    rb[3 * n + i] = cd;
    rb[4 * n + i] = Ab[(size_t)i * n + i];
    rb[5 * n + i] = dAb[(size_t)i * n + i];
    ps += r;
    psd += rd;
  }
  part[0][threadIdx.x] = ps;
  part[1][threadIdx.x] = psd;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      part[0][threadIdx.x] += part[0][threadIdx.x + s];
      part[1][threadIdx.x] += part[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    rb[6 * n] = part[0][0];
    rb[7 * n] = part[1][0];
  }
}

// inv[b,i] = rsqrt(mean(z^2) + eps); m = (z*inv*rw + rb) W^T + bias.  z = relu(prev pre) if relu_in.
__global__ void v_rms_linear(int n, int din, int dout, const float* __restrict__ Z, int relu_in,
                             const float* __restrict__ rw, const float* __restrict__ rbias,
                             const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ m,
                             float* __restrict__ inv_out) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)n * dout) return;
  const int i = (int)(e / dout), o = (int)(e % dout);
  const float* z = Z + ((size_t)b * n + i) * din;
  float ss = 0.f;
  for (int k = 0; k < din; ++k) {
    const float v = relu_in ? fmaxf(z[k], 0.f) : z[k];
    ss = fmaf(v, v, ss);
  }
  const float inv = 1.0f / sqrtf(ss / (float)din + 1e-5f);
  float acc = bias[o];
  const float* w = W + (size_t)o * din;
  for (int k = 0; k < din; ++k) {
    const float v = relu_in ? fmaxf(z[k], 0.f) : z[k];
    acc = fmaf(fmaf(v * inv, rw[k], rbias[k]), w[k], acc);
  }
  m[((size_t)b * n + i) * dout + o] = acc;
  if (o == 0) inv_out[(size_t)b * n + i] = inv;
}

__device__ __forceinline__ void row_terms(const float* fc, const float* rb, int n, int i, float& wi, float& ui) {
  const float s = rb[6 * n], sd = rb[7 * n];
  wi = fc[GNCDE_FC_WR_A] * rb[i] + fc[GNCDE_FC_WR_DA] * rb[n + i] + fc[GNCDE_FC_WC_A] * rb[2 * n + i] +
       fc[GNCDE_FC_WC_DA] * rb[3 * n + i] + fc[GNCDE_FC_WS_A] * s + fc[GNCDE_FC_WS_DA] * sd;
  ui = fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * rb[4 * n + i] + fc[GNCDE_FC_UD_DA] * rb[5 * n + i] +
       fc[GNCDE_FC_UR_A] * rb[i] + fc[GNCDE_FC_UR_DA] * rb[n + i] + fc[GNCDE_FC_UC_A] * rb[2 * n + i] +
       fc[GNCDE_FC_UC_DA] * rb[3 * n + i] + fc[GNCDE_FC_US_A] * s + fc[GNCDE_FC_US_DA] * sd;
}

__device__ __forceinline__ float abar(const float* fc, const float* A, const float* dA, const float* rb, int n,
                                      int i, int k) {
  const float aik = A[(size_t)i * n + k], aki = A[(size_t)k * n + i];
  const float dik = dA[(size_t)i * n + k], dki = dA[(size_t)k * n + i];
  float wi, ui;
  row_terms(fc, rb, n, i, wi, ui);
  const float vk = fc[GNCDE_FC_VR_A] * rb[k] + fc[GNCDE_FC_VR_DA] * rb[n + k] + fc[GNCDE_FC_VC_A] * rb[2 * n + k] +
                   fc[GNCDE_FC_VC_DA] * rb[3 * n + k];
  float v = fc[GNCDE_FC_E_A] * aik + fc[GNCDE_FC_E_DA] * dik + fc[GNCDE_FC_ET_A] * aki + fc[GNCDE_FC_ET_DA] * dki;
  v += wi + vk;
  if (i == k) v += ui;
  return v;
}

// out[b,i,o] = sum_k M[i,k] x[b,k,o] with M = (I+Abar) (trans=0) or its transpose (trans=1)
__global__ void __launch_bounds__(256) v_prop(int n, int d, const float* __restrict__ fc, const float* __restrict__ A,
                                              const float* __restrict__ dA, const float* __restrict__ red,
                                              const float* __restrict__ x, float* __restrict__ out, int trans) {
  const int b = blockIdx.z;
  const int o0 = blockIdx.x * 16, i0 = blockIdx.y * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const size_t nn = (size_t)n * n;
  const float* Ab = A + b * nn;
  const float* dAb = dA + b * nn;
  const float* rb = red + (size_t)b * kRedStride * n;
  const float* xb = x + (size_t)b * n * d;
  __shared__ float sA[16][17];
  __shared__ float sX[16][17];
  float acc = 0.f;
  for (int k0 = 0; k0 < n; k0 += 16) {
    const int i = i0 + ty, k = k0 + tx;
    sA[ty][tx] = (i < n && k < n) ? (trans ? abar(fc, Ab, dAb, rb, n, k, i) : abar(fc, Ab, dAb, rb, n, i, k)) : 0.f;
    const int kk = k0 + ty, o = o0 + tx;
    sX[ty][tx] = (kk < n && o < d) ? xb[(size_t)kk * d + o] : 0.f;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) acc = fmaf(sA[ty][q], sX[q][tx], acc);
    __syncthreads();
  }
  const int i = i0 + ty, o = o0 + tx;
  if (i < n && o < d) out[((size_t)b * n + i) * d + o] = acc;
}

// ---- backward pieces ---------------------------------------------------------------------------------
// gZ_{L-1}: ODE g = tg * gF; CDE g[i, (m*de+l)*2+k] = tg[i] gF[i,m] dX[i,l,k]
__global__ void v_out_grad(int n, int dL, int h, int de, int T, const float* __restrict__ ts,
                           const float* __restrict__ data_coef, const float* __restrict__ t,
                           const float* __restrict__ tg, const float* __restrict__ gF, float* __restrict__ gZ) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)n * dL) return;
  const int i = (int)(e / dL), q = (int)(e % dL);
  const float g = tg[(size_t)b * n + i];
  if (h == 0) {
    gZ[((size_t)b * n + i) * dL + q] = g * gF[((size_t)b * n + i) * dL + q];
    return;
  }
  const int mo = q / (de * 2), lk = q % (de * 2);
  const float tb = t[b];
  const float* tsb = ts + (size_t)b * T;
  const int idx = interval_index(tsb, T, tb);
  const float f = tb - tsb[idx];
  const size_t blk = (size_t)n * de * 2;
  const float* cb = data_coef + ((size_t)b * (T - 1) + idx) * 4 * blk + (size_t)i * de * 2 + lk;
  const float dX = fmaf(f, fmaf(3.0f * f, cb[0], 2.0f * cb[blk]), cb[2 * blk]);
  gZ[((size_t)b * n + i) * dL + q] = g * gF[((size_t)b * n + i) * h + mo] * dX;
}

// gpre = gZ * 1[pre > 0] when the layer has a ReLU (l < L-1), else gZ
__global__ void v_relu_mask(size_t total, const float* __restrict__ pre, float* __restrict__ g) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < total && !(pre[e] > 0.f)) g[e] = 0.f;
}

// column sums over nodes: out[b, o] = sum_i x[b, i, o]
__global__ void v_colsum(int n, int d, const float* __restrict__ x, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= d) return;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += x[((size_t)b * n + i) * d + o];
  out[(size_t)b * d + o] = s;
}

// Fusion-table gradient of one layer for one sample.  With G = gpre m^T (G[i,k] = gpre[i].m[k]):
//   g[E_A] = <G, A>, g[E_DA] = <G, dA>, g[ET_A] = <G, A^T>, g[ET_DA] = <G, dA^T>   (block partials here)
// The row/column/diagonal families use R_i = gpre[i].colsum(m), C_k = m[k].colsum(gpre),
// D_i = gpre[i].m[i] (v_fusion_rank) — no n x n intermediate is stored.
__global__ void __launch_bounds__(256) v_fusion_dense(int n, int d, const float* __restrict__ A,
                                                      const float* __restrict__ dA, const float* __restrict__ gpre,
                                                      const float* __restrict__ m, float* __restrict__ part) {
  const int b = blockIdx.y;
  const int i = blockIdx.x;  // one row per block
  const size_t nn = (size_t)n * n;
  const float* Ab = A + b * nn;
  const float* dAb = dA + b * nn;
  const float* gi = gpre + ((size_t)b * n + i) * d;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const float* mk = m + ((size_t)b * n + k) * d;
    float G = 0.f;
    for (int o = 0; o < d; ++o) G = fmaf(gi[o], mk[o], G);
    s0 = fmaf(G, Ab[(size_t)i * n + k], s0);
    s1 = fmaf(G, dAb[(size_t)i * n + k], s1);
    s2 = fmaf(G, Ab[(size_t)k * n + i], s2);
    s3 = fmaf(G, dAb[(size_t)k * n + i], s3);
  }
  __shared__ float red[4][256];
  red[0][threadIdx.x] = s0;
  red[1][threadIdx.x] = s1;
  red[2][threadIdx.x] = s2;
  red[3][threadIdx.x] = s3;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < 4) part[((size_t)b * n + i) * 4 + threadIdx.x] = red[threadIdx.x][0];
}

// Per-sample accumulation of the 24 fusion-table gradients of layer l into gfc[b, l, :]
__global__ void v_fusion_rank(int n, int d, int L, int l, const float* __restrict__ red,
                              const float* __restrict__ gpre, const float* __restrict__ m,
                              const float* __restrict__ cs_m, const float* __restrict__ cs_g,
                              const float* __restrict__ part, float* __restrict__ gfc) {
  const int b = blockIdx.x;
  const float* rb = red + (size_t)b * kRedStride * n;
  const float s = rb[6 * n], sd = rb[7 * n];
  // one thread per accumulated quantity
  const int q = threadIdx.x;
  if (q >= GNCDE_FC) return;
  float acc = 0.f;
  for (int i = 0; i < n; ++i) {
    const float* gi = gpre + ((size_t)b * n + i) * d;
    const float* mi = m + ((size_t)b * n + i) * d;
    float R = 0.f, C = 0.f, D = 0.f;
    if (q >= GNCDE_FC_WR_A && q <= GNCDE_FC_WS_DA) {
      for (int o = 0; o < d; ++o) R = fmaf(gi[o], cs_m[(size_t)b * d + o], R);
    } else if (q >= GNCDE_FC_VR_A && q <= GNCDE_FC_VC_DA) {
      for (int o = 0; o < d; ++o) C = fmaf(mi[o], cs_g[(size_t)b * d + o], C);
    } else if ((q >= GNCDE_FC_UD_A && q <= GNCDE_FC_US_DA) || q == GNCDE_FC_IDC) {
      for (int o = 0; o < d; ++o) D = fmaf(gi[o], mi[o], D);
    }
    float x = 0.f;
    switch (q) {
      case GNCDE_FC_E_A: case GNCDE_FC_E_DA: case GNCDE_FC_ET_A: case GNCDE_FC_ET_DA:
        x = part[((size_t)b * n + i) * 4 + q];
        break;
      case GNCDE_FC_UD_A: x = D * rb[4 * n + i]; break;
      case GNCDE_FC_UD_DA: x = D * rb[5 * n + i]; break;
      case GNCDE_FC_UR_A: x = D * rb[i]; break;
      case GNCDE_FC_UR_DA: x = D * rb[n + i]; break;
      case GNCDE_FC_UC_A: x = D * rb[2 * n + i]; break;
      case GNCDE_FC_UC_DA: x = D * rb[3 * n + i]; break;
      case GNCDE_FC_US_A: x = D * s; break;
      case GNCDE_FC_US_DA: x = D * sd; break;
      case GNCDE_FC_WR_A: x = R * rb[i]; break;
      case GNCDE_FC_WR_DA: x = R * rb[n + i]; break;
      case GNCDE_FC_WC_A: x = R * rb[2 * n + i]; break;
      case GNCDE_FC_WC_DA: x = R * rb[3 * n + i]; break;
      case GNCDE_FC_WS_A: x = R * s; break;
      case GNCDE_FC_WS_DA: x = R * sd; break;
      case GNCDE_FC_VR_A: x = C * rb[i]; break;
      case GNCDE_FC_VR_DA: x = C * rb[n + i]; break;
      case GNCDE_FC_VC_A: x = C * rb[2 * n + i]; break;
      case GNCDE_FC_VC_DA: x = C * rb[3 * n + i]; break;
      case GNCDE_FC_IDC: x = D; break;
      default: x = 0.f;
    }
    acc += x;
  }
  gfc[((size_t)b * L + l) * GNCDE_FC + q] += acc;
}

// Linear + RMSNorm backward, per (b, i): gzn = gm W; gz = inv (gxh - xh (xh.gxh)/din), gxh = gzn*rw
// (xh = z*inv).  Writes gZ_prev (layer input grad) and the per-node gzn for the parameter sums.
__global__ void v_linear_input_grad(int n, int din, int dout, const float* __restrict__ Z, int relu_in,
                                    const float* __restrict__ inv, const float* __restrict__ rw,
                                    const float* __restrict__ W, const float* __restrict__ gm,
                                    float* __restrict__ gzn, float* __restrict__ gz) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* z = Z + ((size_t)b * n + i) * din;
  const float* g = gm + ((size_t)b * n + i) * dout;
  const float iv = inv[(size_t)b * n + i];
  float dot = 0.f;
  for (int f = 0; f < din; ++f) {
    float acc = 0.f;
    for (int o = 0; o < dout; ++o) acc = fmaf(g[o], W[(size_t)o * din + f], acc);
    gzn[((size_t)b * n + i) * din + f] = acc;
    const float xh = (relu_in ? fmaxf(z[f], 0.f) : z[f]) * iv;
    dot = fmaf(acc * rw[f], xh, dot);
  }
  const float c = dot / (float)din;
  for (int f = 0; f < din; ++f) {
    const float zf = relu_in ? fmaxf(z[f], 0.f) : z[f];
    const float xh = zf * iv;
    const float gxh = gzn[((size_t)b * n + i) * din + f] * rw[f];
    float v = iv * (gxh - xh * c);
    if (relu_in && !(z[f] > 0.f)) v = 0.f;  // through the previous layer's ReLU
    gz[((size_t)b * n + i) * din + f] = v;
  }
}

// Per-sample parameter gradients of one layer (accumulated into gp[b, :] at the layer's offsets):
//   bias += sum_i gm[i];  W[o,f] += sum_i gm[i,o] zn[i,f];  rms_w[f] += sum_i gzn[i,f] xh[i,f];
//   rms_b[f] += sum_i gzn[i,f]
__global__ void v_linear_param_grad(int n, int din, int dout, const float* __restrict__ Z, int relu_in,
                                    const float* __restrict__ inv, const float* __restrict__ rw,
                                    const float* __restrict__ rbias, const float* __restrict__ gm,
                                    const float* __restrict__ gzn, size_t P, size_t off, float* __restrict__ gp) {
  const int b = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int nW = dout * din;
  const int total = 2 * din + nW + dout;
  if (e >= total) return;
  float acc = 0.f;
  if (e < din) {  // rms_w
    const int f = e;
    for (int i = 0; i < n; ++i) {
      const float zf = Z[((size_t)b * n + i) * din + f];
      const float xh = (relu_in ? fmaxf(zf, 0.f) : zf) * inv[(size_t)b * n + i];
      acc = fmaf(gzn[((size_t)b * n + i) * din + f], xh, acc);
    }
  } else if (e < 2 * din) {  // rms_b
    const int f = e - din;
    for (int i = 0; i < n; ++i) acc += gzn[((size_t)b * n + i) * din + f];
  } else if (e < 2 * din + nW) {  // W
    const int q = e - 2 * din, o = q / din, f = q % din;
    for (int i = 0; i < n; ++i) {
      const float zf = Z[((size_t)b * n + i) * din + f];
      const float zn = fmaf((relu_in ? fmaxf(zf, 0.f) : zf) * inv[(size_t)b * n + i], rw[f], rbias[f]);
      acc = fmaf(gm[((size_t)b * n + i) * dout + o], zn, acc);
    }
  } else {  // bias
    const int o = e - 2 * din - nW;
    for (int i = 0; i < n; ++i) acc += gm[((size_t)b * n + i) * dout + o];
  }
  gp[(size_t)b * P + off + e] += acc;
}

// out = sum over b of x[b, :]  (fixed order: deterministic)
__global__ void v_batch_sum(int B, size_t P, const float* __restrict__ x, float* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += x[(size_t)b * P + e];
  out[e] = s;
}

// ---- solver helpers ------------------------------------------------------------------------------------
__global__ void v_step_geom(int B, int G, int k, const float* __restrict__ grid, const int32_t* __restrict__ nsteps,
                            float* __restrict__ tcur, float* __restrict__ hcur) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int ns = nsteps[b];
  ns = ns < 0 ? 0 : (ns > G - 1 ? G - 1 : ns);
  const float* g = grid + (size_t)b * G;
  if (k < ns) {
    tcur[b] = g[k];
    hcur[b] = g[k + 1] - g[k];
  } else {
    tcur[b] = g[ns];
    hcur[b] = 0.f;
  }
}

__global__ void v_stage_time(int B, float c, const float* __restrict__ tcur, const float* __restrict__ hcur,
                             float* __restrict__ tst) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  tst[b] = stage_time(tcur[b], c, hcur[b]);
}

struct Lin {
  const float* x[8];
  float a[8];
  int nx;
  int scale_h;  // multiply the sum by h_b
};
// out = (acc ? out : base) + (scale_h ? h_b : 1) * sum_j a_j x_j
__global__ void v_lincomb(int B, size_t E, const float* __restrict__ base, Lin lc, const float* __restrict__ hcur,
                          float* __restrict__ out, int accumulate) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const size_t o = (size_t)b * E + e;
  float s = 0.f;
  for (int j = 0; j < lc.nx; ++j) s = fmaf(lc.a[j], lc.x[j][o], s);
  const float hb = lc.scale_h ? hcur[b] : 1.0f;
  const float b0 = accumulate ? out[o] : (base ? base[o] : 0.f);
  out[o] = fmaf(hb, s, b0);
}

// row k of a per-step trajectory [B, G, E]: out = (accumulate ? out : 0) + traj[:, k]
__global__ void v_step_row(int B, size_t E, int G, int k, const float* __restrict__ traj, float* __restrict__ out,
                           int accumulate) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float v = traj[((size_t)b * G + k) * E + e];
  out[(size_t)b * E + e] = accumulate ? out[(size_t)b * E + e] + v : v;
}

// ---- workspace ----------------------------------------------------------------------------------------
struct VjpWs {
  float *A, *dA, *red, *tg;
  float* Zin[GNCDE_MAX_LAYERS];  // layer inputs (layer 0: stage input copy; l>0: pre of l-1)
  float* M[GNCDE_MAX_LAYERS];
  float* PRE[GNCDE_MAX_LAYERS];
  float* INV[GNCDE_MAX_LAYERS];
  float *g0, *g1, *gzn, *part, *csm, *csg;
  float *gp, *gfc;               // per-sample accumulators [B, P], [B, L, 24]
  float *y, *lam, *gyacc, *tmp;
  float* U[7];                   // stage inputs
  float* K[7];                   // stage values
  float* gK[7];                  // stage cotangents
  float *tcur, *hcur, *tst;
};

struct Carver {
  char* base;
  size_t off = 0;
  float* take(size_t floats) {
    float* p = reinterpret_cast<float*>(base + off);
    off += align_up(floats * sizeof(float), 256);
    return p;
  }
};

void carve(const GncdeProblem& p, char* ws, VjpWs& w, size_t* bytes) {
  const size_t B = p.B, n = p.n, nn = n * n, D = max_dim(p), E = n * state_dim(p);
  const size_t P = params_floats(p);
  Carver c{ws};
  auto tk = [&](size_t f) { return ws ? c.take(f) : (c.off += align_up(f * sizeof(float), 256), nullptr); };
  w.A = tk(B * nn);
  w.dA = tk(B * nn);
  w.red = tk(B * kRedStride * n);
  w.tg = tk(B * n);
  for (int l = 0; l < p.L; ++l) {
    w.Zin[l] = tk(B * n * D);
    w.M[l] = tk(B * n * D);
    w.PRE[l] = tk(B * n * D);
    w.INV[l] = tk(B * n);
  }
  w.g0 = tk(B * n * D);
  w.g1 = tk(B * n * D);
  w.gzn = tk(B * n * D);
  w.part = tk(B * n * 4);
  w.csm = tk(B * D);
  w.csg = tk(B * D);
  w.gp = tk(B * P);
  w.gfc = tk(B * p.L * GNCDE_FC);
  w.y = tk(B * E);
  w.lam = tk(B * E);
  w.gyacc = tk(B * E);
  w.tmp = tk(B * E);
  for (int j = 0; j < 7; ++j) {
    w.U[j] = tk(B * E);
    w.K[j] = tk(B * E);
    w.gK[j] = tk(B * E);
  }
  w.tcur = tk(B);
  w.hcur = tk(B);
  w.tst = tk(B);
  *bytes = c.off;
}

// The layer activations of F(t, u) kept in the workspace (layer inputs, m_l, pre-activations, 1/rms)
void forward_keep(const GncdeProblem& p, const float* t, const float* u, VjpWs& w, hipStream_t st) {
  const int B = p.B, n = p.n;
  const size_t nn = (size_t)n * n;
  hipLaunchKernelGGL(v_spline, dim3(cdiv(nn > (size_t)n ? nn : n, 256), B), dim3(256), 0, st, n, p.T, p.ts, p.coef,
                     p.tcoef, t, w.A, w.dA, w.tg);
  hipLaunchKernelGGL(v_reduce, dim3(B), dim3(256), 0, st, n, w.A, w.dA, w.red);
  (void)hipMemcpyAsync(w.Zin[0], u, (size_t)B * n * p.dims[0] * sizeof(float), hipMemcpyDeviceToDevice, st);
  for (int l = 0; l < p.L; ++l) {
    const int din = p.dims[l], dout = p.dims[l + 1];
    const LayerOffsets o = layer_offsets(p, l);
    const float* zin = l == 0 ? w.Zin[0] : w.PRE[l - 1];
    hipLaunchKernelGGL(v_rms_linear, dim3(cdiv((size_t)n * dout, 256), B), dim3(256), 0, st, n, din, dout, zin,
                       l > 0 ? 1 : 0, p.params + o.rms_w, p.params + o.rms_b, p.params + o.W, p.params + o.b, w.M[l],
                       w.INV[l]);
    hipLaunchKernelGGL(v_prop, dim3(cdiv(dout, 16), cdiv(n, 16), B), dim3(256), 0, st, n, dout,
                       p.fusion + (size_t)l * GNCDE_FC, w.A, w.dA, w.red, w.M[l], w.PRE[l], 0);
  }
}

}  // namespace

size_t generic_vjp_workspace(const GncdeProblem& p, const GncdeSolver& s) {
  (void)s;
  VjpWs w;
  size_t bytes = 0;
  carve(p, nullptr, w, &bytes);
  return bytes + generic_vf_workspace(p);
}

namespace {

// VJP of F at (t, u) for cotangent gF (B x n x d_out); adds the input cotangent into gu (accumulate) and the
// parameter / fusion gradients into w.gp / w.gfc.
void vf_vjp(const GncdeProblem& p, const float* t, const float* u, const float* gF, float* gu, VjpWs& w,
            hipStream_t st) {
  const int B = p.B, n = p.n, L = p.L;
  const size_t P = params_floats(p);
  forward_keep(p, t, u, w, st);
  const int dL = p.dims[L];
  hipLaunchKernelGGL(v_out_grad, dim3(cdiv((size_t)n * dL, 256), B), dim3(256), 0, st, n, dL, p.cde_hidden,
                     p.cde_embed, p.T, p.ts, p.data_coef, t, w.tg, gF, w.g0);
  float* gZ = w.g0;   // cotangent of Z_l
  float* gm = w.g1;   // cotangent of m_l
  for (int l = L - 1; l >= 0; --l) {
    const int din = p.dims[l], dout = p.dims[l + 1];
    const LayerOffsets o = layer_offsets(p, l);
    if (l < L - 1)
      hipLaunchKernelGGL(v_relu_mask, dim3(cdiv((size_t)B * n * dout, 256)), dim3(256), 0, st,
                         (size_t)B * n * dout, w.PRE[l], gZ);
    const float* fc = p.fusion + (size_t)l * GNCDE_FC;
    // fusion-table gradient (needs gpre = gZ and m)
    hipLaunchKernelGGL(v_fusion_dense, dim3(n, B), dim3(256), 0, st, n, dout, w.A, w.dA, gZ, w.M[l], w.part);
    hipLaunchKernelGGL(v_colsum, dim3(cdiv(dout, 64), B), dim3(64), 0, st, n, dout, w.M[l], w.csm);
    hipLaunchKernelGGL(v_colsum, dim3(cdiv(dout, 64), B), dim3(64), 0, st, n, dout, gZ, w.csg);
    hipLaunchKernelGGL(v_fusion_rank, dim3(B), dim3(64), 0, st, n, dout, L, l, w.red, gZ, w.M[l], w.csm, w.csg,
                       w.part, w.gfc);
    // gm = (I+Abar)^T gpre
    hipLaunchKernelGGL(v_prop, dim3(cdiv(dout, 16), cdiv(n, 16), B), dim3(256), 0, st, n, dout, fc, w.A, w.dA,
                       w.red, gZ, gm, 1);
    // Linear + RMSNorm backward
    const float* zin = l == 0 ? w.Zin[0] : w.PRE[l - 1];
    const int relu_in = l > 0 ? 1 : 0;
    float* gzprev = gZ;  // reuse: gZ is dead after gm is formed
    hipLaunchKernelGGL(v_linear_input_grad, dim3(cdiv(n, 64), B), dim3(64), 0, st, n, din, dout, zin, relu_in,
                       w.INV[l], p.params + o.rms_w, p.params + o.W, gm, w.gzn, gzprev);
    const int tot = 2 * din + dout * din + dout;
    hipLaunchKernelGGL(v_linear_param_grad, dim3(cdiv(tot, 128), B), dim3(128), 0, st, n, din, dout, zin, relu_in,
                       w.INV[l], p.params + o.rms_w, p.params + o.rms_b, gm, w.gzn, P, o.rms_w, w.gp);
    gZ = gzprev;
  }
  // gu += gZ (cotangent of the stage input)
  Lin lc{};
  lc.x[0] = gZ;
  lc.a[0] = 1.0f;
  lc.nx = 1;
  lc.scale_h = 0;
  const size_t E = (size_t)n * state_dim(p);
  hipLaunchKernelGGL(v_lincomb, dim3(cdiv(E, 256), B), dim3(256), 0, st, B, E, nullptr, lc, w.hcur, gu, 1);
}

struct Tableau {
  int stages;
  float c[7];
  float a[7][7];
  float b[7];
};

Tableau rk4_tab() {
  Tableau t{};
  t.stages = 4;
  t.c[0] = 0.f; t.c[1] = 0.5f; t.c[2] = 0.5f; t.c[3] = 1.f;
  t.a[1][0] = 0.5f;
  t.a[2][1] = 0.5f;
  t.a[3][2] = 1.f;
  t.b[0] = 1.f / 6.f; t.b[1] = 2.f / 6.f; t.b[2] = 2.f / 6.f; t.b[3] = 1.f / 6.f;
  return t;
}

Tableau tsit5_tab() {
  Tableau t{};
  t.stages = 6;  // stage 7 (FSAL) does not enter y1
  t.c[0] = 0.f; t.c[1] = TSIT5_C2; t.c[2] = TSIT5_C3; t.c[3] = TSIT5_C4; t.c[4] = TSIT5_C5; t.c[5] = 1.f;
  t.a[1][0] = TSIT5_A21;
  t.a[2][0] = TSIT5_A31; t.a[2][1] = TSIT5_A32;
  t.a[3][0] = TSIT5_A41; t.a[3][1] = TSIT5_A42; t.a[3][2] = TSIT5_A43;
  t.a[4][0] = TSIT5_A51; t.a[4][1] = TSIT5_A52; t.a[4][2] = TSIT5_A53; t.a[4][3] = TSIT5_A54;
  t.a[5][0] = TSIT5_A61; t.a[5][1] = TSIT5_A62; t.a[5][2] = TSIT5_A63; t.a[5][3] = TSIT5_A64; t.a[5][4] = TSIT5_A65;
  t.b[0] = TSIT5_B1; t.b[1] = TSIT5_B2; t.b[2] = TSIT5_B3; t.b[3] = TSIT5_B4; t.b[4] = TSIT5_B5; t.b[5] = TSIT5_B6;
  return t;
}

}  // namespace

int generic_integrate_vjp(const GncdeProblem& p, const GncdeSolver& s, const float* ys, const float* gys, float* gy0,
                          float* gparams, float* gfusion, char* ws, hipStream_t st) {
  if (s.controller != GNCDE_CTRL_GRID) return GNCDE_ERR_UNSUPPORTED;
  const int B = p.B, G = s.grid_len;
  const size_t E = (size_t)p.n * state_dim(p);
  const size_t P = params_floats(p);
  VjpWs w;
  size_t bytes = 0;
  carve(p, ws, w, &bytes);
  char* vf_ws = ws + bytes;
  const Tableau tab = s.method == GNCDE_RK4 ? rk4_tab() : tsit5_tab();
  generic_vf_prepare(p, vf_ws, st);
  const unsigned gb = cdiv(B, 256);
  const dim3 ge(cdiv(E, 256), B);
  (void)hipMemsetAsync(w.gp, 0, (size_t)B * P * sizeof(float), st);
  (void)hipMemsetAsync(w.gfc, 0, (size_t)B * p.L * GNCDE_FC * sizeof(float), st);
  // lambda = cotangent of the final state (every saved state's cotangent is added as the sweep passes it)
  if (s.save_mode == GNCDE_SAVE_STEPS)
    hipLaunchKernelGGL(v_step_row, ge, dim3(256), 0, st, B, E, G, G - 1, gys, w.lam, 0);
  else
    (void)hipMemcpyAsync(w.lam, gys, (size_t)B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  for (int k = G - 2; k >= 0; --k) {
    hipLaunchKernelGGL(v_step_geom, dim3(gb), dim3(256), 0, st, B, G, k, s.grid, s.nsteps, w.tcur, w.hcur);
    // checkpoint y_k (the forward's SAVE_STEPS output)
    hipLaunchKernelGGL(v_step_row, ge, dim3(256), 0, st, B, E, G, k, ys, w.y, 0);
    // recompute stage inputs U_i and values K_i
    for (int i = 0; i < tab.stages; ++i) {
      Lin lc{};
      lc.nx = 0;
      lc.scale_h = 1;
      for (int j = 0; j < i; ++j)
        if (tab.a[i][j] != 0.f) {
          lc.x[lc.nx] = w.K[j];
          lc.a[lc.nx++] = tab.a[i][j];
        }
      hipLaunchKernelGGL(v_lincomb, ge, dim3(256), 0, st, B, E, w.y, lc, w.hcur, w.U[i], 0);
      hipLaunchKernelGGL(v_stage_time, dim3(gb), dim3(256), 0, st, B, tab.c[i], w.tcur, w.hcur, w.tst);
      if (i + 1 < tab.stages) {  // the last stage's value is not needed for the reverse sweep
        const int rc = generic_vf_eval(p, w.tst, w.U[i], w.K[i], vf_ws, st, true);
        if (rc) return rc;
      }
    }
    // reverse: gK_i = h b_i lam ; gy = lam
    for (int i = 0; i < tab.stages; ++i) {
      Lin lc{};
      lc.x[0] = w.lam;
      lc.a[0] = tab.b[i];
      lc.nx = 1;
      lc.scale_h = 1;
      hipLaunchKernelGGL(v_lincomb, ge, dim3(256), 0, st, B, E, nullptr, lc, w.hcur, w.gK[i], 0);
    }
    (void)hipMemcpyAsync(w.gyacc, w.lam, (size_t)B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
    for (int i = tab.stages - 1; i >= 0; --i) {
      hipLaunchKernelGGL(v_stage_time, dim3(gb), dim3(256), 0, st, B, tab.c[i], w.tcur, w.hcur, w.tst);
      // tmp = cotangent of U_i
      (void)hipMemsetAsync(w.tmp, 0, (size_t)B * E * sizeof(float), st);
      vf_vjp(p, w.tst, w.U[i], w.gK[i], w.tmp, w, st);
      // gy += tmp ; gK_j += h a_ij tmp
      Lin one{};
      one.x[0] = w.tmp;
      one.a[0] = 1.0f;
      one.nx = 1;
      hipLaunchKernelGGL(v_lincomb, ge, dim3(256), 0, st, B, E, nullptr, one, w.hcur, w.gyacc, 1);
      for (int j = 0; j < i; ++j)
        if (tab.a[i][j] != 0.f) {
          Lin lc{};
          lc.x[0] = w.tmp;
          lc.a[0] = tab.a[i][j];
          lc.nx = 1;
          lc.scale_h = 1;
          hipLaunchKernelGGL(v_lincomb, ge, dim3(256), 0, st, B, E, nullptr, lc, w.hcur, w.gK[j], 1);
        }
    }
    (void)hipMemcpyAsync(w.lam, w.gyacc, (size_t)B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
    if (s.save_mode == GNCDE_SAVE_STEPS)
      hipLaunchKernelGGL(v_step_row, ge, dim3(256), 0, st, B, E, G, k, gys, w.lam, 1);
  }
  (void)hipMemcpyAsync(gy0, w.lam, (size_t)B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  hipLaunchKernelGGL(v_batch_sum, dim3(cdiv(P, 256)), dim3(256), 0, st, B, P, w.gp, gparams);
  hipLaunchKernelGGL(v_batch_sum, dim3(cdiv((size_t)p.L * GNCDE_FC, 256)), dim3(256), 0, st, B,
                     (size_t)p.L * GNCDE_FC, w.gfc, gfusion);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

}  // namespace gncde
