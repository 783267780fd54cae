// Generic (any n, any layer widths, CDE wrapper, all fusion kinds) multi-kernel path.
//
// One launch per phase of a vector-field evaluation; used for shapes the fused persistent kernel
// (gncde_fused.hip) does not cover and as the second HIP implementation the parity tests compare
// against.  Every kernel is batched over samples on grid.y/grid.z.
//
// Reference semantics: spline (perm_equiv_graph_vector_field.py:98-102), fusion (layers.py:102-160,
// :256-337 via the factored table of gncde.h), ConvLayer (layers.py:36-48), VF epilogue
// (perm_equiv_graph_vector_field.py:122-128), CDE wrapper (cde_wrapper_vector_field.py:19-26).
#include "gncde_internal.h"

namespace gncde {
namespace {

constexpr int kRedStride = 8;  // red[b][q][n]: r, rd, c, cd, diagA, diagdA, {s}, {sd}

// ---- spline: A(t), dA(t), tg(t) -------------------------------------------------------------------
__global__ void k_spline(int n, int T, const float* __restrict__ ts, const float* __restrict__ coef,
                         const float* __restrict__ tcoef, const float* __restrict__ t,
                         float* __restrict__ A, float* __restrict__ dA, float* __restrict__ tg) {
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

// ---- row/col sums, diagonals, totals --------------------------------------------------------------
// grid (B, 4): q = blockIdx.y selects row sums of A / dA (one wave per row, lanes along the row: coalesced;
// these blocks also write the diagonals and the totals) or column sums of A / dA (one thread per column,
// walking down the rows: coalesced across the threads).
__global__ void __launch_bounds__(256) k_reduce(int n, const float* __restrict__ A, const float* __restrict__ dA,
                                                float* __restrict__ red) {
  const int b = blockIdx.x, q = blockIdx.y;
  const size_t nn = (size_t)n * n;
  const float* M = ((q & 1) ? dA : A) + b * nn;
  float* rb = red + (size_t)b * kRedStride * n;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (q >= 2) {
    for (int j = tid; j < n; j += blockDim.x) {
      float c0 = 0.f, c1 = 0.f;
      int k = 0;
      for (; k + 1 < n; k += 2) {
        c0 += M[(size_t)k * n + j];
        c1 += M[(size_t)(k + 1) * n + j];
      }
      if (k < n) c0 += M[(size_t)k * n + j];
      rb[q * n + j] = c0 + c1;
    }
    return;
  }
  __shared__ float part[4];
  float tot = 0.f;
  for (int i = w; i < n; i += 4) {
    const float* row = M + (size_t)i * n;
    float s = 0.f;
    for (int k = lane; k < n; k += 64) s += row[k];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) {
      rb[q * n + i] = s;
      rb[(4 + q) * n + i] = row[i];
    }
    tot += s;
  }
  if (lane == 0) part[w] = tot;
  __syncthreads();
  if (tid == 0) rb[(6 + q) * n] = (part[0] + part[1]) + (part[2] + part[3]);
}

// ---- epilogue: ODE dy = tg * Z; CDE dy[i,m] = tg[i] * sum_{l,k} Z[i,(m*de+l)*2+k] dX[i,l,k] --------
__global__ void k_finalize(int n, int dL, int h, int de, int T, const float* __restrict__ ts,
                           const float* __restrict__ data_coef, const float* __restrict__ t,
                           const float* __restrict__ tg, const float* __restrict__ Z,
                           float* __restrict__ dy) {
  const int b = blockIdx.y;
  const int dout = h > 0 ? h : dL;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)n * dout) return;
  const int i = (int)(e / dout), o = (int)(e % dout);
  const float g = tg[(size_t)b * n + i];
  const float* z = Z + ((size_t)b * n + i) * dL;
  if (h == 0) {
    dy[((size_t)b * n + i) * dout + o] = g * z[o];
    return;
  }
  const float tb = t[b];
  const float* tsb = ts + (size_t)b * T;
  const int idx = interval_index(tsb, T, tb);
  const float f = tb - tsb[idx];
  const size_t blk = (size_t)n * de * 2;
  const float* cb = data_coef + ((size_t)b * (T - 1) + idx) * 4 * blk + (size_t)i * de * 2;
  float acc = 0.f;
  for (int l = 0; l < de; ++l) {
    for (int k = 0; k < 2; ++k) {
      const int q = l * 2 + k;
      const float dX = fmaf(f, fmaf(3.0f * f, cb[q], 2.0f * cb[blk + q]), cb[2 * blk + q]);
      acc = fmaf(g * z[(o * de + l) * 2 + k], dX, acc);
    }
  }
  dy[((size_t)b * n + i) * dout + o] = acc;
}

// ---- solver helpers ---------------------------------------------------------------------------------
// Per-sample step geometry for step k of the host-planned grid.
__global__ void k_grid_step(int B, int G, int k, const float* __restrict__ grid,
                            const int32_t* __restrict__ nsteps, float* __restrict__ tcur,
                            float* __restrict__ hcur) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* g = grid + (size_t)b * G;
  int ns = nsteps[b];
  ns = ns < 0 ? 0 : (ns > G - 1 ? G - 1 : ns);
  if (k < ns) {
    tcur[b] = g[k];
    hcur[b] = g[k + 1] - g[k];
  } else {
    tcur[b] = g[ns];
    hcur[b] = 0.f;
  }
}

__global__ void k_stage_time(int B, float c, const float* __restrict__ tcur,
                             const float* __restrict__ hcur, float* __restrict__ tst) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  tst[b] = stage_time(tcur[b], c, hcur[b]);
}

// out = y + h_b * sum_j a_j K_j   (up to 7 terms; K_j == nullptr terms skipped)
struct Combo {
  const float* K[7];
  float a[7];
  int nk;
};
__global__ void k_combo(int B, size_t E, const float* __restrict__ y, Combo cb,
                        const float* __restrict__ hcur, float* __restrict__ out) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const size_t o = (size_t)b * E + e;
  float s = 0.f;
  for (int j = 0; j < cb.nk; ++j) s = fmaf(cb.a[j], cb.K[j][o], s);
  out[o] = fmaf(hcur[b], s, y[o]);
}

__global__ void k_save_step(int B, size_t E, int G, int k, const float* __restrict__ y,
                            float* __restrict__ ys) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  ys[((size_t)b * G + k) * E + e] = y[(size_t)b * E + e];
}

__global__ void k_grid_stats(int B, int method, const int32_t* __restrict__ nsteps,
                             int32_t* __restrict__ stats) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int ns = nsteps[b];
  stats[b * 4 + GNCDE_STAT_STEPS] = ns;
  stats[b * 4 + GNCDE_STAT_REJECTS] = 0;
  stats[b * 4 + GNCDE_STAT_EVALS] = method == GNCDE_RK4 ? 4 * ns : 1 + 6 * ns;
  stats[b * 4 + GNCDE_STAT_STATUS] = 0;
}

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

struct VfWs {
  float *A, *dA, *red, *tg, *Z0, *Z1, *m, *abar, *wf, *bf, *inv;
};

size_t carve_vf(const GncdeProblem& p, char* ws, VfWs& w) {
  const size_t B = p.B, n = p.n, nn = n * n, D = max_dim(p);
  size_t wsum = 0, bsum = 0;
  for (int l = 0; l < p.L; ++l) {
    wsum += (size_t)p.dims[l] * p.dims[l + 1];
    bsum += (size_t)p.dims[l + 1];
  }
  size_t off = 0;
  auto take = [&](size_t floats) {
    float* ptr = ws ? reinterpret_cast<float*>(ws + off) : nullptr;
    off += align_up(floats * sizeof(float), 256);
    return ptr;
  };
  w.A = take(B * nn);
  w.dA = take(B * nn);
  w.red = take(B * kRedStride * n);
  w.tg = take(B * n);
  w.Z0 = take(B * n * D);
  w.Z1 = take(B * n * D);
  w.m = take(B * n * D);
  w.abar = take(B * nn);
  w.wf = take(wsum);  // W' = W diag(rms_w) per layer, back to back
  w.bf = take(bsum);  // bias' = bias + W rms_b per layer
  w.inv = take(B * n);
  return off;
}

}  // namespace

size_t generic_vf_workspace(const GncdeProblem& p) {
  VfWs w;
  return carve_vf(p, nullptr, w);
}

// One evaluation = spline + reductions, then per layer two MFMA GEMMs (gncde_gemm.hip): the Linear over all
// B*n node rows with RMSNorm folded in, and the per-sample (I + Abar) m with (I + Abar) materialised once.
// Fold every layer's RMSNorm affine into its Linear (once per solve, not per evaluation).
void vf_forms(const GncdeProblem& p, const float* t, float* A, float* dA, float* tg, float* red, hipStream_t st) {
  const int B = p.B, n = p.n;
  const size_t nn = (size_t)n * n;
  hipLaunchKernelGGL(k_spline, dim3(cdiv(nn > (size_t)n ? nn : n, 256), B), dim3(256), 0, st, n, p.T, p.ts, p.coef,
                     p.tcoef, t, A, dA, tg);
  hipLaunchKernelGGL(k_reduce, dim3(B, 4), dim3(256), 0, st, n, A, dA, red);
}

void generic_vf_prepare(const GncdeProblem& p, char* ws, hipStream_t st) {
  VfWs w;
  carve_vf(p, ws, w);
  size_t wo = 0, bo = 0;
  for (int l = 0; l < p.L; ++l) {
    const int din = p.dims[l], dout = p.dims[l + 1];
    const LayerOffsets o = layer_offsets(p, l);
    fold_linear(din, dout, p.params + o.rms_w, p.params + o.rms_b, p.params + o.W, p.params + o.b, w.wf + wo,
                w.bf + bo, st);
    wo += (size_t)din * dout;
    bo += dout;
  }
}

int generic_vf_eval(const GncdeProblem& p, const float* t, const float* y, float* dy, char* ws,
                    hipStream_t st, bool prepared) {
  const int B = p.B, n = p.n;
  const size_t nn = (size_t)n * n;
  VfWs w;
  carve_vf(p, ws, w);
  if (!prepared) generic_vf_prepare(p, ws, st);
  hipLaunchKernelGGL(k_spline, dim3(cdiv(nn > (size_t)n ? nn : n, 256), B), dim3(256), 0, st, n, p.T,
                     p.ts, p.coef, p.tcoef, t, w.A, w.dA, w.tg);
  hipLaunchKernelGGL(k_reduce, dim3(B, 4), dim3(256), 0, st, n, w.A, w.dA, w.red);
  const float* Zin = y;
  float* bufs[2] = {w.Z0, w.Z1};
  size_t wo = 0, bo = 0;
  for (int l = 0; l < p.L; ++l) {
    const int din = p.dims[l], dout = p.dims[l + 1];
    row_inv(B * n, din, Zin, w.inv, st);
    GemmArgs lin{};
    lin.M = B * n;
    lin.N = dout;
    lin.K = din;
    lin.A = Zin;
    lin.lda = din;
    lin.B = w.wf + wo;
    lin.ldb = din;
    lin.C = w.m;
    lin.ldc = dout;
    lin.rowscale = w.inv;
    lin.colbias = w.bf + bo;
    gemm(lin, 1, true, st);
    wo += (size_t)din * dout;
    bo += dout;
    abar_full(B, n, p.fusion + (size_t)l * GNCDE_FC, w.A, w.dA, w.red, kRedStride, w.abar, st);
    float* Zout = bufs[l & 1];
    GemmArgs pr{};
    pr.M = n;
    pr.N = dout;
    pr.K = n;
    pr.A = w.abar;
    pr.lda = n;
    pr.sA = (long)nn;
    pr.B = w.m;
    pr.ldb = dout;
    pr.sB = (long)n * dout;
    pr.C = Zout;
    pr.ldc = dout;
    pr.sC = (long)n * dout;
    pr.relu = l < p.L - 1 ? 1 : 0;
    gemm(pr, B, false, st);
    Zin = Zout;
  }
  const int dout = out_dim(p);
  hipLaunchKernelGGL(k_finalize, dim3(cdiv((size_t)n * dout, 256), B), dim3(256), 0, st, n,
                     p.dims[p.L], p.cde_hidden, p.cde_embed, p.T, p.ts, p.data_coef, t, w.tg, Zin,
                     dy);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

size_t generic_integrate_workspace(const GncdeProblem& p, const GncdeSolver& s) {
  if (s.controller == GNCDE_CTRL_PID) return generic_pid_workspace(p);
  const size_t B = p.B, E = (size_t)p.n * state_dim(p);
  size_t sz = generic_vf_workspace(p);
  sz += 9 * align_up(B * E * 4, 256);  // y, ytmp, K[7]
  sz += 3 * align_up(B * 4, 256);      // tcur, hcur, tstage
  return sz;
}

int generic_integrate(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys,
                      int32_t* stats, char* ws, hipStream_t st) {
  if (s.controller == GNCDE_CTRL_PID) return generic_integrate_pid(p, s, y0, ys, stats, ws, st);
  if (s.controller != GNCDE_CTRL_GRID) return GNCDE_ERR_UNSUPPORTED;
  const int B = p.B;
  const size_t E = (size_t)p.n * state_dim(p);
  char* cur = ws + generic_vf_workspace(p);
  auto take = [&](size_t floats) {
    float* ptr = reinterpret_cast<float*>(cur);
    cur += align_up(floats * sizeof(float), 256);
    return ptr;
  };
  float* y = take(B * E);
  float* yt = take(B * E);
  float* K[7];
  for (int j = 0; j < 7; ++j) K[j] = take(B * E);
  float* tcur = take(B);
  float* hcur = take(B);
  float* tst = take(B);
  const int G = s.grid_len;
  const unsigned gb = cdiv(B, 256);
  const dim3 ge(cdiv(E, 256), B);
  (void)hipMemcpyAsync(y, y0, B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  if (s.save_mode == GNCDE_SAVE_STEPS)
    hipLaunchKernelGGL(k_save_step, ge, dim3(256), 0, st, B, E, G, 0, y, ys);
  generic_vf_prepare(p, ws, st);

  auto eval = [&](float c, const float* yin, float* out) {
    hipLaunchKernelGGL(k_stage_time, dim3(gb), dim3(256), 0, st, B, c, tcur, hcur, tst);
    return generic_vf_eval(p, tst, yin, out, ws, st, true);
  };
  auto combo = [&](std::initializer_list<std::pair<int, float>> terms, float* out) {
    Combo cb{};
    cb.nk = 0;
    for (auto& tr : terms) {
      cb.K[cb.nk] = K[tr.first];
      cb.a[cb.nk] = tr.second;
      cb.nk++;
    }
    hipLaunchKernelGGL(k_combo, ge, dim3(256), 0, st, B, E, y, cb, hcur, out);
  };

  int rc = GNCDE_OK;
  const int steps = G - 1;
  if (s.method == GNCDE_RK4) {
    for (int k = 0; k < steps && rc == GNCDE_OK; ++k) {
      hipLaunchKernelGGL(k_grid_step, dim3(gb), dim3(256), 0, st, B, G, k, s.grid, s.nsteps, tcur, hcur);
      rc |= eval(0.0f, y, K[0]);
      combo({{0, 0.5f}}, yt);
      rc |= eval(0.5f, yt, K[1]);
      combo({{1, 0.5f}}, yt);
      rc |= eval(0.5f, yt, K[2]);
      combo({{2, 1.0f}}, yt);
      rc |= eval(1.0f, yt, K[3]);
      // y + h/6 (k1 + 2k2 + 2k3 + k4)
      combo({{0, 1.0f / 6.0f}, {1, 2.0f / 6.0f}, {2, 2.0f / 6.0f}, {3, 1.0f / 6.0f}}, yt);
      (void)hipMemcpyAsync(y, yt, B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
      if (s.save_mode == GNCDE_SAVE_STEPS)
        hipLaunchKernelGGL(k_save_step, ge, dim3(256), 0, st, B, E, G, k + 1, y, ys);
    }
  } else {  // Tsit5 on the grid (ConstantStepSize), FSAL
    hipLaunchKernelGGL(k_grid_step, dim3(gb), dim3(256), 0, st, B, G, 0, s.grid, s.nsteps, tcur, hcur);
    rc |= eval(0.0f, y, K[0]);
    for (int k = 0; k < steps && rc == GNCDE_OK; ++k) {
      hipLaunchKernelGGL(k_grid_step, dim3(gb), dim3(256), 0, st, B, G, k, s.grid, s.nsteps, tcur, hcur);
      combo({{0, TSIT5_A21}}, yt);
      rc |= eval(TSIT5_C2, yt, K[1]);
      combo({{0, TSIT5_A31}, {1, TSIT5_A32}}, yt);
      rc |= eval(TSIT5_C3, yt, K[2]);
      combo({{0, TSIT5_A41}, {1, TSIT5_A42}, {2, TSIT5_A43}}, yt);
      rc |= eval(TSIT5_C4, yt, K[3]);
      combo({{0, TSIT5_A51}, {1, TSIT5_A52}, {2, TSIT5_A53}, {3, TSIT5_A54}}, yt);
      rc |= eval(TSIT5_C5, yt, K[4]);
      combo({{0, TSIT5_A61}, {1, TSIT5_A62}, {2, TSIT5_A63}, {3, TSIT5_A64}, {4, TSIT5_A65}}, yt);
      rc |= eval(1.0f, yt, K[5]);
      combo({{0, TSIT5_B1}, {1, TSIT5_B2}, {2, TSIT5_B3}, {3, TSIT5_B4}, {4, TSIT5_B5}, {5, TSIT5_B6}},
            yt);
      rc |= eval(1.0f, yt, K[6]);
      (void)hipMemcpyAsync(y, yt, B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
      (void)hipMemcpyAsync(K[0], K[6], B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
      if (s.save_mode == GNCDE_SAVE_STEPS)
        hipLaunchKernelGGL(k_save_step, ge, dim3(256), 0, st, B, E, G, k + 1, y, ys);
    }
  }
  if (s.save_mode == GNCDE_SAVE_T1)
    (void)hipMemcpyAsync(ys, y, B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  if (stats) hipLaunchKernelGGL(k_grid_stats, dim3(gb), dim3(256), 0, st, B, s.method, s.nsteps, stats);
  if (hipGetLastError() != hipSuccess) return GNCDE_ERR_HIP;
  return rc;
}

}  // namespace gncde
