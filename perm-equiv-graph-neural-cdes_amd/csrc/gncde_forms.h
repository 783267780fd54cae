// The forward forms of one 32 x 32 tile pair of one sample: every layer's (I + Abar_l) straight from the interval's
// four coefficient planes and k_coef_sums' node reductions (fusion: layers.py:102-160, :256-337 via the factored
// table of gncde.h; spline: perm_equiv_graph_vector_field.py:98-102).  Shared by k_abar_direct (gncde_generic.hip)
// and the forms blocks that ride in a hidden-layer launch (gncde_layer.hip).
#pragma once

#include "gncde_internal.h"

namespace gncde {

// Coefficient storage: fp32, or bf16 (GNCDE_COMPUTE_BF16_STORAGE / _BF16_MFMA) widened on load.
__device__ __forceinline__ float coef_at(const float* c, size_t e) { return c[e]; }
__device__ __forceinline__ float coef_at(const uint16_t* c, size_t e) {
  return __builtin_bit_cast(float, (uint32_t)c[e] << 16);
}

__device__ __forceinline__ void abar_store(float* o, size_t e, size_t, float v) { o[e] = v; }
// bf16 pair: hi = rne(v) in the first plane, lo = rne(v - hi) in the second (planes `plane` elements apart);
// hi + lo carries 16 significand bits, so the split products lose ~2^-16, far below the PID tolerances.
__device__ __forceinline__ void abar_store(uint16_t* o, size_t e, size_t plane, float v) {
  const __bf16 h = (__bf16)v;
  o[e] = __builtin_bit_cast(uint16_t, h);
  o[plane + e] = __builtin_bit_cast(uint16_t, (__bf16)(v - (float)h));
}

// csum per (sample, interval): [plane q = d, c, b, a][kind = row sum, column sum, diagonal][n], then the 4 totals.
__host__ __device__ inline size_t csum_stride(int n) { return (size_t)12 * n + 4; }

// a fixed-grid stage time from the grid, with exactly the arithmetic of k_grid_step + the combination (GridTime)
__device__ __forceinline__ float grid_stage_time(const GridTime& gt, int b) {
  const float* g = gt.grid + (size_t)b * gt.G;
  int ns = gt.nsteps[b];
  ns = ns < 0 ? 0 : (ns > gt.G - 1 ? gt.G - 1 : ns);
  const float tc = gt.k < ns ? g[gt.k] : g[ns];
  const float hc = gt.k < ns ? g[gt.k + 1] - g[gt.k] : 0.f;
  return gt.fsal ? (gt.k < ns ? g[gt.k + 1] : g[ns]) : stage_time(tc, gt.c, hc);
}

// LDS of one forms tile block (floats): the fusion table, the four staged tiles, the node vectors, the families
constexpr int kFormsLdsFloats = GNCDE_MAX_LAYERS * GNCDE_FC + 4 * 32 * 33 + 2 * 6 * 32 + GNCDE_MAX_LAYERS * 5 * 32;

// Tile pair `pair` (I <= K of 32 x 32 tiles, row-major over I) of sample b at stage time tb, 256 threads.  The block
// reads the coefficients of tile (I, K) and of its mirror (K, I) once (the two tiles each need the other's transposed
// elements), evaluates A and dA/dt there, and writes both tiles of every layer's (I + Abar_l); the node vectors of
// its two ranges are cubics of k_coef_sums' planes.  Diagonal blocks (I == K) also write q_l = (I + Abar_l) 1 for
// their rows, tg and the CDE data-spline derivative.
template <typename CT, typename OT>
__device__ __forceinline__ void forms_tile(const FormsArgs& fa, int pair, int b, float tb, float* lds) {
  const int n = fa.n, T = fa.T, L = fa.L, de2 = fa.de2, B = fa.B, nt = (n + 31) >> 5;
  const CT* coef = reinterpret_cast<const CT*>(fa.coef);
  OT* out = reinterpret_cast<OT*>(fa.abar);
  const size_t layer_stride = fa.layer_stride;
  float* sF = lds;                                                         // [L][FC]
  float(*tX)[33] = reinterpret_cast<float(*)[33]>(lds + GNCDE_MAX_LAYERS * GNCDE_FC);
  float(*tXd)[33] = tX + 32;
  float(*tY)[33] = tX + 64;
  float(*tYd)[33] = tX + 96;
  float(*sv)[6][32] = reinterpret_cast<float(*)[6][32]>(tX + 128);         // [range][r, rd, c, cd, diag, diag_d][node]
  float(*sW)[2][32] = reinterpret_cast<float(*)[2][32]>(sv + 2);           // [L][range][node]
  float(*sV)[2][32] = sW + GNCDE_MAX_LAYERS;
  float(*sU)[32] = reinterpret_cast<float(*)[32]>(sV + GNCDE_MAX_LAYERS);  // [L][node]
  int I = 0, rem = pair;
  while (rem >= nt - I) {
    rem -= nt - I;
    ++I;
  }
  const int K = I + rem;
  const bool dg = I == K;
  const int i0 = I * 32, k0 = K * 32;
  const size_t nn = (size_t)n * n;
  const float* tsb = fa.ts + (size_t)b * T;
  const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;  // 32 x 8
  const int idx = interval_index_wave(tsb, T, tb);
  const float f = tb - tsb[idx], f3 = 3.0f * f;
  const CT* cb = coef + ((size_t)b * (T - 1) + idx) * 4 * nn;
  const float* cs = fa.csum + ((size_t)b * (T - 1) + idx) * csum_stride(n);

  // Every load of the block is issued before the first use (one memory round trip): the thread's elements of
  // tile (I, K) and of the mirror (K, I), rows ty + 8 u; the node-vector planes; the totals.
  float cx[4][4], cy[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int y = ty + 8 * u;
    const bool okx = i0 + y < n && k0 + tx < n, oky = !dg && k0 + y < n && i0 + tx < n;
    const size_t ex = (size_t)(i0 + y) * n + k0 + tx, ey = (size_t)(k0 + y) * n + i0 + tx;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      cx[u][c] = okx ? coef_at(cb, c * nn + ex) : 0.f;
      cy[u][c] = oky ? coef_at(cb, c * nn + ey) : 0.f;
    }
  }
  // node vectors: thread (range r, kind k, node x) for tid < 192 evaluates value and derivative of one reduction
  float pv[4] = {0.f, 0.f, 0.f, 0.f};
  const int vr = tid / 96, vk = (tid / 32) % 3, vx = tid & 31, vnode = (vr ? k0 : i0) + vx;
  if (tid < 192 && vnode < n)
#pragma unroll
    for (int c = 0; c < 4; ++c) pv[c] = cs[(c * 3 + vk) * n + vnode];
  float pt[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) pt[c] = cs[12 * n + c];
  // the fusion table (to LDS) and, in diagonal blocks, the time-channel and data-spline coefficients of the
  // block's rows: the same round trip, not one more after the first barrier
  const float fv = tid < L * GNCDE_FC ? fa.fus[tid] : 0.f;
  float tcv[3] = {0.f, 0.f, 0.f};
  const size_t blk = (size_t)n * de2;
  float* dx = fa.dx;
  const int drows = n - i0 < 32 ? n - i0 : 32, dn = dx ? drows * de2 : 0;
  const float* dc = dx ? fa.data_coef + ((size_t)b * (T - 1) + idx) * 4 * blk + (size_t)i0 * de2 : nullptr;
  float dcv[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
  if (dg) {
    if (tid < 32 && i0 + tid < n) {
      const float* tc = fa.tcoef + ((size_t)b * (T - 1) + idx) * 3 * n + i0 + tid;
      tcv[0] = tc[0];
      tcv[1] = tc[n];
      tcv[2] = tc[2 * n];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + 256 * h;
      if (e < dn) {
        dcv[h][0] = dc[e];
        dcv[h][1] = dc[blk + e];
        dcv[h][2] = dc[2 * blk + e];
      }
    }
  }

  float ax[4], adx[4], ay[4], ady[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int y = ty + 8 * u;
    ax[u] = fmaf(f, fmaf(f, fmaf(f, cx[u][0], cx[u][1]), cx[u][2]), cx[u][3]);
    adx[u] = fmaf(f, fmaf(f3, cx[u][0], 2.0f * cx[u][1]), cx[u][2]);
    ay[u] = fmaf(f, fmaf(f, fmaf(f, cy[u][0], cy[u][1]), cy[u][2]), cy[u][3]);
    ady[u] = fmaf(f, fmaf(f3, cy[u][0], 2.0f * cy[u][1]), cy[u][2]);
    tX[y][tx] = ax[u];
    tXd[y][tx] = adx[u];
    tY[y][tx] = ay[u];
    tYd[y][tx] = ady[u];
  }
  if (tid < 192) {
    sv[vr][2 * vk][vx] = fmaf(f, fmaf(f, fmaf(f, pv[0], pv[1]), pv[2]), pv[3]);
    sv[vr][2 * vk + 1][vx] = fmaf(f, fmaf(f3, pv[0], 2.0f * pv[1]), pv[2]);
  }
  const float s = fmaf(f, fmaf(f, fmaf(f, pt[0], pt[1]), pt[2]), pt[3]);
  const float sd = fmaf(f, fmaf(f3, pt[0], 2.0f * pt[1]), pt[2]);
  if (tid < L * GNCDE_FC) sF[tid] = fv;
  if (dg) {
    if (tid < 32 && i0 + tid < n) fa.tg[(size_t)b * n + i0 + tid] = fmaf(f, fmaf(f3, tcv[0], 2.0f * tcv[1]), tcv[2]);
    float* dxo = dx + (size_t)b * blk + (size_t)i0 * de2;  // CDE wrapper: dX[i][q] at t for the block's rows
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + 256 * h;
      if (e < dn) dxo[e] = fmaf(f, fmaf(f3, dcv[h][0], 2.0f * dcv[h][1]), dcv[h][2]);
    }
    for (int e = tid + 512; e < dn; e += 256) dxo[e] = fmaf(f, fmaf(f3, dc[e], 2.0f * dc[blk + e]), dc[2 * blk + e]);
  }
  __syncthreads();

  // the rank-1 and diagonal families per layer: w_l over the rows, v_l over the columns of each range, u_l on
  // the diagonal (diagonal blocks only)
  for (int e = tid; e < L * 64; e += 256) {
    const int l = e >> 6, r = (e >> 5) & 1, x = e & 31;
    const float* fc = sF + l * GNCDE_FC;
    const float ri = sv[r][0][x], rdi = sv[r][1][x], ci = sv[r][2][x], cdi = sv[r][3][x];
    sW[l][r][x] = fc[GNCDE_FC_WR_A] * ri + fc[GNCDE_FC_WR_DA] * rdi + fc[GNCDE_FC_WC_A] * ci +
                  fc[GNCDE_FC_WC_DA] * cdi + fc[GNCDE_FC_WS_A] * s + fc[GNCDE_FC_WS_DA] * sd;
    sV[l][r][x] = fc[GNCDE_FC_VR_A] * ri + fc[GNCDE_FC_VR_DA] * rdi + fc[GNCDE_FC_VC_A] * ci + fc[GNCDE_FC_VC_DA] * cdi;
    if (r == 0)
      sU[l][x] = fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * sv[0][4][x] + fc[GNCDE_FC_UD_DA] * sv[0][5][x] +
                 fc[GNCDE_FC_UR_A] * ri + fc[GNCDE_FC_UR_DA] * rdi + fc[GNCDE_FC_UC_A] * ci +
                 fc[GNCDE_FC_UC_DA] * cdi + fc[GNCDE_FC_US_A] * s + fc[GNCDE_FC_US_DA] * sd;
  }
  if (dg) {
    const int i = i0 + tid;
    if (tid < 32 && i < n) {
      // q_l[i] = sum_k (I + Abar_l)[i][k]: the dense terms give their row / column sums, the w (row) family n
      // copies, the v (column) family sum_k v_k (sum_k r_k = sum_k c_k = s), the diagonal once.
      const float ri = sv[0][0][tid], rdi = sv[0][1][tid], ci = sv[0][2][tid], cdi = sv[0][3][tid];
      const float dgi = sv[0][4][tid], dgdi = sv[0][5][tid], fn = (float)n;
      if (fa.qrow)
        for (int l = 0; l < L; ++l) {
          const float* fc = sF + l * GNCDE_FC;
          float q = fc[GNCDE_FC_E_A] * ri + fc[GNCDE_FC_E_DA] * rdi + fc[GNCDE_FC_ET_A] * ci + fc[GNCDE_FC_ET_DA] * cdi;
          q += fn * (fc[GNCDE_FC_WR_A] * ri + fc[GNCDE_FC_WR_DA] * rdi + fc[GNCDE_FC_WC_A] * ci +
                     fc[GNCDE_FC_WC_DA] * cdi + fc[GNCDE_FC_WS_A] * s + fc[GNCDE_FC_WS_DA] * sd);
          q += (fc[GNCDE_FC_VR_A] + fc[GNCDE_FC_VC_A]) * s + (fc[GNCDE_FC_VR_DA] + fc[GNCDE_FC_VC_DA]) * sd;
          q += fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * dgi + fc[GNCDE_FC_UD_DA] * dgdi + fc[GNCDE_FC_UR_A] * ri +
               fc[GNCDE_FC_UR_DA] * rdi + fc[GNCDE_FC_UC_A] * ci + fc[GNCDE_FC_UC_DA] * cdi +
               fc[GNCDE_FC_US_A] * s + fc[GNCDE_FC_US_DA] * sd;
          fa.qrow[((size_t)l * B + b) * n + i] = q;
        }
    }
  }
  __syncthreads();
  const float(*sX)[33] = dg ? tX : tY;  // transposed source of tile (I, K)
  const float(*sXd)[33] = dg ? tXd : tYd;
  const size_t plane = (size_t)L * layer_stride;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int y = ty + 8 * u;
    if (i0 + y < n && k0 + tx < n) {  // tile (I, K): element (i0 + y, k0 + tx)
      const float aki = sX[tx][y], dki = sXd[tx][y];
      const size_t e = (size_t)b * nn + (size_t)(i0 + y) * n + k0 + tx;
      for (int l = 0; l < L; ++l) {
        const float* fc = sF + l * GNCDE_FC;
        float v = fc[GNCDE_FC_E_A] * ax[u] + fc[GNCDE_FC_E_DA] * adx[u] + fc[GNCDE_FC_ET_A] * aki +
                  fc[GNCDE_FC_ET_DA] * dki;
        v += sW[l][0][y] + sV[l][1][tx];
        if (dg && y == tx) v += sU[l][y];
        abar_store(out, l * layer_stride + e, plane, v);
      }
    }
    if (!dg && k0 + y < n && i0 + tx < n) {  // mirror tile (K, I): element (k0 + y, i0 + tx)
      const float aik = tX[tx][y], dik = tXd[tx][y];
      const size_t e = (size_t)b * nn + (size_t)(k0 + y) * n + i0 + tx;
      for (int l = 0; l < L; ++l) {
        const float* fc = sF + l * GNCDE_FC;
        float v = fc[GNCDE_FC_E_A] * ay[u] + fc[GNCDE_FC_E_DA] * ady[u] + fc[GNCDE_FC_ET_A] * aik +
                  fc[GNCDE_FC_ET_DA] * dik;
        v += sW[l][1][y] + sV[l][0][tx];
        abar_store(out, l * layer_stride + e, plane, v);
      }
    }
  }
}

}  // namespace gncde
