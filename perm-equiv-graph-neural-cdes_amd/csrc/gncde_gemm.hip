// Batched fp32 MFMA GEMM + the small kernels that turn the generic vector field into two GEMMs per layer:
//
//   m      = inv_row * (Z  W'^T) + bias'      (Linear with RMSNorm folded: W' = W diag(rms_w),
//                                              bias' = bias + W rms_b; one GEMM over all B*n node rows)
//   Z_next = act((I + Abar)  m)               (per-sample GEMM; (I + Abar) materialised once per layer)
//
// This is what makes the wide CDE-wrapper layers of configs 3 / 5 (d_L = 1024 / 512, MFMA-bound, SURVEY
// §8d) run on the matrix cores instead of scalar FMAs.  The GEMM is a 64x64-tile, K-chunk-32 LDS kernel on
// v_mfma_f32_16x16x4f32 (each wave a 32x32 sub-tile, 4 independent accumulators) whose next chunk is
// prefetched into registers while the current one is consumed; bounds are zero-filled so any M, N, K
// (n = 129, 255 ...) works.
#include "gncde_internal.h"

namespace gncde {

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <bool TRANS_A, bool TRANS_B>
__global__ void __launch_bounds__(256) k_gemm(GemmArgs g) {
  constexpr int KC = 32;
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const float* A = g.A + (size_t)b * g.sA;
  const float* B = g.B + (size_t)b * g.sB;
  float* C = g.C + (size_t)b * g.sC;
  __shared__ float As[64][KC + 1];  // As[r][k]
  __shared__ float Bs[KC][68];      // Bs[k][j]
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  // which of the wave's 16x16 sub-tiles hold any valid row / column (padding tiles skip their MFMAs)
  const bool mi0 = m0 + wm < g.M, mi1 = m0 + wm + 16 < g.M;
  const bool nj0 = n0 + wn < g.N, nj1 = n0 + wn + 16 < g.N;
  floatx4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // Per-thread slices of the next chunk (prefetched into registers while the current one is consumed), laid out
  // so that consecutive lanes read consecutive addresses (coalesced 128-256 B per row per instruction):
  //   A row-major (A[r][k]):  r = tid/32 + 8q,  k = tid%32          TRANS_A (At[k][r]): k = tid/64 + 4q, r = tid%64
  //   B row-major (B[k][j]):  k = tid/64 + 4q,  j = tid%64          TRANS_B (Bt[j][k]): j = tid/32 + 8q, k = tid%32
  float ra[8], rb[8];
  float ss = 0.f;  // rownorm: sum of squares of this thread's A elements (row tid/32 + 8q)
  float ssq[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) ssq[q] = 0.f;
  auto fetch = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (TRANS_A) {
        const int kk = k0 + (tid >> 6) + 4 * q, r = m0 + (tid & 63);
        ra[q] = (r < g.M && kk < g.K) ? A[(size_t)kk * g.lda + r] : 0.f;
      } else {
        const int r = m0 + (tid >> 5) + 8 * q, kk = k0 + (tid & 31);
        ra[q] = (r < g.M && kk < g.K) ? A[(size_t)r * g.lda + kk] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (TRANS_B) {
        const int j = n0 + (tid >> 5) + 8 * q, kk = k0 + (tid & 31);
        rb[q] = (j < g.N && kk < g.K) ? B[(size_t)j * g.ldb + kk] : 0.f;
      } else {
        const int kk = k0 + (tid >> 6) + 4 * q, j = n0 + (tid & 63);
        rb[q] = (kk < g.K && j < g.N) ? B[(size_t)kk * g.ldb + j] : 0.f;
        if (g.kscale && kk < g.K) rb[q] *= g.kscale[(size_t)b * g.sK + kk];
      }
    }
    if (!TRANS_A && g.rownorm)
#pragma unroll
      for (int q = 0; q < 8; ++q) ssq[q] = fmaf(ra[q], ra[q], ssq[q]);
  };
  fetch(0);
  for (int k0 = 0; k0 < g.K; k0 += KC) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (TRANS_A)
        As[tid & 63][(tid >> 6) + 4 * q] = ra[q];
      else
        As[(tid >> 5) + 8 * q][tid & 31] = ra[q];
      if (TRANS_B)
        Bs[tid & 31][(tid >> 5) + 8 * q] = rb[q];
      else
        Bs[(tid >> 6) + 4 * q][tid & 63] = rb[q];
    }
    __syncthreads();
    const int ksteps = (g.K - k0 >= KC) ? KC / 4 : (g.K - k0 + 3) / 4;  // the K tail skips its zero steps
    if (k0 + KC < g.K) fetch(k0 + KC);
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      if (kk < ksteps) {
        float av[2], bv[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          av[t] = As[wm + 16 * t + lo][4 * kk + hi];
          bv[t] = Bs[4 * kk + hi][wn + 16 * t + lo];
        }
        if (mi0 && nj0) acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], acc[0][0], 0, 0, 0);
        if (mi0 && nj1) acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[1], acc[0][1], 0, 0, 0);
        if (mi1 && nj0) acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[0], acc[1][0], 0, 0, 0);
        if (mi1 && nj1) acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], acc[1][1], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  __shared__ float sInv[64];
  if (!TRANS_A && g.rownorm) {  // RMSNorm's 1/rms of the A rows (the whole row is this tile's K range)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float v = ssq[q];
      for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);  // the 32 lanes of row tid/32 + 8q
      if ((tid & 31) == 0) {
        const int r = (tid >> 5) + 8 * q;
        const float iv = rms_inv(v, 1.0f / (float)g.K);
        sInv[r] = iv;
        if (g.inv_out && blockIdx.x == 0 && m0 + r < g.M) g.inv_out[(size_t)b * g.sR + m0 + r] = iv;
      }
    }
    __syncthreads();
  }
  (void)ss;
  if (!TRANS_A && g.cde_out) {  // CDE contraction: one 16x16 tile = 16 rows x one hidden channel's 16 columns
    const int hch = g.N / 16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + 4 * hi + r;
        const size_t grow = (size_t)b * g.M + (row < g.M ? row : 0);
        const float dX = g.cde_dx[grow * 16 + lo];
        const float qb = g.biasrow ? g.biasrow[(size_t)b * g.sR + (row < g.M ? row : 0)] : 1.0f;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v = acc[i][j][r];
          if (g.colbias) {
            const int col = n0 + wn + 16 * j + lo;
            v = fmaf(qb, col < g.N ? g.colbias[col] : 0.f, v);
          }
          v *= dX;
          v += __shfl_xor(v, 8);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 1);
          const int ch = (n0 + wn + 16 * j) / 16;
          if (lo == 0 && row < g.M && ch < hch) g.cde_out[grow * hch + ch] = g.cde_tg[grow] * v;
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + 4 * hi + r, col = n0 + wn + 16 * j + lo;
        if (row < g.M && col < g.N) {
          float v = acc[i][j][r];
          if (!TRANS_A && g.rownorm) v *= sInv[row - m0];
          if (g.colbias) v = g.biasrow ? fmaf(g.biasrow[(size_t)b * g.sR + row], g.colbias[col], v) : v + g.colbias[col];
          if (g.rowscale) v *= g.rowscale[(size_t)b * g.sR + row];
          if (g.relu) v = fmaxf(v, 0.f);
          if (g.accumulate) v += C[(size_t)row * g.ldc + col];
          C[(size_t)row * g.ldc + col] = v;
        }
      }
}

// Four consecutive K values p[0..3] of one row (the lane's 4 MFMA K steps of a 16-chunk): one dwordx4 when the row
// is 16-byte aligned and the chunk is inside K, else four guarded scalars.
__device__ __forceinline__ floatx4 load_k4(const float* p, bool vec, int k, int K) {
  if (vec) return *reinterpret_cast<const floatx4*>(p);
  floatx4 v;
#pragma unroll
  for (int s = 0; s < 4; ++s) v[s] = k + s < K ? p[s] : 0.f;
  return v;
}

// Fixed-order reduction of the four waves' K partials of a 32-row x 16*NB-column block, then the GEMM epilogue;
// wave w finishes tiles (t, j) with (t * NB + j) % 4 == w.  ss: per-lane rownorm partials (row lo of each t).
template <int NB>
__device__ __forceinline__ void finish_split_k(const GemmArgs& g, const floatx4 (&acc)[2][NB], const float (&ss)[2],
                                               int b, int m0, int n0, int w, int lane) {
  const int tid = threadIdx.x, lo = lane & 15, hi = lane >> 4;
  float* C = g.C + (size_t)b * g.sC;
  __shared__ floatx4 red[4][2 * NB][64];
  __shared__ float sInv[32];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < NB; ++j) red[w][t * NB + j][lane] = acc[t][j];
  if (g.rownorm) {
    __shared__ float sSS[4][2][64];
    sSS[w][0][lane] = ss[0];
    sSS[w][1][lane] = ss[1];
    __syncthreads();
    if (tid < 32) {  // row tid: its 4 lanes (hi) of each of the 4 waves
      const int t = tid >> 4, l16 = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww)
#pragma unroll
        for (int h4 = 0; h4 < 4; ++h4) v += sSS[ww][t][l16 + 16 * h4];
      const float iv = rms_inv(v, 1.0f / (float)g.K);
      sInv[tid] = iv;
      if (g.inv_out && n0 == 0 && m0 + tid < g.M) g.inv_out[(size_t)b * g.sR + m0 + tid] = iv;
    }
  }
  __syncthreads();
  const int hch = g.N / 16;
  for (int tile = w; tile < 2 * NB; tile += 4) {
    const int t = tile / NB, j = tile % NB;
    floatx4 v4 = red[0][tile][lane];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) {
      const floatx4 o = red[ww][tile][lane];
      v4 = floatx4{v4[0] + o[0], v4[1] + o[1], v4[2] + o[2], v4[3] + o[3]};
    }
    const int col = n0 + 16 * j + lo;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = 16 * t + 4 * hi + r, row = m0 + rl;
      const bool rok = row < g.M;
      const size_t rsafe = rok ? row : 0;
      float v = v4[r];
      if (g.rownorm) v *= sInv[rl];
      if (g.colbias && col < g.N)
        v = g.biasrow ? fmaf(g.biasrow[(size_t)b * g.sR + rsafe], g.colbias[col], v) : v + g.colbias[col];
      if (g.cde_out) {  // one 16-column tile = one hidden channel (de = 8)
        const size_t grow = (size_t)b * g.M + rsafe;
        v *= g.cde_dx[grow * 16 + lo];
        v += __shfl_xor(v, 8);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 1);
        const int ch = (n0 + 16 * j) / 16;
        if (lo == 0 && rok && ch < hch) g.cde_out[grow * hch + ch] = g.cde_tg[grow] * v;
        continue;
      }
      if (!rok || col >= g.N) continue;
      if (g.rowscale) v *= g.rowscale[(size_t)b * g.sR + row];
      if (g.relu) v = fmaxf(v, 0.f);
      if (g.accumulate) v += C[(size_t)row * g.ldc + col];
      C[(size_t)row * g.ldc + col] = v;
    }
  }
}

// ---- narrow GEMM (N <= 64): 32-row blocks, K split over the 4 waves ---------------------------------------
// The n x n products of the narrow layers (N = d <= 64, K = n = 129 / 255) and the Linears of width <= 64 are
// latency-bound on the 64x64 kernel: few workgroups and a serial K loop of one HBM round trip per 32-chunk.
// Here a workgroup owns 32 rows x N columns; wave w takes the 16-wide K chunks w, w+4, ... and issues every load
// of its round (up to 4 chunks = 64 K per wave, 256 per workgroup) before the first MFMA, straight into the MFMA
// operand layout (MFMA step s of a chunk at k0: lane (lo, hi) holds A[row lo][k0 + 4hi + s] and
// B[k0 + 4hi + s][col lo], so a lane's four steps are one dwordx4 of an A row; no LDS staging).  The four K
// partials meet once in LDS, summed in a fixed order.
template <bool TRANS_B, int NB>
__global__ void __launch_bounds__(256) k_gemm_narrow(GemmArgs g) {
  constexpr int CPW = 4;  // chunks (16 K) per wave per round
  const int b = blockIdx.z;
  const int m0 = blockIdx.x * 32;
  const float* A = g.A + (size_t)b * g.sA;
  const float* B = g.B + (size_t)b * g.sB;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  floatx4 acc[2][NB];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[t][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float ss[2] = {0.f, 0.f};  // rownorm: this lane's share of sum_k A[row][k]^2
  const int rowA0 = m0 + lo, rowA1 = m0 + 16 + lo;
  const bool avec = ((g.lda | g.sA) & 3) == 0 && ((uintptr_t)g.A & 15) == 0;
  const bool bvec = TRANS_B && ((g.ldb | g.sB) & 3) == 0 && ((uintptr_t)g.B & 15) == 0;
  for (int kr = 0; kr < g.K; kr += 4 * 16 * CPW) {
    floatx4 av[CPW][2], bv[CPW][NB];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int k = kr + 16 * (w + 4 * c) + 4 * hi;  // this lane's K steps k .. k+3 of chunk c
      const bool kfull = k + 4 <= g.K;
      av[c][0] = rowA0 < g.M ? load_k4(A + (size_t)rowA0 * g.lda + k, avec && kfull, k, g.K) : floatx4{0.f, 0.f, 0.f, 0.f};
      av[c][1] = rowA1 < g.M ? load_k4(A + (size_t)rowA1 * g.lda + k, avec && kfull, k, g.K) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int col = 16 * j + lo;
        floatx4 v = {0.f, 0.f, 0.f, 0.f};
        if (col < g.N) {
          if (TRANS_B) {
            v = load_k4(B + (size_t)col * g.ldb + k, bvec && kfull, k, g.K);
          } else {
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) v[s4] = k + s4 < g.K ? B[(size_t)(k + s4) * g.ldb + col] : 0.f;
          }
        }
        if (g.kscale)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) v[s4] *= k + s4 < g.K ? g.kscale[(size_t)b * g.sK + k + s4] : 0.f;
        bv[c][j] = v;
      }
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        if (g.rownorm) {
          ss[0] = fmaf(av[c][0][s4], av[c][0][s4], ss[0]);
          ss[1] = fmaf(av[c][1][s4], av[c][1][s4], ss[1]);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < NB; ++j)
            acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[c][t][s4], bv[c][j][s4], acc[t][j], 0, 0, 0);
      }
  }
  finish_split_k<NB>(g, acc, ss, b, m0, 0, w, lane);
}

// ---- bf16 n x n products (GNCDE_COMPUTE_BF16*): C = A B on v_mfma_f32_16x16x32_bf16 -------------------------
// A = (I + Abar) as bf16 (hi, lo) planes, B = the fp32 state split on load into hi = rne(x), lo = rne(x - hi);
// C accumulates Ahi Bhi + Ahi Blo + Alo Bhi in fp32 (the dropped lo*lo term and the split residuals are ~2^-16
// relative: the adaptive controller's error estimate does not see bf16 rounding noise).  Same split-K
// organisation as the narrow kernel: a 32-deep chunk is one MFMA step per product, lane (lo, hi) holding
// A[row lo][k0 + 8hi .. +7] (one 16-byte load per plane) and B[k0 + 8hi .. +7][col lo]; grid.y walks 16*NB-column
// blocks so any N works.  fp32 epilogue.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 load_a8(const uint16_t* pa, bool vec, int k, int K) {
  uint4 raw;
  if (vec) {
    raw = *reinterpret_cast<const uint4*>(pa);
  } else {
    uint16_t e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) e[q] = k + q < K ? pa[q] : (uint16_t)0;
    raw = uint4{e[0] | ((uint32_t)e[1] << 16), e[2] | ((uint32_t)e[3] << 16), e[4] | ((uint32_t)e[5] << 16),
                e[6] | ((uint32_t)e[7] << 16)};
  }
  return __builtin_bit_cast(bf16x8, raw);
}

template <int NB>
__global__ void __launch_bounds__(256) k_gemm_bf16(GemmArgs g) {
  constexpr int CPW = 2;  // 32-deep chunks per wave per round
  const int b = blockIdx.z;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 16 * NB;
  const uint16_t* A = reinterpret_cast<const uint16_t*>(g.A) + (size_t)b * g.sA;
  const float* B = g.B + (size_t)b * g.sB;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  floatx4 acc[2][NB];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[t][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const bool avec = ((g.lda | g.sA | g.a_lo) & 7) == 0 && ((uintptr_t)g.A & 15) == 0;
  for (int kr = 0; kr < g.K; kr += 4 * 32 * CPW) {
    bf16x8 ah[CPW][2], al[CPW][2], bh[CPW][NB], bl[CPW][NB];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int k = kr + 32 * (w + 4 * c) + 8 * hi;  // this lane's 8 K values
      const bool vec = avec && k + 8 <= g.K;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int row = m0 + 16 * t + lo;
        if (row < g.M) {
          const uint16_t* pa = A + (size_t)row * g.lda + k;
          ah[c][t] = load_a8(pa, vec, k, g.K);
          al[c][t] = load_a8(pa + g.a_lo, vec, k, g.K);
        } else {
          ah[c][t] = al[c][t] = __builtin_bit_cast(bf16x8, uint4{0u, 0u, 0u, 0u});
        }
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int col = n0 + 16 * j + lo;
        bf16x8 vh, vl;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float x = 0.f;
          if (k + q < g.K && col < g.N) {
            x = B[(size_t)(k + q) * g.ldb + col];
            if (g.kscale) x *= g.kscale[(size_t)b * g.sK + k + q];
          }
          vh[q] = (__bf16)x;
          vl[q] = (__bf16)(x - (float)vh[q]);
        }
        bh[c][j] = vh;
        bl[c][j] = vl;
      }
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[c][t], bh[c][j], acc[t][j], 0, 0, 0);
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c][t], bl[c][j], acc[t][j], 0, 0, 0);
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c][t], bh[c][j], acc[t][j], 0, 0, 0);
        }
  }
  const float ss[2] = {0.f, 0.f};
  finish_split_k<NB>(g, acc, ss, b, m0, n0, w, lane);
}

__global__ void k_fold(int din, int dout, const float* __restrict__ rw, const float* __restrict__ rb,
                       const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ Wf,
                       float* __restrict__ bf) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < dout * din) {
    const int k = e % din;
    Wf[e] = W[e] * rw[k];
  }
  if (e < dout) {
    float acc = bias[e];
    for (int k = 0; k < din; ++k) acc = fmaf(W[(size_t)e * din + k], rb[k], acc);
    bf[e] = acc;
  }
}

// inv[r] = rsqrt(mean(Z[r]^2) + eps), one wave per row
__global__ void k_row_inv(int rows, int d, const float* __restrict__ Z, float* __restrict__ inv) {
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* z = Z + (size_t)r * d;
  float ss = 0.f;
  for (int k = lane; k < d; k += 64) ss = fmaf(z[k], z[k], ss);
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  if (lane == 0) inv[r] = rms_inv(ss, 1.0f / (float)d);
}

}  // namespace

void gemm(const GemmArgs& g, int batch, bool trans_b, hipStream_t st, bool trans_a) {
  if (g.a_bf16) {  // (I + Abar) in bf16 times the fp32 state: NN only
    const int nb = g.N <= 16 ? 1 : (g.N <= 32 ? 2 : 4);
    const dim3 gb((g.M + 31) / 32, (g.N + 16 * nb - 1) / (16 * nb), batch);
    if (nb == 1)
      hipLaunchKernelGGL((k_gemm_bf16<1>), gb, dim3(256), 0, st, g);
    else if (nb == 2)
      hipLaunchKernelGGL((k_gemm_bf16<2>), gb, dim3(256), 0, st, g);
    else
      hipLaunchKernelGGL((k_gemm_bf16<4>), gb, dim3(256), 0, st, g);
    return;
  }
  if (!trans_a && g.N <= 64) {
    const dim3 gn((g.M + 31) / 32, 1, batch);
    const int nb = (g.N + 15) / 16;
#define GNCDE_NARROW(NB)                                                                                 \
  if (nb == NB) {                                                                                        \
    if (trans_b)                                                                                         \
      hipLaunchKernelGGL((k_gemm_narrow<true, NB>), gn, dim3(256), 0, st, g);                            \
    else                                                                                                 \
      hipLaunchKernelGGL((k_gemm_narrow<false, NB>), gn, dim3(256), 0, st, g);                           \
    return;                                                                                              \
  }
    GNCDE_NARROW(1)
    GNCDE_NARROW(2)
    GNCDE_NARROW(3)
    GNCDE_NARROW(4)
#undef GNCDE_NARROW
  }
  const dim3 grid((g.N + 63) / 64, (g.M + 63) / 64, batch);
  if (trans_a) {
    if (trans_b)
      hipLaunchKernelGGL((k_gemm<true, true>), grid, dim3(256), 0, st, g);
    else
      hipLaunchKernelGGL((k_gemm<true, false>), grid, dim3(256), 0, st, g);
  } else {
    if (trans_b)
      hipLaunchKernelGGL((k_gemm<false, true>), grid, dim3(256), 0, st, g);
    else
      hipLaunchKernelGGL((k_gemm<false, false>), grid, dim3(256), 0, st, g);
  }
}

void fold_linear(int din, int dout, const float* rw, const float* rb, const float* W, const float* bias, float* Wf,
                 float* bf, hipStream_t st) {
  const int tot = din * dout > dout ? din * dout : dout;
  hipLaunchKernelGGL(k_fold, dim3((tot + 255) / 256), dim3(256), 0, st, din, dout, rw, rb, W, bias, Wf, bf);
}

void row_inv(int rows, int d, const float* Z, float* inv, hipStream_t st) {
  hipLaunchKernelGGL(k_row_inv, dim3((rows + 3) / 4), dim3(256), 0, st, rows, d, Z, inv);
}


}  // namespace gncde
