// One fused launch per ConvLayer for the generic (multi-kernel) vector field — configs 3 / 5 and every shape the
// persistent kernel does not take (layers.py:36-48, ConvEquivFusionLayer.__call__ layers.py:162-177):
//
//   Z_next[R, :] = act( ((I + Abar) diag(inv) Z)[R, :] W'^T + q[R] b'^T )
//
// in the reassociated order: W' = W diag(rms_w), b' = b + W rms_b (RMSNorm's affine folded, once per solve),
// inv = the RMSNorm factor of each node row, q = (I + Abar) 1.  A workgroup owns 32 node rows R of one sample, so
// nothing crosses workgroups inside a layer (the Linear-first order needs every row of m before the n x n product):
//
//   1. Z[b] (n x d_in, HBM/L2) -> LDS with every load of a round in flight; each row's RMSNorm factor from LDS.
//   2. P = (I + Abar)[R, :] diag(inv) Zs on v_mfma_f32_16x16x4f32: A operand = rows R of (I + Abar) straight from
//      HBM/L2 (one dwordx4 per lane per 16-deep K chunk, K permuted so a lane's 4 steps are 4 consecutive columns)
//      scaled by inv, B operand = Zs from LDS; the K range split over the four waves (each element loaded once per
//      workgroup), the partials summed in LDS in a fixed order.  bf16 modes: v_mfma_f32_16x16x32_bf16 on the
//      (hi, lo) planes of (I + Abar) against diag(inv) Zs split into (hi, lo) on the fly (three products).
//   3. Z_next[R, :] = P W'^T on MFMA (P from LDS, W' pre-permuted into the lane order: one coalesced 1 KB load per
//      wave per operand), epilogue q b'^T + ReLU, or tg * (.) for the ODE output layer.
//   3'. The CDE-wrapper output layer (cde_wrapper_vector_field.py:19-26, de = 8) never forms the n x h*16 read-out:
//      dZ[i, m] = tg_i sum_{c, j} P[i, c] dX[i, j] W'[16 m + j, c] + tg_i q_i sum_j b'[16 m + j] dX[i, j]
//      is one GEMM with K = (j, c) whose A operand P[i, c] dX[i, j] is formed in registers (one multiply per MFMA
//      step), so the 16-column contraction happens inside the MFMA accumulation.
//
// This replaces, per layer, two GEMM launches, the row-norm kernel and the read-out's 16-lane shuffle epilogue.
#include "gncde_forms.h"
#include "gncde_internal.h"

#include <type_traits>

namespace gncde {

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx4u __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned rows (n = 129, 255)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x8u __attribute__((ext_vector_type(8), aligned(2)));  // 8 bf16 of an (I + Abar) plane row

constexpr int kTiles = 2;  // 16-row MFMA tiles per workgroup (hidden / ODE output layers; the CDE read-out picks 2 or 5)
constexpr int kSplit = 2;  // CDE read-out: workgroups per row block (channel groups)
constexpr int kDxS = 20;   // row stride of the read-out's dX rows in LDS: 16-byte rows, 16 rows on 16 distinct banks

struct LayerArgs {
  int n;
  const float* abar;   // (I + Abar_l) [B, n, n]
  const uint16_t* abar16;  // bf16 modes: its hi plane [B, n, n] (lo plane a_lo elements later)
  long a_lo;
  const float* Z;      // [B, n, DIN]
  const float* wperm;  // W' in the lane order of the kernel (permute_linear)
  const float* bf;     // b' [DOUT] (CDE: [16 H])
  const float* q;      // q_l [B, n]
  float* out;          // [B, n, DOUT] (CDE: dy [B, n, H])
  const float* tg;     // [B n] time-channel derivative (MODE 1, 2)
  const float* dx;     // [B n, 16] data-spline derivative (MODE 2)
  FormsRide ride;      // fp32 hidden layers: the next evaluation's forms as the grid's z >= 1 workgroups
  // fp32 CDE read-out (post.blocks != 0): the stage combination that follows this evaluation, folded into the
  // epilogue.  Its last term is this launch's own output; every thread sums its elements' earlier terms (the same
  // fmaf order as k_combo) from loads issued right after its K loop, then adds the output read back from LDS.
  PendingCombo post;
};

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int DIN>
__host__ __device__ constexpr int zs_stride() {
  return DIN + 4;  // row stride of Zs / Ps: 16-byte rows, hi-groups of a column read 16 banks apart
}

// MODE 0: hidden layer, ReLU.  MODE 1: ODE output layer, out = tg * Z_next.  MODE 2: CDE output layer (DOUT = h).
// NT: 16-row tiles per workgroup.  The CDE read-out's MFMA chain (K = 16 h per output) dominates its launch, and with
// NT = 2 config 3's 640 workgroups were 2.5 per CU: the CUs holding three ran 3 x (P product + read-out) MFMA chains,
// every workgroup staged its sample's whole Z first, and no staging overlapped an MFMA chain.  With NT = 5 (when the
// batch still gives every CU a workgroup) config 3 is 256 workgroups, one per CU, each staging Z once for 5 tiles.
// BF: the n x n product on v_mfma_f32_16x16x32_bf16 (GNCDE_COMPUTE_BF16*): (I + Abar) from its bf16 (hi, lo) planes,
// diag(inv) Z split into (hi, lo) on the fly, three products (hi hi, hi lo, lo hi) with fp32 accumulation.
// Phase stamps of the fp32 CDE read-out launch (diagnostic build -DGNCDE_LAYER_STAMPS only: tools/diag_layer_stamps.py):
// the first wave of every workgroup records s_memrealtime at 7 points of the last such launch.
#ifdef GNCDE_LAYER_STAMPS
__device__ unsigned long long g_layer_stamps[1024 * 8];
#define LAYER_STAMP(k)                                                                                              \
  do {                                                                                                              \
    const int wg_ = blockIdx.x + gridDim.x * blockIdx.y;                                                            \
    if (MODE == 2 && !BF && threadIdx.x == 0 && wg_ < 1024) g_layer_stamps[wg_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LAYER_STAMP(k) do {} while (0)
#endif

// Wave count: 4, or 8 for the five-tile CDE read-out with two channel tiles per workgroup (config 3's h = 64): one
// workgroup per CU then has two waves per SIMD, so one wave's operand formation and waits run under the other's
// MFMAs.  The product's K parts and the read-out's j quarters keep one summation order for every wave count.
template <int DOUT, int MODE, bool BF, int NT>
constexpr int layer_waves() {
  return (MODE == 2 && !BF && NT > 2 && DOUT / 16 / ((DOUT / 16 >= kSplit) ? kSplit : 1) == 2) ? 8 : 4;
}

template <int DIN, int DOUT, int MODE, bool BF, int NT>
__global__ void __launch_bounds__((64 * layer_waves<DOUT, MODE, BF, NT>()), (NT > 2 ? 1 : 2)) k_layer(LayerArgs a) {
  static_assert(MODE == 2 || NT == 2, "the Linear epilogue's tile split assumes two row tiles");
  static_assert(!BF || NT == 2, "bf16 modes: two row tiles");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (blockIdx.z) {  // a block riding in this launch (FormsRide; 256 threads): the next evaluation's forms, then
                     // the partial sums of the following read-out's stage combination
    if constexpr (MODE == 0 && !BF && NT == 2) {
      const unsigned fb = (blockIdx.z - 1) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
      if (fb < a.ride.blocks) {
        const int nt = (a.n + 31) >> 5, np = nt * (nt + 1) / 2, b = a.ride.b0 + (int)fb / np;
        forms_tile<float, float>(a.ride.f, (int)fb % np, b, grid_stage_time(a.ride.gt, b), smem);
      } else if (fb - a.ride.blocks < a.ride.pbs * (unsigned)a.ride.nb) {
        const unsigned pb = fb - a.ride.blocks;
        const int b = a.ride.b0 + (int)(pb / a.ride.pbs);
        const size_t e0 = (size_t)(pb % a.ride.pbs) * (kComboThreads * kComboU) + threadIdx.x;
        float kv[6][kComboU];
#pragma unroll
        for (int u = 0; u < kComboU; ++u) {  // every load first (one round trip), then k_combo's summation order
          const size_t e = e0 + (size_t)u * kComboThreads, o = (size_t)b * a.ride.pE + e;
#pragma unroll
          for (int j = 0; j < 6; ++j) kv[j][u] = (e < a.ride.pE && j < a.ride.pnk) ? a.ride.pK[j][o] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kComboU; ++u) {
          const size_t e = e0 + (size_t)u * kComboThreads;
          if (e >= a.ride.pE) break;
          float sp = 0.f;
#pragma unroll
          for (int j = 0; j < 6; ++j)
            if (j < a.ride.pnk) sp = fmaf(a.ride.pa[j], kv[j][u], sp);
          a.ride.part[(size_t)b * a.ride.pE + e] = sp;
        }
      }
    }
    return;
  }
  constexpr int WV = layer_waves<DOUT, MODE, BF, NT>();
  constexpr int NTH = 64 * WV;   // threads
  constexpr int kRows = 16 * NT;
  constexpr int ZS = zs_stride<DIN>();
  constexpr int CTP = DIN / 16;  // product column tiles
  constexpr int KPP = 4;         // product K parts (waves w and w + 4 share one: each takes half the column tiles)
  constexpr int CTW = CTP * 4 / WV;  // product column tiles per wave
  constexpr int NCC = DIN / 16;  // 16-deep K chunks of the Linear
  const int n = a.n;
  const int nk = BF ? (n + 31) & ~31 : (n + 15) & ~15;  // K rows of Zs: whole MFMA K chunks
  floatx4* red = reinterpret_cast<floatx4*>(smem);  // [WV][NT][64] read-out partials (MODE 2)
  float* sDx = smem + WV * NT * 64 * 4;             // [kRows][kDxS] (MODE 2)
  float* Zs = sDx + kRows * kDxS;                   // [nk][ZS] (16-byte aligned)
  float* Ps = Zs;                                   // [KPP][32][ZS] after the product (max(nk, 128) rows reserved)
  float* sInv = Zs + (nk > 4 * kRows ? nk : 4 * kRows) * ZS;  // [nk] RMSNorm factors of the Z rows
  // MODE 2 splits the read-out's channels over kSplit workgroups per row block (each recomputes P: the product is
  // 1/16 of the read-out's MFMA work) so that the grid balances over the 256 CUs.
  constexpr int SPLIT = (MODE == 2 && DOUT / 16 >= kSplit) ? kSplit : 1;
  // (one sample's workgroups on one XCD: they all stage that sample's Z)
  const int wx = xcd_work((int)(blockIdx.x + gridDim.x * blockIdx.y), (int)(gridDim.x * gridDim.y));
  const int bx = wx % (int)gridDim.x;
  const int b = wx / (int)gridDim.x, r0 = (bx / SPLIT) * kRows, ch = bx % SPLIT;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  const int kpp = w & 3, ct0 = (w >> 2) * CTW;  // this wave's product K part and first column tile
  const size_t nb = (size_t)b * n;
  LAYER_STAMP(0);

  const bool two = r0 + 16 < n;  // the second row tile holds a valid row (else its MFMAs are skipped)
  const int ntl = (n - r0 + 15) >> 4 < NT ? (n - r0 + 15) >> 4 : NT;  // tiles holding a valid row
  // f(integral_constant<int, ntl>) (uniform; counts 1..NT, NT <= 5)
  auto with_count = [&](int cnt, auto&& f) __attribute__((always_inline)) {
    if (cnt >= NT) f(std::integral_constant<int, NT>{});
    else if (NT > 4 && cnt == 4) f(std::integral_constant<int, (NT > 4 ? 4 : 1)>{});
    else if (NT > 3 && cnt == 3) f(std::integral_constant<int, (NT > 3 ? 3 : 1)>{});
    else if (NT > 2 && cnt == 2) f(std::integral_constant<int, (NT > 2 ? 2 : 1)>{});
    else f(std::integral_constant<int, 1>{});
  };
  // The fp32 product's first round of (I + Abar) operand loads is issued before Z is staged: the two HBM / L2 round
  // trips overlap instead of following each other (the operand does not depend on Z; diag(inv) is applied later).
  const int nch16 = nk >> 4;
  int ra[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) ra[t] = r0 + 16 * t + lo < n ? r0 + 16 * t + lo : n - 1;
  floatx4 av[4][NT];
  auto load_round = [&](int kr) __attribute__((always_inline)) {
    const float* Ab = a.abar + nb * n;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int kc = kr + 4 * c;
      const int k = 16 * kc + 4 * hi;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float* pa = Ab + (size_t)ra[t] * n + k;
        floatx4 v = {0.f, 0.f, 0.f, 0.f};
        if (kc < nch16 && (NT == 2 || t < ntl)) {
          if (k + 4 <= n) {
            const floatx4u u = *reinterpret_cast<const floatx4u*>(pa);
            v = floatx4{u.x, u.y, u.z, u.w};
          } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) v[s] = k + s < n ? pa[s] : 0.f;
          }
        }
        av[c][t] = v;
      }
    }
  };
  // The Z rows (and the read-out tiles' dX rows) are loaded into registers FIRST and the (I + Abar) rows after them,
  // so the wait for Z (loads complete in issue order) does not include the (I + Abar) round, which lands while Z is
  // stored, normed and the barriers pass (five-tile read-out: staging 5.36 -> 3.90 us)
  constexpr int G4Z = DIN / 4, UZ = 3072 / NTH, UD = (kRows * 16 + NTH - 1) / NTH;
  constexpr bool ZF = !BF;  // (every fp32 launch; the bf16 product splits Z on the fly and keeps the old order)
  const bool zfirst = ZF && nk * G4Z <= NTH * UZ;
  floatx4 zpre[ZF ? UZ : 1];
  float dxpre[ZF && MODE == 2 ? UD : 1];
  if constexpr (ZF) {
    if (zfirst) {
      const floatx4* Z4 = reinterpret_cast<const floatx4*>(a.Z + nb * DIN);
#pragma unroll
      for (int u = 0; u < UZ; ++u) {
        const int e = tid + NTH * u;
        zpre[u] = e < n * G4Z ? Z4[e] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (MODE == 2)
#pragma unroll
        for (int u = 0; u < UD; ++u) {
          const int e = tid + NTH * u, row = e >> 4, R = r0 + row;
          dxpre[u] = e < kRows * 16 && R < n ? a.dx[(nb + R) * 16 + (e & 15)] : 0.f;
        }
    }
  }
  if constexpr (!BF) load_round(kpp);
  // The epilogue's operands (W' B operands of the wave's output tiles, b', q, tg of its rows) do not depend on the
  // product either: issued here, so the tail after the last barrier is MFMA + stores, not two more L2 round trips.
  constexpr int CTO = MODE != 2 ? DOUT / 16 : 1;
  constexpr int NCCE = MODE != 2 ? DIN / 16 : 1;
  floatx4 wpre[2][NCCE];
  float bpre[2], qpre[NT][4], gpre[NT][4];
  if constexpr (MODE != 2) {
    const floatx4* W4p = reinterpret_cast<const floatx4*>(a.wperm);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int tile = w + 4 * tt, rt = tile / CTO, ct = tile % CTO;
      const bool ok = tile < 2 * CTO;
#pragma unroll
      for (int cc = 0; cc < NCCE; ++cc) wpre[tt][cc] = ok ? W4p[(ct * NCCE + cc) * 64 + lane] : floatx4{0.f, 0.f, 0.f, 0.f};
      bpre[tt] = ok ? a.bf[16 * ct + lo] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = r0 + 16 * rt + 4 * hi + r;
        qpre[tt][r] = ok && R < n ? a.q[nb + R] : 0.f;
        gpre[tt][r] = MODE == 1 && ok && R < n ? a.tg[nb + R] : 0.f;
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = r0 + 16 * t + 4 * hi + r;
        qpre[t][r] = R < n ? a.q[nb + R] : 0.f;
        gpre[t][r] = R < n ? a.tg[nb + R] : 0.f;
      }
  }

  // ---- 1. Zs = Z[b] (zero rows up to nk), every load of a round in flight before the first store; then the
  // RMSNorm factor of each row from LDS (diag(inv) is applied to the (I + Abar) operand of the product).
  {
    constexpr int G = DIN / 4;  // float4 per row
    constexpr int U = 8;
    const floatx4* Z4 = reinterpret_cast<const floatx4*>(a.Z + nb * DIN);
    const int tot = nk * G, valid = n * G;
    if (zfirst) {  // stores of the registers loaded first
#pragma unroll
      for (int u = 0; u < (ZF ? UZ : 1); ++u) {
        const int e = tid + NTH * u;
        if (e < tot) *reinterpret_cast<floatx4*>(Zs + (e / G) * ZS + 4 * (e % G)) = zpre[u];
      }
      if constexpr (MODE == 2)
#pragma unroll
        for (int u = 0; u < (ZF ? UD : 1); ++u) {
          const int e = tid + NTH * u;
          if (e < kRows * 16) sDx[(e >> 4) * kDxS + (e & 15)] = dxpre[u];
        }
    }
    for (int e0 = zfirst ? tot : tid; e0 < tot; e0 += NTH * U) {
      floatx4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + NTH * u;
        v[u] = e < valid ? Z4[e] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + NTH * u;
        if (e < tot) *reinterpret_cast<floatx4*>(Zs + (e / G) * ZS + 4 * (e % G)) = v[u];
      }
    }
    if (MODE == 2 && !zfirst)
      for (int e = tid; e < kRows * 16; e += NTH) {
        const int row = e >> 4, j = e & 15, R = r0 + row;
        sDx[row * kDxS + j] = R < n ? a.dx[(nb + R) * 16 + j] : 0.f;
      }
    __syncthreads();
    LAYER_STAMP(1);
    for (int r = tid; r < nk; r += NTH) {
      float ss = 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const floatx4 z = *reinterpret_cast<const floatx4*>(Zs + r * ZS + 4 * g);
        ss = fmaf(z.x, z.x, fmaf(z.y, z.y, fmaf(z.z, z.z, fmaf(z.w, z.w, ss))));
      }
      sInv[r] = r < n ? rms_inv(ss, 1.0f / (float)DIN) : 0.f;
    }
  }
  __syncthreads();
  LAYER_STAMP(2);

  // ---- 2. P = (I + Abar)[R, :] Zs: wave w takes the 16-deep K chunks w, w + 4, ... for every column tile, so each
  // (I + Abar) element is loaded once per workgroup; the four K partials meet in LDS (aliasing Zs) in a fixed order.
  if constexpr (BF) {
    // K chunks of 32: wave w takes chunks w, w + 4, ...; lane (lo, hi) holds A[row lo][32 kc + 8 hi .. +7] of each
    // plane and B[32 kc + 8 hi + j][col lo], j < 8 (the MFMA 16x16x32 operand layout)
    const uint16_t* Ab = a.abar16 + nb * n;
    const int nch = nk >> 5;
    floatx4 acc[2][CTP];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ct = 0; ct < CTP; ++ct) acc[t][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto ld8 = [&](const uint16_t* pa, int k) -> bf16x8 {
      u16x8u u;
      if (k + 8 <= n) {
        u = *reinterpret_cast<const u16x8u*>(pa);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = k + j < n ? pa[j] : (uint16_t)0;
      }
      return __builtin_bit_cast(bf16x8, u);
    };
    for (int kc = w; kc < nch; kc += 4) {
      const int k = 32 * kc + 8 * hi;
      bf16x8 ah[2], al[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint16_t* pa = Ab + (size_t)ra[t] * n + k;
        ah[t] = ld8(pa, k);
        al[t] = ld8(pa + a.a_lo, k);
      }
      float iv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) iv[j] = sInv[k + j];
#pragma unroll
      for (int ct = 0; ct < CTP; ++ct) {
        bf16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = Zs[(k + j) * ZS + 16 * ct + lo] * iv[j];
          bh[j] = (__bf16)x;
          bl[j] = (__bf16)(x - (float)bh[j]);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (t == 1 && !two) break;
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[t], bh, acc[t][ct], 0, 0, 0);
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[t], bl, acc[t][ct], 0, 0, 0);
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[t], bh, acc[t][ct], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // Zs reads done: the partials alias it
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ct = 0; ct < CTP; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) Ps[(w * kRows + 16 * t + 4 * hi + r) * ZS + 16 * ct + lo] = acc[t][ct][r];
  } else {
    const int nch = nch16;
    floatx4 acc[NT][CTW];  // this wave's K part of P[., 16 (ct0 + ct) ...] (the same MFMA order for any CTW)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) acc[t][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int kr = kpp; kr < nch; kr += 16) {  // rounds of up to 4 chunks: kr, kr + 4, kr + 8, kr + 12
      if (kr != kpp) load_round(kr);  // the first round was issued before the Z staging
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // (I + Abar) diag(inv): column k of the operand scaled by inv[k]
        const int kc = kr + 4 * c;
        if (kc < nch) {
          const floatx4 iv = *reinterpret_cast<const floatx4*>(sInv + 16 * kc + 4 * hi);
#pragma unroll
          for (int t = 0; t < NT; ++t) av[c][t] *= iv;
        }
      }
      // the first CNT tiles (NT = 2: both, or the first when the second holds no row; NT > 2: the ntl tiles holding a
      // row, one copy of the loop per count: a runtime test per MFMA compiled to a branch around each of them)
      auto mm = [&](auto cnt_c) __attribute__((always_inline)) {
        constexpr int CNT = decltype(cnt_c)::value;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int kc = kr + 4 * c;
          if (kc >= nch) break;
          // NT > 2: MFMA steps s whose K rows 16 kc + 4 hi + s all lie past n add exact zeros and are skipped
          const int ks = NT > 2 && n - 16 * kc < 4 ? n - 16 * kc : 4;
          const float* zb = Zs + (16 * kc + 4 * hi) * ZS + lo;
          float bv[4][CTW];  // the chunk's B operands: every LDS read issued before the first MFMA
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int ct = 0; ct < CTW; ++ct) bv[s][ct] = zb[s * ZS + 16 * (ct0 + ct)];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            if (NT > 2 && s >= ks) break;
#pragma unroll
            for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
              for (int t = 0; t < NT; ++t)
                if (t < CNT) acc[t][ct] = mfma4(av[c][t][s], bv[s][ct], acc[t][ct]);
          }
        }
      };
      with_count(ntl, mm);
    }
    __syncthreads();  // Zs reads done: the partials alias it
    LAYER_STAMP(3);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Ps[(kpp * kRows + 16 * t + 4 * hi + r) * ZS + 16 * (ct0 + ct) + lo] = acc[t][ct][r];
  }
  __syncthreads();
  LAYER_STAMP(4);

  // P row (16 t + lo), columns 16 cc + 4 hi .. +3, summed over the K parts in a fixed order
  auto prow = [&](int t, int cc) -> floatx4 {
    const float* p = Ps + (16 * t + lo) * ZS + 16 * cc + 4 * hi;
    floatx4 v = *reinterpret_cast<const floatx4*>(p);
#pragma unroll
    for (int kp = 1; kp < KPP; ++kp) v += *reinterpret_cast<const floatx4*>(p + kp * kRows * ZS);
    return v;
  };
  const floatx4* W4 = reinterpret_cast<const floatx4*>(a.wperm);

  if constexpr (MODE != 2) {
    // ---- 3. Z_next = P W'^T + q b'^T -------------------------------------------------------------------------
    constexpr int CTO = DOUT / 16;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int tile = w + 4 * tt;
      if (tile >= 2 * CTO) break;
      const int rt = tile / CTO, ct = tile % CTO;
      if (rt == 1 && !two) break;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int cc = 0; cc < NCC; ++cc) {
        const floatx4 pv = prow(rt, cc);
        const floatx4 wv = wpre[tt][cc];
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(pv[s], wv[s], acc);
      }
      const int col = 16 * ct + lo;
      const float bc = bpre[tt];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = r0 + 16 * rt + 4 * hi + r;
        if (R >= n) continue;
        float v = fmaf(qpre[tt][r], bc, acc[r]);
        if (MODE == 0) v = fmaxf(v, 0.f);
        if (MODE == 1) v *= gpre[tt][r];
        const size_t o = (nb + R) * DOUT + col;
        a.out[o] = v;
      }
    }
  } else {
    // ---- 3'. CDE output layer: dZ = tg * (sum_{c,j} P[., c] dX[., j] W'[16 m + j, c] + q sum_j b'[16 m + j] dX) --
    constexpr int CT = DOUT / 16 / SPLIT;  // this workgroup's output column tiles (channels m)
    constexpr int KP = WV / CT;            // waves per column tile, splitting j (2 or 4)
    constexpr int JP = 16 / KP;
    // The canonical order for every wave count: one partial per QUARTER of the 16 j (sequential over c chunks, its
    // 4 j and the MFMA steps, then its share of the bias term), combined as (q0 + q1) + (q2 + q3)
    constexpr int QW = JP / 4;             // quarters per wave
    static_assert(KP == 2 || KP == 4, "read-out j split");
    const int ct = ch * CT + w % CT, kp = w / CT, j0 = kp * JP;
    float dxr[NT][JP];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < JP; ++j) dxr[t][j] = sDx[(16 * t + lo) * kDxS + j0 + j];
    floatx4 acc[QW][NT];
#pragma unroll
    for (int q = 0; q < QW; ++q)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[q][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    // one copy of the K loop per row-tile count (a per-MFMA test of the count compiles to a branch per MFMA)
    // Per 16-deep c chunk: all JP W' operand loads are issued first (one L2 round trip per chunk), the next chunk's
    // while this one's MFMAs run; the j loop is fully unrolled so dX stays in statically indexed registers.
    const int m = 16 * ct + lo;  // this lane's output channel
    float bfr[JP];                 // b'[16 m + j0 + j]: loaded under the last c chunk's MFMAs (its W' slot is free)
    auto kloop = [&](auto cnt_c) __attribute__((always_inline)) {
      constexpr int CNT = decltype(cnt_c)::value;
      floatx4 wv[2][JP];
#pragma unroll
      for (int j = 0; j < JP; ++j) wv[0][j] = W4[((ct * 16 + j0 + j) * NCC + 0) * 64 + lane];
#pragma unroll
      for (int cc = 0; cc < NCC; ++cc) {
        if (cc + 1 < NCC) {
#pragma unroll
          for (int j = 0; j < JP; ++j) wv[(cc + 1) & 1][j] = W4[((ct * 16 + j0 + j) * NCC + cc + 1) * 64 + lane];
        } else {
#pragma unroll
          for (int j = 0; j < JP; ++j) bfr[j] = a.bf[16 * m + j0 + j];
        }
        floatx4 pv[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) pv[t] = t < CNT ? prow(t, cc) : floatx4{0.f, 0.f, 0.f, 0.f};
        // A operands P[., c] dX[., j]: CNT > 2 (one wave per SIMD, no other wave to cover a VALU -> MFMA operand
        // wait) forms those of step j + 1 between the MFMA groups of step j, a whole step ahead of their use
        floatx4 av4[NT], nx4[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) av4[t] = pv[t] * dxr[t][0];
#pragma unroll
        for (int j = 0; j < JP; ++j) {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
              if (t < CNT) acc[j >> 2][t] = mfma4(av4[t][s], wv[cc & 1][j][s], acc[j >> 2][t]);
            if constexpr (CNT > 2) {
              if (j + 1 < JP)
#pragma unroll
                for (int t = 0; t < NT; ++t)
                  if (t % 4 == s) nx4[t] = pv[t] * dxr[t][j + 1];
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          if (j + 1 < JP) {
#pragma unroll
            for (int t = 0; t < NT; ++t) av4[t] = CNT > 2 ? nx4[t] : pv[t] * dxr[t][j + 1];
          }
        }
      }
    };
    with_count(ntl, kloop);
    LAYER_STAMP(5);
    // The folded stage combination: element k = tid + NTH u of the workgroup's (row, channel) block, row-major over
    // its CW channels; y and the earlier stage outputs are loaded here, under the bias term and the partials' barrier.
    constexpr int CW = 16 * CT;
    constexpr int CE = 16 * NT * CW / NTH;  // elements per thread (5 / 4 / 2 for the launches here)
    static_assert(CE * NTH == 16 * NT * CW, "combination elements per thread");
    const bool post = !BF && a.post.blocks != 0;
    const Combo& cb = a.post.cb;
    const size_t pE = (size_t)n * DOUT;
    float ppre[CE], pyv[CE], phb = 0.f, ptc = 0.f;
    if (post && a.post.part) {  // the earlier terms were summed by blocks riding in the hidden launches: two loads
#pragma unroll
      for (int u = 0; u < CE; ++u) {
        const int k = tid + NTH * u, R = r0 + k / CW;
        const size_t o = (size_t)b * pE + (size_t)R * DOUT + 16 * ch * CT + k % CW;
        pyv[u] = R < n ? a.post.y[o] : 0.f;
        ppre[u] = R < n ? a.post.part[o] : 0.f;
      }
      if (cb.grid) {
        const float* g = cb.grid + (size_t)b * cb.G;
        int ns = cb.nsteps[b];
        ns = ns < 0 ? 0 : (ns > cb.G - 1 ? cb.G - 1 : ns);
        ptc = cb.gk < ns ? g[cb.gk] : g[ns];
        phb = cb.gk < ns ? g[cb.gk + 1] - g[cb.gk] : 0.f;
      } else {
        phb = a.post.hcur[b];
      }
    } else if (post) {
      float kv[6][CE];
#pragma unroll
      for (int u = 0; u < CE; ++u) {
        const int k = tid + NTH * u, R = r0 + k / CW;
        const size_t o = (size_t)b * pE + (size_t)R * DOUT + 16 * ch * CT + k % CW;
        pyv[u] = R < n ? a.post.y[o] : 0.f;
#pragma unroll
        for (int j = 0; j < 6; ++j) kv[j][u] = (R < n && j < cb.nk - 1) ? cb.K[j][o] : 0.f;
      }
      if (cb.grid) {  // the step's geometry, as k_grid_step forms it
        const float* g = cb.grid + (size_t)b * cb.G;
        int ns = cb.nsteps[b];
        ns = ns < 0 ? 0 : (ns > cb.G - 1 ? cb.G - 1 : ns);
        ptc = cb.gk < ns ? g[cb.gk] : g[ns];
        phb = cb.gk < ns ? g[cb.gk + 1] - g[cb.gk] : 0.f;
      } else {
        phb = a.post.hcur[b];
      }
#pragma unroll
      for (int u = 0; u < CE; ++u) {
        float sp = 0.f;
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (j < cb.nk - 1) sp = fmaf(cb.a[j], kv[j][u], sp);
        ppre[u] = sp;
      }
    }
    // bias term of each j quarter; rows 16 t + 4 hi + r, channel m
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = 16 * t + 4 * hi + r, R = r0 + rl;
#pragma unroll
        for (int q = 0; q < QW; ++q) {  // dX[row, j0 + 4 q .. + 3]: one aligned 16-byte read (a row's 16 lanes share it)
          const floatx4 v = *reinterpret_cast<const floatx4*>(sDx + rl * kDxS + j0 + 4 * q);
          float sb = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) sb = fmaf(bfr[4 * q + e], v[e], sb);
          acc[q][t][r] = fmaf(R < n ? qpre[t][r] : 0.f, sb, acc[q][t][r]);
        }
      }
    floatx4 fin[NT];  // (q0 + q1) + (q2 + q3)
#pragma unroll
    for (int t = 0; t < NT; ++t) fin[t] = QW == 2 ? acc[0][t] + acc[QW - 1][t] : acc[0][t];
#pragma unroll
    for (int t = 0; t < NT; ++t) red[(w * NT + t) * 64 + lane] = fin[t];
    __syncthreads();
    if (kp == 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (KP == 2) {
          fin[t] += red[((w + CT) * NT + t) * 64 + lane];
        } else {
          fin[t] = (fin[t] + red[((w + CT) * NT + t) * 64 + lane]) +
                   (red[((w + 2 * CT) * NT + t) * 64 + lane] + red[((w + 3 * CT) * NT + t) * 64 + lane]);
        }
      }
    }
    if (kp == 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = r0 + 16 * t + 4 * hi + r;
          if (R < n) {
            const size_t o = (nb + R) * DOUT + m;
            const float v = gpre[t][r] * fin[t][r];
            a.out[o] = v;
            if (post) Zs[(16 * t + 4 * hi + r) * CW + 16 * w + lo] = v;  // (Ps is dead: every K loop is done)
          }
        }
    }
    LAYER_STAMP(6);
    if (post) {  // out = y + h (sum of the earlier terms + a_last K_last), K_last this launch's output
      __syncthreads();
      const float al = cb.a[cb.nk - 1];
#pragma unroll
      for (int u = 0; u < CE; ++u) {
        const int k = tid + NTH * u, R = r0 + k / CW;
        if (R < n) {
          const size_t e = (size_t)R * DOUT + 16 * ch * CT + k % CW;
          const float v = fmaf(phb, fmaf(al, Zs[k], ppre[u]), pyv[u]);
          a.post.out[(size_t)b * pE + e] = v;
          if (cb.rec) cb.rec[(size_t)b * cb.rec_stride + e] = v;
        }
      }
      if (r0 == 0 && ch == 0 && tid == 0) {  // (the sample's first workgroup, like k_combo's block 0)
        if (cb.grid) {
          const float* g = cb.grid + (size_t)b * cb.G;
          int ns = cb.nsteps[b];
          ns = ns < 0 ? 0 : (ns > cb.G - 1 ? cb.G - 1 : ns);
          cb.tcur_out[b] = ptc;
          cb.hcur_out[b] = phb;
          cb.tnx_out[b] = cb.gk < ns ? g[cb.gk + 1] : g[ns];
        }
        if (cb.tst) cb.tst[b] = cb.tend ? cb.tend[b] : stage_time(cb.grid ? ptc : cb.tcur[b], cb.c, phb);
      }
    }
  }
}

// W' [rows, din] -> the lane order of k_layer's B operands:
//   Linear (cde = 0): out[(ct NCC + cc) 64 + lane][s] = W'[16 ct + lo][16 cc + 4 hi + s]
//   CDE    (cde = 1): out[((ct 16 + j) NCC + cc) 64 + lane][s] = W'[16 (16 ct + lo) + j][16 cc + 4 hi + s]
__global__ void k_permute_linear(int rows, int din, int cde, const float* __restrict__ W, float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * din) return;
  const int ncc = din / 16;
  const int s = e & 3, lane = (e >> 2) & 63, lo = lane & 15, hi = lane >> 4;
  int blk = e >> 8;
  const int cc = blk % ncc;
  blk /= ncc;
  int row;
  if (cde) {
    const int j = blk % 16, ct = blk / 16;
    row = 16 * (16 * ct + lo) + j;
  } else {
    row = 16 * blk + lo;
  }
  out[e] = W[(size_t)row * din + 16 * cc + 4 * hi + s];
}

template <int DIN>
size_t layer_smem(int n, bool bf, int nt = kTiles, int waves = 4) {
  constexpr int ZS = zs_stride<DIN>();
  const int nk = bf ? (n + 31) & ~31 : (n + 15) & ~15, rows = 16 * nt;
  return sizeof(float) * ((size_t)waves * nt * 64 * 4 + rows * kDxS + (size_t)(nk > 4 * rows ? nk : 4 * rows) * ZS + nk);
}

constexpr size_t kMaxSmem = 64 * 1024;  // the default dynamic-LDS limit of a launch (NT = 2)
constexpr int kWideTiles = 5;           // the CDE read-out's wide workgroups (one per CU)
constexpr size_t kMaxWideSmem = 150 * 1024;

// The fp32 CDE read-out takes kWideTiles tiles per workgroup when the batch still puts a workgroup on every CU (config
// 3: 64 samples x 2 row groups x 2 channel groups = 256); GNCDE_READOUT_TILES=2 forces the two-tile launch (A/B).
template <int DIN, int DOUT>
bool readout_wide(int n, int B) {
  const char* e = getenv("GNCDE_READOUT_TILES");  // read per launch: the parity test flips it in one process
  const int forced = e ? atoi(e) : 0;
  if (forced == kTiles) return false;
  const int split = DOUT / 16 >= kSplit ? kSplit : 1;
  const long wgs = (long)B * ((n + 16 * kWideTiles - 1) / (16 * kWideTiles)) * split;
  if (layer_smem<DIN>(n, false, kWideTiles, layer_waves<DOUT, 2, false, kWideTiles>()) > kMaxWideSmem) return false;
  return forced == kWideTiles || wgs >= device_cu_count();
}

template <int DIN, int DOUT, int MODE, bool BF>
void launch(const LayerArgs& a, int B, hipStream_t st) {
  const int split = (MODE == 2 && DOUT / 16 >= kSplit) ? kSplit : 1;
  if constexpr (MODE == 2 && !BF) {
    if (readout_wide<DIN, DOUT>(a.n, B)) {
      constexpr int wv = layer_waves<DOUT, MODE, BF, kWideTiles>();
      const size_t sm = layer_smem<DIN>(a.n, false, kWideTiles, wv);
      auto k = k_layer<DIN, DOUT, MODE, BF, kWideTiles>;
      if (ensure_dyn_lds(reinterpret_cast<const void*>(k), sm)) {
        const int rows = 16 * kWideTiles;
        hipLaunchKernelGGL(k, dim3((a.n + rows - 1) / rows * split, B), dim3(64 * wv), sm, st, a);
        return;
      }
    }
  }
  size_t sm = layer_smem<DIN>(a.n, BF);
  const int rows = 16 * kTiles;
  const unsigned gx = (a.n + rows - 1) / rows * split;
  unsigned gz = 1;
  if (MODE == 0 && !BF && a.ride.blocks) {  // the riding blocks: whole z planes after the layer's plane
    gz += (a.ride.blocks + a.ride.pbs * (unsigned)a.ride.nb + gx * B - 1) / (gx * B);
    sm = sm > sizeof(float) * kFormsLdsFloats ? sm : sizeof(float) * kFormsLdsFloats;
  }
  hipLaunchKernelGGL((k_layer<DIN, DOUT, MODE, BF, kTiles>), dim3(gx, B, gz), dim3(256), sm, st, a);
}

template <int DIN, bool BF>
bool dispatch_dout(const LayerArgs& a, int B, int dout, int mode, hipStream_t st) {
#define GNCDE_LAYER_CASE(D)                                      \
  if (dout == D) {                                               \
    if (mode == 0) launch<DIN, D, 0, BF>(a, B, st);              \
    else if (mode == 1) launch<DIN, D, 1, BF>(a, B, st);         \
    else launch<DIN, D, 2, BF>(a, B, st);                        \
    return true;                                                 \
  }
  GNCDE_LAYER_CASE(16)
  GNCDE_LAYER_CASE(32)
  GNCDE_LAYER_CASE(64)
#undef GNCDE_LAYER_CASE
  return false;
}

bool width_ok(int d) { return d == 16 || d == 32 || d == 64; }

}  // namespace

int layer_mode(const GncdeProblem& p, int l) {
  const int din = p.dims[l], dout = p.dims[l + 1];
  if (!width_ok(din)) return -1;
  const bool last = l == p.L - 1;
  int mode;
  if (last && p.cde_hidden > 0) {
    if (p.cde_embed != 8 || dout != 16 * p.cde_hidden || !width_ok(p.cde_hidden)) return -1;
    mode = 2;
  } else {
    if (!width_ok(dout)) return -1;
    mode = last ? 1 : 0;
  }
  const bool bf = p.compute != GNCDE_COMPUTE_FP32;
  size_t sm = din == 16 ? layer_smem<16>(p.n, bf) : (din == 32 ? layer_smem<32>(p.n, bf) : layer_smem<64>(p.n, bf));
  return sm <= kMaxSmem ? mode : -1;
}

void permute_linear(int rows, int din, bool cde, const float* W, float* out, hipStream_t st) {
  const int tot = rows * din;
  hipLaunchKernelGGL(k_permute_linear, dim3((tot + 255) / 256), dim3(256), 0, st, rows, din, cde ? 1 : 0, W, out);
}

bool layer_fused(const GncdeProblem& p, int l, int mode, const float* abar, const float* Z, const float* wperm,
                 const float* bf, const float* q, float* out, const float* tg, const float* dx, hipStream_t st,
                 const FormsRide* ride, const PendingCombo* post) {
  LayerArgs a{};
  if (ride && mode == 0 && p.compute == GNCDE_COMPUTE_FP32) a.ride = *ride;
  const bool folded = post && mode == 2 && p.compute == GNCDE_COMPUTE_FP32 && p.cde_hidden > 0 && post->cb.nk >= 1 &&
                      post->cb.nk <= 7 && post->cb.K[post->cb.nk - 1] == out;
  if (folded) a.post = *post;
  a.n = p.n;
  a.abar = abar;
  a.Z = Z;
  a.wperm = wperm;
  a.bf = bf;
  a.q = q;
  a.out = out;
  a.tg = tg;
  a.dx = dx;
  const int din = p.dims[l];
  const int dout = mode == 2 ? p.cde_hidden : p.dims[l + 1];
  if (p.compute != GNCDE_COMPUTE_FP32) {  // abar is the hi plane of the layer's bf16 (hi, lo) pair (abar_layer)
    a.abar16 = reinterpret_cast<const uint16_t*>(abar);
    a.a_lo = (long)p.L * p.B * p.n * p.n;
    if (din == 16) dispatch_dout<16, true>(a, p.B, dout, mode, st);
    else if (din == 32) dispatch_dout<32, true>(a, p.B, dout, mode, st);
    else dispatch_dout<64, true>(a, p.B, dout, mode, st);
    return false;
  }
  if (din == 16) dispatch_dout<16, false>(a, p.B, dout, mode, st);
  else if (din == 32) dispatch_dout<32, false>(a, p.B, dout, mode, st);
  else dispatch_dout<64, false>(a, p.B, dout, mode, st);
  return folded;
}

}  // namespace gncde

#ifdef GNCDE_LAYER_STAMPS
extern "C" int gncde_debug_layer_stamps(unsigned long long* host, int count) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gncde::g_layer_stamps), sizeof(unsigned long long) * count) == hipSuccess
             ? 0
             : -1;
}
#endif
