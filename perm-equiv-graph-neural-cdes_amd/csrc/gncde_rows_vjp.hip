// Reverse mode of one vector-field evaluation, one launch per ConvLayer (configs 3 and 5 training: n <= 256, one
// hidden width H in {16, 32, 64}, ODE output or the de = 8 CDE read-out).  It replaces the generic sweep's ~14
// launches per layer (gncde_vjp.hip vf_vjp) with one, and needs no (I + Abar) or G in HBM.
//
// Every layer is taken in the reassociated order the forward evaluates (gncde_rows.hip, gncde_layer.hip):
//   zhat = diag(inv) Z_l,  P = (I + Abar_l) zhat,  q = (I + Abar_l) 1,  out_l = P W'^T + q b'^T
// (W' = W diag(rms_w), b' = b + W rms_b; out_l is Z_{l+1} before the ReLU, or the read-out).  For a cotangent
// g_out of out_l, with g_P = g_out W' and g_q = g_out b':
//   g_W' += g_out^T P,  g_b' += g_out^T q
//   G = g_P zhat^T + g_q 1^T                     the cotangent of (I + Abar_l) -> fusion-table gradient
//   g_zhat = (I + Abar_l)^T g_P,  g_Z = RMSNorm^T(g_zhat),  g_out_{l-1} = g_Z * [Z_l > 0]
// The fusion-table gradient needs, besides the four dense contractions sum_ik G_ik X_ik (X = A, dA, A^T, dA^T),
// only the row sums R_i = g_P_i . sum_k zhat_k + n g_q_i, the diagonal D_i = g_P_i . zhat_i + g_q_i and
// sum_k C_k f_k = sum_i (g_P_i . sum_k zhat_k f_k + g_q_i sum_k f_k) against the form's node features — all O(n H).
//
// Launches per stage (after the forward kept Z_1 .. Z_{L-1}, generic_vf_eval keep mode):
//   k_bwd_head      per 16-row block: the interval's A, dA rows (Horner of the coefficient planes, once per
//                   evaluation for every layer launch), g_out, g_P, g_q of the output layer from the stage cotangent
//                   gF (ODE g_out = tg gF; CDE g_P_i = tg_i sum_{m,j} gF_im dX_ij W'[16m+j, :] without the n x 16h
//                   g_out, and the factors tg gF, dX for the read-out weight gradient)
//   k_bwd_layer<H>  per 16-row block, l = L-1 .. 0: the block's rows and columns of A, dA -> A, dA, A^T, dA^T in
//                   the product's operand layout, zhat and g_P of every node in LDS, then one K
//                   loop over the block's node chunks that runs three MFMA products per chunk: P = (I+Abar) zhat,
//                   g_zhat = (I+Abar)^T g_P (the same registers, the transposed coefficients) and the G^T tile
//                   zhat g_P^T, which meets A, dA, A^T, dA^T in registers for the dense contractions; then g_W'
//                   partials, RMSNorm^T, the ReLU mask and the next layer's g_out, g_P, g_q (or the stage input's
//                   cotangent at l = 0)
//   k_bwd_head_gemm (CDE) g_P, g_q of the read-out layer as one GEMM over all samples' rows
//   k_bwd_readout   (CDE) the read-out weight and bias gradient on MFMA, K = all samples' rows in a few chunks,
//                   one workgroup per (chunk, 4 output m)
//   k_bwd_data      (CDE data-spline cotangent, TGB) g_dX_ij = tg_i sum_m gF_im (P_i . W'[16m+j,:] + q_i b'[16m+j])
// Parameter and fusion partials accumulate in per-(sample, row block) / per-chunk slots that only their owner
// workgroup updates (fixed order, no atomics); k_bwd_finish reduces them once per reverse sweep and maps g_W', g_b'
// to the reference's W, b, rms_w, rms_b.
#include "gncde_internal.h"

#include <cstdlib>

namespace gncde {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kRB = 16;
constexpr int kMaxN = 256;

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float cubic(const float (&c)[4], float f) { return fmaf(f, fmaf(f, fmaf(f, c[0], c[1]), c[2]), c[3]); }
__device__ __forceinline__ float dcubic(const float (&c)[4], float f) {
  return fmaf(f, fmaf(3.0f * f, c[0], 2.0f * c[1]), c[2]);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float u2f(unsigned x) { return __builtin_bit_cast(float, x); }

__host__ __device__ constexpr int bwd_zs(int H) { return H + 4; }
__host__ __device__ inline int bwd_np(int n) { return (n + 15) & ~15; }
constexpr int kMaxRbw = 3;  // row blocks per workgroup (one 256-thread group each)

// Phase stamps of k_bwd_layer (diagnostic build -DGNCDE_BWD_STAMPS only: tools/diag_bwd_stamps.py): the first wave
// of every workgroup records s_memrealtime at 12 points of the last launch.
#ifdef GNCDE_BWD_STAMPS
__device__ unsigned long long g_bwd_stamps[1024 * 16];
#define BWD_STAMP(k) \
  do { if (threadIdx.x == 0 && a.l == 1 && blockIdx.x < 1024) g_bwd_stamps[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// a stamp once the value v has arrived
#define BWD_STAMP_AFTER(k, v) \
  do { asm volatile("" ::"v"(v)); BWD_STAMP(k); } while (0)
#else
#define BWD_STAMP(k) do {} while (0)
#define BWD_STAMP_AFTER(k, v) do {} while (0)
#endif
// The union region, used in turn as (1) zhat and g_P of every node [NP][H+4] each, shared by the groups, (2) every
// group's product partials: P rows [80][H+4] (64 partial rows, 16 result rows), then the g_zhat rows [80][H+4]
__host__ __device__ inline int bwd_union(int n, int H, int rbw) {
  const int z = 2 * bwd_np(n) * bwd_zs(H), e = rbw * 160 * bwd_zs(H);
  return ((z > e ? z : e) + 3) & ~3;
}
inline size_t bwd_smem(int n, int H, int rbw) {
  const int np = bwd_np(n);
  // union | inv, gq, r, rd, c, cd, dg, dgd, v, w [10][NP] | u, q [kMaxRbw][2][16] | scratch [1280 kMaxRbw]
  // | fusion sums [kMaxRbw][24][4]
  return sizeof(float) * ((size_t)bwd_union(n, H, rbw) + 10 * (size_t)np + 32 * kMaxRbw + 1280 * kMaxRbw +
                          (size_t)kMaxRbw * GNCDE_FC * 4);
}

struct BwdArgs {
  int B, n, T, L, l, nb;
  const float* ts;
  const float* aev;        // A, dA at the evaluation time [B][2][NP][NP] (k_bwd_head; zero past n)
  const float* csum;       // k_coef_sums [B, T-1, 12 n + 4]
  const float* fusion;     // [L, GNCDE_FC]
  const float* t;          // [B] stage times
  const float* zin;        // Z_l [B, n, H] (the stage input at l = 0, else the forward's kept hidden output)
  const float* gP;         // this layer's g_P [B, n, H]
  const float* gq;         // g_q [B, n]
  const float* gout;       // g_out [B, n, H] (layers with d_out = H; unused for the CDE read-out layer)
  const float* wprev;      // W'_{l-1} natural [H, H] (l > 0)
  const float* bprev;      // b'_{l-1} [H]
  float* gP_next;          // layer l-1's g_P, g_q, g_out (l > 0)
  float* gq_next;
  float* gout_next;
  float* gz;               // l = 0: the stage input's cotangent [B, n, H]
  float* pq;               // CDE read-out layer: P | q per node [B, n, H + 1]
  float* gfc;              // [B * nb, L, GNCDE_FC] accumulated
  float* gw;               // [B * nb, gw_stride] accumulated; this layer's H x H g_W' then H g_b' at gw_off
  int gw_stride, gw_off;
  int cde_out;             // layer l is the CDE read-out layer
  int scatter;             // l = 0: apply sc to the stage input's cotangent instead of writing gz
  StageScatter sc;
};

// One ConvLayer's reverse mode for rbw = blockDim.x / 256 row blocks R of one sample (see the file comment): each
// 256-thread group owns one 16-row block; the groups share the staging of every node's zhat and g_P (the widest
// part of the launch's memory traffic) and the per-node reductions.  At config 3 (B = 64, nb = 9) three groups per
// workgroup make the grid 192 workgroups, one round on 256 CUs, where one block per workgroup took three rounds (its
// 90 KB of LDS admits one workgroup per CU).
template <int H>
__global__ void __launch_bounds__(256 * kMaxRbw, 1) k_bwd_layer(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int ZS = bwd_zs(H);
  constexpr int CT = H / 16;
  constexpr int KH = H / 4;  // MFMA K steps over a width-H contraction
  const int n = a.n, T = a.T, l = a.l;
  const int NP = bwd_np(n), nch = NP >> 4;
  const int NT = (int)blockDim.x, rbw = NT >> 8, grp = (int)threadIdx.x >> 8;
  float* U = sm;
  float* big = U;                          // zhat of every node [NP][ZS] (shared)
  float* sG = U + (size_t)NP * ZS;         // g_P of every node [NP][ZS] (shared)
  float* epP = U + (size_t)grp * 160 * ZS;  // this group's P partials [64][ZS] + P[R] [16][ZS]
  float* epG = epP + 80 * ZS;               // this group's g_zhat partials + g_zhat[R]
  float* sInv = U + bwd_union(n, H, rbw);
  float* sGq = sInv + NP;
  float* sF = sGq + NP;                // r, rd, c, cd, dg, dgd [6][NP]
  float* sV = sF + 6 * NP;             // v_l [NP]
  float* sW = sV + NP;                 // w_l [NP]
  float* sRow = sW + NP + 32 * grp;    // u_l [16], q_l [16] of this group's rows
  float* sScr = sW + NP + 32 * kMaxRbw;  // [1280 kMaxRbw] reduction scratch (5 H floats per node group)
  float* sFus = sScr + 1280 * kMaxRbw + grp * GNCDE_FC * 4;  // [GNCDE_FC][4] of this group

  // A group's four wave roles rotate by the group index: the waves of one role index share a SIMD, and the K loop's
  // node chunks kc = w + 4 j do not split evenly over four waves (config 3: 9 chunks, 3 / 2 / 2 / 2), so the rotation
  // spreads the long role over the SIMDs.  A permutation of the roles inside the group leaves every result unchanged.
  const int tid = ((((int)threadIdx.x >> 6) + grp) & 3) << 6 | ((int)threadIdx.x & 63);
  const int w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  const int nbw = (a.nb + rbw - 1) / rbw;
  const int wx = xcd_work((int)blockIdx.x, (int)gridDim.x);
  const int b = wx / nbw, rbr = (wx % nbw) * rbw + grp;
  // a group past the sample's last block recomputes that block (every barrier is the whole workgroup's) and stores
  // nothing
  const bool gact = rbr < a.nb;
  const int rb = gact ? rbr : a.nb - 1, slot = b * a.nb + rb;
  const int r0 = rb * kRB, ri = r0 + lo;
  BWD_STAMP(0);
  const size_t zgroup = (size_t)n * H;
  const float tb = a.t[b];
  const float* tsb = a.ts + (size_t)b * T;
  const int idx = interval_index_wave(tsb, T, tb);
  const float f = tb - tsb[idx];
  const float* fc = a.fusion + l * GNCDE_FC;
  BWD_STAMP_AFTER(12, f);
  // independent global reads of the epilogue issued now (their round trips overlap the form): the slot's fusion
  // partial and this group's g_out rows
  const float gfc_old = gact && tid < GNCDE_FC ? a.gfc[((size_t)slot * a.L + l) * GNCDE_FC + tid] : 0.f;
  constexpr int GOU = 16 * H / 256;  // g_out[R] elements per thread
  float gor[GOU];
#pragma unroll
  for (int u = 0; u < GOU; ++u) {
    const int e = tid + 256 * u, i = e / H, c = e % H;
    gor[u] = !a.cde_out && r0 + i < n ? a.gout[((size_t)b * n + r0 + i) * H + c] : 0.f;
  }

  // ---- form: the block's rows and columns of A, dA straight into the operand registers: (ri, k) and (k, ri),
  // k = 16 kc + 4 hi + s, kc = w + 4 j (k_bwd_head evaluated the interval's cubics once for every layer launch)
  const size_t pl = (size_t)NP * NP;
  const float* A0 = a.aev + (size_t)b * 2 * pl;
  const float* A1 = A0 + pl;
  float Ar[4][4], dAr[4][4], At[4][4], dAt[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kc = w + 4 * j, k0 = 16 * kc + 4 * hi;
    const bool in = kc < nch;
    const floatx4 ar = in ? *reinterpret_cast<const floatx4*>(A0 + (size_t)ri * NP + k0) : floatx4{0.f, 0.f, 0.f, 0.f};
    const floatx4 dr = in ? *reinterpret_cast<const floatx4*>(A1 + (size_t)ri * NP + k0) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      Ar[j][s] = ar[s];
      dAr[j][s] = dr[s];
      At[j][s] = in ? A0[(size_t)(k0 + s) * NP + ri] : 0.f;
      dAt[j][s] = in ? A1[(size_t)(k0 + s) * NP + ri] : 0.f;
    }
  }
  const float* cs = a.csum + ((size_t)b * (T - 1) + idx) * ((size_t)12 * n + 4);
  const int nd = tid < n ? tid : n - 1;
  float pv[3][4], pt[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) pv[kd][q] = cs[(q * 3 + kd) * n + nd];
    pt[q] = cs[12 * n + q];
  }
  // ---- Z_l and g_P of every node into LDS (their round trips overlap the operand loads') ----------------------
  {
    constexpr int G4 = H / 4;
    const floatx4* Z4 = reinterpret_cast<const floatx4*>(a.zin + (size_t)b * zgroup);
    const floatx4* P4 = reinterpret_cast<const floatx4*>(a.gP + (size_t)b * zgroup);
    const int tot = NP * G4, valid = n * G4;
    for (int e0 = (int)threadIdx.x; e0 < tot; e0 += NT * 4) {
      floatx4 vz[4], vp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + NT * u;
        vz[u] = e < valid ? Z4[e] : floatx4{0.f, 0.f, 0.f, 0.f};
        vp[u] = e < valid ? P4[e] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + NT * u;
        if (e < tot) {
          *reinterpret_cast<floatx4*>(big + (e / G4) * ZS + 4 * (e % G4)) = vz[u];
          *reinterpret_cast<floatx4*>(sG + (e / G4) * ZS + 4 * (e % G4)) = vp[u];
        }
      }
    }
    for (int k = (int)threadIdx.x; k < NP; k += NT) sGq[k] = k < n ? a.gq[(size_t)b * n + k] : 0.f;
  }
  BWD_STAMP_AFTER(13, dAt[3][3]);
  BWD_STAMP_AFTER(14, pv[2][3]);
  // node features and this layer's families at every node (thread = node)
  const float s_t = cubic(pt, f), sd_t = dcubic(pt, f);
  {
    const bool nin = tid < n;
    const float r = nin ? cubic(pv[0], f) : 0.f, rd = nin ? dcubic(pv[0], f) : 0.f;
    const float c = nin ? cubic(pv[1], f) : 0.f, cd = nin ? dcubic(pv[1], f) : 0.f;
    const float dg = nin ? cubic(pv[2], f) : 0.f, dgd = nin ? dcubic(pv[2], f) : 0.f;
    if (grp == 0 && tid < NP) {  // the node vectors: one group writes them
      sF[tid] = r;
      sF[NP + tid] = rd;
      sF[2 * NP + tid] = c;
      sF[3 * NP + tid] = cd;
      sF[4 * NP + tid] = dg;
      sF[5 * NP + tid] = dgd;
      sV[tid] = fc[GNCDE_FC_VR_A] * r + fc[GNCDE_FC_VR_DA] * rd + fc[GNCDE_FC_VC_A] * c + fc[GNCDE_FC_VC_DA] * cd;
      const float wv = fc[GNCDE_FC_WR_A] * r + fc[GNCDE_FC_WR_DA] * rd + fc[GNCDE_FC_WC_A] * c + fc[GNCDE_FC_WC_DA] * cd +
                       fc[GNCDE_FC_WS_A] * s_t + fc[GNCDE_FC_WS_DA] * sd_t;
      sW[tid] = nin ? wv : 0.f;
    }
    if (tid >= r0 && tid < r0 + kRB && nin) {
      const float wv = fc[GNCDE_FC_WR_A] * r + fc[GNCDE_FC_WR_DA] * rd + fc[GNCDE_FC_WC_A] * c + fc[GNCDE_FC_WC_DA] * cd +
                       fc[GNCDE_FC_WS_A] * s_t + fc[GNCDE_FC_WS_DA] * sd_t;
      const float uv = fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * dg + fc[GNCDE_FC_UD_DA] * dgd + fc[GNCDE_FC_UR_A] * r +
                       fc[GNCDE_FC_UR_DA] * rd + fc[GNCDE_FC_UC_A] * c + fc[GNCDE_FC_UC_DA] * cd + fc[GNCDE_FC_US_A] * s_t +
                       fc[GNCDE_FC_US_DA] * sd_t;
      float qv = fc[GNCDE_FC_E_A] * r + fc[GNCDE_FC_E_DA] * rd + fc[GNCDE_FC_ET_A] * c + fc[GNCDE_FC_ET_DA] * cd;
      qv += (float)n * wv;
      qv += (fc[GNCDE_FC_VR_A] + fc[GNCDE_FC_VC_A]) * s_t + (fc[GNCDE_FC_VR_DA] + fc[GNCDE_FC_VC_DA]) * sd_t;
      qv += uv;
      sRow[tid - r0] = uv;
      sRow[16 + tid - r0] = qv;
    } else if (tid >= r0 && tid < r0 + kRB) {
      sRow[tid - r0] = 0.f;
      sRow[16 + tid - r0] = 0.f;
    }
  }
  __syncthreads();
  BWD_STAMP(1);
  BWD_STAMP(2);
  BWD_STAMP(3);
  for (int k = (int)threadIdx.x; k < NP; k += NT) {
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < H / 4; ++q) {
      const floatx4 z = *reinterpret_cast<const floatx4*>(big + k * ZS + 4 * q);
      ss = fmaf(z.x, z.x, fmaf(z.y, z.y, fmaf(z.z, z.z, fmaf(z.w, z.w, ss))));
    }
    sInv[k] = k < n ? rms_inv(ss, 1.0f / (float)H) : 0.f;
  }
  __syncthreads();
  BWD_STAMP(4);
  // zsum = sum_k zhat_k and zf_x = sum_k zhat_k x_k (x = r, rd, c, cd) as one [16 x NP] x [NP x H] MFMA product
  // (A rows 1, r, rd, c, cd times inv, rows 5.. zero; B = Z_l): work unit kq < NG = the k steps 4 (kq + NG i) for
  // every column tile (the A operand shared), the units spread over every wave of the workgroup; NG is fixed, so the
  // sums do not depend on the row blocks per workgroup
  constexpr int NG = 4 * kMaxRbw;
  {
    const int gw = (int)threadIdx.x >> 6, nw = NT >> 6;
    const int x = lo < 5 ? lo : 0;
    const float* fx = sF + (x > 0 ? x - 1 : 0) * NP;
    constexpr int KS = (kMaxN / 4 + NG - 1) / NG;  // k steps of one unit at most
    for (int kq = gw; kq < NG; kq += nw) {
      // every operand of the unit read first (the steps past NP read row NP - 1 and contribute zero)
      float av[KS];
#pragma unroll
      for (int i = 0; i < KS; ++i) {
        const int k4 = 4 * (kq + NG * i), k = k4 + hi < NP ? k4 + hi : NP - 1;
        const float iv = sInv[k], fv = x == 0 ? 1.f : fx[k];
        av[i] = k4 < NP && lo < 5 ? fv * iv : 0.f;
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        float bv[KS];
#pragma unroll
        for (int i = 0; i < KS; ++i) {
          const int k4 = 4 * (kq + NG * i), k = k4 + hi < NP ? k4 + hi : NP - 1;
          const float bz = big[k * ZS + 16 * ct + lo];
          bv[i] = k4 < NP ? bz : 0.f;
        }
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < KS; ++i) acc = mfma4(av[i], bv[i], acc);
        // rows 0..3 in the lanes of hi = 0, row 4 in acc[0] of hi = 1
        if (hi == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) sScr[(kq * 5 + r) * H + 16 * ct + lo] = acc[r];
        } else if (hi == 1) {
          sScr[(kq * 5 + 4) * H + 16 * ct + lo] = acc[0];
        }
      }
    }
  }
  __syncthreads();
  float* sZv = sScr + 5 * NG * H - 5 * H;  // zsum, zf_r, zf_rd, zf_c, zf_cd [5][H] (after the group partials)
  for (int e = (int)threadIdx.x; e < 5 * H; e += NT) {
    // (the total for (x, c) lands in the last group's slot for (x, c), which only this thread reads, after reading
    // it)
    const int x = e / H, c = e % H;
    float v = 0.f;
    for (int g = 0; g < NG; ++g) v += sScr[(g * 5 + x) * H + c];
    sZv[x * H + c] = v;
  }
  __syncthreads();
  BWD_STAMP(5);

  // ---- the K loop: P = (I+Abar) zhat, g_zhat = (I+Abar)^T g_P, G^T tiles meeting A, dA, A^T, dA^T ----------
  const float eA = fc[GNCDE_FC_E_A], edA = fc[GNCDE_FC_E_DA], eTA = fc[GNCDE_FC_ET_A], eTdA = fc[GNCDE_FC_ET_DA];
  const float wi = sW[ri < NP ? ri : 0], vi = sV[ri < NP ? ri : 0], ui = sRow[lo], gqi = sGq[ri < NP ? ri : 0];
  // this lane's B operand of the G^T tiles, g_P[ri][4 s + hi]: held in registers below H = 64 (at H = 64 its 16
  // registers would spill the 3-group workgroup's 170; read from LDS per chunk)
  constexpr bool kGpr = H < 64;
  float gpr[kGpr ? KH : 1];
#pragma unroll
  for (int s = 0; s < (kGpr ? KH : 0); ++s) gpr[s] = sG[ri * ZS + 4 * s + hi];
  floatx4 accP[CT], accT[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    accP[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    accT[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  float dsum[4] = {0.f, 0.f, 0.f, 0.f};  // sum G.*A, G.*dA, G.*A^T, G.*dA^T over this lane's elements
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kc = w + 4 * j;
    if (kc >= nch) break;
    const int k0 = 16 * kc + 4 * hi;
    const floatx4 vk = *reinterpret_cast<const floatx4*>(sV + k0);
    const floatx4 wk = *reinterpret_cast<const floatx4*>(sW + k0);
    const floatx4 iv = *reinterpret_cast<const floatx4*>(sInv + k0);
    // G^T tile rows k = 16 kc + (0..15), columns R: A operand zhat[16 kc + lo][4 s + hi], B operand g_P[ri][4 s + hi]
    floatx4 gt = {0.f, 0.f, 0.f, 0.f};
    {
      const int kr = 16 * kc + lo;
      const float ik = sInv[kr];
#pragma unroll
      for (int s = 0; s < KH; ++s) {
        float gp;
        if constexpr (kGpr) gp = gpr[s];
        else gp = sG[ri * ZS + 4 * s + hi];
        gt = mfma4(big[kr * ZS + 4 * s + hi] * ik, gp, gt);
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float g = gt[s] + gqi;  // G[ri][k0 + s] (zero operands past n: padded k add nothing below)
      dsum[0] = fmaf(g, Ar[j][s], dsum[0]);
      dsum[1] = fmaf(g, dAr[j][s], dsum[1]);
      dsum[2] = fmaf(g, At[j][s], dsum[2]);
      dsum[3] = fmaf(g, dAt[j][s], dsum[3]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // (the B operands one k at a time: at H = 64 all four k's at once cost the registers a 3-group workgroup
      // does not have)
      float bz[1][CT], bg[1][CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        bz[0][ct] = big[(k0 + s) * ZS + 16 * ct + lo];
        bg[0][ct] = sG[(k0 + s) * ZS + 16 * ct + lo];
      }
      float v = fmaf(eA, Ar[j][s], fmaf(edA, dAr[j][s], fmaf(eTA, At[j][s], fmaf(eTdA, dAt[j][s], wi + vk[s]))));
      float vt = fmaf(eA, At[j][s], fmaf(edA, dAt[j][s], fmaf(eTA, Ar[j][s], fmaf(eTdA, dAr[j][s], wk[s] + vi))));
      if (k0 + s == ri) {
        v += ui;
        vt += ui;
      }
      const float op = v * iv[s];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        accP[ct] = mfma4(op, bz[0][ct], accP[ct]);
        accT[ct] = mfma4(vt, bg[0][ct], accT[ct]);
      }
    }
  }
  // row terms of the fusion gradient (threads 0..15: row r0 + tid), from every node's zhat / g_P still in LDS
  float facc[GNCDE_FC];
#pragma unroll
  for (int q = 0; q < GNCDE_FC; ++q) facc[q] = 0.f;
  {  // row ir of the block: its 16 lanes take columns cl + 16 u, then a fixed 16-lane butterfly
    const int ir = tid >> 4, cl = tid & 15, i = r0 + ir < n ? r0 + ir : n - 1;
    float gz = 0.f, gd = 0.f, gfr = 0.f, gfrd = 0.f, gfc_ = 0.f, gfcd = 0.f;
#pragma unroll
    for (int u = 0; u < H / 16; ++u) {
      const int c = cl + 16 * u;
      const float g = sG[i * ZS + c];
      gz = fmaf(g, sZv[c], gz);
      gd = fmaf(g, big[i * ZS + c], gd);
      gfr = fmaf(g, sZv[H + c], gfr);
      gfrd = fmaf(g, sZv[2 * H + c], gfrd);
      gfc_ = fmaf(g, sZv[3 * H + c], gfc_);
      gfcd = fmaf(g, sZv[4 * H + c], gfcd);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      gz += __shfl_xor(gz, o);
      gd += __shfl_xor(gd, o);
      gfr += __shfl_xor(gfr, o);
      gfrd += __shfl_xor(gfrd, o);
      gfc_ += __shfl_xor(gfc_, o);
      gfcd += __shfl_xor(gfcd, o);
    }
    if (cl == 0 && r0 + ir < n) {
      const float gqv = sGq[i];
      const float R = fmaf((float)n, gqv, gz);
      const float D = fmaf(gd, sInv[i], gqv);
      const float r = sF[i], rd = sF[NP + i], c = sF[2 * NP + i], cd = sF[3 * NP + i];
      const float dg = sF[4 * NP + i], dgd = sF[5 * NP + i];
      facc[GNCDE_FC_WR_A] = R * r;
      facc[GNCDE_FC_WR_DA] = R * rd;
      facc[GNCDE_FC_WC_A] = R * c;
      facc[GNCDE_FC_WC_DA] = R * cd;
      facc[GNCDE_FC_WS_A] = R * s_t;
      facc[GNCDE_FC_WS_DA] = R * sd_t;
      facc[GNCDE_FC_UD_A] = D * dg;
      facc[GNCDE_FC_UD_DA] = D * dgd;
      facc[GNCDE_FC_UR_A] = D * r;
      facc[GNCDE_FC_UR_DA] = D * rd;
      facc[GNCDE_FC_UC_A] = D * c;
      facc[GNCDE_FC_UC_DA] = D * cd;
      facc[GNCDE_FC_US_A] = D * s_t;
      facc[GNCDE_FC_US_DA] = D * sd_t;
      facc[GNCDE_FC_IDC] = D;
      facc[GNCDE_FC_VR_A] = fmaf(gqv, s_t, gfr);
      facc[GNCDE_FC_VR_DA] = fmaf(gqv, sd_t, gfrd);
      facc[GNCDE_FC_VC_A] = fmaf(gqv, s_t, gfc_);
      facc[GNCDE_FC_VC_DA] = fmaf(gqv, sd_t, gfcd);
    }
  }
  facc[GNCDE_FC_E_A] += dsum[0];
  facc[GNCDE_FC_E_DA] += dsum[1];
  facc[GNCDE_FC_ET_A] += dsum[2];
  facc[GNCDE_FC_ET_DA] += dsum[3];
  // this layer's own g_zhat / zhat rows are needed after the partials overwrite the node regions: the rows' Z and
  // inv stay available through HBM (zin) and sInv
  __syncthreads();  // every group's reads of zhat / g_P of all nodes done: the partial rows alias them
  BWD_STAMP(6);
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      epP[(w * 16 + 4 * hi + r) * ZS + 16 * ct + lo] = accP[ct][r];
      epG[(w * 16 + 4 * hi + r) * ZS + 16 * ct + lo] = accT[ct][r];
    }
  // fusion sums: a DPP / row-swap reduction per wave (no LDS), then the four wave partials in order
#pragma unroll
  for (int q = 0; q < GNCDE_FC; ++q) {
    const float v = wave_sum64(facc[q]);
    if (lane == 0) sFus[q * 4 + w] = v;
  }
  __syncthreads();
  BWD_STAMP(7);
  if (gact && tid < GNCDE_FC)
    a.gfc[((size_t)slot * a.L + l) * GNCDE_FC + tid] =
        gfc_old + ((sFus[tid * 4] + sFus[tid * 4 + 1]) + (sFus[tid * 4 + 2] + sFus[tid * 4 + 3]));
  // P[R], g_zhat[R]: the four K parts in a fixed order, into rows 64..79 of the two regions
  for (int e = tid; e < 16 * H; e += 256) {
    const int i = e / H, c = e % H;
    float p = epP[i * ZS + c], g = epG[i * ZS + c];
#pragma unroll
    for (int kp = 1; kp < 4; ++kp) {
      p += epP[(kp * 16 + i) * ZS + c];
      g += epG[(kp * 16 + i) * ZS + c];
    }
    epP[(64 + i) * ZS + c] = p;
    epG[(64 + i) * ZS + c] = g;
  }
  __syncthreads();
  BWD_STAMP(8);
  const float* sP = epP + 64 * ZS;   // P[R] [16][ZS]
  const float* sGz = epG + 64 * ZS;  // g_zhat[R]
  // ---- parameter partials: g_W' += g_out[R]^T P[R], g_b' += g_out[R]^T q[R] (d_out = H), or P | q out (CDE) ----
  if (a.cde_out) {
    for (int e = tid; e < 16 * (H + 1); e += 256) {
      const int i = e / (H + 1), c = e % (H + 1);
      if (gact && r0 + i < n) a.pq[((size_t)b * n + r0 + i) * (H + 1) + c] = c < H ? sP[i * ZS + c] : sRow[16 + i];
    }
  } else {
    float* go = epG;  // g_out[R] staged in rows 0..15 of the group's g partial region (the partials are consumed)
#pragma unroll
    for (int u = 0; u < GOU; ++u) {
      const int e = tid + 256 * u;
      go[(e / H) * ZS + e % H] = gor[u];
    }
    __syncthreads();
    float* gw = a.gw + (size_t)slot * a.gw_stride + a.gw_off;
    // g_W'[j][c] += sum_{i in R} g_out[i][j] P[i][c]: CT x CT MFMA tiles over the waves, K = the 16 rows
    for (int tile = w; gact && tile < CT * CT; tile += 4) {
      const int jt = tile / CT, ct = tile % CT;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma4(go[(4 * s + hi) * ZS + 16 * jt + lo], sP[(4 * s + hi) * ZS + 16 * ct + lo], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) gw[(16 * jt + 4 * hi + r) * H + 16 * ct + lo] += acc[r];
    }
    if (gact && tid < H) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < kRB; ++i) acc = fmaf(go[i * ZS + tid], sRow[16 + i], acc);
      gw[H * H + tid] += acc;
    }
    __syncthreads();  // go is reused below
  }
  BWD_STAMP(9);
  // ---- RMSNorm^T of the block's rows and the next cotangents ------------------------------------------------
  // thread = (row tid / 16, columns (tid % 16) + 16 u): a row's 16 threads are 16 consecutive lanes
  {
    const int i = tid >> 4, cl = tid & 15;
    constexpr int U = H / 16;
    const bool iin = gact && r0 + i < n;
    const float inv = iin ? sInv[r0 + i] : 0.f;
    float z[U], gzh[U];
    float dot = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      z[u] = iin ? a.zin[((size_t)b * n + r0 + i) * H + cl + 16 * u] : 0.f;
      gzh[u] = sGz[i * ZS + cl + 16 * u];
      dot = fmaf(gzh[u], z[u] * inv, dot);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    const float cdot = dot / (float)H;
    float gZ[U];
#pragma unroll
    for (int u = 0; u < U; ++u) gZ[u] = inv * (gzh[u] - z[u] * inv * cdot);
    if (l == 0) {
      if (iin && a.scatter) {  // gncde_vjp.hip's v_stage_scatter arithmetic, fused
        const float hb = a.sc.hcur[b];
        const int nsc = a.sc.n;  // <= 7 earlier stages
        // every accumulator element is read before any is written (gy and the gk[j] are distinct buffers): loaded
        // one after another behind their own stores, they were a chain of up to eight dependent round trips
        float gyv[U], gkv[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const size_t o = ((size_t)b * n + r0 + i) * H + cl + 16 * u;
          gyv[u] = a.sc.gy[o];
#pragma unroll
          for (int j = 0; j < 8; ++j) gkv[u][j] = j < nsc ? a.sc.gk[j][o] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const size_t o = ((size_t)b * n + r0 + i) * H + cl + 16 * u;
          const float v = gZ[u];
          a.sc.gy[o] = fmaf(1.0f, v, gyv[u]);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nsc) a.sc.gk[j][o] = fmaf(hb, a.sc.a[j] * v, gkv[u][j]);
        }
      } else if (iin) {
#pragma unroll
        for (int u = 0; u < U; ++u) a.gz[((size_t)b * n + r0 + i) * H + cl + 16 * u] = gZ[u];
      }
    } else {
      float* go = epG;  // g_out_{l-1}[R] = g_Z * [Z_l > 0]
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float g = z[u] > 0.f ? gZ[u] : 0.f;
        go[i * ZS + cl + 16 * u] = g;
        if (iin) a.gout_next[((size_t)b * n + r0 + i) * H + cl + 16 * u] = g;
      }
    }
  }
  if (l == 0) return;
  __syncthreads();
  BWD_STAMP(10);
  {
    const float* go = epG;
    // g_P_{l-1}[i][c] = sum_j g_out[i][j] W'_{l-1}[j][c]: wave ct's 16 x 16 tile, K = H (W' rows from L2)
    if (gact && w < CT) {
      const int ct = w;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KH; ++s)
        acc = mfma4(go[lo * ZS + 4 * s + hi], a.wprev[(4 * s + hi) * H + 16 * ct + lo], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r0 + 4 * hi + r < n) a.gP_next[((size_t)b * n + r0 + 4 * hi + r) * H + 16 * ct + lo] = acc[r];
    }
    BWD_STAMP(11);
    if (gact && tid < kRB && r0 + tid < n) {
      float acc = 0.f;
      for (int jo = 0; jo < H; ++jo) acc = fmaf(go[tid * ZS + jo], a.bprev[jo], acc);
      a.gq_next[(size_t)b * n + r0 + tid] = acc;
    }
  }
}

struct HeadArgs {
  int B, n, T, H, cde;
  const float* ts;
  const float* coef;       // [B, T-1, 4, n, n]
  const float* tcoef;      // [B, T-1, 3, n]
  const float* data_coef;  // [B, T-1, 4, n, 8, 2]
  const float* t;
  const float* gF;         // [B, n, H] the stage value's cotangent
  const float* wl;         // W'_{L-1} natural [d_L, H]
  const float* bl;         // b'_{L-1} [d_L]
  float* gout;             // ODE: [B, n, H]
  float* gP;               // [B, n, H]
  float* gq;               // [B, n]
  float* tgF;              // CDE: tg gF [B, n, H]
  float* dxo;              // CDE: dX [B, n, 16]
  float* aev;              // A, dA at the evaluation time [B][2][NP][NP]
};

// Output layer's cotangents for a 16-row block (thread = (row tid / 16, column tid % 16 + 16 u) for the elementwise
// parts; the products on MFMA).
template <int H>
__global__ void __launch_bounds__(256) k_bwd_head(HeadArgs a) {
  constexpr int CT = H / 16, KH = H / 4;
  const int nb = (a.n + kRB - 1) / kRB;
  const int wx = xcd_work((int)blockIdx.x, (int)gridDim.x);
  const int b = wx / nb, r0 = (wx % nb) * kRB;
  const int n = a.n, T = a.T, tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  const int i = tid >> 4, cl = tid & 15;
  __shared__ float sgo[kRB][H + 1];  // ODE g_out rows
  const float tb = a.t[b];
  const float* tsb = a.ts + (size_t)b * T;
  const int idx = interval_index_wave(tsb, T, tb);
  const float f = tb - tsb[idx];
  {
    // the interval's A, dA rows r0 .. r0 + 15 at every column (zero past n), read by every layer launch: thread =
    // (row tid / 16, columns 4 (tid % 16) + 64 u)
    const size_t nn = (size_t)n * n;
    const int NP = bwd_np(n), rr = tid >> 4, cq = 4 * (tid & 15);
    const auto crs = rsrc(a.coef + ((size_t)b * (T - 1) + idx) * 4 * nn, (unsigned)(4 * nn * sizeof(float)));
    u32x4 rc[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        rc[u][q] = __builtin_amdgcn_raw_buffer_load_b128(crs, (int)((q * nn + (size_t)(r0 + rr) * n + cq + 64 * u) * 4), 0, 0);
    float* a0 = a.aev + ((size_t)b * 2 * NP + r0 + rr) * NP;
    float* a1 = a0 + (size_t)NP * NP;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c0 = cq + 64 * u;
      if (c0 < NP) {
        floatx4 va, vd;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = r0 + rr < n && c0 + e < n;
          const float cc[4] = {u2f(rc[u][0][e]), u2f(rc[u][1][e]), u2f(rc[u][2][e]), u2f(rc[u][3][e])};
          va[e] = in ? cubic(cc, f) : 0.f;
          vd[e] = in ? dcubic(cc, f) : 0.f;
        }
        *reinterpret_cast<floatx4*>(a0 + c0) = va;
        *reinterpret_cast<floatx4*>(a1 + c0) = vd;
      }
    }
  }
  const bool iin = r0 + i < n;
  const int row = iin ? r0 + i : n - 1;
  const float* tc = a.tcoef + ((size_t)b * (T - 1) + idx) * 3 * n + row;
  // every input of the epilogue is requested before its first store (a store to tgF / gout may alias gF for the
  // compiler, so loads left behind the stores each cost a dependent round trip)
  const float tc0 = tc[0], tc1 = tc[n], tc2 = tc[2 * n];
  float gf[H / 16];
#pragma unroll
  for (int u = 0; u < H / 16; ++u) gf[u] = a.gF[((size_t)b * n + row) * H + cl + 16 * u];
  const size_t blk = (size_t)n * 16;
  float dc0 = 0.f, dc1 = 0.f, dc2 = 0.f;
  if (a.cde) {
    const float* dc = a.data_coef + ((size_t)b * (T - 1) + idx) * 4 * blk + (size_t)row * 16 + cl;
    dc0 = dc[0];
    dc1 = dc[blk];
    dc2 = dc[2 * blk];
  }
  const float tg = iin ? fmaf(f, fmaf(3.0f * f, tc0, 2.0f * tc1), tc2) : 0.f;
#pragma unroll
  for (int u = 0; u < H / 16; ++u) {
    const int c = cl + 16 * u;
    const float g = iin ? tg * gf[u] : 0.f;
    sgo[i][c] = g;
    if (iin) (a.cde ? a.tgF : a.gout)[((size_t)b * n + row) * H + c] = g;
  }
  if (a.cde) {  // tg gF and dX only: g_P, g_q are k_bwd_head_gemm's GEMM over all samples' rows
    const float dx = iin ? fmaf(f, fmaf(3.0f * f, dc0, 2.0f * dc1), dc2) : 0.f;
    if (iin) a.dxo[((size_t)b * n + row) * 16 + cl] = dx;
    return;
  }
  __syncthreads();
  if (!a.cde) {
    // g_P = g_out W': wave ct's 16 x 16 tile, K = H
    if (w < CT) {
      const int ct = w;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KH; ++s) acc = mfma4(sgo[lo][4 * s + hi], a.wl[(4 * s + hi) * H + 16 * ct + lo], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r0 + 4 * hi + r < n) a.gP[((size_t)b * n + r0 + 4 * hi + r) * H + 16 * ct + lo] = acc[r];
    }
    if (tid < kRB) {
      float acc = 0.f;
      for (int jo = 0; jo < H; ++jo) acc = fmaf(sgo[tid][jo], a.bl[jo], acc);
      if (r0 + tid < n) a.gq[(size_t)b * n + r0 + tid] = acc;
    }
    return;
  }
}

// The CDE read-out layer's input cotangents as ONE GEMM over the node rows of every sample (the read-out is
// row-wise; k_bwd_head wrote tgF = tg gF and dX per row):
//   g_P[i][c] = sum_{m, j} (tgF_im dX_ij) W'[16 m + j][c],   g_q[i] = sum_m tgF_im sum_j dX_ij b'[16 m + j]
// A workgroup takes 16 consecutive rows of [B n] (no padded per-sample blocks: n = 129 left a one-row block per
// sample), wave w the output columns 16 (w % CT) .. and the m range of its K part (H < 64: the waves split m, summed
// in LDS in a fixed order).  The A operand tgF_im dX_ij is formed in registers (dX_i. held for the whole K loop); W'
// operands are issued a batch of m ahead, held apart from their use by scheduling barriers (the compiler otherwise
// sinks each load to its MFMA: one L2 round trip per MFMA).
template <int H>
__global__ void __launch_bounds__(256) k_bwd_head_gemm(int rows, const float* __restrict__ tgF,
                                                       const float* __restrict__ dxo, const float* __restrict__ wl,
                                                       const float* __restrict__ bl, float* __restrict__ gP,
                                                       float* __restrict__ gq) {
  constexpr int CT = H / 16, KP = 4 / CT, MP = H / KP;  // column tiles, waves per tile, m per wave
  constexpr int MB = MP < 8 ? MP : 8;                   // m per W' batch
  __shared__ float sg[16][H + 1];
  __shared__ float sx[16][17];
  __shared__ floatx4 red[4][64];
  const int r0 = blockIdx.x * 16;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  const int ct = w % CT, kp = w / CT, m0 = kp * MP;
  // this wave's W' operands: row 16 m + 4 s + hi, column 16 ct + lo (issued before the staging waits)
  const float* wb = wl + (size_t)(16 * m0 + hi) * H + 16 * ct + lo;
  float wv[2][MB][4];
#pragma unroll
  for (int mm = 0; mm < MB; ++mm)
#pragma unroll
    for (int q = 0; q < 4; ++q) wv[0][mm][q] = wb[(size_t)(16 * mm + 4 * q) * H];
  for (int e = tid; e < 16 * H; e += 256) {
    const int R = e / H, c = e % H;
    sg[R][c] = r0 + R < rows ? tgF[(size_t)(r0 + R) * H + c] : 0.f;
  }
  {
    const int R = tid >> 4, j = tid & 15;
    sx[R][j] = r0 + R < rows ? dxo[(size_t)(r0 + R) * 16 + j] : 0.f;
  }
  __syncthreads();
  float dxr[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) dxr[q] = sx[lo][4 * q + hi];
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int mb = 0; mb < MP; mb += MB) {
    const int cur = (mb / MB) & 1;
    if (mb + MB < MP)
#pragma unroll
      for (int mm = 0; mm < MB; ++mm)
#pragma unroll
        for (int q = 0; q < 4; ++q) wv[cur ^ 1][mm][q] = wb[(size_t)(16 * (mb + MB + mm) + 4 * q) * H];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mm = 0; mm < MB; ++mm) {
      const float g = sg[lo][m0 + mb + mm];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = mfma4(g * dxr[q], wv[cur][mm][q], acc);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (KP > 1) {
    red[w][lane] = acc;
    __syncthreads();
    if (kp == 0)
#pragma unroll
      for (int p = 1; p < KP; ++p) acc += red[w + p * CT][lane];
  }
  if (kp == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r0 + 4 * hi + r < rows) gP[(size_t)(r0 + 4 * hi + r) * H + 16 * ct + lo] = acc[r];
  // g_q: row R = tid / 16, m = cl, cl + 16, ... then the 16 lanes of the row in a fixed butterfly
  {
    const int R = tid >> 4, cl = tid & 15;
    float p = 0.f;
    for (int m = cl; m < H; m += 16) {
      float k = 0.f;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) k = fmaf(sx[R][jj], bl[16 * m + jj], k);
      p = fmaf(sg[R][m], k, p);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) p += __shfl_xor(p, o);
    if (cl == 0 && r0 + R < rows) gq[r0 + R] = p;
  }
}

// CDE read-out weight / bias gradient on MFMA, K = the node rows of every sample:
//   part[slot][(16 m + j) (H + 1) + c] += sum_rows (tgF[r][m] dX[r][j]) (P | q)[r][c]
// Workgroup (row chunk kc, m group): wave w owns m = 4 blockIdx.y + w, its 16 x 16 output tiles (rows j, columns c
// = 0 .. H, zero past H) over the chunk's rows; the four waves share the chunk's dX and (P | q) rows, staged in LDS in
// 64-row blocks whose global loads are issued one block ahead.  The chunks are few (one partial slot each, summed
// by k_bwd_reduce once per sweep): the per-evaluation partial traffic is chunks x 16 H (H + 1) floats, and the grid
// is chunks x H / 4 workgroups (~512: two per CU hide each other's LDS and staging latency).
constexpr int kRoBlk = 64;
inline int readout_chunks(int rows, int H) {
  const int groups = H / 4, blocks = (rows + kRoBlk - 1) / kRoBlk;
  int kc = (512 + groups - 1) / groups;
  return kc < blocks ? kc : (blocks > 0 ? blocks : 1);
}
template <int H>
__global__ void __launch_bounds__(256) k_bwd_readout(int rows, int rpc, const float* __restrict__ tgF,
                                                     const float* __restrict__ dxo, const float* __restrict__ pq,
                                                     float* __restrict__ part) {
  constexpr int NT = (H + 1 + 15) / 16, NC = NT * 16, RB = kRoBlk;
  constexpr int NPQ = (RB * (H + 1) + 255) / 256;
  __shared__ float sx[RB][17];
  __shared__ float sp[RB][NC + 1];
  __shared__ float sg[RB][4];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
  const int kc = blockIdx.x, mg = 4 * (int)blockIdx.y, m = mg + w;
  const int rbeg = kc * rpc, rend = rows < rbeg + rpc ? rows : rbeg + rpc;
  for (int e = tid; e < RB * (NC + 1); e += 256) (&sp[0][0])[e] = 0.f;  // columns past H stay zero
  float rdx[4], rpq[NPQ], rtg;
  auto gload = [&](int rb) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, row = rb + (e >> 4);
      rdx[u] = row < rend ? dxo[(size_t)row * 16 + (e & 15)] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NPQ; ++u) {
      const int e = tid + 256 * u, row = rb + e / (H + 1);
      rpq[u] = (e < RB * (H + 1) && row < rend) ? pq[(size_t)row * (H + 1) + e % (H + 1)] : 0.f;
    }
    const int row = rb + (tid >> 2);
    rtg = row < rend ? tgF[(size_t)row * H + mg + (tid & 3)] : 0.f;
  };
  floatx4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (rbeg < rend) gload(rbeg);
  for (int rb = rbeg; rb < rend; rb += RB) {
    __syncthreads();  // the previous block's reads are done (and the zero fill)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      sx[e >> 4][e & 15] = rdx[u];
    }
#pragma unroll
    for (int u = 0; u < NPQ; ++u) {
      const int e = tid + 256 * u;
      if (e < RB * (H + 1)) sp[e / (H + 1)][e % (H + 1)] = rpq[u];
    }
    sg[tid >> 2][tid & 3] = rtg;
    __syncthreads();
    if (rb + RB < rend) gload(rb + RB);  // the next block's loads fly under this block's MFMAs
#pragma unroll 4
    for (int s4 = 0; s4 < RB / 4; ++s4) {
      const int r = 4 * s4 + hi;
      const float av = sg[r][w] * sx[r][lo];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma4(av, sp[r][16 * nt + lo], acc[nt]);
    }
  }
  if (m < H) {
    float* dst = part + (size_t)kc * 16 * H * (H + 1);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int c = 16 * nt + lo;
        if (c <= H) dst[(size_t)(16 * m + 4 * hi + rr) * (H + 1) + c] += acc[nt][rr];
      }
  }
}

// CDE data-spline cotangent (TGB): g_dX[i][j] = sum_m tgF_im (P_i . W'[16m+j, :] + q_i b'[16m+j]), scattered onto
// the stage interval's (d, c, b) with weights (3 f^2, 2 f, 1) (as v_data_grad).  One thread per (sample, node, j).
__global__ void k_bwd_data(int B, int n, int H, int T, const float* __restrict__ ts, const float* __restrict__ t,
                           const float* __restrict__ tgF, const float* __restrict__ pq, const float* __restrict__ wl,
                           const float* __restrict__ bl, float* __restrict__ gcoef) {
  const int b = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * 16) return;
  const int i = e >> 4, jj = e & 15;
  const float* g = tgF + ((size_t)b * n + i) * H;
  const float* p = pq + ((size_t)b * n + i) * (H + 1);
  float s = 0.f;
  for (int m = 0; m < H; ++m) {
    const float* wr = wl + (size_t)(16 * m + jj) * H;
    float fv = p[H] * bl[16 * m + jj];
    for (int c = 0; c < H; ++c) fv = fmaf(p[c], wr[c], fv);
    s = fmaf(g[m], fv, s);
  }
  const float tb = t[b];
  const float* tsb = ts + (size_t)b * T;
  const int idx = interval_index(tsb, T, tb);
  const float f = tb - tsb[idx];
  const size_t blk = (size_t)n * 16;
  float* cb = gcoef + ((size_t)b * (T - 1) + idx) * 4 * blk + e;
  cb[0] = fmaf(3.0f * f * f, s, cb[0]);
  cb[blk] = fmaf(2.0f * f, s, cb[blk]);
  cb[2 * blk] += s;
}

// Reduce the partial slots (fixed order) into gW'[l] [d_out, H] and gb'[l] [d_out] per layer, and the fusion gradient.
// sum_k p[k * stride] for k = 0 .. count-1 in order, 16 loads in flight per batch of the chain
__device__ __forceinline__ float ordered_sum(const float* __restrict__ p, size_t stride, int count) {
  float s = 0.f;
  int k = 0;
  for (; k + 16 <= count; k += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = p[(size_t)(k + u) * stride];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  for (; k < count; ++k) s += p[(size_t)k * stride];
  return s;
}

__global__ void k_bwd_reduce(int slots, int L, int H, int gw_stride, int cde, int ro_chunks,
                             const float* __restrict__ gfc, const float* __restrict__ gw, const float* __restrict__ gwo,
                             float* __restrict__ gfusion, float* __restrict__ gwp, float* __restrict__ gbp) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int nfc = L * GNCDE_FC;
  const int nh = (cde ? L - 1 : L) * (H * H + H);
  if (e < nfc) {
    gfusion[e] = ordered_sum(gfc + e, nfc, slots);
    return;
  }
  int q = e - nfc;
  if (q < nh) {
    const float s = ordered_sum(gw + q, gw_stride, slots);
    const int l = q / (H * H + H), r = q % (H * H + H);
    if (r < H * H) gwp[(size_t)l * H * H + r] = s;  // layers < L-1 (and the ODE output) are H x H
    else gbp[(size_t)l * H + r - H * H] = s;
    return;
  }
  q -= nh;
  if (cde && q < 16 * H * (H + 1)) {
    const float s = ordered_sum(gwo + q, (size_t)16 * H * (H + 1), ro_chunks);
    const int mj = q / (H + 1), c = q % (H + 1);
    const size_t wo = (size_t)(L - 1) * H * H, bo = (size_t)(L - 1) * H;
    if (c < H) gwp[wo + (size_t)mj * H + c] = s;
    else gbp[bo + mj] = s;
  }
}

// g_W'[l], g_b'[l] -> the packed parameter gradient: g_W = g_W' diag(rms_w) + g_b' rms_b^T, g_b = g_b',
// g_rms_w[c] = sum_j g_W'[j][c] W[j][c], g_rms_b[c] = sum_j g_b'[j] W[j][c].  One block per layer.
__global__ void k_bwd_params(int L, int H, int dlast, const float* __restrict__ params, const float* __restrict__ gwp,
                             const float* __restrict__ gbp, float* __restrict__ gparams) {
  const int l = blockIdx.x;
  const int din = H, dout = l == L - 1 ? dlast : H;
  size_t off = 0;
  for (int j = 0; j < l; ++j) off += 2 * (size_t)H + (size_t)H * H + H;
  const float* rw = params + off;
  const float* rb = rw + din;
  const float* W = rb + din;
  const float* gW_ = gwp + (size_t)l * H * H;
  const float* gb_ = gbp + (size_t)l * H;
  float* g = gparams + off;
  for (int e = threadIdx.x; e < dout * din; e += blockDim.x) {
    const int jo = e / din, c = e % din;
    g[2 * din + e] = fmaf(gW_[e], rw[c], gb_[jo] * rb[c]);
  }
  for (int jo = threadIdx.x; jo < dout; jo += blockDim.x) g[2 * din + dout * din + jo] = gb_[jo];
  for (int c = threadIdx.x; c < din; c += blockDim.x) {
    float sw = 0.f, sb = 0.f;
    int jo = 0;
    for (; jo + 8 <= dout; jo += 8) {  // the same order, the loads of 8 rows in flight
      float gw8[8], w8[8], gb8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        gw8[u] = gW_[(size_t)(jo + u) * din + c];
        w8[u] = W[(size_t)(jo + u) * din + c];
        gb8[u] = gb_[jo + u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sw = fmaf(gw8[u], w8[u], sw);
        sb = fmaf(gb8[u], w8[u], sb);
      }
    }
    for (; jo < dout; ++jo) {
      sw = fmaf(gW_[(size_t)jo * din + c], W[(size_t)jo * din + c], sw);
      sb = fmaf(gb_[jo], W[(size_t)jo * din + c], sb);
    }
    g[c] = sw;
    g[din + c] = sb;
  }
}

template <int H>
void launch_layer(const BwdArgs& a, int grid, int rbw, size_t smem, hipStream_t st) {
  hipLaunchKernelGGL((k_bwd_layer<H>), dim3(grid), dim3(256 * rbw), smem, st, a);
}

// Row blocks per k_bwd_layer workgroup: the fewest that put the grid in one round on the device's CUs (one
// workgroup per CU: the LDS), within kMaxRbw and the LDS limit.
int bwd_rbw(const GncdeProblem& p, int nb) {
  static int cus = 0;
  if (!cus) {
    int dev = 0, v = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  if (const char* e = getenv("GNCDE_BWD_RBW")) {  // test hook: a fixed count (the partials do not depend on it)
    const int v = atoi(e);
    if (v >= 1 && v <= kMaxRbw && bwd_smem(p.n, p.dims[0], v) <= 160 * 1024) return v;
  }
  int r = 1;
  while (r < kMaxRbw && (size_t)p.B * ((nb + r - 1) / r) > (size_t)cus && bwd_smem(p.n, p.dims[0], r + 1) <= 160 * 1024)
    ++r;
  return r;
}

bool set_smem(int H, size_t smem) {
  const void* fn = H == 16 ? reinterpret_cast<const void*>(&k_bwd_layer<16>)
                           : (H == 32 ? reinterpret_cast<const void*>(&k_bwd_layer<32>)
                                      : reinterpret_cast<const void*>(&k_bwd_layer<64>));
  return ensure_dyn_lds(fn, smem);
}

}  // namespace

// Envelope: fp32 (the reverse mode of every compute mode runs on the fp32 view), n <= 256, one hidden width
// H in {16, 32, 64} for every layer input, and an ODE output of width H or the de = 8 read-out with h = H.
bool rows_vjp_supported(const GncdeProblem& p) {
  if (p.compute != GNCDE_COMPUTE_FP32 || p.n < 1 || p.n > kMaxN) return false;
  const int H = p.dims[0];
  if (H != 16 && H != 32 && H != 64) return false;
  for (int l = 0; l < p.L; ++l)
    if (p.dims[l] != H) return false;
  if (p.cde_hidden > 0) return p.cde_embed == 8 && p.cde_hidden == H && p.dims[p.L] == 16 * H;
  if (p.dims[p.L] != H) return false;
  // the forward keep needs every layer on the one-launch path or on k_layer (gncde_generic.hip generic_vf_eval)
  if (rows_eval_used(p)) return true;
  for (int l = 0; l < p.L; ++l)
    if (layer_mode(p, l) < 0) return false;
  return true;
}

namespace {
struct RowsVjpWs {
  float *keep, *gP[2], *gq[2], *gout[2], *tgF, *dx, *pq, *gfc, *gw, *gwo, *gwp, *gbp, *dy, *aev;
  int nb, slots, gw_stride, ro_chunks;
};
size_t carve_rows_vjp(const GncdeProblem& p, char* ws, RowsVjpWs& w) {
  const size_t B = p.B, n = p.n, H = p.dims[0];
  const bool cde = p.cde_hidden > 0;
  w.nb = (int)((n + kRB - 1) / kRB);
  w.slots = (int)B * w.nb;
  w.gw_stride = (int)((cde ? p.L - 1 : p.L) * (H * H + H));
  w.ro_chunks = cde ? readout_chunks((int)(B * n), (int)H) : 0;
  size_t off = 0;
  auto take = [&](size_t floats) {
    float* ptr = ws ? reinterpret_cast<float*>(ws + off) : nullptr;
    off += align_up((floats ? floats : 1) * sizeof(float), 256);
    return ptr;
  };
  const size_t E = B * n * H;
  w.keep = take((size_t)(p.L - 1) * E);
  for (int k = 0; k < 2; ++k) {
    w.gP[k] = take(E);
    w.gq[k] = take(B * n);
    w.gout[k] = take(E);
  }
  w.tgF = take(cde ? E : 0);
  w.dx = take(cde ? B * n * 16 : 0);
  w.pq = take(cde ? B * n * (H + 1) : 0);
  w.gfc = take((size_t)w.slots * p.L * GNCDE_FC);
  w.gw = take((size_t)w.slots * w.gw_stride);
  w.gwo = take((size_t)w.ro_chunks * 16 * H * (H + 1));
  w.gwp = take((size_t)(p.L - 1) * H * H + (size_t)p.dims[p.L] * H);
  w.gbp = take((size_t)(p.L - 1) * H + p.dims[p.L]);
  w.dy = take(B * n * (size_t)out_dim(p));
  const size_t np = bwd_np(p.n);
  w.aev = take(B * 2 * np * np);
  return off;
}
}  // namespace

size_t rows_vjp_workspace(const GncdeProblem& p) {
  RowsVjpWs w;
  return carve_rows_vjp(p, nullptr, w);
}

void rows_vjp_begin(const GncdeProblem& p, char* ws, hipStream_t st) {
  RowsVjpWs w;
  carve_rows_vjp(p, ws, w);
  const size_t H = p.dims[0];
  (void)hipMemsetAsync(w.gfc, 0, (size_t)w.slots * p.L * GNCDE_FC * sizeof(float), st);
  (void)hipMemsetAsync(w.gw, 0, (size_t)w.slots * w.gw_stride * sizeof(float), st);
  if (w.ro_chunks) (void)hipMemsetAsync(w.gwo, 0, (size_t)w.ro_chunks * 16 * H * (H + 1) * sizeof(float), st);
}

// The VJP of one evaluation at (t, u) for the cotangent gF: the stage input's cotangent into gu (overwritten), the
// parameter / fusion partials accumulated in the workspace, gdata (optional) accumulated.  wf / bfold: W', b' of
// every layer back to back (generic_vf_prepare's fold).
int rows_vf_vjp(const GncdeProblem& p, const float* t, const float* u, const float* gF, float* gu, float* gdata,
                const float* csum, const float* wf, const float* bfold, char* ws, char* vf_ws, unsigned* bars,
                hipStream_t st, const float* kept, const StageScatter* scat) {
  RowsVjpWs w;
  carve_rows_vjp(p, ws, w);
  const int B = p.B, n = p.n, H = p.dims[0], L = p.L;
  const bool cde = p.cde_hidden > 0;
  // the hidden outputs: the forward's activation record, or a forward in keep mode now
  const float* keep = kept;
  if (!keep) {
    const int rc = generic_vf_eval(p, t, u, w.dy, vf_ws, st, true, bars, w.keep, false);
    if (rc) return rc;
    keep = w.keep;
  }
  const size_t E = (size_t)B * n * H;
  size_t wo_last = 0, bo_last = 0;
  for (int l = 0; l + 1 < L; ++l) {
    wo_last += (size_t)H * H;
    bo_last += H;
  }
  {
    HeadArgs h{};
    h.B = B;
    h.n = n;
    h.T = p.T;
    h.H = H;
    h.cde = cde ? 1 : 0;
    h.ts = p.ts;
    h.coef = p.coef;
    h.aev = w.aev;
    h.tcoef = p.tcoef;
    h.data_coef = p.data_coef;
    h.t = t;
    h.gF = gF;
    h.wl = wf + wo_last;
    h.bl = bfold + bo_last;
    h.gout = w.gout[0];
    h.gP = w.gP[0];
    h.gq = w.gq[0];
    h.tgF = w.tgF;
    h.dxo = w.dx;
    if (H == 16) hipLaunchKernelGGL(k_bwd_head<16>, dim3(B * w.nb), dim3(256), 0, st, h);
    else if (H == 32) hipLaunchKernelGGL(k_bwd_head<32>, dim3(B * w.nb), dim3(256), 0, st, h);
    else hipLaunchKernelGGL(k_bwd_head<64>, dim3(B * w.nb), dim3(256), 0, st, h);
    if (cde) {
      const dim3 g((B * n + 15) / 16);
      if (H == 16) hipLaunchKernelGGL(k_bwd_head_gemm<16>, g, dim3(256), 0, st, B * n, w.tgF, w.dx, h.wl, h.bl, h.gP, h.gq);
      else if (H == 32) hipLaunchKernelGGL(k_bwd_head_gemm<32>, g, dim3(256), 0, st, B * n, w.tgF, w.dx, h.wl, h.bl, h.gP, h.gq);
      else hipLaunchKernelGGL(k_bwd_head_gemm<64>, g, dim3(256), 0, st, B * n, w.tgF, w.dx, h.wl, h.bl, h.gP, h.gq);
    }
  }
  const int rbw = bwd_rbw(p, w.nb), grid = B * ((w.nb + rbw - 1) / rbw);
  const size_t smem = bwd_smem(n, H, rbw);
  if (!set_smem(H, smem)) return GNCDE_ERR_HIP;
  int cur = 0;
  for (int l = L - 1; l >= 0; --l) {
    BwdArgs a{};
    a.B = B;
    a.n = n;
    a.T = p.T;
    a.L = L;
    a.l = l;
    a.nb = w.nb;
    a.ts = p.ts;
    a.aev = w.aev;
    a.csum = csum;
    a.fusion = p.fusion;
    a.t = t;
    a.zin = l == 0 ? u : keep + (size_t)(l - 1) * E;
    a.gP = w.gP[cur];
    a.gq = w.gq[cur];
    a.gout = w.gout[cur];
    a.wprev = l > 0 ? wf + (size_t)(l - 1) * H * H : nullptr;
    a.bprev = l > 0 ? bfold + (size_t)(l - 1) * H : nullptr;
    a.gP_next = w.gP[cur ^ 1];
    a.gq_next = w.gq[cur ^ 1];
    a.gout_next = w.gout[cur ^ 1];
    a.gz = gu;
    a.scatter = scat != nullptr;
    if (scat) a.sc = *scat;
    a.pq = w.pq;
    a.gfc = w.gfc;
    a.gw = w.gw;
    a.gw_stride = w.gw_stride;
    a.gw_off = l * (H * H + H);
    a.cde_out = (cde && l == L - 1) ? 1 : 0;
    if (H == 16) launch_layer<16>(a, grid, rbw, smem, st);
    else if (H == 32) launch_layer<32>(a, grid, rbw, smem, st);
    else launch_layer<64>(a, grid, rbw, smem, st);
    cur ^= 1;
  }
  if (cde) {
    const int rows = B * n, rpc = ((rows + w.ro_chunks - 1) / w.ro_chunks + kRoBlk - 1) / kRoBlk * kRoBlk;
    const dim3 g(w.ro_chunks, H / 4);
    if (H == 16) hipLaunchKernelGGL(k_bwd_readout<16>, g, dim3(256), 0, st, rows, rpc, w.tgF, w.dx, w.pq, w.gwo);
    else if (H == 32) hipLaunchKernelGGL(k_bwd_readout<32>, g, dim3(256), 0, st, rows, rpc, w.tgF, w.dx, w.pq, w.gwo);
    else hipLaunchKernelGGL(k_bwd_readout<64>, g, dim3(256), 0, st, rows, rpc, w.tgF, w.dx, w.pq, w.gwo);
    if (gdata)
      hipLaunchKernelGGL(k_bwd_data, dim3((n * 16 + 255) / 256, B), dim3(256), 0, st, B, n, H, p.T, p.ts, t, w.tgF,
                         w.pq, wf + wo_last, bfold + bo_last, gdata);
  }
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

void rows_vjp_finish(const GncdeProblem& p, char* ws, float* gparams, float* gfusion, hipStream_t st) {
  RowsVjpWs w;
  carve_rows_vjp(p, ws, w);
  const int H = p.dims[0], L = p.L;
  const bool cde = p.cde_hidden > 0;
  const int tot = L * GNCDE_FC + (cde ? L - 1 : L) * (H * H + H) + (cde ? 16 * H * (H + 1) : 0);
  hipLaunchKernelGGL(k_bwd_reduce, dim3((tot + 255) / 256), dim3(256), 0, st, w.slots, L, H, w.gw_stride, cde ? 1 : 0,
                     w.ro_chunks, w.gfc, w.gw, w.gwo, gfusion, w.gwp, w.gbp);
  hipLaunchKernelGGL(k_bwd_params, dim3(L), dim3(256), 0, st, L, H, p.dims[L], p.params, w.gwp, w.gbp, gparams);
}

}  // namespace gncde

#ifdef GNCDE_BWD_STAMPS
extern "C" int gncde_debug_bwd_stamps(unsigned long long* host, int count) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gncde::g_bwd_stamps), sizeof(unsigned long long) * count) == hipSuccess ? 0
                                                                                                                  : -1;
}
#endif

#ifdef GNCDE_DIAG
// Diagnostic builds only (-DGNCDE_DIAG; not part of include/gncde.h): one evaluation with the hidden outputs kept.
extern "C" int gncde_diag_keep(const GncdeProblem* prob, const float* t, const float* y, float* dy, float* keep,
                               void* ws, size_t ws_bytes, void* stream) {
  using namespace gncde;
  const int rc = validate_problem(prob);
  if (rc) return rc;
  if (ws_bytes < generic_vf_workspace(*prob)) return GNCDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  generic_vf_prepare(*prob, static_cast<char*>(ws), st);
  unsigned bars = 0;
  return generic_vf_eval(*prob, t, y, dy, static_cast<char*>(ws), st, true, &bars, keep);
}

// Diagnostic (not part of include/gncde.h): the reverse mode of ONE evaluation through the per-layer kernels.
extern "C" int gncde_diag_vf_vjp(const GncdeProblem* prob, const float* t, const float* y, const float* gF, float* gy,
                                 float* gparams, float* gfusion, void* ws, size_t ws_bytes, void* stream) {
  using namespace gncde;
  const int rc0 = validate_problem(prob);
  if (rc0) return rc0;
  const GncdeProblem& p = *prob;
  if (!rows_vjp_supported(p)) return GNCDE_ERR_UNSUPPORTED;
  const size_t L = p.L, H = p.dims[0];
  size_t wfs = 0, bfs = 0;
  for (size_t l = 0; l < L; ++l) {
    wfs += (size_t)p.dims[l] * p.dims[l + 1];
    bfs += p.dims[l + 1];
  }
  const size_t need = align_up((wfs + bfs) * sizeof(float), 256) + rows_vjp_workspace(p) + generic_vf_workspace(p);
  if (ws_bytes < need || !ws) return GNCDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* wf = static_cast<float*>(ws);
  float* bf = wf + wfs;
  char* rows_ws = static_cast<char*>(ws) + align_up((wfs + bfs) * sizeof(float), 256);
  char* vf_ws = rows_ws + rows_vjp_workspace(p);
  size_t wo = 0, bo = 0;
  for (int l = 0; l < p.L; ++l) {
    const LayerOffsets o = layer_offsets(p, l);
    fold_linear(p.dims[l], p.dims[l + 1], p.params + o.rms_w, p.params + o.rms_b, p.params + o.W, p.params + o.b,
                wf + wo, bf + bo, st);
    wo += (size_t)p.dims[l] * p.dims[l + 1];
    bo += p.dims[l + 1];
  }
  (void)H;
  generic_vf_prepare(p, vf_ws, st);
  rows_vjp_begin(p, rows_ws, st);
  unsigned bars = 0;
  const int rc = rows_vf_vjp(p, t, y, gF, gy, nullptr, generic_vf_csum(p, vf_ws), wf, bf, rows_ws, vf_ws, &bars, st);
  if (rc) return rc;
  rows_vjp_finish(p, rows_ws, gparams, gfusion, st);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

extern "C" size_t gncde_diag_vf_vjp_bytes(const GncdeProblem* prob) {
  using namespace gncde;
  const GncdeProblem& p = *prob;
  size_t wfs = 0, bfs = 0;
  for (int l = 0; l < p.L; ++l) {
    wfs += (size_t)p.dims[l] * p.dims[l + 1];
    bfs += p.dims[l + 1];
  }
  return align_up((wfs + bfs) * sizeof(float), 256) + rows_vjp_workspace(p) + generic_vf_workspace(p);
}
#endif  // GNCDE_DIAG
