// Fused persistent integrate kernel for the dyn family (GraphNeuralCDE: use_control=False, all layer
// widths equal H) — the BASELINE hot path (configs 1, 2, 4).
//
// One workgroup integrates one sample over its whole step grid.  NP/16 waves; wave w owns the node
// block [16w, 16w+16).  Everything between the HBM coefficient reads and the final state stays on
// chip:
//
//   per distinct stage time t (RK4: 2 per step, since k2/k3 share t+h/2 and k4/k1' share t+h):
//     interval index (wave ballot over ts in LDS) -> Horner of the interval's (d,c,b,a) [4,n,n]
//     (coalesced float4 HBM/L2 reads) -> A(t), dA(t) in LDS (padded row stride NP+1: conflict-free row AND
//     column access) -> row/col sums, diagonals, totals -> each lane builds its slice of
//     (I + Abar_l) for every layer l IN REGISTERS (the MFMA B-operand layout), fusing the
//     15-term equivariant basis (layers.py:102-160) into the operand construction.
//   per vector-field evaluation (perm_equiv_graph_vector_field.py:122-128, layers.py:36-48):
//     RMSNorm (in-register + 2 cross-lane shuffles) -> Linear on MFMA 16x16x4 f32 with the state
//     tile as B operand (no LDS) -> m^T tile to LDS -> barrier -> (I+Abar) m on MFMA 16x16x4 f32,
//     A operand = m^T from LDS (ds_read_b128), B operand = Abar registers -> ReLU -> next layer.
//   RK stage combinations in registers; only y0 in and the saved states out touch HBM.
//
// State layout per wave ("T-layout", the MFMA 16x16 C/D map): lane l holds Y[f][i] for node
// i = 16w + (l&15) and features f = 16*fb + 4*(l>>4) + r, r = 0..3, fb = 0..H/16-1.
#include "gncde_internal.h"

#include <cstdio>
#include <cstring>

namespace gncde {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));  // v_pk_fma_f32 / v_pk_add_f32 operands
typedef __attribute__((address_space(4))) const float CFloat;  // constant address space: uniform reads are s_load

constexpr int kTMax = 256;  // knots per sample held in LDS

struct FusedArgs {
  int B, n, T, G, save_mode;
  const float* ts;
  const float* coef;
  const float* tcoef;
  const float* fusion;
  const float* params;
  const float* grid;
  const int32_t* nsteps;
  const float* y0;
  float* ys;
  int32_t* stats;
  // adaptive (PID) controller
  const float* t0;
  const float* t1;
  const float* dt0;  // NULL -> Hairer initial step (diffrax dt0=None)
  const float* save_ts;
  int n_save, max_steps;
  float rtol, atol;
  float* step_ts;  // [B, step_len] accepted step times (GncdeSolver.step_ts) or nullptr
  int step_len;
  float* rec;      // GRID: stage record [B, G-1, S-1, n, H] (GncdeSolver.stage_rec) or nullptr
};

constexpr int kTsit5Pid = 2;  // internal METHOD id: Tsit5 + PIDController (diffrax defaults)

// A(t)/dA(t) LDS images use a padded row stride NP+1: row AND column walks are bank-conflict free
// and every address is lane base + compile-time offset (no per-element address registers).
template <int NP>
__device__ __forceinline__ int swz(int i, int k) {
  return i * (NP + 1) + k;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int NP, int H, int L, int METHOD>
constexpr int min_waves_per_eu() {
  constexpr int regs = L * (NP / 4) + (METHOD != GNCDE_RK4 ? 9 : 4) * (H / 4) + 4 * (H / 4) + 40;
  return NP >= 128 ? 2 : (regs > 120 ? 2 : 4);
}

template <int NP, int H, int L, int METHOD>
__global__ void __launch_bounds__(NP * 4, (min_waves_per_eu<NP, H, L, METHOD>())) k_fused(FusedArgs a) {
  constexpr int NT = NP * 4;
  constexpr int FB = H / 16;
  constexpr int KS = NP / 4;
  constexpr int MS = NP + 4;
  constexpr int AS = NP * (NP + 1);  // one padded A image
  constexpr int R0 = (2 * AS > 2 * H * MS) ? 2 * AS : 2 * H * MS;
  constexpr int PL = H + FB * FB * 4 * 64;  // bias', W' operands (RMSNorm affine folded)

  __shared__ __attribute__((aligned(16))) float sR0[R0];
  __shared__ __attribute__((aligned(16))) float sVec[(6 + L) * NP];
  __shared__ float sTs[kTMax];
  __shared__ __attribute__((aligned(16))) float sPar[L * PL];
  __shared__ float sFus[L * GNCDE_FC];
  __shared__ float sRed[2][NP / 16];  // per-wave partials for workgroup sums (double-buffered)

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int w = tid >> 6;
  const int lane = tid & 63;
  const int lo = lane & 15, hi = lane >> 4;
  const int n = a.n, T = a.T;
  const size_t nn = (size_t)n * n;
  const int node = 16 * w + lo;
  const bool node_ok = node < n;

  // ---- stage per-sample knots and the layer parameters in LDS --------------------------------------
  // RMSNorm's affine is folded into the Linear (exact algebra, fp32 rounding only):
  //   W (z*inv*w + b_rms) + bias = inv * (W diag(w)) z + (W b_rms + bias)
  // so a layer needs W' = W diag(w) as MFMA A-operands and bias' = bias + W b_rms.
  for (int j = tid; j < T; j += NT) sTs[j] = a.ts[(size_t)b * T + j];
  for (int j = tid; j < L * GNCDE_FC; j += NT) sFus[j] = a.fusion[j];
  {
    size_t off = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      float* P = sPar + l * PL;
      const float* g = a.params + off;
      const float* rw = g;
      const float* rb = g + H;
      const float* W = g + 2 * H;
      const float* bias = g + 2 * H + H * H;
      for (int j = tid; j < H; j += NT) {
        float acc = bias[j];
        for (int k = 0; k < H; ++k) acc = fmaf(W[j * H + k], rb[k], acc);
        P[j] = acc;  // bias'
      }
      // W' operand for (ob, fb, r) at lane: W'[16ob + lo'][16fb + 4hi' + r]
      for (int j = tid; j < FB * FB * 4 * 64; j += NT) {
        const int ln = j & 63, r = (j >> 6) & 3, fb = (j >> 8) % FB, ob = (j >> 8) / FB;
        const int row = 16 * ob + (ln & 15), col = 16 * fb + 4 * (ln >> 4) + r;
        P[H + j] = W[row * H + col] * rw[col];
      }
      off += 2 * H + H * H + H;
    }
  }
  __syncthreads();

  float* sA = sR0;
  float* sdA = sR0 + AS;
  float Ab[L][KS];   // (D_l + w_l 1^T + 1 v_l^T)[node][k], k = hi*KS + sl  (MFMA B operand)
  float ul[L];       // diagonal u_l[node] (incl. ConvLayer residual 1), applied in eval
  float tg = 0.f;
  int msel = 0;
  float* sVl = sVec + 6 * NP;  // v_l[k], L x NP

  // ---- (I + Abar_l) operands for stage time t --------------------------------------------------------
  int widx = 0;  // interval index of the previous form (wave-uniform)
  auto form = [&](float t) __attribute__((always_inline)) {
    // The form phase (HBM loads, VALU, LDS) runs at raised wave priority: the co-resident waves of the other
    // samples on this SIMD are mostly in their MFMA-bound eval phase and fill the gaps (config 2: -6%).
    __builtin_amdgcn_s_setprio(1);
    __syncthreads();  // readers of the aliased M buffers are done
    // Opaque per-call copy of the thread id: keeps this phase's per-lane LDS bases from being hoisted
    // out of the time loop (they would stay live in registers across the whole solve).
    int ftid = tid;
    asm volatile("" : "+v"(ftid));
    const int lane = ftid & 63, lo = lane & 15, hi = lane >> 4;
    const int i = 16 * (ftid >> 6) + lo;
    const float* fus = sFus;  // fusion table staged in LDS (uniform broadcast reads)
    // interval index clip(searchsorted(ts, t, 'left') - 1, 0, T-2), i.e. the largest j <= T-2 with ts[j] < t (or 0),
    // walked from the previous form's index on wave-uniform LDS reads: a stage time moves by about one knot per
    // form, and the walk also runs backwards for the PID controller's rejected attempts
    int idx = widx;
    while (idx < T - 2 && sTs[idx + 1] < t) ++idx;
    while (idx > 0 && !(sTs[idx] < t)) --idx;
    widx = idx;
    const float f = t - sTs[idx];
    const float f3 = 3.0f * f;
    const float* cb = a.coef + ((size_t)b * (T - 1) + idx) * 4 * nn;
    // time-channel coefficients: loaded first so their HBM round trip overlaps the interval's Horner pass.
    // Buffer loads: the (sample, interval) base is wave-uniform (descriptor in SGPRs), so a load costs no
    // 64-bit VALU address arithmetic; the plane / iteration offsets ride in soffset.
    float tc0, tc1, tc2;
    {
      const auto trs = rsrc(a.tcoef + ((size_t)b * (T - 1) + idx) * 3 * n, 12u * (unsigned)n);
      const int vo = (i < n ? i : 0) * 4;
      tc0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(trs, vo, 0, 0));
      tc1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(trs, vo, 4 * n, 0));
      tc2 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(trs, vo, 8 * n, 0));
    }
    if (n == NP) {
      constexpr int NQ = NP * NP / 4;   // float4s per plane
      constexpr int QR = NP / 4;        // float4s per image row
      constexpr int RPI = NT / QR;      // image rows per iteration (16)
      static_assert(NQ % NT == 0 && NT % QR == 0, "Horner tiling");
      // thread -> (row, 4 columns) of the first iteration; later iterations move RPI rows down, so every LDS
      // address is one per-lane base plus a compile-time offset
      const unsigned uft = (unsigned)ftid;
      const int rr = (int)(uft / QR), kq = (int)(uft % QR) * 4;
      const int vo = (int)uft * 16;
      const auto crs = rsrc(cb, 16u * NQ * 4);
      float* pa0 = sA + swz<NP>(rr, kq);
      float* pd0 = sdA + swz<NP>(rr, kq);
      // every coefficient load of the interval is issued before the first use (one HBM round trip per form
      // instead of NQ/NT dependent ones)
      // (in groups of at most 4 iterations = 64 VGPRs of loads: NP = 128 takes two round trips)
      constexpr int NIT = NQ / NT, GRP = NIT > 4 ? 4 : NIT;
#pragma unroll
      for (int g0 = 0; g0 < NIT; g0 += GRP) {
      floatx4 cq[GRP][4];
#pragma unroll
      for (int u = 0; u < GRP; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          cq[u][q] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(crs, vo, (q * NQ + (g0 + u) * NT) * 16, 0));
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int it = g0 + u;
        const floatx4 d = cq[u][0], c = cq[u][1], bb = cq[u][2], aa = cq[u][3];
        float* pa = pa0 + it * RPI * (NP + 1);
        float* pd = pd0 + it * RPI * (NP + 1);
        // element pairs on packed FMAs (same per-element Horner order as a scalar chain)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const floatx2 d2 = h2 ? floatx2{d.z, d.w} : floatx2{d.x, d.y};
          const floatx2 c2 = h2 ? floatx2{c.z, c.w} : floatx2{c.x, c.y};
          const floatx2 b2 = h2 ? floatx2{bb.z, bb.w} : floatx2{bb.x, bb.y};
          const floatx2 a2 = h2 ? floatx2{aa.z, aa.w} : floatx2{aa.x, aa.y};
          const floatx2 ff = {f, f}, f33 = {f3, f3}, two = {2.0f, 2.0f};
          const floatx2 va = __builtin_elementwise_fma(ff, __builtin_elementwise_fma(ff, __builtin_elementwise_fma(ff, d2, c2), b2), a2);
          const floatx2 vd = __builtin_elementwise_fma(ff, __builtin_elementwise_fma(f33, d2, two * c2), b2);
          pa[2 * h2] = va.x;
          pa[2 * h2 + 1] = va.y;
          pd[2 * h2] = vd.x;
          pd[2 * h2 + 1] = vd.y;
        }
      }
      }
    } else {  // padded image: rows/cols >= n are zero, so they add nothing to sums or operands
      for (int e = ftid; e < NP * NP; e += NT) {
        const int r = e / NP, k = e % NP;
        float va = 0.f, vd = 0.f;
        if (r < n && k < n) {
          const int ce = r * n + k;
          const float d = cb[ce], c = cb[nn + ce], bb = cb[2 * nn + ce], aa = cb[3 * nn + ce];
          va = fmaf(f, fmaf(f, fmaf(f, d, c), bb), aa);
          vd = fmaf(f, fmaf(f3, d, 2.0f * c), bb);
        }
        sA[swz<NP>(r, k)] = va;
        sdA[swz<NP>(r, k)] = vd;
      }
    }
    __syncthreads();
    {  // r, rd (row sums), c, cd (column sums), diagonals: 4 NP threads, one line each
      const int q = ftid / NP, j = ftid % NP;
      const float* M = (q & 1) ? sdA : sA;
      float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;  // 4 chains: latency, not adds, bound this
      if (q < 2) {
        const float* row = M + swz<NP>(j, 0);
#pragma unroll 4
        for (int k = 0; k < NP; k += 4) {
          acc0 += row[k];
          acc1 += row[k + 1];
          acc2 += row[k + 2];
          acc3 += row[k + 3];
        }
        sVec[(4 + q) * NP + j] = M[swz<NP>(j, j)];
      } else {
        const float* col = M + j;
#pragma unroll 4
        for (int k = 0; k < NP; k += 4) {
          acc0 += col[swz<NP>(k, 0)];
          acc1 += col[swz<NP>(k + 1, 0)];
          acc2 += col[swz<NP>(k + 2, 0)];
          acc3 += col[swz<NP>(k + 3, 0)];
        }
      }
      sVec[q * NP + j] = (acc0 + acc1) + (acc2 + acc3);
    }
    __syncthreads();
    // The per-layer fusion coefficients are read through the constant address space: wave-uniform scalar loads
    // into SGPRs, so the factored families below are one FMA per term with no VALU spent on the coefficients.
    const CFloat* fz = (const CFloat*)(a.fusion);
    // v_l[k] = vR_A r_k + vR_dA rd_k + vC_A c_k + vC_dA cd_k  (zero for padded k: sums are zero)
    if constexpr (NP >= 64) {  // one layer per wave (or wave pair): the layer index is wave-uniform
      constexpr int WPL = NP / 64;
      const int wv = __builtin_amdgcn_readfirstlane(ftid >> 6);
      const int l = wv / WPL;
      if (l < L) {
        const int k = (wv % WPL) * 64 + lane;
        const CFloat* fc = fz + l * GNCDE_FC;
        sVl[l * NP + k] = fmaf(fc[GNCDE_FC_VR_A], sVec[k], fmaf(fc[GNCDE_FC_VR_DA], sVec[NP + k],
                          fmaf(fc[GNCDE_FC_VC_A], sVec[2 * NP + k], fc[GNCDE_FC_VC_DA] * sVec[3 * NP + k])));
      }
    } else {
      for (unsigned e = (unsigned)ftid; e < (unsigned)(L * NP); e += NT) {
        const unsigned l = e / NP, k = e % NP;
        const float* fc = fus + l * GNCDE_FC;
        sVl[e] = fc[GNCDE_FC_VR_A] * sVec[k] + fc[GNCDE_FC_VR_DA] * sVec[NP + k] +
                 fc[GNCDE_FC_VC_A] * sVec[2 * NP + k] + fc[GNCDE_FC_VC_DA] * sVec[3 * NP + k];
      }
    }
    float s = 0.f, sd = 0.f;
    for (int j = lane; j < NP; j += 64) {
      s += sVec[j];
      sd += sVec[NP + j];
    }
    s = wave_sum64(s);
    sd = wave_sum64(sd);
    __syncthreads();
    const float ri = sVec[i], rdi = sVec[NP + i], ci = sVec[2 * NP + i], cdi = sVec[3 * NP + i];
    const float dgi = sVec[4 * NP + i], dgdi = sVec[5 * NP + i];
    float wl[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const CFloat* fc = fz + l * GNCDE_FC;
      const float ws = fmaf(fc[GNCDE_FC_WS_A], s, fc[GNCDE_FC_WS_DA] * sd);
      const float w = fmaf(fc[GNCDE_FC_WR_A], ri, fmaf(fc[GNCDE_FC_WR_DA], rdi,
                      fmaf(fc[GNCDE_FC_WC_A], ci, fmaf(fc[GNCDE_FC_WC_DA], cdi, ws))));
      wl[l] = i < n ? w : 0.f;
      ul[l] = fmaf(fc[GNCDE_FC_UD_A], dgi, fmaf(fc[GNCDE_FC_UD_DA], dgdi, fmaf(fc[GNCDE_FC_UR_A], ri,
              fmaf(fc[GNCDE_FC_UR_DA], rdi, fmaf(fc[GNCDE_FC_UC_A], ci, fmaf(fc[GNCDE_FC_UC_DA], cdi,
              fmaf(fc[GNCDE_FC_US_A], s, fmaf(fc[GNCDE_FC_US_DA], sd, fc[GNCDE_FC_IDC]))))))));
    }
    // operand slice: row i of A/dA at columns k = hi*KS + sl, column i at rows k.  Each of the four image
    // elements is read ONCE and feeds every layer's operand (4 + L LDS reads per element instead of 5 L);
    // the per-layer coefficients are wave-uniform and live in SGPRs.  Offsets are opaque integers (the
    // accesses stay ds_read, not flat) and every operand is pinned as soon as it is formed, so the loaded
    // values stay short-lived.
    float ec[L][4];
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
      for (int q = 0; q < 4; ++q) ec[l][q] = fz[l * GNCDE_FC + q];
    {
      // Chunks of 4 slices: all 16 image reads and the L float4 reads of v_l are issued before the first
      // use, so a chunk waits on LDS once; the pins at the end of a chunk keep the next chunk's loads
      // from being hoisted (register pressure), not the loads of this one.
      // v0 stays a visible multiple of 16 floats (hi comes from the opaque ftid), so the v_l reads are aligned
      // ds_read_b128 with immediate offsets
      int r0 = swz<NP>(i, hi * KS), c0 = swz<NP>(hi * KS, i);
      const int v0 = 6 * NP + hi * KS;
      asm volatile("" : "+v"(r0), "+v"(c0));
#pragma unroll
      for (int s4 = 0; s4 < KS; s4 += 4) {
        float ar[4], dr[4], ac[4], dc[4];
        floatx4 vv[L];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ar[j] = sR0[r0 + s4 + j];
          dr[j] = sR0[AS + r0 + s4 + j];
          ac[j] = sR0[c0 + (s4 + j) * (NP + 1)];
          dc[j] = sR0[AS + c0 + (s4 + j) * (NP + 1)];
        }
#pragma unroll
        for (int l = 0; l < L; ++l) vv[l] = *reinterpret_cast<const floatx4*>(sVec + v0 + l * NP + s4);
        // two adjacent slices per packed op (v_pk_fma_f32 with the SGPR coefficient broadcast): half the
        // VALU issue of the scalar chain, same operation order
#pragma unroll
        for (int j = 0; j < 4; j += 2)
#pragma unroll
          for (int l = 0; l < L; ++l) {
            const floatx2 a2 = {ar[j], ar[j + 1]}, d2 = {dr[j], dr[j + 1]};
            const floatx2 at2 = {ac[j], ac[j + 1]}, dt2 = {dc[j], dc[j + 1]};
            floatx2 x = floatx2{vv[l][j], vv[l][j + 1]} + floatx2{wl[l], wl[l]};
            x = __builtin_elementwise_fma(floatx2{ec[l][3], ec[l][3]}, dt2, x);
            x = __builtin_elementwise_fma(floatx2{ec[l][2], ec[l][2]}, at2, x);
            x = __builtin_elementwise_fma(floatx2{ec[l][1], ec[l][1]}, d2, x);
            x = __builtin_elementwise_fma(floatx2{ec[l][0], ec[l][0]}, a2, x);
            Ab[l][s4 + j] = x.x;
            Ab[l][s4 + j + 1] = x.y;
          }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int l = 0; l < L; ++l) asm volatile("" : "+v"(Ab[l][s4 + j]));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    tg = i < n ? fmaf(f, fmaf(f3, tc0, 2.0f * tc1), tc2) : 0.f;
    __syncthreads();  // all A/dA reads done before the aliased M buffers are written
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- one vector-field evaluation: Kout = VF(Yin) at the formed time --------------------------------
  auto eval = [&](const float (&Yin)[FB][4], float (&Kout)[FB][4]) __attribute__((always_inline)) {
    float Z[FB][4];
#pragma unroll
    for (int fb = 0; fb < FB; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) Z[fb][r] = Yin[fb][r];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      // Opaque base: keeps the (invariant) parameter reads inside the loop instead of hoisting
      // L*(3H/4 + FB*FB*4) values into registers for the whole solve.
      int po = l * PL;
      asm volatile("" : "+v"(po));
      const float* P = sPar + po;
      float ss = 0.f;
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) ss = fmaf(Z[fb][r], Z[fb][r], ss);
      const float inv = rms_inv(xor_sum_rows4(ss), 1.0f / (float)H);
      float* Mb = sR0 + msel * (H * MS);
      msel ^= 1;
      floatx4 mown[FB];  // this lane's own m tile (T-layout), for the diagonal term u_l * m
#pragma unroll
      for (int ob = 0; ob < FB; ++ob) {
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int fb = 0; fb < FB; ++fb)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc = mfma4(P[H + ((ob * FB + fb) * 4 + r) * 64 + lane], Z[fb][r], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[r] = fmaf(inv, acc[r], P[16 * ob + 4 * hi + r]);
          // padded nodes contribute zero rows of m (their Abar columns are not masked)
          Mb[(16 * ob + 4 * hi + r) * MS + node] = node_ok ? acc[r] : 0.f;
        }
        mown[ob] = acc;
      }
      __syncthreads();
#pragma unroll
      for (int ob = 0; ob < FB; ++ob) {
        floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
        const float* mrow = Mb + (16 * ob + lo) * MS + hi * KS;
#pragma unroll
        for (int q = 0; q < KS / 4; ++q) {
          const float4 mv = *reinterpret_cast<const float4*>(mrow + 4 * q);
          c0 = mfma4(mv.x, Ab[l][4 * q + 0], c0);
          c1 = mfma4(mv.y, Ab[l][4 * q + 1], c1);
          c0 = mfma4(mv.z, Ab[l][4 * q + 2], c0);
          c1 = mfma4(mv.w, Ab[l][4 * q + 3], c1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = fmaf(ul[l], mown[ob][r], c0[r] + c1[r]);
          Z[ob][r] = (l < L - 1) ? fmaxf(z, 0.f) : z;
        }
      }
    }
#pragma unroll
    for (int fb = 0; fb < FB; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) Kout[fb][r] = node_ok ? tg * Z[fb][r] : 0.f;
  };

  bool have = false;
  float tcache = 0.f;
  auto vf = [&](float t, const float (&Yin)[FB][4], float (&Kout)[FB][4]) __attribute__((always_inline)) {
    if (!have || t != tcache) {
      form(t);
      tcache = t;
      have = true;
    }
    eval(Yin, Kout);
  };

  // ---- state I/O (reference layout [n, H]) -------------------------------------------------------------
  float y[FB][4];
  const float* y0b = a.y0 + (size_t)b * n * H;
#pragma unroll
  for (int fb = 0; fb < FB; ++fb)
#pragma unroll
    for (int r = 0; r < 4; ++r) y[fb][r] = node_ok ? y0b[(size_t)node * H + 16 * fb + 4 * hi + r] : 0.f;

  auto store_from = [&](float* dst, const float (&v)[FB][4]) __attribute__((always_inline)) {
    if (!node_ok) return;
#pragma unroll
    for (int fb = 0; fb < FB; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(size_t)node * H + 16 * fb + 4 * hi + r] = v[fb][r];
  };
  auto store = [&](float* dst) __attribute__((always_inline)) { store_from(dst, y); };

  const size_t E = (size_t)n * H;

  // Single vf() call site per method (one inlined copy of form/eval keeps the register budget).
  if constexpr (METHOD == GNCDE_RK4 || METHOD == GNCDE_TSIT5) {
  const int G = a.G;
  const float* g = a.grid + (size_t)b * G;
  int ns = a.nsteps[b];
  ns = ns < 0 ? 0 : (ns > G - 1 ? G - 1 : ns);  // never index past the grid row
  if (a.save_mode == GNCDE_SAVE_STEPS) store(a.ys + ((size_t)b * G) * E);
  if constexpr (METHOD == GNCDE_RK4) {
    float K[FB][4], acc[FB][4], yt[FB][4];
    for (int k = 0; k < ns; ++k) {
      const float t = g[k];
      const float h = g[k + 1] - t;
      const float hh = 0.5f * h;
      const float tm = stage_time(t, 0.5f, h);
      const float te = __fadd_rn(t, h);
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) yt[fb][r] = y[fb][r];
#pragma unroll 1
      for (int st = 0; st < 4; ++st) {
        const float tst = st == 0 ? t : (st == 3 ? te : tm);
        vf(tst, yt, K);
        const float wk = (st == 0 || st == 3) ? 1.0f : 2.0f;  // k1 + 2k2 + 2k3 + k4
        const float hn = st < 2 ? hh : h;                      // next stage input y + hn*K
#pragma unroll
        for (int fb = 0; fb < FB; ++fb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc[fb][r] = st == 0 ? K[fb][r] : fmaf(wk, K[fb][r], acc[fb][r]);
            yt[fb][r] = fmaf(hn, K[fb][r], y[fb][r]);
          }
        if (a.rec && st < 3) store_from(a.rec + (((size_t)b * (G - 1) + k) * 3 + st) * E, yt);  // U_{st+1}
      }
      const float h6 = h / 6.0f;
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[fb][r] = fmaf(h6, acc[fb][r], y[fb][r]);
      if (a.save_mode == GNCDE_SAVE_STEPS) store(a.ys + ((size_t)b * G + k + 1) * E);
    }
  } else {
    // Tsit5 on the grid (ConstantStepSize), FSAL: stage s (1..6) input y + h*sum_j a[s][j] k_j,
    // stage 7 input == y1 (a[7][:] = b) and its evaluation is the next step's k_1.
    float kk[7][FB][4], yt[FB][4], K[FB][4];
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) kk[j][fb][r] = 0.f;
    const float t0 = g[0];
#pragma unroll
    for (int fb = 0; fb < FB; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) yt[fb][r] = y[fb][r];
    float tst = t0;
    int st = 0;   // 0 = initial k1 evaluation; then stages 1..6 of every step
    int k = 0;
    float t = t0, h = 0.f;
    while (true) {
      vf(tst, yt, K);
#pragma unroll
      for (int j = 0; j < 7; ++j)
        if (j == st)
#pragma unroll
          for (int fb = 0; fb < FB; ++fb)
#pragma unroll
            for (int r = 0; r < 4; ++r) kk[j][fb][r] = K[fb][r];
      if (st == 6) {  // y1 accepted; stage-7 value is the next k1
#pragma unroll
        for (int fb = 0; fb < FB; ++fb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            y[fb][r] = yt[fb][r];
            kk[0][fb][r] = K[fb][r];
          }
        if (a.save_mode == GNCDE_SAVE_STEPS) store(a.ys + ((size_t)b * G + k + 1) * E);
        ++k;
        st = 0;
      }
      if (k >= ns) break;
      if (st == 0) {
        t = g[k];
        h = g[k + 1] - t;
      }
      // next stage st+1 (1..6): coefficients a[st+1][0..st]
      const int ns1 = st + 1;
      float arow[6], cst;
      tsit5_row(ns1, arow, cst);
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sacc = 0.f;
#pragma unroll
          for (int j = 0; j < 6; ++j) sacc = fmaf(arow[j], kk[j][fb][r], sacc);
          yt[fb][r] = fmaf(h, sacc, y[fb][r]);
        }
      if (a.rec && ns1 <= 5) store_from(a.rec + (((size_t)b * (G - 1) + k) * 5 + ns1 - 1) * E, yt);  // U_ns1
      tst = ns1 == 6 ? g[k + 1] : ns1 == 5 ? __fadd_rn(t, h) : stage_time(t, cst, h);  // FSAL stage at the knot
      st = ns1;
    }
  }
  if (a.rec) {  // padded steps (h = 0): every stage input is the final state, as the generic forward records it
    const int S1 = METHOD == GNCDE_RK4 ? 3 : 5;
    for (int k = ns; k < G - 1; ++k)
      for (int i = 0; i < S1; ++i) store(a.rec + (((size_t)b * (G - 1) + k) * S1 + i) * E);
  }
  if (a.save_mode == GNCDE_SAVE_STEPS) {
    for (int k = ns + 1; k < G; ++k) store(a.ys + ((size_t)b * G + k) * E);
  } else {
    store(a.ys + (size_t)b * E);
  }
  if (a.stats && tid == 0) {
    a.stats[b * 4 + GNCDE_STAT_STEPS] = ns;
    a.stats[b * 4 + GNCDE_STAT_REJECTS] = 0;
    a.stats[b * 4 + GNCDE_STAT_EVALS] = METHOD == GNCDE_RK4 ? 4 * ns : 1 + 6 * ns;
    a.stats[b * 4 + GNCDE_STAT_STATUS] = 0;
  }
  } else {
    // ---- Tsit5 + PIDController(rtol, atol) (graph_neural_cde.py:53-54,94-104; diffrax defaults:
    // pcoeff 0, icoeff 1, dcoeff 0, safety 0.9, factormin 0.2 (1 on accept), factormax 10, RMS norm,
    // error order 5), FSAL, optional Hairer initial step (dt0 = None), SaveAt(ts) via the Tsit5
    // dense interpolant or SaveAt(t1).  Every wave follows the same (uniform) control flow.
    int wsel = 0;
    const float inv_cnt = 1.0f / (float)(n * H);
    auto wg_sum = [&](float v) __attribute__((always_inline)) -> float {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      wsel ^= 1;
      if (lane == 0) sRed[wsel][w] = v;
      __syncthreads();
      float tot = 0.f;
#pragma unroll
      for (int j = 0; j < NP / 16; ++j) tot += sRed[wsel][j];
      return tot;
    };
    const float rtol = a.rtol, atol = a.atol;
    const float t0 = a.t0[b], t1 = a.t1[b];
    const int S = a.save_mode == GNCDE_SAVE_TS ? a.n_save : 0;
    const float* sts = a.save_ts ? a.save_ts + (size_t)b * S : nullptr;
    float* ysb = a.ys + (size_t)b * (S > 0 ? S : 1) * E;
    int si = 0;
    while (si < S && sts[si] <= t0) store(ysb + (size_t)(si++) * E);
    float kk[7][FB][4], yt[FB][4], K[FB][4];
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) kk[j][fb][r] = 0.f;
#pragma unroll
    for (int fb = 0; fb < FB; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) yt[fb][r] = y[fb][r];
    const bool auto_dt = a.dt0 == nullptr;
    float dt = auto_dt ? 0.f : a.dt0[b];
    float t = t0, tn = t0, h = 0.f, tst = t0, h0 = 0.f, d1 = 0.f;
    int phase = 0, st = 0, steps = 0, rejects = 0, evals = 0, status = 0;
    if (a.step_ts && tid == 0) a.step_ts[(size_t)b * a.step_len] = t0;
    while (true) {
      vf(tst, yt, K);
      ++evals;
      if (phase == 0) {  // f(t0, y0): FSAL k1 (and f0 of the initial-step heuristic)
#pragma unroll
        for (int fb = 0; fb < FB; ++fb)
#pragma unroll
          for (int r = 0; r < 4; ++r) kk[0][fb][r] = K[fb][r];
        phase = 2;
        if (auto_dt) {
          float p0 = 0.f, p1 = 0.f;
#pragma unroll
          for (int fb = 0; fb < FB; ++fb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float sc = fmaf(fabsf(y[fb][r]), rtol, atol);
              const float u = y[fb][r] / sc, v = K[fb][r] / sc;
              p0 = node_ok ? fmaf(u, u, p0) : p0;
              p1 = node_ok ? fmaf(v, v, p1) : p1;
            }
          const float d0 = sqrtf(wg_sum(p0) * inv_cnt);
          d1 = sqrtf(wg_sum(p1) * inv_cnt);
          h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : 0.01f * (d0 / d1);
#pragma unroll
          for (int fb = 0; fb < FB; ++fb)
#pragma unroll
            for (int r = 0; r < 4; ++r) yt[fb][r] = fmaf(h0, K[fb][r], y[fb][r]);
          tst = t0 + h0;
          phase = 1;
          continue;
        }
      } else if (phase == 1) {  // f(t0 + h0, y0 + h0 f0)
        float p2 = 0.f;
#pragma unroll
        for (int fb = 0; fb < FB; ++fb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float sc = fmaf(fabsf(y[fb][r]), rtol, atol);
            const float v = (K[fb][r] - kk[0][fb][r]) / sc;
            p2 = node_ok ? fmaf(v, v, p2) : p2;
          }
        const float d2 = sqrtf(wg_sum(p2) * inv_cnt) / h0;
        const float md = fmaxf(d1, d2);
        const float h1 = md <= 1e-15f ? fmaxf(1e-6f, h0 * 1e-3f) : powf(0.01f / md, 0.2f);
        dt = fminf(100.0f * h0, h1);
        phase = 2;
      } else {
#pragma unroll
        for (int j = 1; j < 7; ++j)
          if (j == st)
#pragma unroll
            for (int fb = 0; fb < FB; ++fb)
#pragma unroll
              for (int r = 0; r < 4; ++r) kk[j][fb][r] = K[fb][r];
        if (st == 6) {  // attempt done: yt = y1 candidate, kk[6] = f(tn, y1)
          float pe = 0.f;
#pragma unroll
          for (int fb = 0; fb < FB; ++fb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float e = h * (TSIT5_E1 * kk[0][fb][r] + TSIT5_E2 * kk[1][fb][r] + TSIT5_E3 * kk[2][fb][r] +
                                   TSIT5_E4 * kk[3][fb][r] + TSIT5_E5 * kk[4][fb][r] + TSIT5_E6 * kk[5][fb][r] +
                                   TSIT5_E7 * kk[6][fb][r]);
              const float sc = fmaf(fmaxf(fabsf(y[fb][r]), fabsf(yt[fb][r])), rtol, atol);
              const float v = e / sc;
              pe = node_ok ? fmaf(v, v, pe) : pe;
            }
          const float err = sqrtf(wg_sum(pe) * inv_cnt);
          const bool finite = isfinite(err);
          const bool keep = finite && err < 1.0f;
          float factor;
          if (!finite) {
            factor = 0.2f;
          } else {
            const float f1 = err == 0.f ? 10.0f : 0.9f * powf(1.0f / err, 0.2f);
            factor = fminf(fmaxf(f1, keep ? 1.0f : 0.2f), 10.0f);
          }
          if (keep) {
            while (si < S && sts[si] <= tn) {  // dense output inside (t, tn]
              float wts[7];
              tsit5_dense((sts[si] - t) / h, wts);
              if (node_ok) {
                float* dst = ysb + (size_t)si * E;
#pragma unroll
                for (int fb = 0; fb < FB; ++fb)
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    float acc = 0.f;
#pragma unroll
                    for (int j = 0; j < 7; ++j) acc = fmaf(wts[j], kk[j][fb][r], acc);
                    dst[(size_t)node * H + 16 * fb + 4 * hi + r] = fmaf(h, acc, y[fb][r]);
                  }
              }
              ++si;
            }
#pragma unroll
            for (int fb = 0; fb < FB; ++fb)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                y[fb][r] = yt[fb][r];
                kk[0][fb][r] = kk[6][fb][r];
              }
            if (a.step_ts && tid == 0 && steps + 1 < a.step_len) a.step_ts[(size_t)b * a.step_len + steps + 1] = tn;
            t = tn;
            ++steps;
          } else {
            ++rejects;
          }
          dt = factor * h;
          st = 0;
        }
      }
      if (st == 0) {  // start a new attempt
        if (!(t < t1)) break;
        if (steps + rejects >= a.max_steps) {
          status = 1;
          break;
        }
        tn = t + dt;
        if (tn > t1 - 1e-6f) tn = t1;  // diffrax _clip_to_end
        h = tn - t;
      }
      const int ns1 = st + 1;
      float arow[6], cst;
      tsit5_row(ns1, arow, cst);
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sacc = 0.f;
#pragma unroll
          for (int j = 0; j < 6; ++j) sacc = fmaf(arow[j], kk[j][fb][r], sacc);
          yt[fb][r] = fmaf(h, sacc, y[fb][r]);
        }
      tst = ns1 == 6 ? tn : ns1 == 5 ? __fadd_rn(t, h) : stage_time(t, cst, h);  // FSAL stage at the step end
      st = ns1;
    }
    if (a.step_ts && status == 0 && steps + 1 > a.step_len) status = 3;  // step record truncated
    if (S == 0) {
      store(ysb);
    } else {
      while (si < S) store(ysb + (size_t)(si++) * E);  // only reached on failure (status != 0)
    }
    if (a.stats && tid == 0) {
      a.stats[b * 4 + GNCDE_STAT_STEPS] = steps;
      a.stats[b * 4 + GNCDE_STAT_REJECTS] = rejects;
      a.stats[b * 4 + GNCDE_STAT_EVALS] = evals;
      a.stats[b * 4 + GNCDE_STAT_STATUS] = status;
    }
  }
}

using FusedFn = void (*)(FusedArgs);

struct FusedEntry {
  int np, h, l, method;
  FusedFn fn;
};

#define GNCDE_FUSED(NP, H, L)                                        \
  {NP, H, L, GNCDE_RK4, k_fused<NP, H, L, GNCDE_RK4>},             \
  {NP, H, L, GNCDE_TSIT5, k_fused<NP, H, L, GNCDE_TSIT5>},         \
  {NP, H, L, kTsit5Pid, k_fused<NP, H, L, kTsit5Pid>}

const FusedEntry kFused[] = {
    GNCDE_FUSED(16, 16, 1),  GNCDE_FUSED(16, 16, 2),  GNCDE_FUSED(16, 16, 3),  GNCDE_FUSED(16, 16, 4),
    GNCDE_FUSED(32, 16, 1),  GNCDE_FUSED(32, 16, 2),  GNCDE_FUSED(32, 16, 3),  GNCDE_FUSED(32, 16, 4),
    GNCDE_FUSED(64, 16, 1),  GNCDE_FUSED(64, 16, 2),  GNCDE_FUSED(64, 16, 3),  GNCDE_FUSED(64, 16, 4),
    GNCDE_FUSED(128, 16, 1), GNCDE_FUSED(128, 16, 2), GNCDE_FUSED(128, 16, 3),
    GNCDE_FUSED(16, 32, 1),  GNCDE_FUSED(16, 32, 2),  GNCDE_FUSED(16, 32, 3),  GNCDE_FUSED(16, 32, 4),
    GNCDE_FUSED(32, 32, 1),  GNCDE_FUSED(32, 32, 2),  GNCDE_FUSED(32, 32, 3),  GNCDE_FUSED(32, 32, 4),
    GNCDE_FUSED(64, 32, 1),  GNCDE_FUSED(64, 32, 2),  GNCDE_FUSED(64, 32, 3),  GNCDE_FUSED(64, 32, 4),
    GNCDE_FUSED(128, 32, 1), GNCDE_FUSED(128, 32, 2),
};

const FusedEntry* find_fused(const GncdeProblem& p, const GncdeSolver& s) {
  if (p.cde_hidden != 0 || p.compute != GNCDE_COMPUTE_FP32) return nullptr;
  int method = s.method;
  if (s.controller == GNCDE_CTRL_GRID) {
    if (s.save_mode != GNCDE_SAVE_T1 && s.save_mode != GNCDE_SAVE_STEPS) return nullptr;
  } else {  // PID: Tsit5 only (the reference's adaptive configuration)
    if (s.method != GNCDE_TSIT5) return nullptr;
    if (s.save_mode != GNCDE_SAVE_T1 && s.save_mode != GNCDE_SAVE_TS) return nullptr;
    method = kTsit5Pid;
  }
  if (p.T > kTMax) return nullptr;
  const int H = p.dims[0];
  for (int l = 1; l <= p.L; ++l)
    if (p.dims[l] != H) return nullptr;
  int np = 0;
  for (int c : {16, 32, 64, 128})
    if (p.n <= c) {
      np = c;
      break;
    }
  if (np == 0) return nullptr;
  for (const FusedEntry& e : kFused)
    if (e.np == np && e.h == H && e.l == p.L && e.method == method) return &e;
  return nullptr;
}

}  // namespace

bool fused_supported(const GncdeProblem& p, const GncdeSolver& s, char* name, size_t name_len) {
  const FusedEntry* e = find_fused(p, s);
  if (!e) return false;
  if (name && name_len)
    snprintf(name, name_len, "fused<%d,%d,%d,%s>", e->np, e->h, e->l,
             e->method == GNCDE_RK4 ? "rk4" : (e->method == GNCDE_TSIT5 ? "tsit5" : "tsit5_pid"));
  return true;
}

int fused_integrate(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys,
                    int32_t* stats, hipStream_t st) {
  const FusedEntry* e = find_fused(p, s);
  if (!e) return GNCDE_ERR_UNSUPPORTED;
  FusedArgs a;
  a.B = p.B;
  a.n = p.n;
  a.T = p.T;
  a.G = s.grid_len;
  a.save_mode = s.save_mode;
  a.ts = p.ts;
  a.coef = p.coef;
  a.tcoef = p.tcoef;
  a.fusion = p.fusion;
  a.params = p.params;
  a.grid = s.grid;
  a.nsteps = s.nsteps;
  a.y0 = y0;
  a.ys = ys;
  a.stats = stats;
  a.t0 = s.t0;
  a.t1 = s.t1;
  a.dt0 = s.dt0;
  a.save_ts = s.save_ts;
  a.n_save = s.n_save;
  a.max_steps = s.max_steps;
  a.rtol = s.rtol;
  a.atol = s.atol;
  a.step_ts = s.controller == GNCDE_CTRL_PID ? s.step_ts : nullptr;
  a.step_len = s.step_ts_len;
  a.rec = s.controller == GNCDE_CTRL_GRID && s.grid_len >= 2 ? s.stage_rec : nullptr;
  hipLaunchKernelGGL(e->fn, dim3(p.B), dim3(e->np * 4), 0, st, a);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

}  // namespace gncde
