// Fused per-stage kernels for the reverse sweep of a fixed-grid solve (the discrete adjoint
// that jax.grad takes through diffrax, trainer.py:315).  One workgroup per sample, NP/16 wave64s, wave w
// owns nodes [16w, 16w+16), all layer widths H = 16 (the dyn family: configs 1, 2, 4).
//
//   k_stage<NP, L, false>  (EVAL):  K = VF(t, U)                       — stage recompute
//   k_stage<NP, L, true>   (VJP):   gU = (dVF/dU)^T gK, and the per-sample parameter / fusion-table
//                                   gradients accumulated into gp[b] (+=), gU scattered into up to 7
//                                   cotangent accumulators (lambda and the earlier stages' gK_j)
//
// Per launch the sample's interval is formed once (Horner of (d,c,b,a) into padded LDS images of A(t) and
// dA(t), row/col/diag/total reductions, the factored fusion vectors u, w, v).  The VJP then:
//   forward (kept): per layer RMSNorm -> Linear (MFMA, RMSNorm affine folded) -> (I+Abar) m (MFMA, operand
//     built from LDS just for that layer) -> ReLU; inputs, m, pre-activations and 1/rms stay in registers;
//   backward, layer by layer:
//     gpre = gZ * relu'(pre);  G = gpre m^T on MFMA, 16 rows at a time — contracted on the fly with the
//     A, dA, A^T, dA^T elements that the transposed operand build reads anyway (the 4 dense fusion-table
//     gradients cost no extra LDS traffic); the rank-1 / diagonal families use R_i = gpre_i . colsum(m),
//     C_k = m_k . colsum(gpre), D_i = gpre_i . m_i;  gm = (I+Abar)^T gpre on MFMA with the column slice of
//     Abar as operand;  gW += gm^T zn (MFMA over the wave's nodes), gzn = W^T gm (MFMA), RMSNorm backward.
// Gradients stay lane-distributed in registers until one cross-wave reduction at the end (fixed order:
// deterministic, no atomics).
#include "gncde_internal.h"

namespace gncde {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

// v_pk_fma_f32: two independent fp32 FMAs per VALU issue (same per-element operation order as fmaf)
__device__ __forceinline__ floatx2 pkfma(floatx2 a, floatx2 b, floatx2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ floatx2 bc2(float v) { return floatx2{v, v}; }

constexpr int H = 16;
constexpr int kTMaxS = 256;
// per-layer operand block prepared by k_stage_prep
constexpr int kOpBias = 0;     // bias' = bias + W rms_b                       [16]
constexpr int kOpWf = 16;      // forward operand  W'[lo][4hi+r] = W[lo][4hi+r] rms_w[4hi+r]   [4][64]
constexpr int kOpWb = 272;     // backward operand W[4hi+r][lo]                 [4][64]
constexpr int kOpRw = 528;     // rms_w                                         [16]
constexpr int kOpRb = 544;     // rms_b                                         [16]
constexpr int kOpStride = 560;
constexpr int kLayerP = 2 * H + H * H + H;   // packed params of one layer (gncde.h order)
constexpr int kGradStride = kLayerP + GNCDE_FC;  // per-sample accumulator block of one layer

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Orders this wave's LDS accesses across lanes (a store by one lane, a later load of it by another) without a
// workgroup barrier: the LDS executes one wave's DS instructions in issue order, so only the compiler must not
// move memory accesses across this point.
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int NP>
__device__ __forceinline__ int swz(int i, int k) {
  return i * (NP + 1) + k;
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

template <int MASK>
__device__ __forceinline__ float swzf(float v) {  // lane ^ MASK within each 32-lane half (MASK < 32)
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), (MASK << 10) | 0x1F));
}

// Sum over the 16 lanes sharing lane>>4, all on DPP (quad swaps, half-row and row mirrors): no LDS traffic.
__device__ __forceinline__ float xor_sum16(float v) {
  v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppf<0x141>(v);  // row_half_mirror
  v += dppf<0x140>(v);  // row_mirror
  return v;
}

// Reduce 32 per-lane values over the wave: recursive halving (xor 16, 8, 4, 2, 1 inside each 32-lane half, then
// one xor 32) -> lane l holds the wave total of value (l & 31).  31 + 1 exchanges instead of 32 x 6.
__device__ __forceinline__ float reduce_scatter32(float (&v)[32], int lane) {
#define GNCDE_RS_STEP(M, XCH)                                   \
  {                                                             \
    const bool up = (lane & (M)) != 0;                          \
    _Pragma("unroll") for (int i = 0; i < (M); ++i) {           \
      const float send = up ? v[i] : v[(M) + i];                \
      const float keep = up ? v[(M) + i] : v[i];                \
      v[i] = keep + XCH(send);                                  \
    }                                                           \
  }
  GNCDE_RS_STEP(16, swzf<16>)
  GNCDE_RS_STEP(8, swzf<8>)
  GNCDE_RS_STEP(4, swzf<4>)
  GNCDE_RS_STEP(2, dppf<0x4E>)
  GNCDE_RS_STEP(1, dppf<0xB1>)
#undef GNCDE_RS_STEP
  return v[0] + __shfl_xor(v[0], 32);
}

__device__ __forceinline__ float xor_sum4(float v) {  // sum over the 4 lane groups (same lane&15)
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

__global__ void k_stage_prep(const float* __restrict__ params, float* __restrict__ ops) {
  const int l = blockIdx.x;
  const float* g = params + (size_t)l * kLayerP;
  const float* rw = g;
  const float* rb = g + H;
  const float* W = g + 2 * H;
  const float* bias = g + 2 * H + H * H;
  float* o = ops + (size_t)l * kOpStride;
  for (int j = threadIdx.x; j < kOpStride; j += blockDim.x) {
    float v;
    if (j < kOpWf) {
      v = bias[j];
      for (int k = 0; k < H; ++k) v = fmaf(W[j * H + k], rb[k], v);
    } else if (j < kOpWb) {
      const int q = j - kOpWf, ln = q & 63, r = q >> 6;
      const int row = ln & 15, col = 4 * (ln >> 4) + r;
      v = W[row * H + col] * rw[col];
    } else if (j < kOpRw) {
      const int q = j - kOpWb, ln = q & 63, r = q >> 6;
      v = W[(4 * (ln >> 4) + r) * H + (ln & 15)];
    } else if (j < kOpRb) {
      v = rw[j - kOpRw];
    } else {
      v = rb[j - kOpRb];
    }
    o[j] = v;
  }
}

enum { kEval1 = 0, kEval2 = 1, kVjpMid = 2, kVjpPair = 3, kBoundary = 4, kEvalRk4 = 5, kBoundaryPair = 6, kStepRk4 = 7 };

struct RevArgs {
  int n, T, G, k, S, stage, has_next, has_cur, write_next;
  const float* ts;
  const float* coef;
  const float* tcoef;
  const float* fusion;
  const float* ops;     // [L, kOpStride]
  const float* grid;    // [B, G]
  const int32_t* nsteps;
  const float* ys;      // checkpoints [B, G, n, H]
  const float* gys;     // saved-state cotangents [B, G, n, H] (SAVE_STEPS) or nullptr
  const float* gst;     // extra stage-value cotangents [B, G-1, S, n, H] (gncde_integrate_vjp_ex) or nullptr
  const float* rec;     // the forward's stage record [B, G-1, S-1, n, H] (GncdeSolver.stage_rec) or nullptr
  float* K[6];          // stage values      [B, n, H] each
  float* U[6];          // stage inputs
  float* gK[6];         // stage cotangents
  float* gyacc;         // cotangent of y_k being accumulated
  float* lam;           // lambda at the last grid point (boundary with has_next == 0)
  float* gy0;           // boundary with has_cur == 0: output
  float* gp;            // [B, L, kGradStride] (+=)
  float c[6], bw[6], a[6][6];
};

// Reverse-sweep kernels.  PROG:
//   kEval1    stage `stage` of step k: U = y_k + h sum_j a[stage][j] K_j; K_stage = VF(U)   (write_next: also
//             U_{stage+1}, the input of the last stage)
//   kEval2    RK4 stages 1, 2 (shared time t + h/2): U1, K1, U2, K2 and U3 = y + h K2
//   kVjpMid   one middle stage: gU = J^T gK_stage; gyacc += gU; gK_j += h a[stage][j] gU
//   kVjpPair  RK4 stages 2 then 1 at t + h/2 (gK1 updated in registers between them)
//   kBoundary at t_{k+1}: stage 0 of step k+1 (has_next) -> lambda_{k+1}; seeds gK_j = h b_j lambda of step
//             k and its last stage (has_cur) -> gyacc, gK_j.  has_cur == 0 writes gy0 = lambda_0.
template <int NP, int L, int PROG>
__global__ void __launch_bounds__(NP * 4, 1) k_rev(RevArgs a) {
  constexpr bool EVAL_RK4 = PROG == kEvalRk4 || PROG == kStepRk4;  // stage 0 at t, then stages 1, 2 at t + h/2
  constexpr bool BOUND_PAIR = PROG == kBoundaryPair || PROG == kStepRk4;  // boundary at t_{k+1}, then stages 2, 1
  constexpr bool VJP = PROG == kVjpMid || PROG == kVjpPair || PROG == kBoundary || BOUND_PAIR;
  constexpr int NT = NP * 4;
  constexpr int NW = NP / 16;
  constexpr int KS = NP / 4;
  constexpr int MS = NP + 4;
  constexpr int AS = NP * (NP + 1);
  constexpr int RED = VJP ? NW * L * kGradStride : 0;
  constexpr int R0 = (2 * AS > RED) ? 2 * AS : RED;

  __shared__ __attribute__((aligned(16))) float sR0[R0];
  __shared__ __attribute__((aligned(16))) float sMb[H * MS];
  __shared__ __attribute__((aligned(16))) float sGb[H * MS];
  __shared__ float sVec[(6 + 2 * L) * NP];
  __shared__ float sTs[kTMaxS];
  __shared__ float sFus[L * GNCDE_FC];
  __shared__ float sCol[1][NW][H];
  // the layers' operand blocks (k_stage_prep), staged once: read from global memory, every Linear and RMSNorm
  // parameter access was a dependent L1/L2 round trip on the evaluation's critical path (up to seven in a row per
  // backward layer: tools/isa_review.py disassembly, round 6)
  __shared__ __attribute__((aligned(16))) float sOp[L * kOpStride];

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int w = tid >> 6;
  const int lane = tid & 63;
  const int lo = lane & 15, hi = lane >> 4;
  const int n = a.n, T = a.T, G = a.G;
  const size_t nn = (size_t)n * n;
  const int node = 16 * w + lo;
  const bool node_ok = node < n;
  const size_t E = (size_t)n * H;
  const size_t rowoff = (size_t)b * E + (size_t)(node_ok ? node : 0) * H + 4 * hi;
  auto rowk = [&](int k) -> size_t { return ((size_t)b * G + k) * E + (size_t)(node_ok ? node : 0) * H + 4 * hi; };
  auto rowst = [&](int k, int j) -> size_t {
    return (((size_t)b * (G - 1) + k) * a.S + j) * E + (size_t)(node_ok ? node : 0) * H + 4 * hi;
  };
  float* sA = sR0;
  float* sdA = sR0 + AS;
  float* sW = sVec + 6 * NP;
  float* sV = sVec + (6 + L) * NP;

  for (int j = tid; j < T; j += NT) sTs[j] = a.ts[(size_t)b * T + j];
  for (int j = tid; j < L * GNCDE_FC; j += NT) sFus[j] = a.fusion[j];
  for (int j = tid; j < L * kOpStride; j += NT) sOp[j] = a.ops[j];

  // step geometry of this sample (padded steps past nsteps have h = 0 and contribute nothing)
  const float* gr = a.grid + (size_t)b * G;
  int ns = a.nsteps[b];
  ns = ns < 0 ? 0 : (ns > G - 1 ? G - 1 : ns);
  auto geom = [&](int k, float& t, float& h) {
    t = k < ns ? gr[k] : gr[ns];
    h = k < ns ? gr[k + 1] - gr[k] : 0.f;
  };

  // ---- form: interval at t -> LDS images, reductions, fusion vectors, per-node terms ------------------
  float ul[L];
  float tg = 0.f, rn = 0.f, rdn = 0.f, cn = 0.f, cdn = 0.f, dgn = 0.f, dgdn = 0.f, s = 0.f, sd = 0.f;
  auto form = [&](float t) __attribute__((always_inline)) {
    __syncthreads();  // previous readers of the LDS images / staging buffers are done
    int cnt = 0;
    for (int j0 = 0; j0 < T; j0 += 64) {
      const int j = j0 + lane;
      const bool p = (j < T) && (sTs[j < T ? j : 0] < t);
      cnt += __popcll(__ballot(p));
    }
    int idx = cnt - 1;
    idx = idx < 0 ? 0 : (idx > T - 2 ? T - 2 : idx);
    const float f = t - sTs[idx];
    const float f3 = 3.0f * f;
    const float* cb = a.coef + ((size_t)b * (T - 1) + idx) * 4 * nn;
    // time-channel coefficients first: their HBM round trip overlaps the interval's Horner pass
    float tc0, tc1, tc2;
    {
      const float* tc = a.tcoef + ((size_t)b * (T - 1) + idx) * 3 * n;
      const int ii = node_ok ? node : 0;
      tc0 = tc[ii];
      tc1 = tc[n + ii];
      tc2 = tc[2 * n + ii];
    }
    if (n == NP) {
      const float4* c4 = reinterpret_cast<const float4*>(cb);
      constexpr int NQ = NP * NP / 4;
      // fully unrolled: every coefficient load of the interval is in flight before the first use (one HBM
      // round trip per form instead of NP/16 dependent ones; the form is the sweep's HBM-bound phase)
#pragma unroll
      for (int it = 0; it < NQ / NT; ++it) {
        const int e4 = tid + it * NT;
        const float4 d = c4[e4], c = c4[NQ + e4], bb = c4[2 * NQ + e4], aa = c4[3 * NQ + e4];
        const int r = (e4 * 4) / NP, k = (e4 * 4) % NP;
        float* pa = sA + swz<NP>(r, k);
        float* pd = sdA + swz<NP>(r, k);
        // element pairs on packed FMAs (same per-element Horner order as the scalar form)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const floatx2 d2 = h2 ? floatx2{d.z, d.w} : floatx2{d.x, d.y};
          const floatx2 c2 = h2 ? floatx2{c.z, c.w} : floatx2{c.x, c.y};
          const floatx2 b2 = h2 ? floatx2{bb.z, bb.w} : floatx2{bb.x, bb.y};
          const floatx2 a2 = h2 ? floatx2{aa.z, aa.w} : floatx2{aa.x, aa.y};
          const floatx2 va = pkfma(bc2(f), pkfma(bc2(f), pkfma(bc2(f), d2, c2), b2), a2);
          const floatx2 vd = pkfma(bc2(f), pkfma(bc2(f3), d2, bc2(2.0f) * c2), b2);
          pa[2 * h2] = va.x;
          pa[2 * h2 + 1] = va.y;
          pd[2 * h2] = vd.x;
          pd[2 * h2 + 1] = vd.y;
        }
      }
    } else {
#pragma unroll 8
      for (int e = tid; e < NP * NP; e += NT) {
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
    {
      const int q = tid / NP, j = tid % NP;
      const float* M = (q & 1) ? sdA : sA;
      float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
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
    s = 0.f;
    sd = 0.f;
    for (int j = lane; j < NP; j += 64) {
      s += sVec[j];
      sd += sVec[NP + j];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_xor(s, o);
      sd += __shfl_xor(sd, o);
    }
    for (int e = tid; e < L * NP; e += NT) {
      const int l = e / NP, k = e % NP;
      const float* fc = sFus + l * GNCDE_FC;
      const float r = sVec[k], rd = sVec[NP + k], c = sVec[2 * NP + k], cd = sVec[3 * NP + k];
      sV[e] = fc[GNCDE_FC_VR_A] * r + fc[GNCDE_FC_VR_DA] * rd + fc[GNCDE_FC_VC_A] * c + fc[GNCDE_FC_VC_DA] * cd;
      const float wv = fc[GNCDE_FC_WR_A] * r + fc[GNCDE_FC_WR_DA] * rd + fc[GNCDE_FC_WC_A] * c +
                       fc[GNCDE_FC_WC_DA] * cd + fc[GNCDE_FC_WS_A] * s + fc[GNCDE_FC_WS_DA] * sd;
      sW[e] = k < n ? wv : 0.f;
    }
    rn = sVec[node];
    rdn = sVec[NP + node];
    cn = sVec[2 * NP + node];
    cdn = sVec[3 * NP + node];
    dgn = sVec[4 * NP + node];
    dgdn = sVec[5 * NP + node];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const float* fc = sFus + l * GNCDE_FC;
      ul[l] = fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * dgn + fc[GNCDE_FC_UD_DA] * dgdn + fc[GNCDE_FC_UR_A] * rn +
              fc[GNCDE_FC_UR_DA] * rdn + fc[GNCDE_FC_UC_A] * cn + fc[GNCDE_FC_UC_DA] * cdn + fc[GNCDE_FC_US_A] * s +
              fc[GNCDE_FC_US_DA] * sd;
    }
    tg = node_ok ? fmaf(f, fmaf(f3, tc0, 2.0f * tc1), tc2) : 0.f;
    __syncthreads();  // sW / sV visible
  };

  // ---- forward at the formed time, activations kept for the backward ----------------------------------
  // activations of up to two stage evaluations at the formed time (slot 0 / 1; forward2 fills both)
  float Zin[2][L][4], invl[2][L], ml[2][L][4], prel[2][L][4];
  // K range of lane group hi: [hi*KS, hi*KS + KS), walked from offset kRot: at NP = 128 the groups hi = 0 / 1 (and
  // 2 / 3) of one 32-lane half would otherwise hit the same banks (hi*KS = 32 = 0 mod 32) — 2-way conflicts on
  // every operand-build read; rotating the odd groups by 16 puts them on the other 16 banks.
  const int kRot = KS == 32 ? 16 * (hi & 1) : 0;
  const int oAr = swz<NP>(node, hi * KS), oAc = swz<NP>(hi * KS, node);
  // full == false (a forward whose backward follows): the last layer's (I+Abar) m product is skipped — the
  // backward needs only its m (and the earlier layers' pre-activations), never the stage value itself.
  auto forward = [&](float (&Z)[4], bool full) __attribute__((always_inline)) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const float* op = sOp + l * kOpStride;
      const float* fc = sFus + l * GNCDE_FC;
#pragma unroll
      for (int r = 0; r < 4; ++r) Zin[0][l][r] = Z[r];
      float ss = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) ss = fmaf(Z[r], Z[r], ss);
      ss = xor_sum4(ss);
      const float inv = 1.0f / sqrtf(ss / (float)H + 1e-5f);
      invl[0][l] = inv;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = mfma4(op[kOpWf + r * 64 + lane], Z[r], acc);
      float mown[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mown[r] = fmaf(inv, acc[r], op[kOpBias + 4 * hi + r]);
        ml[0][l][r] = node_ok ? mown[r] : 0.f;
      }
      if (!full && l == L - 1) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) sMb[(4 * hi + r) * MS + node] = ml[0][l][r];
      float Ab[KS];
      {
        const float e0 = fc[GNCDE_FC_E_A], e1 = fc[GNCDE_FC_E_DA], e2 = fc[GNCDE_FC_ET_A], e3 = fc[GNCDE_FC_ET_DA];
        const float wi = sW[l * NP + node];
        const float* vv = sV + l * NP + hi * KS;
#pragma unroll
        for (int sl = 0; sl < KS; sl += 2) {  // slice pairs on packed FMAs
          const int kr = (sl + kRot) & (KS - 1);
          const floatx2 ar = {sA[oAr + kr], sA[oAr + kr + 1]}, dr = {sdA[oAr + kr], sdA[oAr + kr + 1]};
          const floatx2 ac = {sA[oAc + kr * (NP + 1)], sA[oAc + (kr + 1) * (NP + 1)]};
          const floatx2 dc = {sdA[oAc + kr * (NP + 1)], sdA[oAc + (kr + 1) * (NP + 1)]};
          floatx2 x = floatx2{vv[kr], vv[kr + 1]} + bc2(wi);
          x = pkfma(bc2(e3), dc, x);
          x = pkfma(bc2(e2), ac, x);
          x = pkfma(bc2(e1), dr, x);
          x = pkfma(bc2(e0), ar, x);
          Ab[sl] = x.x;
          Ab[sl + 1] = x.y;
        }
      }
      __syncthreads();
      floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      const float* mrow = sMb + lo * MS + hi * KS;
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const float4 mv = *reinterpret_cast<const float4*>(mrow + ((4 * q + kRot) & (KS - 1)));
        c0 = mfma4(mv.x, Ab[4 * q + 0], c0);
        c1 = mfma4(mv.y, Ab[4 * q + 1], c1);
        c0 = mfma4(mv.z, Ab[4 * q + 2], c0);
        c1 = mfma4(mv.w, Ab[4 * q + 3], c1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = fmaf(ul[l], mown[r], c0[r] + c1[r]);
        prel[0][l][r] = z;
        Z[r] = (l < L - 1) ? fmaxf(z, 0.f) : z;
      }
      __syncthreads();  // m^T reads done before sMb is rewritten
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) Z[r] = node_ok ? tg * Z[r] : 0.f;
  };
  // Two independent stage evaluations at the formed time (the boundary's stage 0 of step k+1 and last stage of step
  // k; the pair's stages 2 and 1), forward only as far as their backwards need: each layer's operand slice Ab is
  // built once for both, their m^T go to sMb / sGb (sGb is free until a backward), and their product MFMA chains
  // interleave.
  auto forward2 = [&](float (&Za)[4], float (&Zb)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const float* op = sOp + l * kOpStride;
      const float* fc = sFus + l * GNCDE_FC;
      float mown[2][4];
#pragma unroll
      for (int sl2 = 0; sl2 < 2; ++sl2) {
        float (&Z)[4] = sl2 ? Zb : Za;
#pragma unroll
        for (int r = 0; r < 4; ++r) Zin[sl2][l][r] = Z[r];
        float ss = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) ss = fmaf(Z[r], Z[r], ss);
        ss = xor_sum4(ss);
        const float inv = 1.0f / sqrtf(ss / (float)H + 1e-5f);
        invl[sl2][l] = inv;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma4(op[kOpWf + r * 64 + lane], Z[r], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          mown[sl2][r] = fmaf(inv, acc[r], op[kOpBias + 4 * hi + r]);
          ml[sl2][l][r] = node_ok ? mown[sl2][r] : 0.f;
        }
      }
      if (l == L - 1) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sMb[(4 * hi + r) * MS + node] = ml[0][l][r];
        sGb[(4 * hi + r) * MS + node] = ml[1][l][r];
      }
      float Ab[KS];
      {
        const float e0 = fc[GNCDE_FC_E_A], e1 = fc[GNCDE_FC_E_DA], e2 = fc[GNCDE_FC_ET_A], e3 = fc[GNCDE_FC_ET_DA];
        const float wi = sW[l * NP + node];
        const float* vv = sV + l * NP + hi * KS;
#pragma unroll
        for (int sl = 0; sl < KS; sl += 2) {
          const int kr = (sl + kRot) & (KS - 1);
          const floatx2 ar = {sA[oAr + kr], sA[oAr + kr + 1]}, dr = {sdA[oAr + kr], sdA[oAr + kr + 1]};
          const floatx2 ac = {sA[oAc + kr * (NP + 1)], sA[oAc + (kr + 1) * (NP + 1)]};
          const floatx2 dc = {sdA[oAc + kr * (NP + 1)], sdA[oAc + (kr + 1) * (NP + 1)]};
          floatx2 x = floatx2{vv[kr], vv[kr + 1]} + bc2(wi);
          x = pkfma(bc2(e3), dc, x);
          x = pkfma(bc2(e2), ac, x);
          x = pkfma(bc2(e1), dr, x);
          x = pkfma(bc2(e0), ar, x);
          Ab[sl] = x.x;
          Ab[sl + 1] = x.y;
        }
      }
      __syncthreads();
      floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f}, d0 = c0, d1 = c0;
      const float* mrow = sMb + lo * MS + hi * KS;
      const float* grow = sGb + lo * MS + hi * KS;
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const int o = (4 * q + kRot) & (KS - 1);
        const float4 mv = *reinterpret_cast<const float4*>(mrow + o);
        const float4 gv = *reinterpret_cast<const float4*>(grow + o);
        c0 = mfma4(mv.x, Ab[4 * q + 0], c0);
        d0 = mfma4(gv.x, Ab[4 * q + 0], d0);
        c1 = mfma4(mv.y, Ab[4 * q + 1], c1);
        d1 = mfma4(gv.y, Ab[4 * q + 1], d1);
        c0 = mfma4(mv.z, Ab[4 * q + 2], c0);
        d0 = mfma4(gv.z, Ab[4 * q + 2], d0);
        c1 = mfma4(mv.w, Ab[4 * q + 3], c1);
        d1 = mfma4(gv.w, Ab[4 * q + 3], d1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float za = fmaf(ul[l], mown[0][r], c0[r] + c1[r]);
        const float zb = fmaf(ul[l], mown[1][r], d0[r] + d1[r]);
        prel[0][l][r] = za;
        prel[1][l][r] = zb;
        Za[r] = (l < L - 1) ? fmaxf(za, 0.f) : za;
        Zb[r] = (l < L - 1) ? fmaxf(zb, 0.f) : zb;
      }
      __syncthreads();  // m^T reads done before sMb / sGb are rewritten
    }
  };

  // ---- backward of the last forward: gU = J^T gK; gradients accumulated lane-distributed ---------------
  floatx4 gWacc[L];
  float gbA[L][4], grwA[L][4], grbA[L][4], gfA[L];
  if constexpr (VJP) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      gWacc[l] = floatx4{0.f, 0.f, 0.f, 0.f};
      gfA[l] = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) gbA[l][r] = grwA[l][r] = grbA[l][r] = 0.f;
    }
  }
  auto backward = [&](const float (&gK)[4], float (&gU)[4], const int slot) __attribute__((always_inline)) {
    float gZ[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) gZ[r] = node_ok ? tg * gK[r] : 0.f;
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
      const float* op = sOp + l * kOpStride;
      const float* fc = sFus + l * GNCDE_FC;
      float gpre[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gpre[r] = (l < L - 1 && !(prel[slot][l][r] > 0.f)) ? 0.f : gZ[r];
        sGb[(4 * hi + r) * MS + node] = gpre[r];  // (m itself enters G from registers: no m^T staging)
      }
      {
        float cm[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) cm[r] = xor_sum16(ml[slot][l][r]);
        if (lo == 0)
#pragma unroll
          for (int r = 0; r < 4; ++r) sCol[0][w][4 * hi + r] = cm[r];
      }
      __syncthreads();
      // R_i = gpre_i . colsum(m), D_i = gpre_i . m_i here; C_k = colsum(gpre) . m_k = sum_i G_ik comes from the
      // G blocks below (no column sum of gpre needed)
      float R = 0.f, D = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float colm = xor_sum16(lo < NW ? sCol[0][lo < NW ? lo : 0][4 * hi + r] : 0.f);
        R = fmaf(gpre[r], colm, R);
        D = fmaf(gpre[r], ml[slot][l][r], D);
      }
      R = xor_sum4(R);
      D = xor_sum4(D);
      if (hi != 0) R = D = 0.f;  // every node once
      float fq[GNCDE_FC];
#pragma unroll
      for (int q = 0; q < GNCDE_FC; ++q) fq[q] = 0.f;
      fq[GNCDE_FC_UD_A] = D * dgn;
      fq[GNCDE_FC_UD_DA] = D * dgdn;
      fq[GNCDE_FC_UR_A] = D * rn;
      fq[GNCDE_FC_UR_DA] = D * rdn;
      fq[GNCDE_FC_UC_A] = D * cn;
      fq[GNCDE_FC_UC_DA] = D * cdn;
      fq[GNCDE_FC_US_A] = D * s;
      fq[GNCDE_FC_US_DA] = D * sd;
      fq[GNCDE_FC_IDC] = D;
      fq[GNCDE_FC_WR_A] = R * rn;
      fq[GNCDE_FC_WR_DA] = R * rdn;
      fq[GNCDE_FC_WC_A] = R * cn;
      fq[GNCDE_FC_WC_DA] = R * cdn;
      fq[GNCDE_FC_WS_A] = R * s;
      fq[GNCDE_FC_WS_DA] = R * sd;
      const float e0 = fc[GNCDE_FC_E_A], e1 = fc[GNCDE_FC_E_DA], e2 = fc[GNCDE_FC_ET_A], e3 = fc[GNCDE_FC_ET_DA];
      const float vk = sV[l * NP + node];
      // Row order of the G blocks: MFMA output row R = 4g + r (lane group g) stands for row base(it) + og(g) + r.
      // Pairing blocks into 32-row windows puts lane groups 0 / 1 (2 / 3) of one 32-lane half 16 rows apart, so
      // the A / dA reads of both the row (A[i][node]) and the column (A[node][i]) walk hit 32 distinct banks
      // (with consecutive 16-row blocks they were 4 rows apart: 2-way conflicts).
      constexpr bool PAIR = NW % 2 == 0;
      auto og = [](int g) { return PAIR ? 16 * (g & 1) + 4 * (g >> 1) : 4 * g; };
      auto base = [](int it) { return PAIR ? 32 * (it >> 1) + 8 * (it & 1) : 16 * it; };
      const float* wv = sW + l * NP + og(hi);
      const int oCol = swz<NP>(og(hi), node), oRow = swz<NP>(node, og(hi));
      const int rA = og(lo >> 2) + (lo & 3);  // A-operand row of this lane
      floatx2 q0 = {0.f, 0.f}, q1 = {0.f, 0.f}, q2 = {0.f, 0.f}, q3 = {0.f, 0.f}, cs = {0.f, 0.f};
      float AbT[KS];
#pragma unroll
      for (int it = 0; it < NW; ++it) {
        floatx4 Gt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) Gt = mfma4(sGb[(4 * hi + j) * MS + base(it) + rA], ml[slot][l][j], Gt);
#pragma unroll
        for (int r = 0; r < 4; r += 2) {  // row pairs on packed FMAs
          const int di = base(it) + r;
          const floatx2 g2 = {Gt[r], Gt[r + 1]};
          const floatx2 aik = {sA[oCol + di * (NP + 1)], sA[oCol + (di + 1) * (NP + 1)]};
          const floatx2 dik = {sdA[oCol + di * (NP + 1)], sdA[oCol + (di + 1) * (NP + 1)]};
          const floatx2 aki = {sA[oRow + di], sA[oRow + di + 1]}, dki = {sdA[oRow + di], sdA[oRow + di + 1]};
          q0 = pkfma(g2, aik, q0);
          q1 = pkfma(g2, dik, q1);
          q2 = pkfma(g2, aki, q2);
          q3 = pkfma(g2, dki, q3);
          cs = cs + g2;
          floatx2 x = floatx2{wv[di], wv[di + 1]} + bc2(vk);
          x = pkfma(bc2(e3), dki, x);
          x = pkfma(bc2(e2), aki, x);
          x = pkfma(bc2(e1), dik, x);
          x = pkfma(bc2(e0), aik, x);
          AbT[4 * it + r] = x.x;
          AbT[4 * it + r + 1] = x.y;
        }
      }
      fq[GNCDE_FC_E_A] = q0.x + q0.y;
      fq[GNCDE_FC_E_DA] = q1.x + q1.y;
      fq[GNCDE_FC_ET_A] = q2.x + q2.y;
      fq[GNCDE_FC_ET_DA] = q3.x + q3.y;
      {
        float C = xor_sum4(cs.x + cs.y);
        if (hi != 0) C = 0.f;
        fq[GNCDE_FC_VR_A] = C * rn;
        fq[GNCDE_FC_VR_DA] = C * rdn;
        fq[GNCDE_FC_VC_A] = C * cn;
        fq[GNCDE_FC_VC_DA] = C * cdn;
      }
      floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      const float* grow = sGb + lo * MS + og(hi);
#pragma unroll
      for (int it = 0; it < NW; ++it) {
        const float4 gv = *reinterpret_cast<const float4*>(grow + base(it));
        c0 = mfma4(gv.x, AbT[4 * it + 0], c0);
        c1 = mfma4(gv.y, AbT[4 * it + 1], c1);
        c0 = mfma4(gv.z, AbT[4 * it + 2], c0);
        c1 = mfma4(gv.w, AbT[4 * it + 3], c1);
      }
      float gm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) gm[r] = node_ok ? fmaf(ul[l], gpre[r], c0[r] + c1[r]) : 0.f;
      {
        float v32[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) v32[q] = q < GNCDE_FC ? fq[q] : 0.f;
        gfA[l] += reduce_scatter32(v32, lane);  // lane q (q < 24) owns fusion-table entry q
      }
      __syncthreads();  // sGb / sMb (G, gm) consumed by every wave before restaging
      float xh[4], zn[4], rw4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rw4[r] = op[kOpRw + 4 * hi + r];
        xh[r] = Zin[slot][l][r] * invl[slot][l];
        zn[r] = node_ok ? fmaf(xh[r], rw4[r], op[kOpRb + 4 * hi + r]) : 0.f;
        sGb[(4 * hi + r) * MS + node] = gm[r];
        sMb[(4 * hi + r) * MS + node] = zn[r];
        gbA[l][r] += gm[r];  // lane partials: reduced over the wave's nodes once, at the end
      }
      // The gW operands below are this wave's own node columns of the restaged gm / zn, so only the wave's own
      // stores must precede them: the LDS executes one wave's DS instructions in order, and the compiler fence
      // keeps the reads behind the stores (no workgroup barrier).
      wave_lds_order();
      {
        const float4 ga = *reinterpret_cast<const float4*>(sGb + lo * MS + 16 * w + 4 * hi);
        const float4 za = *reinterpret_cast<const float4*>(sMb + lo * MS + 16 * w + 4 * hi);
        gWacc[l] = mfma4(ga.x, za.x, gWacc[l]);
        gWacc[l] = mfma4(ga.y, za.y, gWacc[l]);
        gWacc[l] = mfma4(ga.z, za.z, gWacc[l]);
        gWacc[l] = mfma4(ga.w, za.w, gWacc[l]);
      }
      floatx4 gz4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) gz4 = mfma4(op[kOpWb + r * 64 + lane], gm[r], gz4);
      float dot = 0.f, gxh[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        grwA[l][r] = fmaf(gz4[r], xh[r], grwA[l][r]);
        grbA[l][r] += node_ok ? gz4[r] : 0.f;
        gxh[r] = gz4[r] * rw4[r];
        dot = fmaf(gxh[r], xh[r], dot);
      }
      dot = xor_sum4(dot);
#pragma unroll
      for (int r = 0; r < 4; ++r) gZ[r] = node_ok ? invl[slot][l] * (gxh[r] - xh[r] * dot * (1.0f / (float)H)) : 0.f;
      // No barrier here: what follows (the next layer's gpre / m stores, a forward's m^T stores) writes only this
      // wave's own node columns of sGb / sMb, which no other wave reads before the next workgroup barrier, and
      // sCol[w] was last read before the barrier above; a form or the final reduction starts with a barrier.
      wave_lds_order();
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) gU[r] = gZ[r];
  };

  auto load4 = [&](const float* p, size_t off, float (&v)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = node_ok ? p[off + r] : 0.f;
  };
  // stage input U_i (i >= 1) of step k: from the forward's record when there is one (steps past nsteps have h = 0,
  // so their stage inputs are the checkpoint y_k, which the forward never recorded), else as recomputed above
  auto loadU = [&](int kk, int i, float (&v)[4]) {
    if (!a.rec)
      load4(a.U[i], rowoff, v);
    else if (kk < ns)
      load4(a.rec, (((size_t)b * (G - 1) + kk) * (a.S - 1) + i - 1) * E + (size_t)(node_ok ? node : 0) * H + 4 * hi, v);
    else
      load4(a.ys, rowk(kk), v);
  };
  auto store4 = [&](float* p, size_t off, const float (&v)[4]) {
    if (node_ok)
#pragma unroll
      for (int r = 0; r < 4; ++r) p[off + r] = v[r];
  };
  __syncthreads();  // sTs / sFus staged

  const int k = a.k;
  float tk = 0.f, hk = 0.f;
  if (k >= 0) geom(k, tk, hk);

  if constexpr (PROG == kEval1 || EVAL_RK4) {
    const int i = a.stage;
    float y[4], U[4];
    load4(a.ys, rowk(k), y);
#pragma unroll
    for (int r = 0; r < 4; ++r) U[r] = 0.f;
    for (int j = 0; j < i; ++j) {
      float Kj[4];
      load4(a.K[j], rowoff, Kj);
#pragma unroll
      for (int r = 0; r < 4; ++r) U[r] = fmaf(a.a[i][j], Kj[r], U[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) U[r] = fmaf(hk, U[r], y[r]);
    if (i > 0) store4(a.U[i], rowoff, U);
    form(stage_time(tk, a.c[i], hk));
    forward(U, true);
    store4(a.K[i], rowoff, U);
    if (a.write_next) {  // input of stage i+1 (the last stage, whose value the sweep never needs)
      float Un[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) Un[r] = 0.f;
      for (int j = 0; j <= i; ++j) {
        float Kj[4];
        if (j < i) {
          load4(a.K[j], rowoff, Kj);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) Kj[r] = U[r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Un[r] = fmaf(a.a[i + 1][j], Kj[r], Un[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) Un[r] = fmaf(hk, Un[r], y[r]);
      store4(a.U[i + 1], rowoff, Un);
    }
  }
  if constexpr (PROG == kEval2 || EVAL_RK4) {  // RK4: stages 1 and 2 share t + h/2
    float y[4], K0[4], U[4], Kv[4];
    load4(a.ys, rowk(k), y);
    load4(a.K[0], rowoff, K0);
    const float hh = 0.5f * hk;
#pragma unroll
    for (int r = 0; r < 4; ++r) U[r] = fmaf(hh, K0[r], y[r]);
    store4(a.U[1], rowoff, U);
    form(stage_time(tk, 0.5f, hk));
#pragma unroll
    for (int r = 0; r < 4; ++r) Kv[r] = U[r];
    forward(Kv, true);
#pragma unroll
    for (int r = 0; r < 4; ++r) U[r] = fmaf(hh, Kv[r], y[r]);
    store4(a.U[2], rowoff, U);
#pragma unroll
    for (int r = 0; r < 4; ++r) Kv[r] = U[r];
    forward(Kv, true);
#pragma unroll
    for (int r = 0; r < 4; ++r) U[r] = fmaf(hk, Kv[r], y[r]);
    store4(a.U[3], rowoff, U);
  }
  if constexpr (VJP) {
    if constexpr (PROG == kVjpMid) {
      const int i = a.stage;
      float U[4], gK[4], gU[4], acc[4];
      loadU(k, i, U);
      load4(a.gK[i], rowoff, gK);
      form(stage_time(tk, a.c[i], hk));
      forward(U, false);
      backward(gK, gU, 0);
      load4(a.gyacc, rowoff, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += gU[r];
      store4(a.gyacc, rowoff, acc);
      for (int j = 0; j < i; ++j) {
        if (a.a[i][j] == 0.f) continue;
        const float cf = hk * a.a[i][j];
        load4(a.gK[j], rowoff, acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = fmaf(cf, gU[r], acc[r]);
        store4(a.gK[j], rowoff, acc);
      }
    }
    if constexpr (PROG == kBoundary || BOUND_PAIR) {
      const int S = a.S;
      const int il = S - 1;
      const float tl = stage_time(tk, a.c[il], hk);
      float lam[4], Un[4], gKn[4], Uc[4];
      float tn = 0.f, hn = 0.f;
      if (a.has_next) {
        geom(k + 1, tn, hn);
        load4(a.ys, rowk(k + 1), Un);
        load4(a.gK[0], rowoff, gKn);
      }
      if (a.has_cur) loadU(k, il, Uc);
      // both evaluations at t_{k+1} in one two-stage forward when the last stage's time is that same float
      const bool dual = a.has_next && a.has_cur && tl == tn;
      if (a.has_next) {  // stage 0 of step k+1 at t_{k+1}: lambda_{k+1} = gyacc + gU (+ gys[k+1])
        float gU[4];
        form(tn);
        if (dual)
          forward2(Un, Uc);
        else
          forward(Un, false);
        backward(gKn, gU, 0);
        load4(a.gyacc, rowoff, lam);
#pragma unroll
        for (int r = 0; r < 4; ++r) lam[r] += gU[r];
        if (a.gys) {
          float gs[4];
          load4(a.gys, rowk(k + 1), gs);
#pragma unroll
          for (int r = 0; r < 4; ++r) lam[r] += gs[r];
        }
      } else {
        load4(a.lam, rowoff, lam);
      }
      if (a.has_cur) {  // seeds of step k and its last stage
        float gK[4], gU[4], sd[4] = {0.f, 0.f, 0.f, 0.f};
        if (a.gst) load4(a.gst, rowst(k, il), sd);
#pragma unroll
        for (int r = 0; r < 4; ++r) gK[r] = hk * a.bw[il] * lam[r] + sd[r];
        if (dual) {
          backward(gK, gU, 1);
        } else {
          if (!a.has_next || tl != tn) form(tl);
          forward(Uc, false);
          backward(gK, gU, 0);
        }
        float acc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = lam[r] + gU[r];
        store4(a.gyacc, rowoff, acc);
        for (int j = 0; j < il; ++j) {
          if (a.gst) load4(a.gst, rowst(k, j), sd);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = hk * fmaf(a.a[il][j], gU[r], a.bw[j] * lam[r]) + sd[r];
          store4(a.gK[j], rowoff, acc);
        }
      } else {
        store4(a.gy0, rowoff, lam);
      }
    }
    // RK4 stages 2 then 1 at t + h/2 (kBoundaryPair: right after the boundary, one launch and one gradient
    // reduction for both)
    if constexpr (PROG == kVjpPair || BOUND_PAIR) {
      float U[4], U1[4], gK[4], gU[4], gy[4], g1[4];
      loadU(k, 2, U);
      loadU(k, 1, U1);
      load4(a.gK[2], rowoff, gK);
      form(stage_time(tk, 0.5f, hk));
      forward2(U, U1);  // stages 2 and 1 share t + h/2; stage 1's backward waits for stage 2's
      backward(gK, gU, 0);
      load4(a.gyacc, rowoff, gy);
      load4(a.gK[1], rowoff, g1);
      const float hh = 0.5f * hk;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gy[r] += gU[r];
        g1[r] = fmaf(hh, gU[r], g1[r]);  // a[2][1] = 1/2
      }
      backward(g1, gU, 1);
      load4(a.gK[0], rowoff, g1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gy[r] += gU[r];
        g1[r] = fmaf(hh, gU[r], g1[r]);  // a[1][0] = 1/2
      }
      store4(a.gyacc, rowoff, gy);
      store4(a.gK[0], rowoff, g1);
    }
    // ---- cross-wave reduction of the gradient accumulators, += into this sample's block --------------
    __syncthreads();
    float* red = sR0 + w * (L * kGradStride);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      float* blk = red + l * kGradStride;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        blk[2 * H + (4 * hi + r) * H + lo] = gWacc[l][r];
        const float rw = xor_sum16(grwA[l][r]), rb = xor_sum16(grbA[l][r]), bb = xor_sum16(gbA[l][r]);
        if (lo == 0) {
          blk[4 * hi + r] = rw;
          blk[H + 4 * hi + r] = rb;
          blk[2 * H + H * H + 4 * hi + r] = bb;
        }
      }
      if (lane < GNCDE_FC) blk[kLayerP + lane] = gfA[l];
    }
    __syncthreads();
    float* gpb = a.gp + (size_t)b * L * kGradStride;
    for (int j = tid; j < L * kGradStride; j += NT) {
      float sum = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) sum += sR0[q * L * kGradStride + j];
      gpb[j] += sum;
    }
  }
}

// sum over samples of the per-sample accumulators -> gparams [L*kLayerP], gfusion [L, 24]
__global__ void k_stage_grad_sum(int B, int L, const float* __restrict__ gp, float* __restrict__ gparams,
                                 float* __restrict__ gfusion) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int per = L * kGradStride;
  if (j >= per) return;
  // samples in order (the summation order is fixed); 16 loads in flight per batch of the chain
  float sum = 0.f;
  int b = 0;
  for (; b + 16 <= B; b += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = gp[(size_t)(b + u) * per + j];
#pragma unroll
    for (int u = 0; u < 16; ++u) sum += v[u];
  }
  for (; b < B; ++b) sum += gp[(size_t)b * per + j];
  const int l = j / kGradStride, q = j % kGradStride;
  if (q < kLayerP)
    gparams[l * kLayerP + q] = sum;
  else
    gfusion[l * GNCDE_FC + (q - kLayerP)] = sum;
}

// lambda at the last grid point: gys (SAVE_T1) or gys[:, G-1] (SAVE_STEPS)
__global__ void k_lam_init(size_t E, int G, int steps, const float* __restrict__ gys, float* __restrict__ lam) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  lam[(size_t)b * E + e] = steps ? gys[((size_t)b * G + (G - 1)) * E + e] : gys[(size_t)b * E + e];
}

typedef void (*RevFn)(RevArgs);
struct RevEntry {
  int np, l;
  RevFn fn[8];
};

#define GNCDE_REV(NP, L) \
  {NP, L, {k_rev<NP, L, kEval1>, k_rev<NP, L, kEval2>, k_rev<NP, L, kVjpMid>, k_rev<NP, L, kVjpPair>, \
           k_rev<NP, L, kBoundary>, k_rev<NP, L, kEvalRk4>, k_rev<NP, L, kBoundaryPair>, k_rev<NP, L, kStepRk4>}}
const RevEntry kRev[] = {
    GNCDE_REV(16, 1),  GNCDE_REV(16, 2),  GNCDE_REV(16, 3),  GNCDE_REV(16, 4),
    GNCDE_REV(32, 1),  GNCDE_REV(32, 2),  GNCDE_REV(32, 3),  GNCDE_REV(32, 4),
    GNCDE_REV(64, 1),  GNCDE_REV(64, 2),  GNCDE_REV(64, 3),  GNCDE_REV(64, 4),
    GNCDE_REV(128, 1), GNCDE_REV(128, 2), GNCDE_REV(128, 3),
};
#undef GNCDE_REV

const RevEntry* find_rev(const GncdeProblem& p) {
  if (p.cde_hidden != 0 || p.T > kTMaxS) return nullptr;
  for (int l = 0; l <= p.L; ++l)
    if (p.dims[l] != H) return nullptr;
  int np = 16;
  while (np < p.n) np *= 2;
  for (const RevEntry& e : kRev)
    if (e.np == np && e.l == p.L) return &e;
  return nullptr;
}

inline unsigned cdivs(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

struct StageWs {
  float *ops, *gp, *lam, *gyacc;
  float *U[6], *K[6], *gK[6];
};

size_t carve_stage(const GncdeProblem& p, char* ws, StageWs& w) {
  const size_t B = p.B, E = (size_t)p.n * H;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    float* ptr = ws ? reinterpret_cast<float*>(ws + off) : nullptr;
    off += align_up(bytes, 256);
    return ptr;
  };
  w.ops = take((size_t)p.L * kOpStride * 4);
  w.gp = take(B * p.L * kGradStride * 4);
  w.lam = take(B * E * 4);
  w.gyacc = take(B * E * 4);
  for (int i = 0; i < 6; ++i) {
    w.U[i] = take(B * E * 4);
    w.K[i] = take(B * E * 4);
    w.gK[i] = take(B * E * 4);
  }
  return off;
}

}  // namespace

bool stage_vjp_supported(const GncdeProblem& p, const GncdeSolver& s) {
  return s.controller == GNCDE_CTRL_GRID && find_rev(p) != nullptr;
}

size_t stage_vjp_workspace(const GncdeProblem& p) {
  StageWs w;
  return carve_stage(p, nullptr, w);
}

// Reverse sweep, per step k = G-2 .. 0 (RK4: one kStepRk4 launch; Tsit5: 10 launches):
//   recompute  RK4: stage 0 at t_k, stages 1-2 at t_k + h/2, and U_3 (inside kStepRk4)
//              Tsit5: kEval1 for stages 0..4 (the last writes U_5)
//              -- skipped when the forward left a stage record (RK4: kBoundaryPair; Tsit5: no kEval1): the
//                 sweep then forms A(t) twice per RK4 step instead of four times and runs no forward-only stage
//   kBoundary  at t_{k+1}: stage 0 of step k+1 closes lambda_{k+1}; seeds + last stage of step k
//   middle     RK4: kVjpPair (stages 2, 1);  Tsit5: kVjpMid for stages 4..1
// and a final kBoundary (stage 0 of step 0 -> gy0).
int stage_integrate_vjp(const GncdeProblem& p, const GncdeSolver& s, const float* ys, const float* gys,
                        const float* gstage, float* gy0, float* gparams, float* gfusion, char* ws, hipStream_t st) {
  const RevEntry* e = find_rev(p);
  if (!e || s.controller != GNCDE_CTRL_GRID) return GNCDE_ERR_UNSUPPORTED;
  const int B = p.B, G = s.grid_len;
  const size_t E = (size_t)p.n * H;
  StageWs w;
  carve_stage(p, ws, w);
  const bool rk4 = s.method == GNCDE_RK4;
  const bool steps = s.save_mode == GNCDE_SAVE_STEPS;
  hipLaunchKernelGGL(k_stage_prep, dim3(p.L), dim3(256), 0, st, p.params, w.ops);
  (void)hipMemsetAsync(w.gp, 0, (size_t)B * p.L * kGradStride * sizeof(float), st);
  hipLaunchKernelGGL(k_lam_init, dim3(cdivs(E, 256), B), dim3(256), 0, st, E, G, steps ? 1 : 0, gys, w.lam);

  RevArgs a{};
  a.n = p.n;
  a.T = p.T;
  a.G = G;
  a.ts = p.ts;
  a.coef = p.coef;
  a.tcoef = p.tcoef;
  a.fusion = p.fusion;
  a.ops = w.ops;
  a.grid = s.grid;
  a.nsteps = s.nsteps;
  a.ys = ys;
  a.gys = steps ? gys : nullptr;
  a.gst = gstage;
  a.rec = G >= 2 ? s.stage_rec : nullptr;
  for (int i = 0; i < 6; ++i) {
    a.K[i] = w.K[i];
    a.U[i] = w.U[i];
    a.gK[i] = w.gK[i];
  }
  a.gyacc = w.gyacc;
  a.lam = w.lam;
  a.gy0 = gy0;
  a.gp = w.gp;
  if (rk4) {
    a.S = 4;
    a.c[1] = a.c[2] = 0.5f;
    a.c[3] = 1.f;
    a.a[1][0] = 0.5f;
    a.a[2][1] = 0.5f;
    a.a[3][2] = 1.f;
    a.bw[0] = a.bw[3] = 1.f / 6.f;
    a.bw[1] = a.bw[2] = 2.f / 6.f;
  } else {
    a.S = 6;
    const float c[6] = {0.f, TSIT5_C2, TSIT5_C3, TSIT5_C4, TSIT5_C5, 1.f};
    const float A[6][6] = {{0, 0, 0, 0, 0, 0},
                           {TSIT5_A21, 0, 0, 0, 0, 0},
                           {TSIT5_A31, TSIT5_A32, 0, 0, 0, 0},
                           {TSIT5_A41, TSIT5_A42, TSIT5_A43, 0, 0, 0},
                           {TSIT5_A51, TSIT5_A52, TSIT5_A53, TSIT5_A54, 0, 0},
                           {TSIT5_A61, TSIT5_A62, TSIT5_A63, TSIT5_A64, TSIT5_A65, 0}};
    const float bw[6] = {TSIT5_B1, TSIT5_B2, TSIT5_B3, TSIT5_B4, TSIT5_B5, TSIT5_B6};
    for (int i = 0; i < 6; ++i) {
      a.c[i] = c[i];
      a.bw[i] = bw[i];
      for (int j = 0; j < 6; ++j) a.a[i][j] = A[i][j];
    }
  }
  const dim3 grid(B), wg(e->np * 4);
  for (int k = G - 2; k >= 0; --k) {
    a.k = k;
    a.has_next = (k + 1 <= G - 2) ? 1 : 0;
    a.has_cur = 1;
    if (rk4) {  // one launch per step: [stage 0 at t, stages 1, 2 at t + h/2,] boundary at t_{k+1}, stages 2, 1
      a.stage = 0;
      a.write_next = 0;
      hipLaunchKernelGGL(e->fn[a.rec ? kBoundaryPair : kStepRk4], grid, wg, 0, st, a);
      continue;
    }
    for (int i = 0; i + 1 < a.S && !a.rec; ++i) {  // recompute (no stage record)
      a.stage = i;
      a.write_next = (i + 2 == a.S) ? 1 : 0;
      hipLaunchKernelGGL(e->fn[kEval1], grid, wg, 0, st, a);
    }
    hipLaunchKernelGGL(e->fn[kBoundary], grid, wg, 0, st, a);
    for (int i = a.S - 2; i >= 1; --i) {
      a.stage = i;
      hipLaunchKernelGGL(e->fn[kVjpMid], grid, wg, 0, st, a);
    }
  }
  // stage 0 of step 0 closes lambda_0 = dL/dy0
  a.k = -1;
  a.has_next = G >= 2 ? 1 : 0;
  a.has_cur = 0;
  hipLaunchKernelGGL(e->fn[kBoundary], grid, wg, 0, st, a);
  hipLaunchKernelGGL(k_stage_grad_sum, dim3(cdivs((size_t)p.L * kGradStride, 256)), dim3(256), 0, st, B, p.L, w.gp,
                     gparams, gfusion);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

}  // namespace gncde
