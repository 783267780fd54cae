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

template <int NP>
__device__ __forceinline__ int swz(int i, int k) {
  return i * (NP + 1) + k;
}

__device__ __forceinline__ float xor_sum16(float v) {  // sum over the 16 lanes sharing lane>>4
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
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

struct StageArgs {
  int n, T;
  const float* ts;
  const float* coef;
  const float* tcoef;
  const float* fusion;
  const float* ops;   // [L, kOpStride]
  const float* t;     // [B] stage time
  const float* h;     // [B] step size (scales the cotangent scatter)
  const float* U;     // [B, n, H]
  const float* gK;    // [B, n, H] (VJP)
  float* out;         // EVAL: K [B, n, H]
  float* gp;          // VJP: [B, L, kGradStride] (+=)
  float* acc[7];      // VJP: acc[j][b] += coef[j] * (scale_h[j] ? h_b : 1) * gU[b]
  float accw[7];
  int scale_h[7];
  int nacc;
};

template <int NP, int L, bool VJP>
__global__ void __launch_bounds__(NP * 4, 1) k_stage(StageArgs a) {
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
  __shared__ float sCol[2][NW][H];

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int w = tid >> 6;
  const int lane = tid & 63;
  const int lo = lane & 15, hi = lane >> 4;
  const int n = a.n, T = a.T;
  const size_t nn = (size_t)n * n;
  const int node = 16 * w + lo;
  const bool node_ok = node < n;
  float* sA = sR0;
  float* sdA = sR0 + AS;
  float* sW = sVec + 6 * NP;        // w_l[i]
  float* sV = sVec + (6 + L) * NP;  // v_l[k]

  for (int j = tid; j < T; j += NT) sTs[j] = a.ts[(size_t)b * T + j];
  for (int j = tid; j < L * GNCDE_FC; j += NT) sFus[j] = a.fusion[j];
  __syncthreads();

  // ---- form the interval at t: A, dA images, reductions, fusion vectors ------------------------------
  const float t = a.t[b];
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
  if (n == NP) {
    const float4* c4 = reinterpret_cast<const float4*>(cb);
    constexpr int NQ = NP * NP / 4;
    for (int e4 = tid; e4 < NQ; e4 += NT) {
      const float4 d = c4[e4], c = c4[NQ + e4], bb = c4[2 * NQ + e4], aa = c4[3 * NQ + e4];
      const int r = (e4 * 4) / NP, k = (e4 * 4) % NP;
      float* pa = sA + swz<NP>(r, k);
      float* pd = sdA + swz<NP>(r, k);
      pa[0] = fmaf(f, fmaf(f, fmaf(f, d.x, c.x), bb.x), aa.x);
      pa[1] = fmaf(f, fmaf(f, fmaf(f, d.y, c.y), bb.y), aa.y);
      pa[2] = fmaf(f, fmaf(f, fmaf(f, d.z, c.z), bb.z), aa.z);
      pa[3] = fmaf(f, fmaf(f, fmaf(f, d.w, c.w), bb.w), aa.w);
      pd[0] = fmaf(f, fmaf(f3, d.x, 2.0f * c.x), bb.x);
      pd[1] = fmaf(f, fmaf(f3, d.y, 2.0f * c.y), bb.y);
      pd[2] = fmaf(f, fmaf(f3, d.z, 2.0f * c.z), bb.z);
      pd[3] = fmaf(f, fmaf(f3, d.w, 2.0f * c.w), bb.w);
    }
  } else {
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
      for (int k = 0; k < NP; k += 4) {
        acc0 += row[k];
        acc1 += row[k + 1];
        acc2 += row[k + 2];
        acc3 += row[k + 3];
      }
      sVec[(4 + q) * NP + j] = M[swz<NP>(j, j)];
    } else {
      const float* col = M + j;
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
  float s = 0.f, sd = 0.f;
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
  const float rn = sVec[node], rdn = sVec[NP + node], cn = sVec[2 * NP + node], cdn = sVec[3 * NP + node];
  const float dgn = sVec[4 * NP + node], dgdn = sVec[5 * NP + node];
  float ul[L];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float* fc = sFus + l * GNCDE_FC;
    ul[l] = fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * dgn + fc[GNCDE_FC_UD_DA] * dgdn + fc[GNCDE_FC_UR_A] * rn +
            fc[GNCDE_FC_UR_DA] * rdn + fc[GNCDE_FC_UC_A] * cn + fc[GNCDE_FC_UC_DA] * cdn + fc[GNCDE_FC_US_A] * s +
            fc[GNCDE_FC_US_DA] * sd;
  }
  float tg = 0.f;
  {
    const float* tc = a.tcoef + ((size_t)b * (T - 1) + idx) * 3 * n;
    const int ii = node_ok ? node : 0;
    tg = node_ok ? fmaf(f, fmaf(f3, tc[ii], 2.0f * tc[n + ii]), tc[2 * n + ii]) : 0.f;
  }
  __syncthreads();

  // ---- forward, activations kept ------------------------------------------------------------------------
  const size_t rowoff = ((size_t)b * n + (node_ok ? node : 0)) * H + 4 * hi;
  float Z[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) Z[r] = node_ok ? a.U[rowoff + r] : 0.f;
  float Zin[L][4], invl[L], ml[L][4], prel[L][4];
  const int oAr = swz<NP>(node, hi * KS), oAc = swz<NP>(hi * KS, node);
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float* op = a.ops + (size_t)l * kOpStride;
    const float* fc = sFus + l * GNCDE_FC;
#pragma unroll
    for (int r = 0; r < 4; ++r) Zin[l][r] = Z[r];
    float ss = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) ss = fmaf(Z[r], Z[r], ss);
    ss = xor_sum4(ss);
    const float inv = 1.0f / sqrtf(ss / (float)H + 1e-5f);
    invl[l] = inv;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) acc = mfma4(op[kOpWf + r * 64 + lane], Z[r], acc);
    float mown[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mown[r] = fmaf(inv, acc[r], op[kOpBias + 4 * hi + r]);
      ml[l][r] = node_ok ? mown[r] : 0.f;
      sMb[(4 * hi + r) * MS + node] = ml[l][r];
    }
    // this layer's operand slice: row `node` of (Abar - diag(u)), columns k = hi*KS + sl
    float Ab[KS];
    {
      const float e0 = fc[GNCDE_FC_E_A], e1 = fc[GNCDE_FC_E_DA], e2 = fc[GNCDE_FC_ET_A], e3 = fc[GNCDE_FC_ET_DA];
      const float wi = sW[l * NP + node];
      const float* vv = sV + l * NP + hi * KS;
#pragma unroll
      for (int sl = 0; sl < KS; ++sl)
        Ab[sl] = fmaf(e0, sA[oAr + sl], fmaf(e1, sdA[oAr + sl], fmaf(e2, sA[oAc + sl * (NP + 1)],
                      fmaf(e3, sdA[oAc + sl * (NP + 1)], wi + vv[sl]))));
    }
    __syncthreads();
    floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
    const float* mrow = sMb + lo * MS + hi * KS;
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      const float4 mv = *reinterpret_cast<const float4*>(mrow + 4 * q);
      c0 = mfma4(mv.x, Ab[4 * q + 0], c0);
      c1 = mfma4(mv.y, Ab[4 * q + 1], c1);
      c0 = mfma4(mv.z, Ab[4 * q + 2], c0);
      c1 = mfma4(mv.w, Ab[4 * q + 3], c1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = fmaf(ul[l], mown[r], c0[r] + c1[r]);
      prel[l][r] = z;
      Z[r] = (l < L - 1) ? fmaxf(z, 0.f) : z;
    }
    __syncthreads();  // m^T reads done before the next layer (or the backward) rewrites sMb
  }

  if constexpr (!VJP) {
    if (node_ok) {
      float* o = a.out + rowoff;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = tg * Z[r];
    }
    return;
  } else {
    // ---- backward ---------------------------------------------------------------------------------------
    float gZ[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) gZ[r] = node_ok ? tg * a.gK[rowoff + r] : 0.f;
    floatx4 gWacc[L];
    float gbA[L][4], grwA[L][4], grbA[L][4], gfA[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      gWacc[l] = floatx4{0.f, 0.f, 0.f, 0.f};
      gfA[l] = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) gbA[l][r] = grwA[l][r] = grbA[l][r] = 0.f;
    }
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
      const float* op = a.ops + (size_t)l * kOpStride;
      const float* fc = sFus + l * GNCDE_FC;
      float gpre[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gpre[r] = (l < L - 1 && !(prel[l][r] > 0.f)) ? 0.f : gZ[r];
        sGb[(4 * hi + r) * MS + node] = gpre[r];
        sMb[(4 * hi + r) * MS + node] = ml[l][r];
      }
      {  // per-wave column sums of m and gpre (feature 4hi + r)
        float cm[4], cg[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          cm[r] = xor_sum16(ml[l][r]);
          cg[r] = xor_sum16(gpre[r]);
        }
        if (lo == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sCol[0][w][4 * hi + r] = cm[r];
            sCol[1][w][4 * hi + r] = cg[r];
          }
        }
      }
      __syncthreads();
      float colm[4], colg[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        colm[r] = xor_sum16(lo < NW ? sCol[0][lo < NW ? lo : 0][4 * hi + r] : 0.f);
        colg[r] = xor_sum16(lo < NW ? sCol[1][lo < NW ? lo : 0][4 * hi + r] : 0.f);
      }
      float R = 0.f, C = 0.f, D = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        R = fmaf(gpre[r], colm[r], R);
        C = fmaf(ml[l][r], colg[r], C);
        D = fmaf(gpre[r], ml[l][r], D);
      }
      R = xor_sum4(R);
      C = xor_sum4(C);
      D = xor_sum4(D);
      if (hi != 0) R = C = D = 0.f;  // count every node once
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
      fq[GNCDE_FC_VR_A] = C * rn;
      fq[GNCDE_FC_VR_DA] = C * rdn;
      fq[GNCDE_FC_VC_A] = C * cn;
      fq[GNCDE_FC_VC_DA] = C * cdn;
      // G = gpre m^T (16 rows per MFMA tile) contracted with A, dA, A^T, dA^T while building the column
      // slice of Abar (rows i = 16 it + 4 hi + r, column `node`) as the backward operand
      const float e0 = fc[GNCDE_FC_E_A], e1 = fc[GNCDE_FC_E_DA], e2 = fc[GNCDE_FC_ET_A], e3 = fc[GNCDE_FC_ET_DA];
      const float vk = sV[l * NP + node];
      const float* wv = sW + l * NP + 4 * hi;
      const int oCol = swz<NP>(4 * hi, node), oRow = swz<NP>(node, 4 * hi);
      float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;
      float AbT[KS];
#pragma unroll
      for (int it = 0; it < NW; ++it) {
        floatx4 Gt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) Gt = mfma4(sGb[(4 * hi + j) * MS + 16 * it + lo], ml[l][j], Gt);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int di = 16 * it + r;
          const float aik = sA[oCol + di * (NP + 1)], dik = sdA[oCol + di * (NP + 1)];
          const float aki = sA[oRow + di], dki = sdA[oRow + di];
          q0 = fmaf(Gt[r], aik, q0);
          q1 = fmaf(Gt[r], dik, q1);
          q2 = fmaf(Gt[r], aki, q2);
          q3 = fmaf(Gt[r], dki, q3);
          AbT[4 * it + r] = fmaf(e0, aik, fmaf(e1, dik, fmaf(e2, aki, fmaf(e3, dki, wv[di] + vk))));
        }
      }
      fq[GNCDE_FC_E_A] = q0;
      fq[GNCDE_FC_E_DA] = q1;
      fq[GNCDE_FC_ET_A] = q2;
      fq[GNCDE_FC_ET_DA] = q3;
      // gm^T = gpre^T (I + Abar): A operand gpre^T rows from LDS, B operand the column slice
      floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      const float* grow = sGb + lo * MS + 4 * hi;
#pragma unroll
      for (int it = 0; it < NW; ++it) {
        const float4 gv = *reinterpret_cast<const float4*>(grow + 16 * it);
        c0 = mfma4(gv.x, AbT[4 * it + 0], c0);
        c1 = mfma4(gv.y, AbT[4 * it + 1], c1);
        c0 = mfma4(gv.z, AbT[4 * it + 2], c0);
        c1 = mfma4(gv.w, AbT[4 * it + 3], c1);
      }
      float gm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) gm[r] = node_ok ? fmaf(ul[l], gpre[r], c0[r] + c1[r]) : 0.f;
      // fusion-table gradients of this layer: wave reduction, lane q keeps entry q
#pragma unroll
      for (int q = 0; q < GNCDE_FC; ++q) {
        float v = fq[q];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == q) gfA[l] += v;
      }
      __syncthreads();  // all waves done with sGb / sMb (G, gm) before they are restaged
      // Linear / RMSNorm backward
      float xh[4], zn[4], rw4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rw4[r] = op[kOpRw + 4 * hi + r];
        xh[r] = Zin[l][r] * invl[l];
        zn[r] = node_ok ? fmaf(xh[r], rw4[r], op[kOpRb + 4 * hi + r]) : 0.f;
        sGb[(4 * hi + r) * MS + node] = gm[r];
        sMb[(4 * hi + r) * MS + node] = zn[r];
        gbA[l][r] += xor_sum16(gm[r]);
      }
      __syncthreads();
      {  // gW[o][f] += sum over this wave's nodes of gm[node][o] zn[node][f]
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
        grwA[l][r] += xor_sum16(gz4[r] * xh[r]);
        grbA[l][r] += xor_sum16(node_ok ? gz4[r] : 0.f);
        gxh[r] = gz4[r] * rw4[r];
        dot = fmaf(gxh[r], xh[r], dot);
      }
      dot = xor_sum4(dot);
#pragma unroll
      for (int r = 0; r < 4; ++r) gZ[r] = node_ok ? invl[l] * (gxh[r] - xh[r] * dot * (1.0f / (float)H)) : 0.f;
      if (l > 0) __syncthreads();  // restaged buffers read before the next layer writes them
    }
    // scatter gU into the cotangent accumulators
    if (node_ok) {
      const float hb = a.h[b];
      for (int j = 0; j < a.nacc; ++j) {
        const float cf = a.accw[j] * (a.scale_h[j] ? hb : 1.0f);
        float* o = a.acc[j] + rowoff;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = fmaf(cf, gZ[r], o[r]);
      }
    }
    // ---- cross-wave reduction of the gradient accumulators, then += into this sample's block ----------
    __syncthreads();
    float* red = sR0 + w * (L * kGradStride);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      float* blk = red + l * kGradStride;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        blk[2 * H + (4 * hi + r) * H + lo] = gWacc[l][r];
        if (lo == 0) {
          blk[4 * hi + r] = grwA[l][r];
          blk[H + 4 * hi + r] = grbA[l][r];
          blk[2 * H + H * H + 4 * hi + r] = gbA[l][r];
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
  float sum = 0.f;
  for (int b = 0; b < B; ++b) sum += gp[(size_t)b * per + j];
  const int l = j / kGradStride, q = j % kGradStride;
  if (q < kLayerP)
    gparams[l * kLayerP + q] = sum;
  else
    gfusion[l * GNCDE_FC + (q - kLayerP)] = sum;
}

typedef void (*StageFn)(StageArgs);
struct StageEntry {
  int np, l;
  StageFn eval, vjp;
};

#define GNCDE_STAGE(NP, L) {NP, L, k_stage<NP, L, false>, k_stage<NP, L, true>}
const StageEntry kStage[] = {
    GNCDE_STAGE(16, 1),  GNCDE_STAGE(16, 2),  GNCDE_STAGE(16, 3),  GNCDE_STAGE(16, 4),
    GNCDE_STAGE(32, 1),  GNCDE_STAGE(32, 2),  GNCDE_STAGE(32, 3),  GNCDE_STAGE(32, 4),
    GNCDE_STAGE(64, 1),  GNCDE_STAGE(64, 2),  GNCDE_STAGE(64, 3),  GNCDE_STAGE(64, 4),
    GNCDE_STAGE(128, 1), GNCDE_STAGE(128, 2), GNCDE_STAGE(128, 3),
};
#undef GNCDE_STAGE

const StageEntry* find_stage(const GncdeProblem& p) {
  if (p.cde_hidden != 0 || p.T > kTMaxS) return nullptr;
  for (int l = 0; l <= p.L; ++l)
    if (p.dims[l] != H) return nullptr;
  int np = 16;
  while (np < p.n) np *= 2;
  for (const StageEntry& e : kStage)
    if (e.np == np && e.l == p.L) return &e;
  return nullptr;
}

inline unsigned cdivs(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

__global__ void s_step_geom(int B, int G, int k, const float* __restrict__ grid, const int32_t* __restrict__ nsteps,
                            float* __restrict__ tcur, float* __restrict__ hcur) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int ns = nsteps[b];
  ns = ns < 0 ? 0 : (ns > G - 1 ? G - 1 : ns);
  const float* g = grid + (size_t)b * G;
  tcur[b] = k < ns ? g[k] : g[ns];
  hcur[b] = k < ns ? g[k + 1] - g[k] : 0.f;
}

__global__ void s_stage_time(int B, float c, const float* __restrict__ tcur, const float* __restrict__ hcur,
                             float* __restrict__ tst) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) tst[b] = stage_time(tcur[b], c, hcur[b]);
}

struct SLin {
  const float* x[7];
  float a[7];
  int nx;
};
// out[b] = base[b] + h_b * sum_j a_j x_j[b]  (base row = traj[b, k] when traj != nullptr, else base)
__global__ void s_lincomb(size_t E, int G, int k, const float* __restrict__ traj, SLin lc,
                          const float* __restrict__ hcur, float* __restrict__ out) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const size_t o = (size_t)b * E + e;
  float sum = 0.f;
  for (int j = 0; j < lc.nx; ++j) sum = fmaf(lc.a[j], lc.x[j][o], sum);
  out[o] = fmaf(hcur[b], sum, traj[((size_t)b * G + k) * E + e]);
}

// gK_i = h b_i lam for every stage, gyacc = lam (+ the saved-state cotangent of row k if given)
__global__ void s_seed(size_t E, int S, const float* __restrict__ lam, const float* __restrict__ hcur, SLin bw,
                       float* const* __restrict__ gK, float* __restrict__ gyacc) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const size_t o = (size_t)b * E + e;
  const float l = lam[o], hb = hcur[b];
  for (int i = 0; i < S; ++i) gK[i][o] = hb * bw.a[i] * l;
  gyacc[o] = l;
}

// lam = gyacc (+ gys[:, k] when given)
__global__ void s_lam(size_t E, int G, int k, const float* __restrict__ gyacc, const float* __restrict__ gys,
                      float* __restrict__ lam) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const size_t o = (size_t)b * E + e;
  lam[o] = gyacc[o] + (gys ? gys[((size_t)b * G + k) * E + e] : 0.f);
}

struct Tab {
  int S;
  float c[6], a[6][6], bw[6];
};

Tab make_tab(int method) {
  Tab t{};
  if (method == GNCDE_RK4) {
    t.S = 4;
    t.c[1] = t.c[2] = 0.5f;
    t.c[3] = 1.f;
    t.a[1][0] = 0.5f;
    t.a[2][1] = 0.5f;
    t.a[3][2] = 1.f;
    t.bw[0] = t.bw[3] = 1.f / 6.f;
    t.bw[1] = t.bw[2] = 2.f / 6.f;
  } else {
    t.S = 6;
    const float c[6] = {0.f, TSIT5_C2, TSIT5_C3, TSIT5_C4, TSIT5_C5, 1.f};
    const float A[6][6] = {{0, 0, 0, 0, 0, 0},
                           {TSIT5_A21, 0, 0, 0, 0, 0},
                           {TSIT5_A31, TSIT5_A32, 0, 0, 0, 0},
                           {TSIT5_A41, TSIT5_A42, TSIT5_A43, 0, 0, 0},
                           {TSIT5_A51, TSIT5_A52, TSIT5_A53, TSIT5_A54, 0, 0},
                           {TSIT5_A61, TSIT5_A62, TSIT5_A63, TSIT5_A64, TSIT5_A65, 0}};
    const float bw[6] = {TSIT5_B1, TSIT5_B2, TSIT5_B3, TSIT5_B4, TSIT5_B5, TSIT5_B6};
    for (int i = 0; i < 6; ++i) {
      t.c[i] = c[i];
      t.bw[i] = bw[i];
      for (int j = 0; j < 6; ++j) t.a[i][j] = A[i][j];
    }
  }
  return t;
}

struct StageWs {
  float *ops, *gp, *lam, *gyacc, *tcur, *hcur, *tst;
  float *U[6], *K[6], *gK[6];
  float** gKptr;
};

size_t carve_stage(const GncdeProblem& p, char* ws, StageWs& w) {
  const size_t B = p.B, E = (size_t)p.n * H;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* ptr = ws ? ws + off : nullptr;
    off += align_up(bytes, 256);
    return ptr;
  };
  w.ops = reinterpret_cast<float*>(take((size_t)p.L * kOpStride * 4));
  w.gp = reinterpret_cast<float*>(take(B * p.L * kGradStride * 4));
  w.lam = reinterpret_cast<float*>(take(B * E * 4));
  w.gyacc = reinterpret_cast<float*>(take(B * E * 4));
  for (int i = 0; i < 6; ++i) {
    w.U[i] = reinterpret_cast<float*>(take(B * E * 4));
    w.K[i] = reinterpret_cast<float*>(take(B * E * 4));
    w.gK[i] = reinterpret_cast<float*>(take(B * E * 4));
  }
  w.tcur = reinterpret_cast<float*>(take(B * 4));
  w.hcur = reinterpret_cast<float*>(take(B * 4));
  w.tst = reinterpret_cast<float*>(take(B * 4));
  w.gKptr = reinterpret_cast<float**>(take(6 * sizeof(float*)));
  return off;
}

}  // namespace

bool stage_vjp_supported(const GncdeProblem& p, const GncdeSolver& s) {
  return s.controller == GNCDE_CTRL_GRID && find_stage(p) != nullptr;
}

size_t stage_vjp_workspace(const GncdeProblem& p) {
  StageWs w;
  return carve_stage(p, nullptr, w);
}

int stage_integrate_vjp(const GncdeProblem& p, const GncdeSolver& s, const float* ys, const float* gys, float* gy0,
                        float* gparams, float* gfusion, char* ws, hipStream_t st) {
  const StageEntry* e = find_stage(p);
  if (!e || s.controller != GNCDE_CTRL_GRID) return GNCDE_ERR_UNSUPPORTED;
  const int B = p.B, G = s.grid_len;
  const size_t E = (size_t)p.n * H;
  StageWs w;
  carve_stage(p, ws, w);
  const Tab tab = make_tab(s.method);
  const int S = tab.S;
  const dim3 ge(cdivs(E, 256), B);
  const unsigned gb = cdivs(B, 256);
  const dim3 wg(e->np * 4);
  (void)hipMemcpyAsync(w.gKptr, w.gK, sizeof(w.gK), hipMemcpyHostToDevice, st);
  hipLaunchKernelGGL(k_stage_prep, dim3(p.L), dim3(256), 0, st, p.params, w.ops);
  (void)hipMemsetAsync(w.gp, 0, (size_t)B * p.L * kGradStride * sizeof(float), st);
  const bool steps = s.save_mode == GNCDE_SAVE_STEPS;
  // lambda = cotangent of the final state (saved-state cotangents are added as the sweep passes them)
  if (steps) {
    (void)hipMemsetAsync(w.gyacc, 0, (size_t)B * E * sizeof(float), st);
    hipLaunchKernelGGL(s_lam, ge, dim3(256), 0, st, E, G, G - 1, w.gyacc, gys, w.lam);
  } else {
    (void)hipMemcpyAsync(w.lam, gys, (size_t)B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  }

  StageArgs a{};
  a.n = p.n;
  a.T = p.T;
  a.ts = p.ts;
  a.coef = p.coef;
  a.tcoef = p.tcoef;
  a.fusion = p.fusion;
  a.ops = w.ops;
  a.t = w.tst;
  a.h = w.hcur;
  a.gp = w.gp;
  for (int k = G - 2; k >= 0; --k) {
    hipLaunchKernelGGL(s_step_geom, dim3(gb), dim3(256), 0, st, B, G, k, s.grid, s.nsteps, w.tcur, w.hcur);
    // recompute the stage inputs U_i (U_0 = y_k) and values K_i (i < S-1)
    for (int i = 0; i < S; ++i) {
      SLin lc{};
      for (int j = 0; j < i; ++j)
        if (tab.a[i][j] != 0.f) {
          lc.x[lc.nx] = w.K[j];
          lc.a[lc.nx++] = tab.a[i][j];
        }
      hipLaunchKernelGGL(s_lincomb, ge, dim3(256), 0, st, E, G, k, ys, lc, w.hcur, w.U[i]);
      if (i + 1 < S) {
        hipLaunchKernelGGL(s_stage_time, dim3(gb), dim3(256), 0, st, B, tab.c[i], w.tcur, w.hcur, w.tst);
        a.U = w.U[i];
        a.out = w.K[i];
        hipLaunchKernelGGL(e->eval, dim3(B), wg, 0, st, a);
      }
    }
    // reverse: gK_i = h b_i lam, gy = lam; stage VJPs scatter into gy and the earlier gK_j
    SLin bw{};
    for (int i = 0; i < S; ++i) bw.a[i] = tab.bw[i];
    hipLaunchKernelGGL(s_seed, ge, dim3(256), 0, st, E, S, w.lam, w.hcur, bw, w.gKptr, w.gyacc);
    for (int i = S - 1; i >= 0; --i) {
      hipLaunchKernelGGL(s_stage_time, dim3(gb), dim3(256), 0, st, B, tab.c[i], w.tcur, w.hcur, w.tst);
      a.U = w.U[i];
      a.gK = w.gK[i];
      a.nacc = 0;
      a.acc[a.nacc] = w.gyacc;
      a.accw[a.nacc] = 1.f;
      a.scale_h[a.nacc++] = 0;
      for (int j = 0; j < i; ++j)
        if (tab.a[i][j] != 0.f) {
          a.acc[a.nacc] = w.gK[j];
          a.accw[a.nacc] = tab.a[i][j];
          a.scale_h[a.nacc++] = 1;
        }
      hipLaunchKernelGGL(e->vjp, dim3(B), wg, 0, st, a);
    }
    hipLaunchKernelGGL(s_lam, ge, dim3(256), 0, st, E, G, k, w.gyacc, steps ? gys : nullptr, w.lam);
  }
  (void)hipMemcpyAsync(gy0, w.lam, (size_t)B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  hipLaunchKernelGGL(k_stage_grad_sum, dim3(cdivs((size_t)p.L * kGradStride, 256)), dim3(256), 0, st, B, p.L, w.gp,
                     gparams, gfusion);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

}  // namespace gncde
