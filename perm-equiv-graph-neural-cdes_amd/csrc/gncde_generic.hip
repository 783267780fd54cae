// Generic (any n, any layer widths, CDE wrapper, all fusion kinds) multi-kernel path.
//
// One launch per phase of a vector-field evaluation; used for shapes the fused persistent kernel
// (gncde_fused.hip) does not cover and as the second HIP implementation the parity tests compare
// against.  Every kernel is batched over samples on grid.y/grid.z.
//
// Reference semantics: spline (perm_equiv_graph_vector_field.py:98-102), fusion (layers.py:102-160,
// :256-337 via the factored table of gncde.h), ConvLayer (layers.py:36-48), VF epilogue
// (perm_equiv_graph_vector_field.py:122-128), CDE wrapper (cde_wrapper_vector_field.py:19-26).
#include "gncde_forms.h"
#include "gncde_internal.h"

#include <vector>

#include <utility>

namespace gncde {
namespace {

constexpr int kRedStride = 8;  // red[b][q][n]: r, rd, c, cd, diagA, diagdA, {s}, {sd}

// ---- spline + reductions in one pass ------------------------------------------------------------------
// grid (slabs of kSlab rows, B).  Thread j owns columns k = j, j+256, ...: for the slab's rows it evaluates A and
// dA (coalesced along k), writes them, keeps the column partials and the diagonal, and accumulates per-row
// partials that one block reduction turns into complete row sums (a slab holds whole rows).  Column partials
// go to part[b][slab][2][n]; k_abar_all sums them over slabs (fixed order) and forms the totals.
constexpr int kSlab = 16;

template <typename CT>
__global__ void __launch_bounds__(256) k_spline_slab(int n, int T, const float* __restrict__ ts,
                                                     const CT* __restrict__ coef, const float* __restrict__ tcoef,
                                                     const float* __restrict__ t, float* __restrict__ A,
                                                     float* __restrict__ dA, float* __restrict__ tg,
                                                     float* __restrict__ red, float* __restrict__ part,
                                                     const float* __restrict__ data_coef, int de2,
                                                     float* __restrict__ dx) {
  const int b = blockIdx.y, slab = blockIdx.x;
  const int i0 = slab * kSlab;
  const size_t nn = (size_t)n * n;
  const float tb = t[b];
  const float* tsb = ts + (size_t)b * T;
  const int idx = interval_index_wave(tsb, T, tb);
  const float f = tb - tsb[idx];
  const float f3 = 3.0f * f;
  const CT* cb = coef + ((size_t)b * (T - 1) + idx) * 4 * nn;
  float* Ab = A + (size_t)b * nn;
  float* dAb = dA + (size_t)b * nn;
  float* rb = red + (size_t)b * kRedStride * n;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rows = n - i0 < kSlab ? n - i0 : kSlab;
  float ra[kSlab], rd[kSlab];
#pragma unroll
  for (int r = 0; r < kSlab; ++r) ra[r] = rd[r] = 0.f;
  for (int k = tid; k < n; k += blockDim.x) {
    float ca = 0.f, cd = 0.f;
#pragma unroll
    for (int r = 0; r < kSlab; ++r) {
      if (r < rows) {
        const size_t e = (size_t)(i0 + r) * n + k;
        const float d = coef_at(cb, e), c = coef_at(cb, nn + e), bb = coef_at(cb, 2 * nn + e), a = coef_at(cb, 3 * nn + e);
        const float va = fmaf(f, fmaf(f, fmaf(f, d, c), bb), a);
        const float vd = fmaf(f, fmaf(f3, d, 2.0f * c), bb);
        Ab[e] = va;
        dAb[e] = vd;
        ca += va;
        cd += vd;
        ra[r] += va;
        rd[r] += vd;
        if (k == i0 + r) {
          rb[4 * n + k] = va;
          rb[5 * n + k] = vd;
        }
      }
    }
    float* pb = part + ((size_t)b * gridDim.x + slab) * 2 * n;
    pb[k] = ca;
    pb[n + k] = cd;
  }
  // Row sums: the 2 x kSlab per-thread partials go through LDS (stride 264: the reads below hit 64 distinct banks),
  // then thread t sums partials t % 8, t % 8 + 8, ... of row-sum t / 8 and three lane swaps finish it: 32 LDS
  // writes + 32 reads + 3 shuffles per thread instead of 2 kSlab wave reductions (6 shuffles each).
  constexpr int kPs = 264;
  __shared__ float sp[2 * kSlab][kPs];
#pragma unroll
  for (int r = 0; r < kSlab; ++r) {
    sp[r][tid] = ra[r];
    sp[kSlab + r][tid] = rd[r];
  }
  __syncthreads();
  {
    const int q = tid >> 3, p0 = tid & 7;
    float x = 0.f;
#pragma unroll 8
    for (int j = 0; j < 32; ++j) x += sp[q][p0 + 8 * j];
    x += __shfl_xor(x, 1);
    x += __shfl_xor(x, 2);
    x += __shfl_xor(x, 4);
    const int r = q % kSlab;
    if (p0 == 0 && r < rows) rb[(q / kSlab) * n + i0 + r] = x;
  }
  (void)lane;
  (void)w;
  if (slab == 0) {
    const float* tc = tcoef + ((size_t)b * (T - 1) + idx) * 3 * n;
    for (int e = tid; e < n; e += blockDim.x) tg[(size_t)b * n + e] = fmaf(f, fmaf(f3, tc[e], 2.0f * tc[n + e]), tc[2 * n + e]);
  }
  if (dx) {  // CDE wrapper: the data spline's derivative dX[i][q] at t (same knots), spread over the sample's slabs
    const size_t blk = (size_t)n * de2;
    const float* dc = data_coef + ((size_t)b * (T - 1) + idx) * 4 * blk;
    for (size_t e = (size_t)slab * blockDim.x + tid; e < blk; e += (size_t)gridDim.x * blockDim.x)
      dx[(size_t)b * blk + e] = fmaf(f, fmaf(f3, dc[e], 2.0f * dc[blk + e]), dc[2 * blk + e]);
  }
}

// (I + Abar_l)[b, i, k] for every layer l from one read of the A / dA tiles (32 x 32, the transposed tile staged in
// LDS so both A[i][k] and A[k][i] are read coalesced).  The block also finishes the reductions it needs: column sums
// of its i and k ranges from k_spline_slab's slab partials (fixed order) and the totals; blocks on the first tile
// row / the first tile publish the column sums / totals into red (the reverse sweep reads them later).
template <typename OT>
__global__ void __launch_bounds__(256) k_abar_all(int n, int L, int slabs, const float* __restrict__ fus,
                                                  const float* __restrict__ A, const float* __restrict__ dA,
                                                  float* __restrict__ red, const float* __restrict__ part,
                                                  OT* __restrict__ out, size_t layer_stride,
                                                  float* __restrict__ qrow, int B) {
  const int b = blockIdx.z;
  const int i0 = blockIdx.y * 32, k0 = blockIdx.x * 32;
  const size_t nn = (size_t)n * n;
  const float* Ab = A + b * nn;
  const float* dAb = dA + b * nn;
  float* rb = red + (size_t)b * kRedStride * n;
  const float* pb = part + (size_t)b * slabs * 2 * n;
  __shared__ float tA[32][33], tD[32][33];
  __shared__ float cs[2][2][32];  // [i-range / k-range][A / dA][32]
  __shared__ float tot[2][4];
  const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;  // 32 x 8
  // Every tile load is issued before the first use (one HBM round trip): the transposed tile (for LDS) and this
  // thread's own (i, k) elements, rows ty + 8 q.
  float ta[4], td[4], aik[4], dik[4];
  // ... and the row reductions this tile reads later (r, rd, diagonals of its i range; r, rd of its k range)
  __shared__ float sRb[6][32];
  float rbv = 0.f;
  if (tid < 192) {
    const int q = tid >> 5, x = tid & 31;
    const int idx = (q < 4 ? i0 : k0) + x;
    const int plane = q == 0 ? 0 : (q == 1 ? 1 : (q == 2 ? 4 : (q == 3 ? 5 : q - 4)));
    rbv = idx < n ? rb[plane * n + idx] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int y = ty + 8 * q;
    const bool okt = k0 + y < n && i0 + tx < n, oko = i0 + y < n && k0 + tx < n;
    ta[q] = okt ? Ab[(size_t)(k0 + y) * n + i0 + tx] : 0.f;
    td[q] = okt ? dAb[(size_t)(k0 + y) * n + i0 + tx] : 0.f;
    aik[q] = oko ? Ab[(size_t)(i0 + y) * n + k0 + tx] : 0.f;
    dik[q] = oko ? dAb[(size_t)(i0 + y) * n + k0 + tx] : 0.f;
  }
  if (tid < 128) {  // column sums of A / dA over the slabs for columns i0 + x and k0 + x
    const int which = tid >> 6, q = (tid >> 5) & 1, x = tid & 31;
    const int col = (which ? k0 : i0) + x;
    float c = 0.f;
    if (col < n)
#pragma unroll 8
      for (int sl = 0; sl < slabs; ++sl) c += pb[(size_t)sl * 2 * n + q * n + col];
    cs[which][q][x] = c;
    if (which == 1 && blockIdx.y == 0 && col < n) rb[(2 + q) * n + col] = c;
  } else {  // totals s = sum_i r_i, sd = sum_i rd_i (waves 2, 3)
    const int w = (tid >> 6) - 2, lane = tid & 63;
    float x = 0.f;
    for (int i = lane; i < n; i += 64) x += rb[w * n + i];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) tot[w][0] = x;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    tA[ty + 8 * q][tx] = ta[q];
    tD[ty + 8 * q][tx] = td[q];
  }
  if (tid < 192) sRb[tid >> 5][tid & 31] = rbv;
  __syncthreads();
  const float s = tot[0][0], sd = tot[1][0];
  if (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
    rb[6 * n] = s;
    rb[7 * n] = sd;
  }
  if (qrow && blockIdx.x == 0 && tid < 32 && i0 + tid < n) {
    // q_l[i] = sum_k (I + Abar_l)[i][k] from the reductions: the dense terms give their row / column sums, the
    // w (row) family n copies, the v (column) family sum_k v_k (sum_k r_k = sum_k c_k = s), the diagonal once.
    const int i = i0 + tid;
    const float ri = sRb[0][tid], rdi = sRb[1][tid], ci = cs[0][0][tid], cdi = cs[0][1][tid];
    const float dgi = sRb[2][tid], dgdi = sRb[3][tid], fn = (float)n;
    for (int l = 0; l < L; ++l) {
      const float* fc = fus + l * GNCDE_FC;
      float q = fc[GNCDE_FC_E_A] * ri + fc[GNCDE_FC_E_DA] * rdi + fc[GNCDE_FC_ET_A] * ci + fc[GNCDE_FC_ET_DA] * cdi;
      q += fn * (fc[GNCDE_FC_WR_A] * ri + fc[GNCDE_FC_WR_DA] * rdi + fc[GNCDE_FC_WC_A] * ci + fc[GNCDE_FC_WC_DA] * cdi +
                 fc[GNCDE_FC_WS_A] * s + fc[GNCDE_FC_WS_DA] * sd);
      q += (fc[GNCDE_FC_VR_A] + fc[GNCDE_FC_VC_A]) * s + (fc[GNCDE_FC_VR_DA] + fc[GNCDE_FC_VC_DA]) * sd;
      q += fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * dgi + fc[GNCDE_FC_UD_DA] * dgdi + fc[GNCDE_FC_UR_A] * ri +
           fc[GNCDE_FC_UR_DA] * rdi + fc[GNCDE_FC_UC_A] * ci + fc[GNCDE_FC_UC_DA] * cdi + fc[GNCDE_FC_US_A] * s +
           fc[GNCDE_FC_US_DA] * sd;
      qrow[((size_t)l * B + b) * n + i] = q;
    }
  }
  // The rank-1 and diagonal families per layer, once per tile: w_l (row i), v_l (column k), u_l (diagonal).
  __shared__ float sWv[GNCDE_MAX_LAYERS][3][32];
  for (int e = tid; e < L * 32; e += 256) {
    const int l = e >> 5, x = e & 31;
    const float* fc = fus + l * GNCDE_FC;
    const float ri = sRb[0][x], rdi = sRb[1][x], ci = cs[0][0][x], cdi = cs[0][1][x];
    const float rk = sRb[4][x], rdk = sRb[5][x], ck = cs[1][0][x], cdk = cs[1][1][x];
    sWv[l][0][x] = fc[GNCDE_FC_WR_A] * ri + fc[GNCDE_FC_WR_DA] * rdi + fc[GNCDE_FC_WC_A] * ci +
                   fc[GNCDE_FC_WC_DA] * cdi + fc[GNCDE_FC_WS_A] * s + fc[GNCDE_FC_WS_DA] * sd;
    sWv[l][1][x] = fc[GNCDE_FC_VR_A] * rk + fc[GNCDE_FC_VR_DA] * rdk + fc[GNCDE_FC_VC_A] * ck + fc[GNCDE_FC_VC_DA] * cdk;
    sWv[l][2][x] = fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * sRb[2][x] + fc[GNCDE_FC_UD_DA] * sRb[3][x] +
                   fc[GNCDE_FC_UR_A] * ri + fc[GNCDE_FC_UR_DA] * rdi + fc[GNCDE_FC_UC_A] * ci +
                   fc[GNCDE_FC_UC_DA] * cdi + fc[GNCDE_FC_US_A] * s + fc[GNCDE_FC_US_DA] * sd;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int y = ty + 8 * q;
    const int i = i0 + y, k = k0 + tx;
    if (i >= n || k >= n) continue;
    const float aki = tA[tx][y], dki = tD[tx][y];
    const bool diag = i == k;
    for (int l = 0; l < L; ++l) {
      const float* fc = fus + l * GNCDE_FC;
      float v = fc[GNCDE_FC_E_A] * aik[q] + fc[GNCDE_FC_E_DA] * dik[q] + fc[GNCDE_FC_ET_A] * aki +
                fc[GNCDE_FC_ET_DA] * dki;
      v += sWv[l][0][y] + sWv[l][1][tx];
      if (diag) v += sWv[l][2][y];
      abar_store(out, l * layer_stride + b * nn + (size_t)i * n + k, (size_t)L * layer_stride, v);
    }
  }
}

// ---- forward forms straight from the coefficients -----------------------------------------------------------
// The fusion reads, per evaluation, the row sums, column sums, diagonals and totals of A(t) and dA/dt(t).  On an
// interval A(t) = a + f (b + f (c + f d)) elementwise with one f per sample, so each of those reductions is the
// same cubic of the matching reduction of the four coefficient planes (the time channel's tcoef uses the same
// linearity).  k_coef_sums forms the plane reductions once per solve; an evaluation then evaluates O(n) cubics and
// never sums n^2 values, so one launch (k_abar_direct) goes from the coefficients to every layer's (I + Abar_l)
// with no A / dA round trip through HBM and no reduction pass in front of it.
//
// grid (4 planes, T-1 intervals, B).  Fixed summation orders (deterministic, no atomics).
template <typename CT>
__global__ void __launch_bounds__(256) k_coef_sums(int n, int T, const CT* __restrict__ coef, float* __restrict__ csum) {
  const int q = blockIdx.x, iv = blockIdx.y, b = blockIdx.z;
  const size_t nn = (size_t)n * n;
  const CT* P = coef + (((size_t)b * (T - 1) + iv) * 4 + q) * nn;
  float* o = csum + ((size_t)b * (T - 1) + iv) * csum_stride(n);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int j = tid; j < n; j += 256) {  // column j: one thread walks it (coalesced across the block)
    float s = 0.f;
#pragma unroll 32
    for (int i = 0; i < n; ++i) s += coef_at(P, (size_t)i * n + j);
    o[(q * 3 + 1) * n + j] = s;
    o[(q * 3 + 2) * n + j] = coef_at(P, (size_t)j * n + j);
  }
  float tot = 0.f;  // lane 0 of wave w: the sum of its rows' sums, in row order
  // row i: wave w's lanes across it, one wave reduction; four rows (i0, i0 + 4, i0 + 8, i0 + 12) per pass, so their
  // loads are in flight together (each row's and the total's summation order unchanged)
  for (int i0 = w; i0 < n; i0 += 16) {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = lane; j < n; j += 64)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + 4 * u < n) s[u] += coef_at(P, (size_t)(i0 + 4 * u) * n + j);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int m = 32; m > 0; m >>= 1) s[u] += __shfl_xor(s[u], m);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + 4 * u < n) {
        if (lane == 0) o[(q * 3) * n + i0 + 4 * u] = s[u];
        tot += s[u];
      }
  }
  __shared__ float wt[4];
  if (lane == 0) wt[w] = tot;
  __syncthreads();
  if (tid == 0) o[12 * n + q] = (wt[0] + wt[1]) + (wt[2] + wt[3]);
}

// block bx of sample b's combination (k_combo, or the combination blocks of a merged k_abar_direct launch)
__device__ __forceinline__ void combo_block(size_t E, const float* __restrict__ y, const Combo& cb,
                                            const float* __restrict__ hcur, float* __restrict__ out, int bx, int b) {
  const size_t e0 = (size_t)bx * (kComboThreads * kComboU) + threadIdx.x;
  float hb, tc = 0.f;
  if (cb.grid) {  // the step's geometry, as k_grid_step forms it
    const float* g = cb.grid + (size_t)b * cb.G;
    int ns = cb.nsteps[b];
    ns = ns < 0 ? 0 : (ns > cb.G - 1 ? cb.G - 1 : ns);
    const bool on = cb.gk < ns;
    tc = on ? g[cb.gk] : g[ns];
    hb = on ? g[cb.gk + 1] - g[cb.gk] : 0.f;
    if (e0 == 0) {
      cb.tcur_out[b] = tc;
      cb.hcur_out[b] = hb;
      cb.tnx_out[b] = on ? g[cb.gk + 1] : g[ns];
    }
  } else {
    hb = hcur[b];
  }
  if (cb.tst && e0 == 0) cb.tst[b] = cb.tend ? cb.tend[b] : stage_time(cb.grid ? tc : cb.tcur[b], cb.c, hb);
  float kv[7][kComboU], yv[kComboU];
#pragma unroll
  for (int u = 0; u < kComboU; ++u) {
    const size_t e = e0 + (size_t)u * kComboThreads, o = (size_t)b * E + e;
    const bool in = e < E;
    yv[u] = in ? y[o] : 0.f;
#pragma unroll
    for (int j = 0; j < 7; ++j) kv[j][u] = (in && j < cb.nk) ? cb.K[j][o] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kComboU; ++u) {
    const size_t e = e0 + (size_t)u * kComboThreads;
    if (e >= E) break;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 7; ++j)
      if (j < cb.nk) s = fmaf(cb.a[j], kv[j][u], s);
    const float v = fmaf(hb, s, yv[u]);
    out[(size_t)b * E + e] = v;
    if (cb.rec) cb.rec[(size_t)b * cb.rec_stride + e] = v;
  }
}
__global__ void __launch_bounds__(kComboThreads) k_combo(int B, size_t E, const float* __restrict__ y, Combo cb,
                                                         const float* __restrict__ hcur, float* __restrict__ out) {
  combo_block(E, y, cb, hcur, out, blockIdx.x, blockIdx.y);
}

// grid (tile pairs I <= K of 32 x 32 tiles [+ a pending combination's blocks], B).  A block reads the coefficients of tile (I, K) and of its mirror
// (K, I) once (the two tiles each need the other's transposed elements), evaluates A and dA/dt there, and writes
// both tiles of every layer's (I + Abar_l); the node vectors of its two ranges are cubics of k_coef_sums' planes.
// Diagonal blocks (I == K) also write q_l = (I + Abar_l) 1 for their rows, tg and the CDE data-spline derivative.
template <typename CT, typename OT>
__global__ void __launch_bounds__(256) k_abar_direct(int n, int T, int L, const float* __restrict__ ts,
                                                     const CT* __restrict__ coef, const float* __restrict__ csum,
                                                     const float* __restrict__ tcoef, const float* __restrict__ t,
                                                     const float* __restrict__ fus, OT* __restrict__ out,
                                                     size_t layer_stride, float* __restrict__ qrow,
                                                     float* __restrict__ tg, const float* __restrict__ data_coef,
                                                     int de2, float* __restrict__ dx, int B, PendingCombo pc,
                                                     GridTime gt) {
  const int b = blockIdx.y, nt = (n + 31) >> 5;
  if ((int)blockIdx.x >= nt * (nt + 1) / 2) {  // the pending stage combination's blocks
    combo_block(pc.E, pc.y, pc.cb, pc.hcur, pc.out, (int)blockIdx.x - nt * (nt + 1) / 2, b);
    return;
  }
  // merged launch: the stage time as the combination computes it (it writes tst in this same launch)
  const float tb = gt.grid ? grid_stage_time(gt, b)  // overlapped forms: no combination has written tst yet
                           : (pc.blocks ? (pc.cb.tend ? pc.cb.tend[b] : stage_time(pc.cb.tcur[b], pc.cb.c, pc.hcur[b]))
                                        : t[b]);
  __shared__ float lds[kFormsLdsFloats];
  const FormsArgs fa{n, T, L, de2, B, ts, reinterpret_cast<const float*>(coef), csum, tcoef, fus, data_coef,
                     reinterpret_cast<float*>(out), layer_stride, qrow, tg, dx};
  forms_tile<CT, OT>(fa, (int)blockIdx.x, b, tb, lds);
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
// Per-sample step geometry for step k of the host-planned grid; tst = the first stage's time (c = 0), tnx = the
// step's end knot (Tsit5's FSAL stage is evaluated there: it is the next step's first stage).
__global__ void k_grid_step(int B, int G, int k, const float* __restrict__ grid,
                            const int32_t* __restrict__ nsteps, float* __restrict__ tcur,
                            float* __restrict__ hcur, float* __restrict__ tst, float* __restrict__ tnx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* g = grid + (size_t)b * G;
  int ns = nsteps[b];
  ns = ns < 0 ? 0 : (ns > G - 1 ? G - 1 : ns);
  if (k < ns) {
    tcur[b] = g[k];
    hcur[b] = g[k + 1] - g[k];
    tnx[b] = g[k + 1];
  } else {
    tcur[b] = g[ns];
    hcur[b] = 0.f;
    tnx[b] = g[ns];
  }
  tst[b] = tcur[b];
}

__global__ void k_save_step(int B, size_t E, int G, int k, const float* __restrict__ y,
                            float* __restrict__ ys) {
  const int b = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  ys[((size_t)b * G + k) * E + e] = y[(size_t)b * E + e];
}

__global__ void k_grid_stats(int B, int method, const int32_t* __restrict__ nsteps, const int* __restrict__ fault,
                             int32_t* __restrict__ stats) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int ns = nsteps[b];
  stats[b * 4 + GNCDE_STAT_STEPS] = ns;
  stats[b * 4 + GNCDE_STAT_REJECTS] = 0;
  stats[b * 4 + GNCDE_STAT_EVALS] = method == GNCDE_RK4 ? 4 * ns : 1 + 6 * ns;
  stats[b * 4 + GNCDE_STAT_STATUS] = *fault ? 4 : 0;
}

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

__global__ void k_round_bf16(size_t N, const float* __restrict__ in, uint16_t* __restrict__ out) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (size_t)gridDim.x * blockDim.x)
    out[e] = __builtin_bit_cast(uint16_t, (__bf16)in[e]);
}

// (I + Abar_l) of layer l: [B, n, n] fp32, or the hi plane of its bf16 (hi, lo) pair (bf16 modes: planes
// [L, B, n, n] of uint16 each, the lo plane L*B*n*n elements after the hi plane — the fp32 buffer's bytes)
inline const float* abar_layer(const GncdeProblem& p, const float* abar, int l) {
  const size_t off = (size_t)l * p.B * p.n * p.n;
  if (p.compute != GNCDE_COMPUTE_FP32) return reinterpret_cast<const float*>(reinterpret_cast<const uint16_t*>(abar) + off);
  return abar + off;
}

struct VfWs {
  float *csum, *tg, *Z0, *Z1, *m, *abar, *wf, *wp, *bf, *inv, *q, *dx;
  void* coefT;     // one-launch evaluation: every (sample, interval, plane) transposed, once per solve
  uint16_t* wbf;   // GNCDE_COMPUTE_BF16_MFMA: W' per layer rounded to bfloat16, natural layout
  unsigned* sync;  // one-launch evaluation: per-group arrival counters [B] + the fault word, zeroed per solve
  unsigned* zgran;  // persistent solve: the tagged hand-off granules [2][B][n H][2], zeroed per solve
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
  w.csum = take(B * (size_t)(p.T - 1) * csum_stride(p.n));  // k_coef_sums' plane reductions, once per solve
  w.tg = take(B * n);
  w.Z0 = take(B * n * D);
  w.Z1 = take(B * n * D);
  w.m = take(B * n * D);
  // (I + Abar_l) for every layer (not needed by the one-launch evaluation)
  w.abar = take(rows_eval_used(p) ? 1 : (size_t)p.L * B * nn);
  w.wf = take(wsum);  // W' = W diag(rms_w) per layer, back to back
  w.wp = take(wsum);  // W' in k_layer's operand order (layers with layer_mode >= 0)
  w.bf = take(bsum);  // bias' = bias + W rms_b per layer
  w.inv = take(B * n);
  w.q = take((size_t)p.L * B * n);                          // q_l = (I + Abar_l) 1
  w.dx = take(B * n * (size_t)(p.cde_hidden > 0 ? 2 * p.cde_embed : 1));  // data-spline derivative at t
  w.sync = reinterpret_cast<unsigned*>(take(rows_sync_words(p.B)));
  w.zgran = reinterpret_cast<unsigned*>(take(rows_solve_shape(p) ? 4 * B * n * (size_t)p.dims[0] : 1));
  w.wbf = reinterpret_cast<uint16_t*>(take(p.compute == GNCDE_COMPUTE_BF16_MFMA ? (wsum + 1) / 2 : 1));
  // the one-launch evaluation reads a node block's column strip [:, R] as rows R of the transposed planes (whole
  // cache lines, like its rows block) instead of 16-column segments of every row
  const size_t planes = B * (size_t)(p.T - 1) * 4 * nn;
  const bool strip = rows_supported(p) || rows_solve_shape(p);
  w.coefT = take(strip ? (coef_is_bf16(p) ? (planes + 1) / 2 : planes) : 1);
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
size_t vf_forms_scratch(const GncdeProblem& p) { return (size_t)p.B * cdiv(p.n, kSlab) * 2 * p.n; }

void vf_forms(const GncdeProblem& p, const float* t, float* A, float* dA, float* tg, float* red, float* part,
              float* abar, hipStream_t st, float* qrow, float* dx) {
  const int B = p.B, n = p.n;
  const unsigned slabs = cdiv(n, kSlab);
  const bool bf16 = p.compute != GNCDE_COMPUTE_FP32;
  float* dxo = p.cde_hidden > 0 ? dx : nullptr;
  if (coef_is_bf16(p))
    hipLaunchKernelGGL(k_spline_slab<uint16_t>, dim3(slabs, B), dim3(256), 0, st, n, p.T, p.ts,
                       reinterpret_cast<const uint16_t*>(p.coef), p.tcoef, t, A, dA, tg, red, part, p.data_coef,
                       2 * p.cde_embed, dxo);
  else
    hipLaunchKernelGGL(k_spline_slab<float>, dim3(slabs, B), dim3(256), 0, st, n, p.T, p.ts, p.coef, p.tcoef, t, A,
                       dA, tg, red, part, p.data_coef, 2 * p.cde_embed, dxo);
  const unsigned tiles = cdiv(n, 32);
  if (bf16)
    hipLaunchKernelGGL(k_abar_all<uint16_t>, dim3(tiles, tiles, B), dim3(256), 0, st, n, p.L, (int)slabs, p.fusion,
                       A, dA, red, part, reinterpret_cast<uint16_t*>(abar), (size_t)B * n * n, qrow, B);
  else
    hipLaunchKernelGGL(k_abar_all<float>, dim3(tiles, tiles, B), dim3(256), 0, st, n, p.L, (int)slabs, p.fusion, A,
                       dA, red, part, abar, (size_t)B * n * n, qrow, B);
}

// The forward evaluation's forms: one k_abar_direct launch (every layer's (I + Abar_l), q_l, tg, dX) from the
// coefficients and k_coef_sums' reductions.
void vf_forms_direct(const GncdeProblem& p, const float* t, const float* csum, float* abar, float* qrow, float* tg,
                     float* dx, hipStream_t st, const PendingCombo* pending, const GridTime* gtime = nullptr) {
  const int B = p.B, n = p.n;
  const unsigned nt = cdiv(n, 32);
  PendingCombo pc{};
  if (pending) pc = *pending;
  GridTime gt{};
  if (gtime) gt = *gtime;
  const dim3 grid(nt * (nt + 1) / 2 + pc.blocks, B);
  float* dxo = p.cde_hidden > 0 ? dx : nullptr;
  const size_t ls = (size_t)B * n * n;
  const bool bf16 = p.compute != GNCDE_COMPUTE_FP32;
  if (coef_is_bf16(p))
    hipLaunchKernelGGL((k_abar_direct<uint16_t, uint16_t>), grid, dim3(256), 0, st, n, p.T, p.L, p.ts,
                       reinterpret_cast<const uint16_t*>(p.coef), csum, p.tcoef, t, p.fusion,
                       reinterpret_cast<uint16_t*>(abar), ls, qrow, tg, p.data_coef, 2 * p.cde_embed, dxo, B, pc, gt);
  else if (bf16)
    hipLaunchKernelGGL((k_abar_direct<float, uint16_t>), grid, dim3(256), 0, st, n, p.T, p.L, p.ts, p.coef, csum,
                       p.tcoef, t, p.fusion, reinterpret_cast<uint16_t*>(abar), ls, qrow, tg, p.data_coef,
                       2 * p.cde_embed, dxo, B, pc, gt);
  else
    hipLaunchKernelGGL((k_abar_direct<float, float>), grid, dim3(256), 0, st, n, p.T, p.L, p.ts, p.coef, csum,
                       p.tcoef, t, p.fusion, abar, ls, qrow, tg, p.data_coef, 2 * p.cde_embed, dxo, B, pc, gt);
}

const float* generic_vf_csum(const GncdeProblem& p, char* ws) {
  VfWs w;
  carve_vf(p, ws, w);
  return w.csum;
}

const int* generic_vf_fault(const GncdeProblem& p, char* ws) {
  VfWs w;
  carve_vf(p, ws, w);
  return reinterpret_cast<const int*>(w.sync + rows_fault_word(p.B));
}

// plane z (= (sample, interval, coefficient)) of [*, n, n] -> its transpose, 32 x 32 tiles through LDS
template <typename CT>
__global__ void __launch_bounds__(256) k_transpose_planes(int n, size_t planes, const CT* __restrict__ in,
                                                          CT* __restrict__ out) {
  __shared__ CT tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  for (size_t z = blockIdx.z; z < planes; z += gridDim.z) {
    const size_t base = z * n * n;
    for (int r = threadIdx.y; r < 32; r += 8)
      if (r0 + r < n && c0 + (int)threadIdx.x < n) tile[r][threadIdx.x] = in[base + (size_t)(r0 + r) * n + c0 + threadIdx.x];
    __syncthreads();
    for (int c = threadIdx.y; c < 32; c += 8)
      if (c0 + c < n && r0 + (int)threadIdx.x < n) out[base + (size_t)(c0 + c) * n + r0 + threadIdx.x] = tile[threadIdx.x][c];
    __syncthreads();
  }
}

void generic_vf_transpose(const GncdeProblem& p, char* ws, hipStream_t st) {
  VfWs w;
  carve_vf(p, ws, w);
  const size_t planes = (size_t)p.B * (p.T - 1) * 4;
  const dim3 tg(cdiv(p.n, 32), cdiv(p.n, 32), planes < 65535 ? (unsigned)planes : 65535u);
  if (coef_is_bf16(p))
    hipLaunchKernelGGL(k_transpose_planes<uint16_t>, tg, dim3(32, 8), 0, st, p.n, planes,
                       reinterpret_cast<const uint16_t*>(p.coef), reinterpret_cast<uint16_t*>(w.coefT));
  else
    hipLaunchKernelGGL(k_transpose_planes<float>, tg, dim3(32, 8), 0, st, p.n, planes, p.coef,
                       reinterpret_cast<float*>(w.coefT));
}

void generic_vf_prepare(const GncdeProblem& p, char* ws, hipStream_t st, bool rows_layout) {
  VfWs w;
  carve_vf(p, ws, w);
  (void)hipMemsetAsync(w.sync, 0, rows_sync_words(p.B) * sizeof(unsigned), st);
  const dim3 gs(4, p.T - 1, p.B);
  if (coef_is_bf16(p))
    hipLaunchKernelGGL(k_coef_sums<uint16_t>, gs, dim3(256), 0, st, p.n, p.T,
                       reinterpret_cast<const uint16_t*>(p.coef), w.csum);
  else
    hipLaunchKernelGGL(k_coef_sums<float>, gs, dim3(256), 0, st, p.n, p.T, p.coef, w.csum);
  const bool rows = rows_eval_used(p) || rows_layout;
  if (rows) generic_vf_transpose(p, ws, st);
  size_t wo = 0, bo = 0;
  for (int l = 0; l < p.L; ++l) {
    const int din = p.dims[l], dout = p.dims[l + 1];
    const LayerOffsets o = layer_offsets(p, l);
    fold_linear(din, dout, p.params + o.rms_w, p.params + o.rms_b, p.params + o.W, p.params + o.b, w.wf + wo,
                w.bf + bo, st);
    // W' in the MFMA operand order for every layer the evaluation runs through an operand-ordered kernel: all of
    // them on the one-launch path (whatever k_layer's own LDS envelope says), else k_layer's layers
    const bool cde_out = p.cde_hidden > 0 && l == p.L - 1;
    const int mode = layer_mode(p, l);
    if (rows) permute_linear(dout, din, cde_out, w.wf + wo, w.wp + wo, st);
    else if (mode >= 0) permute_linear(dout, din, mode == 2, w.wf + wo, w.wp + wo, st);
    wo += (size_t)din * dout;
    bo += dout;
  }
  if (p.compute == GNCDE_COMPUTE_BF16_MFMA)
    hipLaunchKernelGGL(k_round_bf16, dim3(cdiv(wo, 256) < 4096 ? cdiv(wo, 256) : 4096), dim3(256), 0, st, wo, w.wf,
                       w.wbf);
}

int generic_vf_eval(const GncdeProblem& p, const float* t, const float* y, float* dy, char* ws,
                    hipStream_t st, bool prepared, unsigned* bars, float* keep, bool need_dy,
                    const PendingCombo* pending, const FormBufs* forms, const FormsRide* ride,
                    const PendingCombo* post, bool* post_done) {
  if (post_done) *post_done = false;
  const int B = p.B, n = p.n;
  const size_t nn = (size_t)n * n;
  VfWs w;
  carve_vf(p, ws, w);
  unsigned local = 0;
  if (!prepared) generic_vf_prepare(p, ws, st);
  if (rows_eval_used(p)) {  // one launch: spline, fusion, every layer (and the read-out) (gncde_rows.hip)
    if (pending)  // (no forms launch to fold the combination into)
      hipLaunchKernelGGL(k_combo, dim3(pending->blocks, B), dim3(kComboThreads), 0, st, B, pending->E, pending->y,
                         pending->cb, pending->hcur, pending->out);
    if (!bars) {
      if (prepared) return GNCDE_ERR_ARG;
      bars = &local;
    }
    // (the workspace holds no (I + Abar_l) planes for these problems: there is no multi-kernel fallback here)
    return rows_vf_eval(p, t, y, dy, w.csum, w.coefT, w.wp, w.wbf, w.bf, w.Z0, w.Z1, w.sync,
                        reinterpret_cast<int*>(w.sync + rows_fault_word(B)), *bars, st, keep);
  }
  if (forms) {  // the caller launched this evaluation's forms into its own buffers
    w.abar = forms->abar;
    w.q = forms->q;
    w.tg = forms->tg;
    w.dx = forms->dx;
  } else {
    vf_forms_direct(p, t, w.csum, w.abar, w.q, w.tg, w.dx, st, pending);
  }
  const bool fused_out = p.cde_hidden == 0 || (p.cde_embed == 8 && p.dims[p.L] == 16 * p.cde_hidden);
  const float* Zin = y;
  float* bufs[2] = {w.Z0, w.Z1};
  size_t wo = 0, bo = 0;
  // the riding forms: samples split evenly over the hidden launches [hf, hf + nh) (the caller checked forms_ride:
  // every hidden layer is a fused launch).  A/B: GNCDE_FORMS_RIDE=2 puts them all in the first one, 3 in the last.
  int nh = ride ? p.L - 1 : 0, hf = 0, hidx = 0;
  if (ride) {
    const char* e = getenv("GNCDE_FORMS_RIDE");
    const int v = e ? atoi(e) : 1;
    if (v == 2 || v == 3) {
      hf = v == 3 ? p.L - 2 : 0;
      nh = 1;
    }
  }
  for (int l = 0; l < p.L; ++l) {
    const int din = p.dims[l], dout = p.dims[l + 1];
    float* Zout = keep && l + 1 < p.L ? keep + (size_t)l * B * n * p.dims[l + 1] : bufs[l & 1];
    const bool last = l == p.L - 1;
    if (!need_dy && last) break;  // a reverse sweep's keep forward reads the kept layers, never dy
    // A widening layer (d_out > d_in: the CDE wrapper's h -> h*de*2 read-out layer) is evaluated in the
    // reassociated order (I + Abar)(diag(inv) Z W'^T + 1 b'^T) = ((I + Abar) diag(inv) Z) W'^T + q b'^T with
    // q = (I + Abar) 1: the n x n product runs at width d_in instead of d_out (configs 3 / 5: 16x / 16x fewer
    // flops for that GEMM).  Exact algebra; only the fp32 summation order changes.
    const bool reassoc = dout > din;
    const int mode = layer_mode(p, l);
    if (mode >= 0 && (mode != 2 || fused_out)) {  // one fused launch (gncde_layer.hip)
      float* out = mode == 0 ? Zout : dy;
      FormsRide r{};
      if (mode == 0 && ride && hidx >= hf && hidx < hf + nh) {
        const int q = hidx - hf;
        r = *ride;
        const unsigned per = ride->blocks / ride->nb;  // tile pairs
        r.b0 = ride->b0 + ride->nb * q / nh;
        r.nb = ride->b0 + ride->nb * (q + 1) / nh - r.b0;
        r.blocks = per * r.nb;
      }
      if (mode == 0) ++hidx;
      const bool folded = layer_fused(p, l, mode, abar_layer(p, w.abar, l), Zin, w.wp + wo, w.bf + bo,
                                      w.q + (size_t)l * B * n, out, w.tg, w.dx, st, r.blocks ? &r : nullptr,
                                      mode == 2 ? post : nullptr);
      if (folded && post_done) *post_done = true;
      wo += (size_t)din * dout;
      bo += dout;
      Zin = Zout;
      continue;
    }
    GemmArgs lin{};
    GemmArgs pr{};
    float* m = w.m;
    if (reassoc) {
      row_inv(B * n, din, Zin, w.inv, st);
      pr.M = n;
      pr.N = din;
      pr.K = n;
      pr.A = abar_layer(p, w.abar, l);
      pr.a_bf16 = p.compute != GNCDE_COMPUTE_FP32;
      pr.a_lo = (long)p.L * B * nn;
      pr.lda = n;
      pr.sA = (long)nn;
      pr.B = Zin;
      pr.ldb = din;
      pr.sB = (long)n * din;
      pr.kscale = w.inv;
      pr.sK = n;
      pr.C = m;
      pr.ldc = din;
      pr.sC = (long)n * din;
      gemm(pr, B, false, st);
      lin.M = B * n;
      lin.N = dout;
      lin.K = din;
      lin.A = m;
      lin.lda = din;
      lin.B = w.wf + wo;
      lin.ldb = din;
      lin.C = Zout;
      lin.ldc = dout;
      lin.colbias = w.bf + bo;
      lin.biasrow = w.q + (size_t)l * B * n;
      lin.relu = last ? 0 : 1;
      if (last && fused_out) {  // the VF epilogue in the GEMM over all B*n rows
        if (p.cde_hidden > 0) {
          lin.cde_out = dy;
          lin.cde_dx = w.dx;
          lin.cde_tg = w.tg;
        } else {
          lin.C = dy;
          lin.rowscale = w.tg;
        }
      }
      gemm(lin, 1, true, st);
    } else {
      lin.M = B * n;
      lin.N = dout;
      lin.K = din;
      lin.A = Zin;
      lin.lda = din;
      lin.B = w.wf + wo;
      lin.ldb = din;
      lin.C = m;
      lin.ldc = dout;
      lin.rownorm = 1;
      lin.colbias = w.bf + bo;
      gemm(lin, 1, true, st);
      pr.M = n;
      pr.N = dout;
      pr.K = n;
      pr.A = abar_layer(p, w.abar, l);
      pr.a_bf16 = p.compute != GNCDE_COMPUTE_FP32;
      pr.a_lo = (long)p.L * B * nn;
      pr.lda = n;
      pr.sA = (long)nn;
      pr.B = m;
      pr.ldb = dout;
      pr.sB = (long)n * dout;
      pr.C = Zout;
      pr.ldc = dout;
      pr.sC = (long)n * dout;
      pr.relu = last ? 0 : 1;
      if (last && fused_out) {  // the VF epilogue in the GEMM: ODE dy = tg * Z, CDE contraction (de = 8)
        if (p.cde_hidden > 0) {
          pr.cde_out = dy;
          pr.cde_dx = w.dx;
          pr.cde_tg = w.tg;
        } else {
          pr.C = dy;
          pr.rowscale = w.tg;
          pr.sR = n;
        }
      }
      gemm(pr, B, false, st);
    }
    wo += (size_t)din * dout;
    bo += dout;
    Zin = Zout;
  }
  if (fused_out || !need_dy) return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
  const int dout = out_dim(p);
  hipLaunchKernelGGL(k_finalize, dim3(cdiv((size_t)n * dout, 256), B), dim3(256), 0, st, n,
                     p.dims[p.L], p.cde_hidden, p.cde_embed, p.T, p.ts, p.data_coef, t, w.tg, Zin,
                     dy);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

int rows_fault_status(const GncdeProblem& p, char* vf_ws, hipStream_t st, bool ran_rows) {
  if (!ran_rows) return GNCDE_OK;
  int fault = 0;
  if (hipMemcpyAsync(&fault, generic_vf_fault(p, vf_ws), sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return GNCDE_ERR_HIP;
  return fault ? GNCDE_ERR_BARRIER : GNCDE_OK;
}

// the whole solve (Tsit5 + PID, or a fixed grid) as ONE persistent launch on the one-launch evaluation (gncde_rows.hip)
int generic_rows_pid(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys, int32_t* stats, char* ws,
                     hipStream_t st) {
  VfWs w;
  carve_vf(p, ws, w);
  generic_vf_prepare(p, ws, st, true);
  float* part = reinterpret_cast<float*>(ws + generic_vf_workspace(p));
  if (rows_solve_granules())  // no tag is current
    (void)hipMemsetAsync(w.zgran, 0, 4 * (size_t)p.B * p.n * p.dims[0] * sizeof(unsigned), st);
  const int rc = rows_integrate_pid(p, s, y0, ys, stats, ws, part, w.csum, w.coefT, w.wp, w.bf, w.Z0, w.Z1, w.sync,
                                    w.zgran, st);
  if (rc) return rc;
  return rows_fault_status(p, ws, st, true);
}

// The fixed-grid solve's forms (k_abar_direct) do not depend on the stage input, only on the stage time, which the
// grid fixes: with GNCDE_FORMS_OVERLAP=1 they run one evaluation ahead on a side stream, into a second set of form
// buffers, while the caller's stream runs the previous evaluation's layers and the stage combination.  Measured at
// config 3 (alternating, one box): 13.2 ms per solve against 11.94 ms in line — the two cross-stream event waits
// per evaluation cost more than the 14.7 us forms launch they hide — so it is off by default (bitwise the same
// results either way: tests/test_gpu_configs.py::test_forms_overlap_bitwise).
bool forms_overlap(const GncdeProblem& p) {
  if (rows_eval_used(p)) return false;  // (the one-launch evaluation forms inside its own launch)
  const char* e = getenv("GNCDE_FORMS_OVERLAP");
  return e && atoi(e) != 0;
}

// The fixed-grid solve's forms of evaluation e + 1 ride as extra workgroups in evaluation e's hidden-layer launches
// (FormsRide, split by samples over them), into the second form buffer set: those launches leave most of every
// CU's registers and LDS idle, and the forms do not depend on the stage input.  Needs every hidden layer on the
// fused fp32 k_layer launch.  GNCDE_FORMS_RIDE=0 keeps one forms launch per evaluation (A/B, bitwise the same).
bool forms_ride(const GncdeProblem& p) {
  if (rows_eval_used(p) || p.compute != GNCDE_COMPUTE_FP32 || p.L < 2) return false;
  for (int l = 0; l + 1 < p.L; ++l)
    if (layer_mode(p, l) != 0) return false;
  const char* e = getenv("GNCDE_FORMS_RIDE");
  return !(e && atoi(e) == 0);
}

size_t form_set_floats(const GncdeProblem& p, int part) {  // abar, q, tg, dx of one form buffer set
  const size_t B = p.B, n = p.n;
  switch (part) {
    case 0: return (size_t)p.L * B * n * n;
    case 1: return (size_t)p.L * B * n;
    case 2: return B * n;
    default: return B * n * (size_t)(p.cde_hidden > 0 ? 2 * p.cde_embed : 1);
  }
}

// per (host thread, device): the side stream of the overlapped forms and its events (created once)
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t ev[6] = {};
  bool ok = false;
};
SideStream* side_stream() {
  static thread_local SideStream cache[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  SideStream& c = cache[dev];
  if (!c.ok) {
    if (hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    for (auto& e : c.ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    c.ok = true;
  }
  return &c;
}

size_t generic_integrate_workspace(const GncdeProblem& p, const GncdeSolver& s) {
  if (s.controller == GNCDE_CTRL_PID) return generic_pid_workspace(p);
  const size_t B = p.B, E = (size_t)p.n * state_dim(p);
  size_t sz = generic_vf_workspace(p);
  sz += 9 * align_up(B * E * 4, 256);  // y, ytmp, K[7]
  sz += 4 * align_up(B * 4, 256);      // tcur, hcur, tstage, tnx
  if (forms_overlap(p) || forms_ride(p)) {
    for (int q = 0; q < 4; ++q) sz += align_up(form_set_floats(p, q) * 4, 256);  // the second form buffer set
    sz += align_up(B * E * 4, 256);  // the riding partial sums of the read-out's combination
  }
  return sz;
}

int generic_integrate(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys, int32_t* stats,
                      char* ws, hipStream_t st) {
  if (s.controller == GNCDE_CTRL_PID) {
    if (rows_pid_supported(p, s)) return generic_rows_pid(p, s, y0, ys, stats, ws, st);
    const int rc = generic_integrate_pid(p, s, y0, ys, stats, ws, st);
    return rc ? rc : rows_fault_status(p, ws, st, rows_eval_used(p));
  }
  if (s.controller != GNCDE_CTRL_GRID) return GNCDE_ERR_UNSUPPORTED;
  if (rows_pid_supported(p, s)) return generic_rows_pid(p, s, y0, ys, stats, ws, st);  // the whole grid: one launch
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
  float* tnx = take(B);
  const int G = s.grid_len;
  // overlapped forms: buffer set e % 2 holds evaluation e's forms; the plan lists every evaluation's stage time
  const bool ovl = forms_overlap(p);
  SideStream* side = ovl ? side_stream() : nullptr;
  if (ovl && !side) return GNCDE_ERR_HIP;
  const bool ride = !ovl && forms_ride(p);
  FormBufs fbs[2];
  float* cpart = nullptr;  // (ride) the read-out combination's earlier terms, summed by blocks riding in the hidden launches
  std::vector<GridTime> plan;
  if (ovl || ride) {
    VfWs w0;
    carve_vf(p, ws, w0);
    fbs[0] = FormBufs{w0.abar, w0.q, w0.tg, w0.dx};
    fbs[1].abar = take(form_set_floats(p, 0));
    fbs[1].q = take(form_set_floats(p, 1));
    fbs[1].tg = take(form_set_floats(p, 2));
    fbs[1].dx = take(form_set_floats(p, 3));
    cpart = take(B * E);
    auto add = [&](int k, float c, int fsal) { plan.push_back(GridTime{s.grid, s.nsteps, G, k, c, fsal}); };
    if (s.method == GNCDE_RK4) {
      for (int k = 0; k < G - 1; ++k) {
        add(k, 0.f, 0);
        add(k, 0.5f, 0);
        add(k, 0.5f, 0);
        add(k, 1.0f, 0);
      }
    } else {  // the FSAL k0, then per step the stages at c2 .. c5, 1 and the FSAL stage at the step's end knot
      add(0, 0.f, 0);
      for (int k = 0; k < G - 1; ++k) {
        add(k, TSIT5_C2, 0);
        add(k, TSIT5_C3, 0);
        add(k, TSIT5_C4, 0);
        add(k, TSIT5_C5, 0);
        add(k, 1.0f, 0);
        add(k, 0.f, 1);
      }
    }
  }
  const unsigned gb = cdiv(B, 256);
  const dim3 ge(cdiv(E, 256), B);
  const dim3 gc(cdiv(E, 256 * kComboU), B);
  (void)hipMemcpyAsync(y, y0, B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  if (s.save_mode == GNCDE_SAVE_STEPS)
    hipLaunchKernelGGL(k_save_step, ge, dim3(256), 0, st, B, E, G, 0, y, ys);
  generic_vf_prepare(p, ws, st);

  // Every evaluation's stage time tst is written by the launch before it (k_grid_step for c = 0, k_combo for the
  // others); the step's y <- y_{k+1} and Tsit5's FSAL k1 <- k7 are pointer swaps, not copies.
  unsigned bars = 0;
  // activation record (GncdeSolver.act_rec): stage i of step k keeps its hidden outputs in slab (k, i)
  const int S = s.method == GNCDE_RK4 ? 4 : 6;
  const size_t slab = (size_t)(p.L - 1) * B * E;
  auto act = [&](int k, int i) -> float* {
    return s.act_rec && k < G - 1 ? s.act_rec + ((size_t)k * S + i) * slab : nullptr;
  };
  float* keep_next = nullptr;  // the keep slab of the next evaluation
  // A combination whose output the next evaluation reads right away rides in that evaluation's forms launch
  // (PendingCombo): one launch per stage fewer.  Anything else in between flushes it as its own k_combo.
  PendingCombo pend{};
  bool has_pend = false;
  const char* nm = getenv("GNCDE_COMBO_SEPARATE");  // A/B: every combination as its own k_combo launch
  const bool merge = !ovl && !ride && !(nm && atoi(nm) != 0);
  int ecur = 0, issued = 0;  // overlapped forms: the next evaluation, the forms launched so far
  const float* csum = generic_vf_csum(p, ws);
  auto issue_forms = [&](int e) {  // side stream: forms of evaluation e into set e % 2, once layers e - 2 are done
    if (e >= (int)plan.size()) return;
    if (e >= 2) (void)hipStreamWaitEvent(side->s, side->ev[2 + (e & 1)], 0);
    const FormBufs& f = fbs[e & 1];
    vf_forms_direct(p, tst, csum, f.abar, f.q, f.tg, f.dx, side->s, nullptr, &plan[e]);
    (void)hipEventRecord(side->ev[e & 1], side->s);
    issued = e + 1;
  };
  const unsigned tpairs = cdiv(p.n, 32) * (cdiv(p.n, 32) + 1) / 2;
  auto ride_of = [&](int e) {  // evaluation e's forms into set e % 2, all samples (generic_vf_eval splits them)
    const FormBufs& f = fbs[e & 1];
    FormsRide r{};
    r.f = FormsArgs{p.n, p.T, p.L, 2 * p.cde_embed, B, p.ts, p.coef, csum, p.tcoef, p.fusion, p.data_coef,
                    f.abar, (size_t)B * p.n * p.n, f.q, f.tg, p.cde_hidden > 0 ? f.dx : nullptr};
    r.gt = plan[e];
    r.b0 = 0;
    r.nb = B;
    r.blocks = tpairs * B;
    return r;
  };
  if (ride) vf_forms_direct(p, tst, csum, fbs[0].abar, fbs[0].q, fbs[0].tg, fbs[0].dx, st, nullptr, &plan[0]);
  if (ovl) {  // the side stream starts after everything queued on st so far (the prepared workspace)
    (void)hipEventRecord(side->ev[4], st);
    (void)hipStreamWaitEvent(side->s, side->ev[4], 0);
    issue_forms(0);
  }
  // With the forms riding, a combination that follows a read-out runs in that launch's epilogue (PendingCombo as
  // `post`); GNCDE_COMBO_FOLD=0 keeps it a k_combo launch (A/B, bitwise the same)
  const char* nf = getenv("GNCDE_COMBO_FOLD");
  const bool fold = ride && !(nf && atoi(nf) == 0);
  const char* npart = getenv("GNCDE_COMBO_PARTIAL");
  const bool partial_ride = fold && !(npart && atoi(npart) == 0);
  PendingCombo post_pc{};
  bool post_on = false, post_done = false;
  auto flush = [&]() {
    if (has_pend)
      hipLaunchKernelGGL(k_combo, gc, dim3(kComboThreads), 0, st, B, E, pend.y, pend.cb, pend.hcur, pend.out);
    has_pend = false;
  };
  auto eval = [&](const float* yin, float* out) {
    if (ovl) {  // the next evaluation's forms go out first, then this one's layers once its forms are done
      if (issued <= ecur + 1) issue_forms(ecur + 1);
      (void)hipStreamWaitEvent(st, side->ev[ecur & 1], 0);
      const int r = generic_vf_eval(p, tst, yin, out, ws, st, true, &bars, keep_next, true, nullptr, &fbs[ecur & 1]);
      (void)hipEventRecord(side->ev[2 + (ecur & 1)], st);
      ++ecur;
      return r;
    }
    if (ride) {  // this evaluation's forms are in set ecur % 2; the next one's ride in its hidden layers
      FormsRide r{};
      if (ecur + 1 < (int)plan.size()) r = ride_of(ecur + 1);
      post_done = false;
      // the folded combination's earlier terms ride too (every sample's, split with the forms over the hidden
      // launches), so the read-out epilogue loads one partial per element; GNCDE_COMBO_PARTIAL=0 keeps them there
      post_pc.part = nullptr;
      if (post_on && r.blocks && post_pc.cb.nk >= 2 && post_pc.cb.nk <= 7 && partial_ride && p.L >= 2) {
        r.pnk = post_pc.cb.nk - 1;
        for (int j = 0; j < r.pnk; ++j) {
          r.pK[j] = post_pc.cb.K[j];
          r.pa[j] = post_pc.cb.a[j];
        }
        r.part = cpart;
        r.pE = E;
        r.pbs = gc.x;
        post_pc.part = cpart;
      }
      const int res = generic_vf_eval(p, tst, yin, out, ws, st, true, &bars, keep_next, true, nullptr,
                                      &fbs[ecur & 1], r.blocks ? &r : nullptr, post_on ? &post_pc : nullptr,
                                      &post_done);
      post_pc.part = nullptr;
      ++ecur;
      return res;
    }
    const PendingCombo* pc = has_pend ? &pend : nullptr;
    has_pend = false;
    return generic_vf_eval(p, tst, yin, out, ws, st, true, &bars, keep_next, true, pc);
  };
  // stage record (GncdeSolver.stage_rec): the stage input U_i of step k goes to slot (k, i-1) as it is formed
  float* rec = G >= 2 ? s.stage_rec : nullptr;
  int rec_k = 0, rec_i = 0;  // slot of the next combination's output (rec_i == 0: not recorded)
  bool fsal_next = false;     // the combination forms Tsit5's FSAL stage input (its time: the step's end knot)
  auto make_combo = [&](std::initializer_list<std::pair<int, float>> terms, float c_next, bool has_next, int gk) {
    Combo cb{};
    if (gk >= 0) {  // step gk's k_grid_step folded in (nothing before this combination reads its outputs)
      cb.grid = s.grid;
      cb.nsteps = s.nsteps;
      cb.G = G;
      cb.gk = gk;
      cb.tcur_out = tcur;
      cb.hcur_out = hcur;
      cb.tnx_out = tnx;
    }
    if (rec && rec_i > 0) {
      cb.rec = rec + ((size_t)rec_k * (S - 1) + rec_i - 1) * E;
      cb.rec_stride = (size_t)(G - 1) * (S - 1) * E;
    }
    cb.nk = 0;
    for (auto& tr : terms) {
      cb.K[cb.nk] = K[tr.first];
      cb.a[cb.nk] = tr.second;
      cb.nk++;
    }
    cb.c = c_next;
    cb.tcur = tcur;
    cb.tend = fsal_next ? tnx : nullptr;
    cb.tst = has_next ? tst : nullptr;
    return cb;
  };
  auto combo = [&](std::initializer_list<std::pair<int, float>> terms, float* out, float c_next, bool has_next,
                   int gk = -1) {
    const Combo cb = make_combo(terms, c_next, has_next, gk);
    flush();
    if (has_next && merge) {  // the next evaluation reads `out` (and its stage time) first: fold it into that launch
      pend = PendingCombo{cb, y, hcur, out, E, gc.x};
      has_pend = true;
    } else {
      hipLaunchKernelGGL(k_combo, gc, dim3(kComboThreads), 0, st, B, E, y, cb, hcur, out);
    }
  };

  // Stage j's evaluation into K[j] followed by the next stage's input out = y + h sum_i a_i K_i (terms end with
  // K[j]).  (Round 2 folded the combination into the read-out k_layer's epilogue and measured it slower at config 3,
  // 15.8 vs 15.15 ms per solve: the epilogue's dependent K loads lengthened the critical launch by more than k_combo
  // cost.  Round 5's fold issues those loads right after each wave's K loop, under the partials' barrier.)
  int rc = GNCDE_OK;
  int cur_k = 0;  // the step eval_combo's evaluations belong to (activation slab (cur_k, j))
  auto eval_combo = [&](const float* yin, int j, std::initializer_list<std::pair<int, float>> terms, float* out,
                        float c_next, bool has_next) {
    keep_next = act(cur_k, j);
    if (fold) {  // the combination rides in the evaluation's read-out epilogue when that launch can take it
      flush();
      post_pc = PendingCombo{make_combo(terms, c_next, has_next, -1), y, hcur, out, E, gc.x};
      post_on = true;
      rc |= eval(yin, K[j]);
      post_on = false;
      if (!post_done)
        hipLaunchKernelGGL(k_combo, gc, dim3(kComboThreads), 0, st, B, E, post_pc.y, post_pc.cb, post_pc.hcur,
                           post_pc.out);
      return;
    }
    rc |= eval(yin, K[j]);
    combo(terms, out, c_next, has_next);
  };

  const int steps = G - 1;
  if (s.method == GNCDE_RK4) {
    for (int k = 0; k < steps && rc == GNCDE_OK; ++k) {
      flush();
      hipLaunchKernelGGL(k_grid_step, dim3(gb), dim3(256), 0, st, B, G, k, s.grid, s.nsteps, tcur, hcur, tst, tnx);
      rec_k = k;
      rec_i = 1;
      cur_k = k;
      eval_combo(y, 0, {{0, 0.5f}}, yt, 0.5f, true);
      rec_i = 2;
      eval_combo(yt, 1, {{1, 0.5f}}, yt, 0.5f, true);
      rec_i = 3;
      eval_combo(yt, 2, {{2, 1.0f}}, yt, 1.0f, true);
      rec_i = 0;
      // y + h/6 (k1 + 2k2 + 2k3 + k4)
      eval_combo(yt, 3, {{0, 1.0f / 6.0f}, {1, 2.0f / 6.0f}, {2, 2.0f / 6.0f}, {3, 1.0f / 6.0f}}, yt, 0.f, false);
      flush();
      std::swap(y, yt);
      if (s.save_mode == GNCDE_SAVE_STEPS)
        hipLaunchKernelGGL(k_save_step, ge, dim3(256), 0, st, B, E, G, k + 1, y, ys);
    }
  } else {  // Tsit5 on the grid (ConstantStepSize), FSAL
    hipLaunchKernelGGL(k_grid_step, dim3(gb), dim3(256), 0, st, B, G, 0, s.grid, s.nsteps, tcur, hcur, tst, tnx);
    keep_next = act(0, 0);
    rc |= eval(y, K[0]);
    for (int k = 0; k < steps && rc == GNCDE_OK; ++k) {
      flush();
      // With the forms riding (timed from the grid) nothing reads the step geometry before the step's first
      // combination, which then forms it itself: one launch per step fewer.
      if (!ride)
        hipLaunchKernelGGL(k_grid_step, dim3(gb), dim3(256), 0, st, B, G, k, s.grid, s.nsteps, tcur, hcur, tst, tnx);
      cur_k = k;
      rec_k = k;
      rec_i = 1;
      combo({{0, TSIT5_A21}}, yt, TSIT5_C2, true, ride ? k : -1);  // K[0] is the FSAL value
      rec_i = 2;
      eval_combo(yt, 1, {{0, TSIT5_A31}, {1, TSIT5_A32}}, yt, TSIT5_C3, true);
      rec_i = 3;
      eval_combo(yt, 2, {{0, TSIT5_A41}, {1, TSIT5_A42}, {2, TSIT5_A43}}, yt, TSIT5_C4, true);
      rec_i = 4;
      eval_combo(yt, 3, {{0, TSIT5_A51}, {1, TSIT5_A52}, {2, TSIT5_A53}, {3, TSIT5_A54}}, yt, TSIT5_C5, true);
      rec_i = 5;
      eval_combo(yt, 4, {{0, TSIT5_A61}, {1, TSIT5_A62}, {2, TSIT5_A63}, {3, TSIT5_A64}, {4, TSIT5_A65}}, yt, 1.0f,
                 true);
      rec_i = 0;
      fsal_next = true;
      eval_combo(yt, 5, {{0, TSIT5_B1}, {1, TSIT5_B2}, {2, TSIT5_B3}, {3, TSIT5_B4}, {4, TSIT5_B5}, {5, TSIT5_B6}},
                 yt, 1.0f, true);
      fsal_next = false;
      keep_next = act(k + 1, 0);  // the FSAL evaluation is the next step's stage 0
      rc |= eval(yt, K[6]);
      flush();
      std::swap(y, yt);
      std::swap(K[0], K[6]);
      if (s.save_mode == GNCDE_SAVE_STEPS)
        hipLaunchKernelGGL(k_save_step, ge, dim3(256), 0, st, B, E, G, k + 1, y, ys);
    }
  }
  flush();
  if (ovl) {  // st resumes after the side stream's last launch (forms issued past a failed evaluation included)
    (void)hipEventRecord(side->ev[5], side->s);
    (void)hipStreamWaitEvent(st, side->ev[5], 0);
  }
  if (s.save_mode == GNCDE_SAVE_T1)
    (void)hipMemcpyAsync(ys, y, B * E * sizeof(float), hipMemcpyDeviceToDevice, st);
  if (stats)
    hipLaunchKernelGGL(k_grid_stats, dim3(gb), dim3(256), 0, st, B, s.method, s.nsteps, generic_vf_fault(p, ws),
                       stats);
  if (hipGetLastError() != hipSuccess) return GNCDE_ERR_HIP;
  return rc ? rc : rows_fault_status(p, ws, st, rows_eval_used(p));
}

}  // namespace gncde
