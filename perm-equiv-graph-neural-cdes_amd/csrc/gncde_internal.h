// Internal declarations shared by the HIP translation units of libgncde_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/gncde.h"

namespace gncde {

// ---- Tsit5 tableau (Tsitouras 2011), restated in oracle/gncde_oracle.py:TSIT5_* ----------------
#define TSIT5_A21 0.161f
#define TSIT5_A31 (-0.008480655492356989f)
#define TSIT5_A32 0.335480655492357f
#define TSIT5_A41 2.897153057105493f
#define TSIT5_A42 (-6.359448489975075f)
#define TSIT5_A43 4.3622954328695815f
#define TSIT5_A51 5.325864828439257f
#define TSIT5_A52 (-11.748883564062828f)
#define TSIT5_A53 7.4955393428898365f
#define TSIT5_A54 (-0.09249506636175525f)
#define TSIT5_A61 5.86145544294642f
#define TSIT5_A62 (-12.92096931784711f)
#define TSIT5_A63 8.159367898576159f
#define TSIT5_A64 (-0.071584973281401f)
#define TSIT5_A65 (-0.028269050394068383f)
#define TSIT5_B1 0.09646076681806523f
#define TSIT5_B2 0.01f
#define TSIT5_B3 0.4798896504144996f
#define TSIT5_B4 1.379008574103742f
#define TSIT5_B5 (-3.290069515436081f)
#define TSIT5_B6 2.324710524099774f
#define TSIT5_E1 0.001780011052226f
#define TSIT5_E2 0.000816434459657f
#define TSIT5_E3 (-0.007880878010262f)
#define TSIT5_E4 0.144711007173263f
#define TSIT5_E5 (-0.582357165452555f)
#define TSIT5_E6 0.458082105929187f
#define TSIT5_E7 (-0.015151515151515152f)
#define TSIT5_C2 0.161f
#define TSIT5_C3 0.327f
#define TSIT5_C4 0.9f
#define TSIT5_C5 0.9800255409045097f

// Stage time t + c*h with exactly two fp32 roundings (no contraction), matching the oracle.
__device__ __forceinline__ float stage_time(float t, float c, float h) {
  return __fadd_rn(t, __fmul_rn(c, h));
}

// Tsit5 row a[s][0..5] for stage s = 1..6 (row 6 = b_sol) and c[s], as compile-time immediates
// selected by a wave-uniform switch (no constant-memory table).
__device__ __forceinline__ void tsit5_row(int s, float (&a)[6], float& c) {
  a[0] = a[1] = a[2] = a[3] = a[4] = a[5] = 0.f;
  c = 1.f;
  switch (s) {
    case 1: a[0] = TSIT5_A21; c = TSIT5_C2; break;
    case 2: a[0] = TSIT5_A31; a[1] = TSIT5_A32; c = TSIT5_C3; break;
    case 3: a[0] = TSIT5_A41; a[1] = TSIT5_A42; a[2] = TSIT5_A43; c = TSIT5_C4; break;
    case 4: a[0] = TSIT5_A51; a[1] = TSIT5_A52; a[2] = TSIT5_A53; a[3] = TSIT5_A54; c = TSIT5_C5; break;
    case 5:
      a[0] = TSIT5_A61; a[1] = TSIT5_A62; a[2] = TSIT5_A63; a[3] = TSIT5_A64; a[4] = TSIT5_A65;
      break;
    default:
      a[0] = TSIT5_B1; a[1] = TSIT5_B2; a[2] = TSIT5_B3; a[3] = TSIT5_B4; a[4] = TSIT5_B5; a[5] = TSIT5_B6;
      break;
  }
}

// Tsit5 free interpolant weights b_i(theta): y(t + theta h) = y + h * sum_i b_i(theta) f_i
// (restated in oracle/gncde_oracle.py:tsit5_dense_weights).
__device__ __forceinline__ void tsit5_dense(float th, float (&w)[7]) {
  const float t2 = th * th;
  w[0] = -1.0530884977290216f * th * (th - 1.3299890189751412f) * (t2 - 1.4364028541716351f * th + 0.7139816917074209f);
  w[1] = 0.1017f * t2 * (t2 - 2.1966568338249754f * th + 1.2949852507374631f);
  w[2] = 2.490627285651252793f * t2 * (t2 - 2.38535645472061657f * th + 1.57803468208092486f);
  w[3] = -16.54810288924490272f * (th - 1.21712927295533244f) * (th - 0.61620406037800089f) * t2;
  w[4] = 47.37952196281928122f * (th - 1.203071208372362603f) * (th - 0.658047292653547382f) * t2;
  w[5] = -34.87065786149660974f * (th - 1.2f) * (th - 0.666666666666666667f) * t2;
  w[6] = 2.5f * (th - 1.0f) * (th - 0.6f) * t2;
}

// Sum over the four 16-lane rows of a wave64 (lane ^ 16, lane ^ 32) on the gfx950 row-swap VALU ops:
// no LDS round trip.  Written as asm because the clang builtins of this toolchain drop the second
// (vsrc) result of the swap; the leading s_nop covers the VALU-write -> permlane-read hazard.
__device__ __forceinline__ float xor_sum_rows4(float v) {
  float x = v, y = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  v = x + y;  // lanes l and l^32 both hold v_l + v_{l^32}
  x = v;
  y = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  return x + y;
}

// Sum over all 64 lanes, result in every lane: DPP within each 16-lane row (quad swaps, then the half-row and row
// mirrors), then the gfx950 row swaps (xor_sum_rows4).  No LDS and no lane-index arithmetic.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum64(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return xor_sum_rows4(v);
}

// equinox RMSNorm scale rsqrt(mean(x^2) + eps) on the hardware reciprocal square root (1 ulp; the
// parity tolerances are fp32-accumulation bounds).
__device__ __forceinline__ float rms_inv(float sumsq, float inv_d) {
  return __builtin_amdgcn_rsqf(fmaf(sumsq, inv_d, 1e-5f));
}

// diffrax CubicInterpolation interval rule: clip(searchsorted(ts, t, 'left') - 1, 0, T-2).
__device__ __forceinline__ int interval_index(const float* ts, int T, float t) {
  int lo = 0, hi = T;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (ts[mid] < t) lo = mid + 1; else hi = mid;
  }
  int i = lo - 1;
  i = i < 0 ? 0 : i;
  return i > T - 2 ? T - 2 : i;
}

// The same index from one round of loads: every lane of the wave reads a knot and the ballot counts the knots
// below t (searchsorted 'left' on sorted knots), instead of log2(T) dependent loads.  Call with the whole wave
// active (uniform control flow).
// XCD-aware work index: workgroup s runs on XCD s % 8, so consecutive work indices (one sample's row blocks, which
// read the same sample's Z, g_P and coefficient columns) go to one XCD and its L2 (a bijection of [0, G) when
// G % 8 == 0)
__device__ __forceinline__ int xcd_work(int s, int G) { return G % 8 ? s : (s % 8) * (G / 8) + s / 8; }

__device__ __forceinline__ int interval_index_wave(const float* ts, int T, float t) {
  const int lane = threadIdx.x & 63;
  int cnt = 0;
  for (int j0 = 0; j0 < T; j0 += 64) {
    const int j = j0 + lane;
    const float v = ts[j < T ? j : T - 1];
    cnt += __popcll(__ballot(j < T && v < t));
  }
  const int i = cnt - 1 < 0 ? 0 : cnt - 1;
  return i > T - 2 ? T - 2 : i;
}

// Offsets of layer l's parameters inside the packed params buffer (see gncde.h).
struct LayerOffsets {
  size_t rms_w, rms_b, W, b;
};
inline LayerOffsets layer_offsets(const GncdeProblem& p, int l) {
  size_t off = 0;
  for (int j = 0; j < l; ++j) {
    const size_t din = p.dims[j], dout = p.dims[j + 1];
    off += 2 * din + dout * din + dout;
  }
  const size_t din = p.dims[l], dout = p.dims[l + 1];
  LayerOffsets o;
  o.rms_w = off;
  o.rms_b = off + din;
  o.W = off + 2 * din;
  o.b = off + 2 * din + dout * din;
  return o;
}
inline size_t params_floats(const GncdeProblem& p) {
  size_t off = 0;
  for (int j = 0; j < p.L; ++j) {
    const size_t din = p.dims[j], dout = p.dims[j + 1];
    off += 2 * din + dout * din + dout;
  }
  return off;
}

inline int state_dim(const GncdeProblem& p) { return p.dims[0]; }
inline int out_dim(const GncdeProblem& p) { return p.cde_hidden > 0 ? p.cde_hidden : p.dims[p.L]; }
inline int max_dim(const GncdeProblem& p) {
  int m = 0;
  for (int l = 0; l <= p.L; ++l) m = p.dims[l] > m ? p.dims[l] : m;
  return m;
}

int validate_problem(const GncdeProblem* p);
int validate_solver(const GncdeProblem* p, const GncdeSolver* s);

// batched fp32 MFMA GEMM and helpers: gncde_gemm.hip
struct GemmArgs {
  int M, N, K;
  const float* A;  // A[b] + r * lda + k
  long lda, sA;
  const float* B;  // NN: B[b] + k * ldb + j;  TRANS_B: B[b] + j * ldb + k
  long ldb, sB;
  float* C;
  long ldc, sC;
  const float* rowscale;  // optional: C = rowscale[b * sR + r] * acc
  long sR;
  const float* colbias;  // optional [N]
  const float* biasrow;  // optional with colbias: C += biasrow[b * sR + r] * colbias[c] (rank-1 bias q b'^T)
  const float* kscale;   // optional (NN only): B row k scaled by kscale[b * sK + k] (a diagonal left of B)
  long sK;
  int a_bf16;      // (NN only) A holds bf16 (hi, lo) pairs: hi at the element offsets of A, lo a_lo elements later
  long a_lo;
  int relu;
  int accumulate;  // C += result
  int rownorm;     // (NN/TRANS_B only) scale row r by 1/sqrt(mean_k A[r][k]^2 + 1e-5): RMSNorm folded into the GEMM
  float* inv_out;  // optional with rownorm: those factors, [b * sR + r]
  // CDE-wrapper epilogue (de = 8 so that one 16-column MFMA tile is one hidden channel): instead of C, write
  // cde_out[b*M + r][c/16] = cde_tg[b*M + r] * sum_{q<16} C[r][c+q] * cde_dx[b*M + r][q], with dX the data
  // spline's derivative at the row's stage time (cde_wrapper_vector_field.py:19-26).  Rows are global node
  // rows, so the same epilogue serves a per-sample batched GEMM (M = n) and one GEMM over all B*n rows.
  float* cde_out;
  const float* cde_dx;  // [rows, 16]
  const float* cde_tg;  // [rows]
};
// TRANS_A: A[b] + k * lda + r (A^T stored row-major)
void gemm(const GemmArgs& g, int batch, bool trans_b, hipStream_t st, bool trans_a = false);
void fold_linear(int din, int dout, const float* rw, const float* rb, const float* W, const float* bias, float* Wf,
                 float* bf, hipStream_t st);
void row_inv(int rows, int d, const float* Z, float* inv, hipStream_t st);

// fused ConvLayer launch of the generic path: gncde_layer.hip.  layer_mode: -1 = not supported (two-GEMM path),
// 0 hidden layer (ReLU), 1 ODE output layer (tg scaling), 2 CDE output layer (de = 8 contraction).
int layer_mode(const GncdeProblem& p, int l);
void permute_linear(int rows, int din, bool cde, const float* W, float* out, hipStream_t st);

struct FormsRide;
struct PendingCombo;
// ride (optional, fp32 hidden layers only): forms blocks launched after the layer's workgroups in the same grid;
// post (optional, the fp32 CDE read-out): the stage combination whose last term is this launch's output, folded into
// its epilogue.  Returns whether post was folded (else the caller launches it).
bool layer_fused(const GncdeProblem& p, int l, int mode, const float* abar, const float* Z, const float* wperm,
                 const float* bf, const float* q, float* out, const float* tg, const float* dx, hipStream_t st,
                 const FormsRide* ride = nullptr, const PendingCombo* post = nullptr);

// generic (any-shape, multi-kernel) path: gncde_generic.hip
size_t generic_vf_workspace(const GncdeProblem& p);
size_t generic_integrate_workspace(const GncdeProblem& p, const GncdeSolver& s);
// A(t), dA/dt(t), the time-channel derivative tg and the row/col/diag/total reductions (stride 8 n per sample)
// part: scratch of vf_forms_scratch(p) floats (per-slab column partials)
size_t vf_forms_scratch(const GncdeProblem& p);
// ... and (I + Abar_l) of every layer into abar [L, B, n, n] (red: stride 8 n per sample, completed here too)
// qrow (optional, [L, B, n]) receives q_l = (I + Abar_l) 1 (the row sums, from the reductions); dx (optional, CDE
// wrapper, [B, n, 2 de]) the data spline's derivative at t.
void vf_forms(const GncdeProblem& p, const float* t, float* A, float* dA, float* tg, float* red, float* part,
              float* abar, hipStream_t st, float* qrow = nullptr, float* dx = nullptr);
// rows_layout: also lay out what the one-launch evaluation reads (transposed planes, every W' permuted) for a caller
// that runs it although rows_supported(p) is false (the persistent solve at batches past one co-resident round)
void generic_vf_prepare(const GncdeProblem& p, char* ws, hipStream_t st, bool rows_layout = false);
// bars: the solve's count of per-group barriers done by one-launch evaluations so far (gncde_rows.hip); nullptr
// only together with prepared = false (a standalone evaluation)
// keep (optional, [L-1, B, n, d]): every hidden layer's output Z_{l+1} kept for the reverse mode (uniform width d);
// need_dy = false (a reverse sweep's keep forward): dy is not wanted and the multi-kernel path skips the read-out
// A Tsit5 / RK4 stage combination (k_combo, gncde_generic.hip):
// out = y + h_b * sum_j a_j K_j   (up to 7 terms; K_j == nullptr terms skipped), and (tst != nullptr) the next
// stage's time t_b + c h_b (the stage-time launch folded in)
struct Combo {
  const float* K[7];
  float a[7];
  int nk;
  float c;
  const float* tcur;
  const float* tend;  // non-null: the next stage is Tsit5's FSAL stage, evaluated at the step's end knot tend[b]
  float* tst;
  float* rec;         // stage record slot of this stage input ([B, G-1, S-1, E] at (k, i-1)) or nullptr
  size_t rec_stride;  // floats between consecutive samples' slots: (G-1)*(S-1)*E
  // grid != nullptr: step gk's geometry from the grid folded in (k_grid_step's work and arithmetic): h and the
  // stage time come from grid / nsteps, and block 0 of each sample writes tcur, hcur_out and tnx
  const float* grid;
  const int32_t* nsteps;
  int G, gk;
  float *tcur_out, *hcur_out, *tnx_out;
};
// A stage combination folded into the next evaluation's k_abar_direct launch: its blocks follow the form tiles in
// the grid (the two are independent: the forms read the coefficients at the stage's time, which they compute from
// tcur / hcur / c / tend exactly as the combination does; the combination reads K and y), so the combination costs
// no launch of its own and runs under the forms' memory round trips.
struct PendingCombo {
  Combo cb;
  const float* y;
  const float* hcur;
  float* out;
  size_t E;
  unsigned blocks;  // combination blocks per sample (0: none)
  const float* part;  // folded read-out epilogue: the earlier terms' sum, formed by riding blocks (FormsRide), or null
};
// A fixed-grid evaluation's stage time computed by the forms launch itself from the grid (the overlapped forms of
// generic_integrate: launched on a side stream ahead of the stage combination that writes tst), with exactly the
// arithmetic of k_grid_step + the combination: tcur = g[min(k, ns)], h = k < ns ? g[k+1] - g[k] : 0,
// t = fsal ? g[min(k + 1, ns)] : tcur + c h (stage_time).
struct GridTime {
  const float* grid;  // [B, G] (nullptr: not used)
  const int32_t* nsteps;
  int G, k;
  float c;
  int fsal;
};
// The outputs of one evaluation's forms launch (every layer's (I + Abar_l), q_l, tg, dX), when the caller owns them
struct FormBufs {
  float *abar, *q, *tg, *dx;
};
// What one forms tile block reads and writes (fp32 coefficients and planes; gncde_forms.h)
struct FormsArgs {
  int n, T, L, de2, B;  // de2 = 2 de (CDE wrapper), B = the batch (q_l rows are [L, B, n])
  const float *ts, *coef, *csum, *tcoef, *fus, *data_coef;
  float* abar;          // (I + Abar_l) planes [L, B, n, n]
  size_t layer_stride;  // B n n
  float *qrow, *tg, *dx;  // dx: nullptr unless the CDE wrapper
};
// A fixed-grid evaluation's forms riding as extra workgroups in the previous evaluation's hidden-layer launches
// (gncde_layer.hip): samples [b0, b0 + nb) of the next evaluation's forms, its stage time from the grid (gt)
// kComboU elements per thread (strided by the block), each element's stage-buffer loads issued together before the
// summation: the load latency is paid once per thread, not once per term.  Same summation order per element.
constexpr int kComboU = 4;
constexpr int kComboThreads = 256;
struct FormsRide {
  FormsArgs f;
  GridTime gt;
  int b0, nb;
  unsigned blocks;  // tile pairs x nb (0: no ride)
  // the following read-out's stage combination, all terms but its last (that evaluation's own output), summed by
  // further riding blocks into part [B, pE] (pbs blocks of kComboThreads x kComboU elements per sample; 0: none), in
  // k_combo's fmaf order: the read-out epilogue then loads one partial per element instead of every earlier term
  const float* pK[6];
  float pa[6];
  int pnk;
  float* part;
  size_t pE;
  unsigned pbs;
};
// pending (optional): a stage combination folded into this evaluation's forms launch; forms (optional): the forms
// were launched by the caller into these buffers (no forms launch here); ride (optional, with forms): the next
// evaluation's forms, split over this evaluation's hidden-layer launches
// post (optional): the stage combination that follows this evaluation; *post_done tells whether the read-out launch
// took it (else the caller launches it)
int generic_vf_eval(const GncdeProblem& p, const float* t, const float* y, float* dy, char* ws,
                    hipStream_t st, bool prepared = false, unsigned* bars = nullptr, float* keep = nullptr,
                    bool need_dy = true, const PendingCombo* pending = nullptr, const FormBufs* forms = nullptr,
                    const FormsRide* ride = nullptr, const PendingCombo* post = nullptr, bool* post_done = nullptr);
// the workspace's fault word (a one-launch evaluation's barrier gave up): solver status 4 when set
const int* generic_vf_fault(const GncdeProblem& p, char* ws);

// one-launch evaluation for one hidden width and n <= 256 (configs 3 / 5): gncde_rows.hip
bool rows_supported(const GncdeProblem& p);
// coefficients stored as bfloat16 (GNCDE_COMPUTE_BF16_STORAGE, GNCDE_COMPUTE_BF16_MFMA)
inline bool coef_is_bf16(const GncdeProblem& p) {
  return p.compute == GNCDE_COMPUTE_BF16_STORAGE || p.compute == GNCDE_COMPUTE_BF16_MFMA;
}
// The one-launch evaluation's synchronisation words: one 128-byte line per group's arrival counter (the groups'
// atomics and polls never share a line), then the fault word and the start-order ticket.
constexpr int kBarStride = 32;
// [B] arrival counter lines, [B] group mailbox lines (the persistent solve's sample queue), then the fault word, the
// ticket counter and the sample queue counter
inline size_t rows_sync_words(int B) { return (size_t)2 * B * kBarStride + 64; }
inline size_t rows_fault_word(int B) { return (size_t)2 * B * kBarStride; }
int rows_vf_eval(const GncdeProblem& p, const float* t, const float* y, float* dy, const float* csum, const void* coefT,
                 const float* wperm, const uint16_t* wbf, const float* bf, float* z0, float* z1, unsigned* bar, int* fault,
                 unsigned& bars_done, hipStream_t st, float* keep = nullptr);
// an evaluation of this problem runs on k_rows: group barriers, a fault word
bool rows_eval_used(const GncdeProblem& p);
int generic_integrate(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys,
                      int32_t* stats, char* ws, hipStream_t st);
// k_coef_sums' per-plane reductions in a prepared evaluation workspace
const float* generic_vf_csum(const GncdeProblem& p, char* ws);
// the transposed coefficient planes of the one-launch evaluation: generic_vf_prepare fills them when
// rows_supported(p) (or for the persistent solve's rows layout)
void generic_vf_transpose(const GncdeProblem& p, char* ws, hipStream_t st);

// reverse mode of one evaluation, one launch per ConvLayer (n <= 256, one width H): gncde_rows_vjp.hip
bool rows_vjp_supported(const GncdeProblem& p);
size_t rows_vjp_workspace(const GncdeProblem& p);
void rows_vjp_begin(const GncdeProblem& p, char* ws, hipStream_t st);
// The step sweep's per-stage scatter of the stage input's cotangent v: gy += v, gk[j] += h a[j] v (h per sample).
struct StageScatter {
  float* gy;
  const float* hcur;
  float* gk[8];
  float a[8];
  int n;
};
// kept (optional): the stage's hidden outputs [L-1, B, n, H] from the forward's activation record (GncdeSolver.act_rec);
// without it the evaluation's forward runs first in keep mode.  scat (optional): the layer-0 launch applies that
// scatter to the stage input's cotangent instead of writing it to gu (one launch per stage fewer, same arithmetic)
int rows_vf_vjp(const GncdeProblem& p, const float* t, const float* u, const float* gF, float* gu, float* gdata,
                const float* csum, const float* wf, const float* bfold, char* ws, char* vf_ws, unsigned* bars,
                hipStream_t st, const float* kept = nullptr, const StageScatter* scat = nullptr);
void rows_vjp_finish(const GncdeProblem& p, char* ws, float* gparams, float* gfusion, hipStream_t st);

// the persistent solve on the one-launch evaluation (gncde_rows.hip): n <= 256, one width; Tsit5 + PIDController
// or a fixed grid (GRID controller)
bool rows_pid_supported(const GncdeProblem& p, const GncdeSolver& s);
bool rows_solve_shape(const GncdeProblem& p);  // the shape part of rows_pid_supported
size_t rows_pid_scratch(const GncdeProblem& p);
// sync: the evaluation workspace's [B] arrival counters, fault word and ticket counter (zeroed by generic_vf_prepare)
int rows_integrate_pid(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys, int32_t* stats,
                       char* vf_ws, float* part, const float* csum, const void* coefT, const float* wperm,
                       const float* bf, float* z0, float* z1, unsigned* sync, unsigned* zgran, hipStream_t st);
void rows_pid_name(const GncdeProblem& p, const GncdeSolver& s, char* buf, size_t len);
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel, size) for launches above 64 KB of LDS
bool ensure_dyn_lds(const void* fn, size_t smem);
// compute units of the current device (cached per device; 0 when the query fails)
int device_cu_count();
// the persistent solve hands off through tagged granules (GNCDE_SOLVE_GRANULES=1) instead of counter barriers
bool rows_solve_granules();
// a one-launch evaluation's group barrier gave up in this call: GNCDE_ERR_BARRIER (reads the workspace's fault word
// back, one stream synchronisation; GNCDE_OK without one-launch evaluations)
int rows_fault_status(const GncdeProblem& p, char* vf_ws, hipStream_t st, bool ran_rows);

// generic Tsit5 + PIDController (any shape, CDE wrapper): gncde_pid.hip
size_t generic_pid_workspace(const GncdeProblem& p);
int generic_integrate_pid(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys, int32_t* stats,
                          char* ws, hipStream_t st);
// reverse mode (discrete adjoint, GRID controller): gncde_vjp.hip
size_t generic_vjp_workspace(const GncdeProblem& p, const GncdeSolver& s);
// gstage (optional): [B, G-1, S, E] cotangents added to the stage values (gncde_integrate_vjp_ex)
int generic_integrate_vjp(const GncdeProblem& p, const GncdeSolver& s, const float* ys, const float* gys,
                          const float* gstage, float* gy0, float* gparams, float* gfusion, float* gdata, char* ws,
                          hipStream_t st);

// fused per-stage reverse sweep (H = 16, n <= 128, ODE): gncde_stage.hip
bool stage_vjp_supported(const GncdeProblem& p, const GncdeSolver& s);
size_t stage_vjp_workspace(const GncdeProblem& p);
int stage_integrate_vjp(const GncdeProblem& p, const GncdeSolver& s, const float* ys, const float* gys,
                        const float* gstage, float* gy0, float* gparams, float* gfusion, char* ws, hipStream_t st);

// fused persistent path: gncde_fused.hip.  Returns GNCDE_ERR_UNSUPPORTED when no kernel fits.
bool fused_supported(const GncdeProblem& p, const GncdeSolver& s, char* name, size_t name_len);
int fused_integrate(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys,
                    int32_t* stats, hipStream_t st);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace gncde
