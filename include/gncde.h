/*
 * gncde.h — C-ABI of the MI355X-native GNCDE integration engine (libgncde_hip.so, gfx950).
 *
 * This is the drop-in boundary for the reference's hot path.  The reference is
 * pure JAX; the calls these entry points replace are:
 *
 *   gncde_vf_eval     <- PermEquivGraphVectorField.__call__(t, y, args)
 *                        src/models/vector_fields/perm_equiv_graph_vector_field.py:85-129
 *                        (+ GraphVectorField.__call__ graph_vector_field.py:80-115,
 *                           PermEquivDirGraphVectorField.__call__ perm_equiv_dir_graph_vector_field.py:86-130,
 *                           CDEWrapperVectorField.__call__ cde_wrapper_vector_field.py:19-26),
 *                        batched over the jax.vmap axis of src/configs/loss_configs.py:44.
 *   gncde_integrate   <- diffrax.diffeqsolve(ODETerm(vf), Tsit5(), t0, t1, dt0, y0, args=spline,
 *                                            stepsize_controller, saveat)
 *                        src/models/graph_neural_cde.py:94-104 (PIDController(1e-3,1e-6), dt0=None),
 *                        src/models/pgt_graph_neural_cde.py:119-129 (ConstantStepSize, dt0=0.1),
 *                        src/models/tgb_graph_neural_cde.py:152-162 (ConstantStepSize, dt0=0.01),
 *                        plus fixed-step RK4 (build extension, BASELINE.json configs[1]).
 *   gncde_node_affine <- jax.vmap(eqx.nn.Linear) per node: graph_neural_cde.py:87 (initial_linear),
 *                        :106-109 (final_linear).
 *   gncde_interval_index <- diffrax CubicInterpolation interval rule (searchsorted, 'left') used at
 *                        perm_equiv_graph_vector_field.py:98-102 — exported so the index can be
 *                        checked bit-exactly.
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer (hipMalloc / torch cuda tensor), fp32 unless stated,
 *     contiguous row-major.  The caller owns all memory; the library never allocates or frees
 *     caller memory.  Scratch comes from a caller-allocated workspace of gncde_workspace_bytes().
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).  All work is enqueued
 *     asynchronously on it; no entry point synchronises the device, so calls are graph-capturable.
 *   - Return value 0 = success, otherwise a GNCDE_ERR_* code; gncde_strerror() describes it.
 *     No C++ exception crosses this boundary.  Per-sample solver failures (max_steps exceeded,
 *     non-finite state) are reported in the stats array, not as a return code.
 *   - Reentrant and thread-safe for distinct streams/workspaces.  No global mutable state.
 *
 * Data layout in HBM (one GPU holds its shard of the batch):
 *   ts        [B, T]               knot times per sample (increasing)
 *   coef      [B, T-1, 4, n, n]    operator-channel spline coefficients in diffrax tuple order
 *                                  (d, c, b, a) — i.e. the reference's coeffs[q][..., 1], de-interleaved
 *   tcoef     [B, T-1, 3, n]       column means over rows of the time-channel coefficients (d, c, b)[..., 0];
 *                                  tg(t)[i] = tb + f*(2*tc + 3*f*td) == jnp.mean(derivative(t)[...,0], axis=0)
 *   data_coef [B, T-1, 4, n, de, 2] CDE data spline (d, c, b, a) (CDE wrapper only, else NULL)
 *   fusion    [L, GNCDE_FC]        factored fusion table (see GNCDE_FC_* below), one row per layer
 *   params    per layer l, packed back to back: rms_w[d_l], rms_b[d_l], W[d_{l+1}, d_l], b[d_{l+1}]
 *   y / y0    [B, n, d_0] state (node-major, like the reference's y [n, h])
 */
#ifndef GNCDE_H
#define GNCDE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNCDE_ABI_VERSION 8
#define GNCDE_MAX_LAYERS 8
#define GNCDE_FC 24

/* Fusion table columns.  For layer l:
 *   (I + Abar) = e_A*A + e_dA*dA + eT_A*A^T + eT_dA*dA^T + diag(u) + w 1^T + 1 v^T
 *   u_i = idc + uD_A*A_ii + uD_dA*dA_ii + uR_A*r_i + uR_dA*rd_i + uC_A*c_i + uC_dA*cd_i + uS_A*s + uS_dA*sd
 *   w_i = wR_A*r_i + wR_dA*rd_i + wC_A*c_i + wC_dA*cd_i + wS_A*s + wS_dA*sd
 *   v_k = vR_A*r_k + vR_dA*rd_k + vC_A*c_k + vC_dA*cd_k
 * r/c = row/column sums, s = total sum (of A; "d" = of dA).  Mapping from the reference's
 * param1..param8 (+ *_prime) is documented in DESIGN.md §3 and layers.py:102-160 / :256-337.
 */
enum {
  GNCDE_FC_E_A = 0, GNCDE_FC_E_DA = 1, GNCDE_FC_ET_A = 2, GNCDE_FC_ET_DA = 3,
  GNCDE_FC_UD_A = 4, GNCDE_FC_UD_DA = 5, GNCDE_FC_UR_A = 6, GNCDE_FC_UR_DA = 7,
  GNCDE_FC_UC_A = 8, GNCDE_FC_UC_DA = 9, GNCDE_FC_US_A = 10, GNCDE_FC_US_DA = 11,
  GNCDE_FC_WR_A = 12, GNCDE_FC_WR_DA = 13, GNCDE_FC_WC_A = 14, GNCDE_FC_WC_DA = 15,
  GNCDE_FC_WS_A = 16, GNCDE_FC_WS_DA = 17,
  GNCDE_FC_VR_A = 18, GNCDE_FC_VR_DA = 19, GNCDE_FC_VC_A = 20, GNCDE_FC_VC_DA = 21,
  GNCDE_FC_IDC = 22
};

enum {
  GNCDE_OK = 0,
  GNCDE_ERR_ARG = 1,          /* NULL pointer / negative size */
  GNCDE_ERR_SHAPE = 2,        /* inconsistent dims (e.g. CDE width != h*de*2) */
  GNCDE_ERR_UNSUPPORTED = 3,  /* configuration outside what any kernel implements */
  GNCDE_ERR_WORKSPACE = 4,    /* workspace smaller than gncde_workspace_bytes() */
  GNCDE_ERR_HIP = 5,          /* a HIP runtime call failed (launch error) */
  GNCDE_ERR_BARRIER = 6       /* a one-launch evaluation's group barrier gave up: the results are invalid (see
                                 gncde_integrate) */
};

enum { GNCDE_RK4 = 0, GNCDE_TSIT5 = 1 };
/* Arithmetic of the n x n stream (BASELINE config 5, "bf16 MFMA path").
 *   FP32:         everything fp32 (the reference's arithmetic).
 *   BF16:         the n x n products (I + Abar_l) Z run on v_mfma_f32_16x16x32_bf16 with both operands split into
 *                 bf16 (hi, lo) pairs (three products, fp32 accumulation, ~2^-16 relative: fp32-class results and
 *                 no rounding noise for the adaptive controller).  Inputs stay fp32.
 *   BF16_STORAGE: `coef` holds bfloat16 values (same shape, uint16 storage): the operator spline's input is
 *                 quantised to bf16, halving the dominant HBM stream.  On the persistent solve (gncde_rows.hip, PREC
 *                 2: configs 5's shapes) every product stays fp32 on the exactly widened values, so its results are
 *                 BITWISE the fp32 solve of the bf16-rounded coefficients; on the multi-kernel path the products
 *                 are BF16's split pairs.
 *   BF16_MFMA:    (retired, round 6) single-plane bf16 operands for every product.  It lives only in an experiment
 *                 build (`make experiment`, GNCDE_EXPERIMENT_BF16_MFMA): 8-15 % from fp32 on a fixed grid, 12-21x
 *                 the steps under the PID controller, and no BASELINE config uses it.  The product library returns
 *                 GNCDE_ERR_UNSUPPORTED for it.
 * Splines, reductions, RMSNorm, solver and epilogues stay fp32.  The bf16 modes always take the generic path.
 * Their reverse mode (gncde_integrate_vjp*) is the fp32 discrete adjoint over the coefficients the forward read
 * (BF16_STORAGE: the bf16 planes widened exactly into the workspace head, which gncde_vjp_workspace_bytes
 * includes): the gradient of the bf16 solve to its own ~2^-16 product rounding. */
enum { GNCDE_COMPUTE_FP32 = 0, GNCDE_COMPUTE_BF16 = 1, GNCDE_COMPUTE_BF16_STORAGE = 2, GNCDE_COMPUTE_BF16_MFMA = 3 };
enum { GNCDE_CTRL_GRID = 0, GNCDE_CTRL_PID = 1 };
enum { GNCDE_SAVE_T1 = 0, GNCDE_SAVE_STEPS = 1, GNCDE_SAVE_TS = 2 };
/* GncdeSolver.flags.  GNCDE_FLAG_GENERIC: take the generic multi-kernel path in gncde_integrate AND the generic
 * reverse sweep in gncde_integrate_vjp*, even where the fused kernels fit.  The two paths compute the same discrete
 * solve (and its adjoint) with different fp32 summation orders; the flag exists so that callers and tests can check
 * one against the other on identical inputs (e.g. the same recorded PID step grid). */
enum { GNCDE_FLAG_GENERIC = 1 };
/* stats[b*4 + k]: k=0 accepted steps, 1 rejected steps, 2 vector-field evaluations, 3 status
 * (0 ok, 1 max_steps exceeded, 2 non-finite error estimate, 3 step record (step_ts) too short, 4 internal: a
 * one-launch evaluation's workgroups did not all become resident, so its barrier gave up and the results are invalid) */
enum { GNCDE_STAT_STEPS = 0, GNCDE_STAT_REJECTS = 1, GNCDE_STAT_EVALS = 2, GNCDE_STAT_STATUS = 3 };

typedef struct GncdeProblem {
  int32_t B;                         /* samples in this call (this rank's shard) */
  int32_t n;                         /* nodes */
  int32_t T;                         /* knots per sample (>= 2) */
  int32_t L;                         /* layers (1..GNCDE_MAX_LAYERS) */
  int32_t dims[GNCDE_MAX_LAYERS + 1];/* d_0 .. d_L */
  int32_t cde_hidden;                /* 0: ODE vector field (output [n, d_L]); >0: CDE wrapper h */
  int32_t cde_embed;                 /* CDE wrapper data_embed_dim de (d_L must equal h*de*2) */
  const float* ts;
  const float* coef;
  const float* tcoef;
  const float* data_coef;
  const float* fusion;
  const float* params;
  int32_t compute;                   /* GNCDE_COMPUTE_* (above) */
} GncdeProblem;

typedef struct GncdeSolver {
  int32_t method;                    /* GNCDE_RK4 | GNCDE_TSIT5 */
  int32_t controller;                /* GNCDE_CTRL_GRID (host-planned grid) | GNCDE_CTRL_PID */
  int32_t save_mode;                 /* GNCDE_SAVE_T1 | GNCDE_SAVE_STEPS | GNCDE_SAVE_TS */
  int32_t max_steps;                 /* PID: accepted+rejected step cap (diffrax default 4096) */
  int32_t grid_len;                  /* G: columns of grid (GRID controller; max steps + 1) */
  int32_t n_save;                    /* S: columns of save_ts (SAVE_TS) */
  float rtol, atol;                  /* PID tolerances */
  const float* grid;                 /* [B, G] step grid (GRID controller) */
  const int32_t* nsteps;             /* [B] steps per sample (GRID controller) */
  const float* t0;                   /* [B] (PID) */
  const float* t1;                   /* [B] (PID) */
  const float* dt0;                  /* [B] (PID) initial step, or NULL for the Hairer heuristic */
  const float* save_ts;              /* [B, S] (SAVE_TS), increasing, within [t0, t1] */
  /* PID only, optional OUTPUT (NULL = not recorded): the accepted step sequence of every sample,
   * step_ts[b, 0] = t0 and step_ts[b, k] = the time reached by the k-th accepted step (k <= stats steps).  It is
   * the grid on which the reverse mode differentiates an adaptive solve (the controller's step sizes are treated
   * as constants, as RecursiveCheckpointAdjoint does through diffrax's while_loop).  A sample with more accepted
   * steps than step_ts_len - 1 gets status 3. */
  float* step_ts;                    /* [B, step_ts_len] */
  int32_t step_ts_len;
  /* GRID only, optional (NULL = not recorded / not used): the stage record, [B, G-1, S-1, n, d_s] with S = 4 (RK4)
   * or 6 (Tsit5): every step's stage inputs U_1 .. U_{S-1} (U_0 is the step's starting state, already in ys).
   * gncde_integrate WRITES it; gncde_integrate_vjp* READ it (the same forward's record), so the reverse sweep
   * evaluates no stage twice: with 288 GB of HBM per GPU the forward stores what the reverse would recompute.
   * Both forward paths (fused, generic) write it and both reverse sweeps (fused, generic, the _data variant)
   * read it; size it with gncde_stage_record_floats().  stage_rec_len is its row length in floats: when stage_rec
   * is set it must equal gncde_stage_record_floats() for this problem and solver (both the forward and the reverse
   * mode check it and return GNCDE_ERR_ARG otherwise), so a record sized for another grid, method or arithmetic is
   * refused instead of read out of bounds.  The caller must pass the reverse mode the record the same forward wrote
   * (the library cannot tell an unwritten buffer from a written one). */
  float* stage_rec;
  int64_t stage_rec_len;
  int32_t flags;                     /* GNCDE_FLAG_* (0 = default dispatch) */
  /* GRID only, optional (NULL = not recorded / recomputed; ABI 7): the activation record, [G-1, S, L-1, B, n, H] —
   * every stage evaluation's hidden-layer outputs Z_1 .. Z_{L-1} (S = 4 RK4 / 6 Tsit5 stages of every step), each
   * (step, stage) slab in the layout the per-layer reverse mode reads.  gncde_integrate WRITES it and
   * gncde_integrate_vjp* READ it instead of re-running every stage's forward (288 GB of HBM per GPU: the forward
   * keeps what the reverse would recompute).  Only where gncde_activation_record_floats() is nonzero (an fp32
   * multi-kernel forward whose reverse takes the per-layer kernels: BASELINE config 3's shape); act_rec_len must
   * equal it (else GNCDE_ERR_ARG).  Batch-major: a caller that shards the batch records per shard.
   * PID controller (ABI 8, see pid_ckpt below): the same slabs, written by the adaptive solve itself. */
  float* act_rec;
  int64_t act_rec_len;
  /* PID only, optional (ABI 8): the adaptive solve records its ACCEPTED steps for the reverse mode, so that no
   * forward has to be re-run over the accepted grid.  Slots k < rec_steps (R) hold, for the k-th accepted step:
   *   pid_ckpt  [B, R, n, d]                 its starting state y_k (slot ns: the final state),
   *   stage_rec [B, R, 5, n, d]              its stage inputs U_1 .. U_5 (stage_rec_len = R * 5 * n * d),
   *   act_rec   [R, 6, L-1, B, n, H]         the hidden outputs Z_1 .. Z_{L-1} of its six stage evaluations, stage 0
   *                                          being the FSAL evaluation of step k - 1 (act_rec_len = R*6*(L-1)*B*n*H).
   * A rejected attempt writes the slots of the step it tried and its retry overwrites them.  A sample is recorded
   * completely iff its accepted steps + 1 <= R; otherwise the caller replays its accepted grid (step_ts).  The
   * layouts are the GRID records' with G - 1 = R (act_rec's leading dimension only), so the fixed-grid reverse
   * sweep reads them directly.  Only the persistent solve writes them (gncde_stage_record_floats /
   * gncde_activation_record_floats return 0 for any other PID path); all three or none. */
  float* pid_ckpt;
  int32_t rec_steps;
} GncdeSolver;

/* Library / error helpers */
int gncde_abi_version(void);
const char* gncde_strerror(int code);
/* Build provenance: lowercase hex sha256 of the kernel sources this library was compiled from (the bytes of the
 * sorted .hip and .h files of csrc, then this header, concatenated).  The Python binding refuses a library whose
 * sha differs from the source tree's, so a stale prebuilt binary cannot stand in for the tree's kernels. */
const char* gncde_source_sha256(void);
/* Name of the kernel path gncde_integrate would take for this problem ("fused<64,16,3,rk4>" or
 * "generic"), written into buf (NUL-terminated).  Returns GNCDE_OK or an error code. */
int gncde_integrate_path(const GncdeProblem* prob, const GncdeSolver* solver, char* buf, size_t buf_len);

/* Floats per sample of the stage record (GncdeSolver.stage_rec) for this problem and solver: (G-1)*(S-1)*n*d_s for
 * an fp32 GRID solve with G >= 2, else 0 (PID controller: its reverse mode replays the accepted steps as a GRID
 * solve, which takes the record; bf16 modes: their reverse sweep recomputes the stages, no record).  Never fails; 0 for invalid arguments. */
size_t gncde_stage_record_floats(const GncdeProblem* prob, const GncdeSolver* solver);

/* Floats of the activation record (GncdeSolver.act_rec, the whole batch) for this problem and solver:
 * (G-1)*S*(L-1)*B*n*H where the forward takes the multi-kernel fixed-grid path and the reverse the per-layer
 * kernels, else 0 (no record is written or read).  Never fails; 0 for invalid arguments.  (ABI 7) */
size_t gncde_activation_record_floats(const GncdeProblem* prob, const GncdeSolver* solver);

/* Workspace bytes needed by gncde_vf_eval (solver == NULL) or gncde_integrate. */
size_t gncde_workspace_bytes(const GncdeProblem* prob, const GncdeSolver* solver);

/* dy[b] = VF(t[b], y[b]) for every sample.  t: [B], y: [B, n, d_0], dy: [B, n, d_out] with
 * d_out = d_L (ODE) or cde_hidden (CDE wrapper). */
int gncde_vf_eval(const GncdeProblem* prob, const float* t, const float* y, float* dy,
                  void* workspace, size_t workspace_bytes, void* stream);

/* Solve dy/dt = VF(t, y) per sample.  y0: [B, n, d_s] (d_s = d_0).  ys:
 *   SAVE_T1: [B, n, d_s]; SAVE_STEPS: [B, G, n, d_s] (GRID controller); SAVE_TS: [B, S, n, d_s].
 * stats: [B, 4] int32 (may be NULL). */
int gncde_integrate(const GncdeProblem* prob, const GncdeSolver* solver, const float* y0, float* ys,
                    int32_t* stats, void* workspace, size_t workspace_bytes, void* stream);

/* Reverse mode of gncde_integrate for the GRID controller (the discrete adjoint that
 * jax.value_and_grad through diffrax.diffeqsolve's RecursiveCheckpointAdjoint computes:
 * trainer.py:315 over graph_neural_cde.py:94-104 / pgt_graph_neural_cde.py:84-93).
 *   ys:  [B, G, n, d_s] the forward's SAVE_STEPS states (the checkpoints; y_0 .. y_G-1)
 *   gys: cotangents of the forward's outputs in solver->save_mode layout: SAVE_T1 [B, n, d_s] (cotangent
 *        of the final state) or SAVE_STEPS [B, G, n, d_s]
 *   gy0:     [B, n, d_s]  cotangent of y0
 *   gparams: [P]          sum over samples of the cotangent of prob->params (packed layout above)
 *   gfusion: [L, GNCDE_FC] sum over samples of the cotangent of the fusion table
 * Deterministic (fixed reduction order, no atomics).  Workspace: gncde_vjp_workspace_bytes. */
size_t gncde_vjp_workspace_bytes(const GncdeProblem* prob, const GncdeSolver* solver);
int gncde_integrate_vjp(const GncdeProblem* prob, const GncdeSolver* solver, const float* ys, const float* gys,
                        float* gy0, float* gparams, float* gfusion, void* workspace, size_t workspace_bytes,
                        void* stream);

/* gncde_integrate_vjp plus the cotangent of the CDE wrapper's data spline (CDE problems only): gdata_coef has the
 * layout of prob->data_coef, [B, T-1, 4, n, de, 2]; the 'a' rows are zero (the wrapper reads dX/dt only,
 * cde_wrapper_vector_field.py:25).  Chained with gncde_hermite_coefficients_vjp it gives the gradient of the
 * data embedding that TGBGraphNeuralCDE rebuilds inside every forward (tgb_graph_neural_cde.py:118-130).
 * Always takes the generic reverse sweep. */
int gncde_integrate_vjp_data(const GncdeProblem* prob, const GncdeSolver* solver, const float* ys, const float* gys,
                             float* gy0, float* gparams, float* gfusion, float* gdata_coef, void* workspace,
                             size_t workspace_bytes, void* stream);

/* gncde_integrate_vjp with two optional extras (NULL = absent):
 *   gstage:     [B, G-1, S, n, d_s], S = 4 (RK4) or 6 (Tsit5): cotangents added to the stage VALUES of each step,
 *               K_j = VF(t_k + c_j h_k, U_j).  This is the reverse mode of output maps that read the stages, above all
 *               the Tsit5 dense interpolant of SaveAt(ts) (graph_neural_cde.py:89-104): y(t_k + th h_k) =
 *               y_k + h_k sum_j b_j(th) K_j, where K_6 (the FSAL value f(t_{k+1}, y_{k+1})) is stage 0 of step k+1 --
 *               so a caller whose last step's K_6 carries a cotangent leaves one padded step (nsteps < G-1) and puts
 *               it on stage 0 of step nsteps.
 *   gdata_coef: the CDE data spline's cotangent, as gncde_integrate_vjp_data. */
int gncde_integrate_vjp_ex(const GncdeProblem* prob, const GncdeSolver* solver, const float* ys, const float* gys,
                           const float* gstage, float* gy0, float* gparams, float* gfusion, float* gdata_coef,
                           void* workspace, size_t workspace_bytes, void* stream);

/* Per-node affine map out[r, :] = W @ x[r, :] + b for `rows` rows.  x: [rows, din], W: [dout, din],
 * b: [dout] (may be NULL), out: [rows, dout]. */
int gncde_node_affine(int32_t rows, int32_t din, int32_t dout, const float* x, const float* W,
                      const float* b, float* out, void* stream);

/* Reverse mode of gncde_node_affine (encoders / read-outs, graph_neural_cde.py:87,106-111):
 *   gx[r, :] = W^T g[r, :]  (gx may be NULL);  gW = sum_r g[r]^T x[r]  (may be NULL);  gb = sum_r g[r]  (may be NULL).
 * g: [rows, dout].  Deterministic. */
int gncde_node_affine_grad(int32_t rows, int32_t din, int32_t dout, const float* x, const float* W,
                           const float* g, float* gx, float* gW, float* gb, void* stream);

/* One optimiser update over a flat fp32 parameter buffer: optax.chain(clip_by_global_norm(max_norm),
 * adamw(lr, b1, b2, eps, weight_decay)) as built by optimiser_configs.py:70-88 (max_norm <= 0: no clipping).
 * step is the 1-based update count (bias correction).  stats[3] (device): global grad norm, max|grad|,
 * max|update| (the values trainer.py:318-326 logs).  Workspace: gncde_adamw_workspace_bytes(P). */
size_t gncde_adamw_workspace_bytes(int32_t P);
int gncde_clip_adamw(int32_t P, float* params, const float* grads, float* m, float* v, int32_t step, float lr,
                     float b1, float b2, float eps, float weight_decay, float max_norm, float* stats,
                     void* workspace, size_t workspace_bytes, void* stream);

/* ---- input side ------------------------------------------------------------------------------ */
/* Graph operators of misc.py:58-113 (get_graph_operator), per graph, fp32:
 *   NORM_LAP        I - D_out^-1/2 (A + I) D_in^-1/2, degrees of A + I   (default, misc.py:83-99)
 *   NORM_ADJ, KIPF  D_out^-1/2 (A + I) D_in^-1/2, degrees of A + I        (misc.py:101-113, zipf_smoothing :16-33)
 *   NORMALIZED_PLUS D_out^-1/2 (A + I) D_in^-1/2, degrees of A (0 -> 0)   (misc.py:36-57)
 * A, out: [graphs, n, n]; workspace: 2 * graphs * n floats (device). */
enum { GNCDE_OP_NORM_LAP = 0, GNCDE_OP_NORM_ADJ = 1, GNCDE_OP_KIPF = 2, GNCDE_OP_NORMALIZED_PLUS = 3 };
int gncde_graph_operator(int32_t kind, int32_t graphs, int32_t n, const float* A, float* out, float* workspace,
                         void* stream);

/* diffrax.backward_hermite_coefficients over knots ts [B, T] of X [B, T, C] (any channel count C), written in
 * the engine layout out [B, T-1, ncoef, C] with (d, c, b, a) order; ncoef = 4, or 3 to drop a (the tcoef
 * layout).  dataset_configs.py:170, tgb_graph_neural_cde.py:130. */
int gncde_hermite_coefficients(int32_t B, int32_t T, int32_t C, int32_t ncoef, const float* ts, const float* X,
                               float* out, void* stream);

/* Reverse mode of gncde_hermite_coefficients with respect to X (the knots ts are data): gX [B, T, C] from
 * gout [B, T-1, ncoef, C].  Overwrites gX. */
int gncde_hermite_coefficients_vjp(int32_t B, int32_t T, int32_t C, int32_t ncoef, const float* ts,
                                   const float* gout, float* gX, void* stream);

/* idx[k] = clip(searchsorted(ts[b], t[k], 'left') - 1, 0, T-2) with b = sample[k].
 * ts: [B, T], t: [count], sample: [count] int32, idx: [count] int32. */
int gncde_interval_index(const float* ts, int32_t B, int32_t T, const float* t, const int32_t* sample,
                         int32_t* idx, int32_t count, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNCDE_H */
