// extern "C" entry points of libgncde_hip.so (declared in include/gncde.h).
//
// Host-side validation and dispatch only: the fused persistent kernel (gncde_fused.hip) when the
// problem fits it, the generic multi-kernel path (gncde_generic.hip) otherwise.  There is no CPU
// fallback: every entry point enqueues HIP work or returns an error code.
#include <cstdio>
#include <cstring>

#include "gncde_internal.h"

namespace gncde {

int validate_problem(const GncdeProblem* p) {
  if (!p) return GNCDE_ERR_ARG;
  if (p->B < 0 || p->n <= 0 || p->T < 2 || p->L < 1 || p->L > GNCDE_MAX_LAYERS) return GNCDE_ERR_SHAPE;
  for (int l = 0; l <= p->L; ++l)
    if (p->dims[l] <= 0) return GNCDE_ERR_SHAPE;
  // (an empty shard may pass NULL data pointers: torch gives empty tensors a null data_ptr)
  if (p->B > 0 && (!p->ts || !p->coef || !p->tcoef)) return GNCDE_ERR_ARG;
  if (!p->fusion || !p->params) return GNCDE_ERR_ARG;
  if (p->compute < GNCDE_COMPUTE_FP32 || p->compute > GNCDE_COMPUTE_BF16_MFMA) return GNCDE_ERR_ARG;
  if (p->cde_hidden > 0) {
    if (p->cde_embed <= 0 || (p->B > 0 && !p->data_coef)) return GNCDE_ERR_ARG;
    if (p->dims[p->L] != p->cde_hidden * p->cde_embed * 2) return GNCDE_ERR_SHAPE;
    if (p->dims[0] != p->cde_hidden) return GNCDE_ERR_SHAPE;
  } else if (p->cde_hidden < 0) {
    return GNCDE_ERR_SHAPE;
  }
  // the single-plane bf16 mode exists only in the one-launch evaluation, and only in an experiment build
  // (GNCDE_EXPERIMENT_BF16_MFMA, `make experiment`): the product library refuses it
#ifdef GNCDE_EXPERIMENT_BF16_MFMA
  if (p->compute == GNCDE_COMPUTE_BF16_MFMA && !rows_supported(*p)) return GNCDE_ERR_UNSUPPORTED;
#else
  if (p->compute == GNCDE_COMPUTE_BF16_MFMA) return GNCDE_ERR_UNSUPPORTED;
#endif
  return GNCDE_OK;
}

bool use_fused(const GncdeProblem& p, const GncdeSolver& s, char* name, size_t len);
bool use_stage_vjp(const GncdeProblem& p, const GncdeSolver& s);

// The persistent adaptive solve records its accepted steps (ABI 8, gncde.h pid_ckpt): Tsit5 on the persistent path
// (fp32, or bf16 coefficient storage: its products are fp32), at least one hidden layer, and a reverse mode that
// takes the per-layer kernels (which read the activation slabs)
bool pid_record_supported(const GncdeProblem& p, const GncdeSolver& s) {
  if (s.controller != GNCDE_CTRL_PID || s.rec_steps < 1 || p.L < 2 || s.method != GNCDE_TSIT5) return false;
  if (p.compute != GNCDE_COMPUTE_FP32 && p.compute != GNCDE_COMPUTE_BF16_STORAGE) return false;
  GncdeProblem q = p;
  q.compute = GNCDE_COMPUTE_FP32;
  return !use_fused(p, s, nullptr, 0) && rows_pid_supported(p, s) && rows_vjp_supported(q);
}

// Floats per sample of the stage record an fp32 GRID solve writes and its reverse sweep reads (gncde.h); under the
// PID controller, the persistent solve's record of its accepted steps (R slots of 5 stage inputs).
size_t record_floats(const GncdeProblem& p, const GncdeSolver& s) {
  if (pid_record_supported(p, s)) return (size_t)s.rec_steps * 5 * (size_t)p.n * (size_t)p.dims[0];
  if (s.controller != GNCDE_CTRL_GRID || p.compute != GNCDE_COMPUTE_FP32 || s.grid_len < 2) return 0;
  const size_t S = s.method == GNCDE_RK4 ? 4 : 6;
  return (size_t)(s.grid_len - 1) * (S - 1) * (size_t)p.n * (size_t)p.dims[0];
}

// Floats of the activation record (gncde.h): the multi-kernel fixed-grid forward (not the fused kernel, not the
// persistent solve) whose reverse sweep takes the per-layer kernels
size_t act_floats(const GncdeProblem& p, const GncdeSolver& s) {
  if (pid_record_supported(p, s))
    return (size_t)s.rec_steps * 6 * (size_t)(p.L - 1) * (size_t)p.B * (size_t)p.n * (size_t)p.dims[0];
  if (s.controller != GNCDE_CTRL_GRID || p.compute != GNCDE_COMPUTE_FP32 || s.grid_len < 2 || p.L < 2) return 0;
  if (use_fused(p, s, nullptr, 0) || use_stage_vjp(p, s) || rows_pid_supported(p, s) || !rows_vjp_supported(p))
    return 0;
  const size_t S = s.method == GNCDE_RK4 ? 4 : 6;
  return (size_t)(s.grid_len - 1) * S * (size_t)(p.L - 1) * (size_t)p.B * (size_t)p.n * (size_t)p.dims[0];
}

int validate_solver(const GncdeProblem* p, const GncdeSolver* s) {
  if (!s) return GNCDE_ERR_ARG;
  if (s->flags & ~GNCDE_FLAG_GENERIC) return GNCDE_ERR_ARG;
  if (s->method != GNCDE_RK4 && s->method != GNCDE_TSIT5) return GNCDE_ERR_ARG;
  if (s->save_mode < GNCDE_SAVE_T1 || s->save_mode > GNCDE_SAVE_TS) return GNCDE_ERR_ARG;
  if (p->cde_hidden == 0 && p->dims[0] != p->dims[p->L]) return GNCDE_ERR_SHAPE;  // ODE state width
  if (s->controller == GNCDE_CTRL_GRID) {
    if (!s->grid || !s->nsteps || s->grid_len < 1) return GNCDE_ERR_ARG;
    if (s->save_mode == GNCDE_SAVE_TS) return GNCDE_ERR_UNSUPPORTED;
    if (s->pid_ckpt) return GNCDE_ERR_ARG;
    // a record must be exactly the one this solve writes / its sweep reads (none exists for the bf16 modes)
    if (s->stage_rec && (s->stage_rec_len <= 0 || (size_t)s->stage_rec_len != record_floats(*p, *s)))
      return GNCDE_ERR_ARG;
    if (s->act_rec) {
      GncdeSolver q = *s;
      q.act_rec = nullptr;
      if (s->act_rec_len <= 0 || (size_t)s->act_rec_len != act_floats(*p, q)) return GNCDE_ERR_ARG;
    }
  } else if (s->controller == GNCDE_CTRL_PID) {
    if (s->act_rec || s->stage_rec || s->pid_ckpt) {  // the accepted-step record (ABI 8): all three, sized exactly
      if (!(s->act_rec && s->stage_rec && s->pid_ckpt) || s->rec_steps < 1) return GNCDE_ERR_ARG;
      GncdeSolver q = *s;
      q.act_rec = q.stage_rec = q.pid_ckpt = nullptr;
      const size_t sf = record_floats(*p, q), af = act_floats(*p, q);
      if (sf == 0 || af == 0) return GNCDE_ERR_UNSUPPORTED;
      if (s->stage_rec_len <= 0 || (size_t)s->stage_rec_len != sf || s->act_rec_len <= 0 ||
          (size_t)s->act_rec_len != af)
        return GNCDE_ERR_ARG;
    }
    // the single-plane bf16 mode puts ~1e-2 relative noise into every stage, which the embedded error estimate
    // reads as truncation error: at rtol 1e-3 the controller takes 12-21x the evaluations, so
    // the mode is for fixed grids (ConstantStepSize, the reference's own PGT / TGB solves) only
    if (p->compute == GNCDE_COMPUTE_BF16_MFMA) return GNCDE_ERR_UNSUPPORTED;
    if (!s->t0 || !s->t1 || s->max_steps < 1) return GNCDE_ERR_ARG;
    if (!(s->rtol >= 0.f) || !(s->atol > 0.f)) return GNCDE_ERR_ARG;
    if (s->save_mode == GNCDE_SAVE_STEPS) return GNCDE_ERR_UNSUPPORTED;
    if (s->save_mode == GNCDE_SAVE_TS && (!s->save_ts || s->n_save < 1)) return GNCDE_ERR_ARG;
    if (s->step_ts && s->step_ts_len < 1) return GNCDE_ERR_ARG;
  } else {
    return GNCDE_ERR_ARG;
  }
  return GNCDE_OK;
}

// ---- reverse mode of the bf16 modes ---------------------------------------------------------------------
// The bf16 modes' forward differs from the fp32 forward only in the n x n products, which run on split (hi, lo)
// bf16 pairs with fp32 accumulation (~2^-16 relative per product), and, for BF16_STORAGE, in reading the operator
// coefficients as bfloat16.  Their reverse mode is the fp32 discrete adjoint over the coefficients that forward
// read: the fp32 planes themselves (BF16), or the bf16 planes widened exactly into the head of the workspace
// (BF16_STORAGE).  It is the gradient of the bf16 solve to the forward's own product rounding.  BF16_MFMA (single-plane
// products, ~2^-8 per operand) gets the same fp32 adjoint over its widened coefficients, evaluated along the
// trajectory the bf16 forward saved: the gradient of the fp32 solve on the bf16 input, not of the bf16 rounding.
namespace {

__global__ void k_widen_bf16(size_t N, const uint16_t* __restrict__ in, float* __restrict__ out) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (size_t)gridDim.x * blockDim.x)
    out[e] = __builtin_bit_cast(float, (uint32_t)in[e] << 16);
}

size_t coef_floats(const GncdeProblem& p) { return (size_t)p.B * (p.T - 1) * 4 * (size_t)p.n * p.n; }

// the fp32 problem the reverse sweep runs on, and the workspace bytes it keeps in front for widened coefficients
GncdeProblem fp32_view(const GncdeProblem& p, size_t& head) {
  GncdeProblem q = p;
  q.compute = GNCDE_COMPUTE_FP32;
  head = coef_is_bf16(p) ? align_up(coef_floats(p) * sizeof(float), 256) : 0;
  return q;
}

}  // namespace

// GNCDE_FLAG_GENERIC forces the generic forward and the generic reverse sweep (gncde.h)
bool use_fused(const GncdeProblem& p, const GncdeSolver& s, char* name, size_t len) {
  return !(s.flags & GNCDE_FLAG_GENERIC) && fused_supported(p, s, name, len);
}
bool use_stage_vjp(const GncdeProblem& p, const GncdeSolver& s) {
  return !(s.flags & GNCDE_FLAG_GENERIC) && stage_vjp_supported(p, s);
}

}  // namespace gncde

using namespace gncde;

extern "C" {

int gncde_abi_version(void) { return GNCDE_ABI_VERSION; }

const char* gncde_strerror(int code) {
  switch (code) {
    case GNCDE_OK: return "ok";
    case GNCDE_ERR_ARG: return "invalid argument (NULL pointer or bad enum)";
    case GNCDE_ERR_SHAPE: return "inconsistent shapes/dims";
    case GNCDE_ERR_UNSUPPORTED: return "configuration not supported by any kernel";
    case GNCDE_ERR_WORKSPACE: return "workspace too small";
    case GNCDE_ERR_HIP: return "HIP runtime error";
    case GNCDE_ERR_BARRIER: return "a one-launch evaluation's group barrier gave up (results invalid)";
    default: return "unknown gncde error";
  }
}

size_t gncde_stage_record_floats(const GncdeProblem* prob, const GncdeSolver* solver) {
  if (validate_problem(prob) != GNCDE_OK || !solver) return 0;
  GncdeSolver s = *solver;  // the records themselves are not part of the question
  s.stage_rec = nullptr;
  s.act_rec = nullptr;
  s.pid_ckpt = nullptr;
  if (validate_solver(prob, &s) != GNCDE_OK) return 0;
  return record_floats(*prob, s);
}

size_t gncde_activation_record_floats(const GncdeProblem* prob, const GncdeSolver* solver) {
  if (validate_problem(prob) != GNCDE_OK || !solver) return 0;
  GncdeSolver s = *solver;  // the records themselves are not part of the question
  s.stage_rec = nullptr;
  s.act_rec = nullptr;
  s.pid_ckpt = nullptr;
  if (validate_solver(prob, &s) != GNCDE_OK) return 0;
  return act_floats(*prob, s);
}

size_t gncde_workspace_bytes(const GncdeProblem* prob, const GncdeSolver* solver) {
  if (validate_problem(prob) != GNCDE_OK) return 0;
  if (!solver) return generic_vf_workspace(*prob);
  if (use_fused(*prob, *solver, nullptr, 0)) return 0;
  return generic_integrate_workspace(*prob, *solver);
}

int gncde_integrate_path(const GncdeProblem* prob, const GncdeSolver* solver, char* buf, size_t buf_len) {
  int rc = validate_problem(prob);
  if (rc) return rc;
  rc = validate_solver(prob, solver);
  if (rc) return rc;
  if (!buf || buf_len == 0) return GNCDE_ERR_ARG;
  if (use_fused(*prob, *solver, buf, buf_len)) return GNCDE_OK;
  if (rows_pid_supported(*prob, *solver))
    rows_pid_name(*prob, *solver, buf, buf_len);
  else if (prob->compute == GNCDE_COMPUTE_FP32)  // generic_rows: every evaluation is one k_rows launch
    snprintf(buf, buf_len, rows_eval_used(*prob) ? "generic_rows" : "generic");
  else
    snprintf(buf, buf_len, prob->compute == GNCDE_COMPUTE_BF16_MFMA ? "rows_bf16" : "generic_bf16");
  return GNCDE_OK;
}

int gncde_vf_eval(const GncdeProblem* prob, const float* t, const float* y, float* dy, void* workspace,
                  size_t workspace_bytes, void* stream) {
  int rc = validate_problem(prob);
  if (rc) return rc;
  if (prob->B == 0) return GNCDE_OK;
  if (!t || !y || !dy) return GNCDE_ERR_ARG;
  if (workspace_bytes < generic_vf_workspace(*prob) || !workspace) return GNCDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int rc2 = generic_vf_eval(*prob, t, y, dy, static_cast<char*>(workspace), st);
  return rc2 ? rc2 : rows_fault_status(*prob, static_cast<char*>(workspace), st, rows_eval_used(*prob));
}

int gncde_integrate(const GncdeProblem* prob, const GncdeSolver* solver, const float* y0, float* ys,
                    int32_t* stats, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = validate_problem(prob);
  if (rc) return rc;
  rc = validate_solver(prob, solver);
  if (rc) return rc;
  if (prob->B == 0) return GNCDE_OK;
  if (!y0 || !ys) return GNCDE_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (use_fused(*prob, *solver, nullptr, 0)) return fused_integrate(*prob, *solver, y0, ys, stats, st);
  if (workspace_bytes < generic_integrate_workspace(*prob, *solver) || !workspace) return GNCDE_ERR_WORKSPACE;
  return generic_integrate(*prob, *solver, y0, ys, stats, static_cast<char*>(workspace), st);
}

size_t gncde_vjp_workspace_bytes(const GncdeProblem* prob, const GncdeSolver* solver) {
  if (validate_problem(prob) != GNCDE_OK || validate_solver(prob, solver) != GNCDE_OK) return 0;
  size_t head = 0;
  const GncdeProblem p = fp32_view(*prob, head);
  if (use_stage_vjp(p, *solver)) return head + stage_vjp_workspace(p);
  return head + generic_vjp_workspace(p, *solver);
}

static int integrate_vjp(const GncdeProblem* prob, const GncdeSolver* solver, const float* ys, const float* gys,
                         const float* gstage, float* gy0, float* gparams, float* gfusion, float* gdata, void* workspace,
                         size_t workspace_bytes, void* stream) {
  using namespace gncde;
  int rc = validate_problem(prob);
  if (rc) return rc;
  rc = validate_solver(prob, solver);
  if (rc) return rc;
  if (solver->controller != GNCDE_CTRL_GRID) return GNCDE_ERR_UNSUPPORTED;
  if (solver->save_mode != GNCDE_SAVE_T1 && solver->save_mode != GNCDE_SAVE_STEPS) return GNCDE_ERR_UNSUPPORTED;
  if (!gparams || !gfusion) return GNCDE_ERR_ARG;
  if (gdata && prob->cde_hidden <= 0) return GNCDE_ERR_ARG;  // only the CDE wrapper reads a data spline
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (prob->B == 0) {  // empty shard: zero gradients (an all-reduce still sees this rank's contribution)
    size_t P = params_floats(*prob);
    (void)hipMemsetAsync(gparams, 0, P * sizeof(float), st);
    (void)hipMemsetAsync(gfusion, 0, (size_t)prob->L * GNCDE_FC * sizeof(float), st);
    return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
  }
  if (!ys || !gys || !gy0) return GNCDE_ERR_ARG;
  size_t head = 0;
  GncdeProblem p = fp32_view(*prob, head);  // bf16 modes: the fp32 adjoint (see fp32_view)
  char* ws = static_cast<char*>(workspace);
  const bool stage = !gdata && use_stage_vjp(p, *solver);
  const size_t need = head + (stage ? stage_vjp_workspace(p) : generic_vjp_workspace(p, *solver));
  if (workspace_bytes < need || !workspace) return GNCDE_ERR_WORKSPACE;
  if (head) {
    float* wide = reinterpret_cast<float*>(ws);
    const size_t N = coef_floats(p);
    hipLaunchKernelGGL(k_widen_bf16, dim3((unsigned)((N + 255) / 256 < 65536 ? (N + 255) / 256 : 65536)), dim3(256), 0,
                       st, N, reinterpret_cast<const uint16_t*>(prob->coef), wide);
    p.coef = wide;
    ws += head;
  }
  if (stage) return stage_integrate_vjp(p, *solver, ys, gys, gstage, gy0, gparams, gfusion, ws, st);
  return generic_integrate_vjp(p, *solver, ys, gys, gstage, gy0, gparams, gfusion, gdata, ws, st);
}

int gncde_integrate_vjp(const GncdeProblem* prob, const GncdeSolver* solver, const float* ys, const float* gys,
                        float* gy0, float* gparams, float* gfusion, void* workspace, size_t workspace_bytes,
                        void* stream) {
  return integrate_vjp(prob, solver, ys, gys, nullptr, gy0, gparams, gfusion, nullptr, workspace, workspace_bytes,
                       stream);
}

int gncde_integrate_vjp_data(const GncdeProblem* prob, const GncdeSolver* solver, const float* ys, const float* gys,
                             float* gy0, float* gparams, float* gfusion, float* gdata_coef, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (!gdata_coef) return GNCDE_ERR_ARG;
  return integrate_vjp(prob, solver, ys, gys, nullptr, gy0, gparams, gfusion, gdata_coef, workspace, workspace_bytes,
                       stream);
}

int gncde_integrate_vjp_ex(const GncdeProblem* prob, const GncdeSolver* solver, const float* ys, const float* gys,
                           const float* gstage, float* gy0, float* gparams, float* gfusion, float* gdata_coef,
                           void* workspace, size_t workspace_bytes, void* stream) {
  return integrate_vjp(prob, solver, ys, gys, gstage, gy0, gparams, gfusion, gdata_coef, workspace, workspace_bytes,
                       stream);
}

}  // extern "C"

namespace {

__global__ void k_node_affine(int rows, int din, int dout, const float* __restrict__ x,
                              const float* __restrict__ W, const float* __restrict__ bias,
                              float* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)rows * dout) return;
  const size_t r = e / dout;
  const int o = (int)(e % dout);
  float acc = bias ? bias[o] : 0.f;
  const float* xr = x + r * din;
  const float* w = W + (size_t)o * din;
  for (int k = 0; k < din; ++k) acc = fmaf(w[k], xr[k], acc);
  out[e] = acc;
}

// gx[r, f] = sum_o g[r, o] W[o, f]
__global__ void k_affine_grad_x(int rows, int din, int dout, const float* __restrict__ W, const float* __restrict__ g,
                                float* __restrict__ gx) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)rows * din) return;
  const size_t r = e / din;
  const int f = (int)(e % din);
  const float* gr = g + r * dout;
  float acc = 0.f;
  for (int o = 0; o < dout; ++o) acc = fmaf(gr[o], W[(size_t)o * din + f], acc);
  gx[e] = acc;
}

// One block per weight entry (o, f) (f == din: the bias): gW[o, f] = sum_r g[r, o] x[r, f], gb[o] = sum_r g[r, o].
// Fixed strided partition + tree reduction: deterministic.
// One workgroup per weight / bias entry, summing over every node row.  1024 threads, each with four independent
// accumulators (rows t + 1024 (4 j + u)), so 8 loads per thread are in flight: the sum over B n rows (131 K at
// config 4) is a handful of memory round trips, not 128 dependent ones.  Fixed order (deterministic, no atomics).
__global__ void __launch_bounds__(1024) k_affine_grad_w(int rows, int din, int dout, const float* __restrict__ x,
                                                        const float* __restrict__ g, float* __restrict__ gW,
                                                        float* __restrict__ gb) {
  const int e = blockIdx.x;
  const int o = e / (din + 1), f = e % (din + 1);
  const bool bias = f == din;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int r = threadIdx.x;
  for (; r + 3 * 1024 < rows; r += 4 * 1024) {
    float gv[4], xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      gv[u] = g[(size_t)(r + u * 1024) * dout + o];
      xv[u] = bias ? 1.f : x[(size_t)(r + u * 1024) * din + f];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = fmaf(gv[u], xv[u], acc[u]);
  }
  for (int u = 0; r < rows; r += 1024, ++u) acc[u & 3] = fmaf(g[(size_t)r * dout + o], bias ? 1.f : x[(size_t)r * din + f], acc[u & 3]);
  float v = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  v = wave_sum64(v);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w];
    if (!bias) {
      if (gW) gW[(size_t)o * din + f] = t;
    } else if (gb) {
      gb[o] = t;
    }
  }
}

// optax.chain(clip_by_global_norm(max_norm), adamw(lr, b1, b2, eps, weight_decay)) over one flat buffer.
// Pass 1 (single block): global norm and max|g|.
__global__ void __launch_bounds__(1024) k_grad_norm(int P, const float* __restrict__ g, float* __restrict__ stats) {
  double ss = 0.0;
  float mx = 0.f;
  for (int e = threadIdx.x; e < P; e += blockDim.x) {
    const float v = g[e];
    ss += (double)v * v;
    mx = fmaxf(mx, fabsf(v));
  }
  __shared__ double rs[1024];
  __shared__ float rm[1024];
  rs[threadIdx.x] = ss;
  rm[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      rs[threadIdx.x] += rs[threadIdx.x + s];
      rm[threadIdx.x] = fmaxf(rm[threadIdx.x], rm[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[0] = (float)sqrt(rs[0]);
    stats[1] = rm[0];
    stats[2] = 0.f;
  }
}

// Pass 2: clip (optax: g if norm < max_norm else g / norm * max_norm), Adam moments with bias correction,
// decoupled weight decay (optax.adamw: u = -lr * (m_hat / (sqrt(v_hat) + eps) + wd * p)).
__global__ void k_adamw(int P, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                        float* __restrict__ v, float lr, float b1, float b2, float eps, float wd, float max_norm,
                        float bc1, float bc2, float* __restrict__ stats, float* __restrict__ upd_max) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  float u = 0.f;
  if (e < P) {
    const float norm = stats[0];
    float gv = g[e];
    if (max_norm > 0.f && !(norm < max_norm)) gv = gv / norm * max_norm;
    const float mn = b1 * m[e] + (1.f - b1) * gv;
    const float vn = b2 * v[e] + (1.f - b2) * gv * gv;
    m[e] = mn;
    v[e] = vn;
    const float mh = mn / bc1, vh = vn / bc2;
    u = -lr * (mh / (sqrtf(vh) + eps) + wd * p[e]);
    p[e] += u;
  }
  // per-block max |update| (reduced by the host-facing entry afterwards)
  __shared__ float red[256];
  red[threadIdx.x] = fabsf(u);
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) upd_max[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(1024) k_max_reduce(int nblk, const float* __restrict__ upd_max,
                                                     float* __restrict__ stats) {
  float mx = 0.f;
  for (int e = threadIdx.x; e < nblk; e += blockDim.x) mx = fmaxf(mx, upd_max[e]);
  __shared__ float red[1024];
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) stats[2] = red[0];
}

__global__ void k_interval_index(const float* __restrict__ ts, int B, int T, const float* __restrict__ t,
                                 const int32_t* __restrict__ sample, int32_t* __restrict__ idx, int count) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  int b = sample[e];
  b = b < 0 ? 0 : (b >= B ? B - 1 : b);
  idx[e] = interval_index(ts + (size_t)b * T, T, t[e]);
}

}  // namespace

extern "C" {

int gncde_node_affine(int32_t rows, int32_t din, int32_t dout, const float* x, const float* W,
                      const float* b, float* out, void* stream) {
  if (rows < 0 || din <= 0 || dout <= 0) return GNCDE_ERR_SHAPE;
  if (rows == 0) return GNCDE_OK;
  if (!x || !W || !out) return GNCDE_ERR_ARG;
  const size_t total = (size_t)rows * dout;
  hipLaunchKernelGGL(k_node_affine, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), rows, din, dout, x, W, b, out);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

int gncde_node_affine_grad(int32_t rows, int32_t din, int32_t dout, const float* x, const float* W,
                           const float* g, float* gx, float* gW, float* gb, void* stream) {
  if (rows < 0 || din <= 0 || dout <= 0) return GNCDE_ERR_SHAPE;
  if (!g || (gx && !W) || (gW && !x)) return GNCDE_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (gx && rows > 0) {
    const size_t total = (size_t)rows * din;
    hipLaunchKernelGGL(k_affine_grad_x, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, rows, din, dout, W,
                       g, gx);
  }
  if (gW || gb)
    hipLaunchKernelGGL(k_affine_grad_w, dim3((unsigned)(dout * (din + 1))), dim3(1024), 0, st, rows, din, dout, x, g,
                       gW, gb);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

size_t gncde_adamw_workspace_bytes(int32_t P) { return P <= 0 ? 0 : (size_t)((P + 255) / 256) * sizeof(float); }

int gncde_clip_adamw(int32_t P, float* params, const float* grads, float* m, float* v, int32_t step, float lr,
                     float b1, float b2, float eps, float weight_decay, float max_norm, float* stats,
                     void* workspace, size_t workspace_bytes, void* stream) {
  if (P < 0 || step < 1) return GNCDE_ERR_ARG;
  if (P == 0) return GNCDE_OK;
  if (!params || !grads || !m || !v || !stats) return GNCDE_ERR_ARG;
  if (!workspace || workspace_bytes < gncde_adamw_workspace_bytes(P)) return GNCDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nblk = (P + 255) / 256;
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  float* upd = static_cast<float*>(workspace);
  hipLaunchKernelGGL(k_grad_norm, dim3(1), dim3(1024), 0, st, P, grads, stats);
  hipLaunchKernelGGL(k_adamw, dim3(nblk), dim3(256), 0, st, P, params, grads, m, v, lr, b1, b2, eps, weight_decay,
                     max_norm, bc1, bc2, stats, upd);
  hipLaunchKernelGGL(k_max_reduce, dim3(1), dim3(1024), 0, st, nblk, upd, stats);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

int gncde_interval_index(const float* ts, int32_t B, int32_t T, const float* t, const int32_t* sample,
                         int32_t* idx, int32_t count, void* stream) {
  if (B <= 0 || T < 2 || count < 0) return GNCDE_ERR_SHAPE;
  if (count == 0) return GNCDE_OK;
  if (!ts || !t || !sample || !idx) return GNCDE_ERR_ARG;
  hipLaunchKernelGGL(k_interval_index, dim3((count + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), ts, B, T, t, sample, idx, count);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

}  // extern "C"
