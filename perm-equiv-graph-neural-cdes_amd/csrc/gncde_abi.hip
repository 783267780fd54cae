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
  if (!p->ts || !p->coef || !p->tcoef || !p->fusion || !p->params) return GNCDE_ERR_ARG;
  if (p->cde_hidden > 0) {
    if (p->cde_embed <= 0 || !p->data_coef) return GNCDE_ERR_ARG;
    if (p->dims[p->L] != p->cde_hidden * p->cde_embed * 2) return GNCDE_ERR_SHAPE;
    if (p->dims[0] != p->cde_hidden) return GNCDE_ERR_SHAPE;
  } else if (p->cde_hidden < 0) {
    return GNCDE_ERR_SHAPE;
  }
  return GNCDE_OK;
}

int validate_solver(const GncdeProblem* p, const GncdeSolver* s) {
  if (!s) return GNCDE_ERR_ARG;
  if (s->method != GNCDE_RK4 && s->method != GNCDE_TSIT5) return GNCDE_ERR_ARG;
  if (s->save_mode < GNCDE_SAVE_T1 || s->save_mode > GNCDE_SAVE_TS) return GNCDE_ERR_ARG;
  if (p->cde_hidden == 0 && p->dims[0] != p->dims[p->L]) return GNCDE_ERR_SHAPE;  // ODE state width
  if (s->controller == GNCDE_CTRL_GRID) {
    if (!s->grid || !s->nsteps || s->grid_len < 1) return GNCDE_ERR_ARG;
    if (s->save_mode == GNCDE_SAVE_TS) return GNCDE_ERR_UNSUPPORTED;
  } else if (s->controller == GNCDE_CTRL_PID) {
    if (!s->t0 || !s->t1 || s->max_steps < 1) return GNCDE_ERR_ARG;
    if (!(s->rtol >= 0.f) || !(s->atol > 0.f)) return GNCDE_ERR_ARG;
    if (s->save_mode == GNCDE_SAVE_STEPS) return GNCDE_ERR_UNSUPPORTED;
    if (s->save_mode == GNCDE_SAVE_TS && (!s->save_ts || s->n_save < 1)) return GNCDE_ERR_ARG;
  } else {
    return GNCDE_ERR_ARG;
  }
  return GNCDE_OK;
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
    default: return "unknown gncde error";
  }
}

size_t gncde_workspace_bytes(const GncdeProblem* prob, const GncdeSolver* solver) {
  if (validate_problem(prob) != GNCDE_OK) return 0;
  if (!solver) return generic_vf_workspace(*prob);
  if (fused_supported(*prob, *solver, nullptr, 0)) return 0;
  return generic_integrate_workspace(*prob, *solver);
}

int gncde_integrate_path(const GncdeProblem* prob, const GncdeSolver* solver, char* buf, size_t buf_len) {
  int rc = validate_problem(prob);
  if (rc) return rc;
  rc = validate_solver(prob, solver);
  if (rc) return rc;
  if (!buf || buf_len == 0) return GNCDE_ERR_ARG;
  if (!fused_supported(*prob, *solver, buf, buf_len)) snprintf(buf, buf_len, "generic");
  return GNCDE_OK;
}

int gncde_vf_eval(const GncdeProblem* prob, const float* t, const float* y, float* dy, void* workspace,
                  size_t workspace_bytes, void* stream) {
  int rc = validate_problem(prob);
  if (rc) return rc;
  if (prob->B == 0) return GNCDE_OK;
  if (!t || !y || !dy) return GNCDE_ERR_ARG;
  if (workspace_bytes < generic_vf_workspace(*prob) || !workspace) return GNCDE_ERR_WORKSPACE;
  return generic_vf_eval(*prob, t, y, dy, static_cast<char*>(workspace),
                         static_cast<hipStream_t>(stream));
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
  if (fused_supported(*prob, *solver, nullptr, 0)) return fused_integrate(*prob, *solver, y0, ys, stats, st);
  if (workspace_bytes < generic_integrate_workspace(*prob, *solver) || !workspace) return GNCDE_ERR_WORKSPACE;
  return generic_integrate(*prob, *solver, y0, ys, stats, static_cast<char*>(workspace), st);
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
