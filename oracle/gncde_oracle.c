/*
 * gncde_oracle.c — CPU restatement of the GNCDE hot path in plain C (fp32, OpenMP over samples).
 * TEST INFRASTRUCTURE ONLY: used by tests/ (cross-check of the numpy oracle) and by bench.py's
 * cpu_baseline leg ("kind": "port").  Never linked into, or called by, the product path.
 *
 * Follows the reference literally, per vector-field evaluation (what XLA executes on CPU):
 *   spline evaluate/derivative  perm_equiv_graph_vector_field.py:98-102 (diffrax CubicInterpolation,
 *                               interval = clip(searchsorted_left(ts, t) - 1, 0, T-2))
 *   Abar materialised from the 8 undirected terms   layers.py:102-160 (term_7 quirk kept)
 *   ConvLayer: RMSNorm -> Linear -> m + Abar @ m     layers.py:36-48
 *   ReLU between layers, tg scaling                  perm_equiv_graph_vector_field.py:122-128
 *   fixed-grid RK4 with fp32 stage times fl(t + fl(0.5h)), fl(t + h) (build extension, BASELINE cfg 2)
 * PARITY UNPINNED (no executable reference in this image); cross-checked against oracle/gncde_oracle.py.
 *
 * Layouts are those of include/gncde.h; `fparams` holds the RAW reference fusion parameters
 * [L][8][2] (param1..param8, each (A, dA)).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int interval_index(const float* ts, int T, float t) {
  int lo = 0, hi = T;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (ts[mid] < t) lo = mid + 1; else hi = mid;
  }
  int i = lo - 1;
  if (i < 0) i = 0;
  if (i > T - 2) i = T - 2;
  return i;
}

typedef struct {
  int n, T, L;
  const int* dims;
  const float* ts;     /* [T] */
  const float* coef;   /* [T-1][4][n][n] */
  const float* tcoef;  /* [T-1][3][n] */
  const float* fp;     /* [L][8][2] */
  const float* params; /* packed */
  float *A, *dA, *Ab, *Z, *Zn, *m, *tg, *r, *rd; /* scratch */
} Ctx;

static void vf(Ctx* c, float t, const float* y, float* out) {
  const int n = c->n, T = c->T;
  const size_t nn = (size_t)n * n;
  const int idx = interval_index(c->ts, T, t);
  const float f = t - c->ts[idx];
  const float* cb = c->coef + (size_t)idx * 4 * nn;
  for (size_t e = 0; e < nn; ++e) {
    const float d = cb[e], cc = cb[nn + e], b = cb[2 * nn + e], a = cb[3 * nn + e];
    c->A[e] = a + f * (b + f * (cc + f * d));
    c->dA[e] = b + f * (2.0f * cc + f * 3.0f * d);
  }
  const float* tc = c->tcoef + (size_t)idx * 3 * n;
  for (int i = 0; i < n; ++i) c->tg[i] = tc[2 * n + i] + f * (2.0f * tc[n + i] + f * 3.0f * tc[i]);
  float sA = 0.f, sdA = 0.f;
  for (int i = 0; i < n; ++i) {
    float r = 0.f, rd = 0.f;
    for (int k = 0; k < n; ++k) {
      r += c->A[(size_t)i * n + k];
      rd += c->dA[(size_t)i * n + k];
    }
    c->r[i] = r;
    c->rd[i] = rd;
    sA += r;
    sdA += rd;
  }
  int din = c->dims[0];
  memcpy(c->Z, y, sizeof(float) * n * din);
  size_t off = 0;
  for (int l = 0; l < c->L; ++l) {
    const int dout = c->dims[l + 1];
    const float* p = c->fp + l * 16;
    const float fn = (float)n, fn2 = (float)n * (float)n;
    /* Abar: the 8 reference terms, elementwise (layers.py:102-160) */
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < n; ++k) {
        const size_t e = (size_t)i * n + k, et = (size_t)k * n + i;
        float v = (1.0f + p[0]) * c->A[e] + (1.0f + p[1]) * c->dA[e];
        v += p[2] * c->A[et] + p[3] * c->dA[et];
        if (i == k) v += p[4] * c->A[e] + p[5] * c->dA[e];
        v += p[6] / fn * c->r[i] + p[7] / fn * c->rd[i];
        v += p[8] / fn * c->r[k] + p[9] / fn * c->rd[k];
        if (i == k) v += p[10] / fn * c->r[i] + p[11] / fn * c->rd[i];
        v += p[12] / fn2 * sA + p[13] / fn2 * sA;
        if (i == k) v += (p[14] * sA + p[15] * sdA) / fn2;
        c->Ab[e] = v;
      }
    const float* rw = c->params + off;
    const float* rb = rw + din;
    const float* W = rb + din;
    const float* bias = W + (size_t)dout * din;
    off += 2 * (size_t)din + (size_t)dout * din + dout;
    for (int i = 0; i < n; ++i) {
      float ss = 0.f;
      for (int k = 0; k < din; ++k) ss += c->Z[i * din + k] * c->Z[i * din + k];
      const float inv = 1.0f / sqrtf(ss / (float)din + 1e-5f);
      for (int k = 0; k < din; ++k) c->Zn[i * din + k] = c->Z[i * din + k] * inv * rw[k] + rb[k];
      for (int o = 0; o < dout; ++o) {
        float acc = bias[o];
        for (int k = 0; k < din; ++k) acc += W[(size_t)o * din + k] * c->Zn[i * din + k];
        c->m[i * dout + o] = acc;
      }
    }
    for (int i = 0; i < n; ++i) {
      float* zr = c->Z + (size_t)i * dout;
      for (int o = 0; o < dout; ++o) zr[o] = c->m[i * dout + o];
      for (int k = 0; k < n; ++k) {
        const float a = c->Ab[(size_t)i * n + k];
        const float* mr = c->m + (size_t)k * dout;
        for (int o = 0; o < dout; ++o) zr[o] += a * mr[o];
      }
      if (l < c->L - 1)
        for (int o = 0; o < dout; ++o) zr[o] = zr[o] > 0.f ? zr[o] : 0.f;
    }
    din = dout;
  }
  for (int i = 0; i < n; ++i)
    for (int o = 0; o < din; ++o) out[i * din + o] = c->tg[i] * c->Z[i * din + o];
}

/* Fixed-grid RK4 over B samples.  Returns the number of vector-field evaluations performed. */
long gncde_oracle_rk4(int B, int n, int T, int L, const int* dims, const float* ts, const float* coef,
                      const float* tcoef, const float* fparams, const float* params, const float* grid,
                      const int* nsteps, int G, const float* y0, float* yT, int nthreads) {
  int Dmax = 0;
  for (int l = 0; l <= L; ++l) Dmax = dims[l] > Dmax ? dims[l] : Dmax;
  const int H = dims[0];
  long total = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
#endif
  for (int b = 0; b < B; ++b) {
    const size_t nn = (size_t)n * n;
    Ctx c;
    c.n = n; c.T = T; c.L = L; c.dims = dims;
    c.ts = ts + (size_t)b * T;
    c.coef = coef + (size_t)b * (T - 1) * 4 * nn;
    c.tcoef = tcoef + (size_t)b * (T - 1) * 3 * n;
    c.fp = fparams; c.params = params;
    float* buf = (float*)malloc(sizeof(float) * (3 * nn + 3 * (size_t)n * Dmax + 3 * n + 8 * (size_t)n * H));
    c.A = buf; c.dA = c.A + nn; c.Ab = c.dA + nn;
    c.Z = c.Ab + nn; c.Zn = c.Z + (size_t)n * Dmax; c.m = c.Zn + (size_t)n * Dmax;
    c.tg = c.m + (size_t)n * Dmax; c.r = c.tg + n; c.rd = c.r + n;
    float* y = c.rd + n;
    float* yt = y + (size_t)n * H;
    float* k1 = yt + (size_t)n * H; float* k2 = k1 + (size_t)n * H;
    float* k3 = k2 + (size_t)n * H; float* k4 = k3 + (size_t)n * H;
    const size_t E = (size_t)n * H;
    memcpy(y, y0 + (size_t)b * E, sizeof(float) * E);
    const float* g = grid + (size_t)b * G;
    const int ns = nsteps[b];
    for (int s = 0; s < ns; ++s) {
      const float t = g[s];
      const float h = g[s + 1] - t;
      const float hh = 0.5f * h;
      const float tm = t + hh;
      const float te = t + h;
      vf(&c, t, y, k1);
      for (size_t e = 0; e < E; ++e) yt[e] = y[e] + hh * k1[e];
      vf(&c, tm, yt, k2);
      for (size_t e = 0; e < E; ++e) yt[e] = y[e] + hh * k2[e];
      vf(&c, tm, yt, k3);
      for (size_t e = 0; e < E; ++e) yt[e] = y[e] + h * k3[e];
      vf(&c, te, yt, k4);
      for (size_t e = 0; e < E; ++e) y[e] += (h / 6.0f) * (k1[e] + 2.0f * k2[e] + 2.0f * k3[e] + k4[e]);
    }
    memcpy(yT + (size_t)b * E, y, sizeof(float) * E);
    total += 4L * ns;
    free(buf);
  }
  return total;
}
