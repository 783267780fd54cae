// Generic (any shape, CDE wrapper included) Tsit5 + PIDController solve — the adaptive configuration of
// graph_neural_cde.py:53-54,94-104 (and BASELINE config 5) for problems the fused persistent kernel does not
// cover.  Same controller as gncde_fused.hip (diffrax defaults: pcoeff 0, icoeff 1, safety 0.9, factormin 0.2
// but 1 after an accepted step, factormax 10, RMS error norm, error order 5, FSAL, _clip_to_end 1e-6, Hairer
// initial step for dt0 = None, SaveAt(ts) through the Tsit5 dense interpolant).
//
// Every sample runs its own step sequence.  The host loop issues one batched vector-field evaluation per
// iteration (each sample at its own stage time and input), then k_pid_advance — one workgroup per sample —
// advances that sample's controller state machine by one stage: norms are workgroup reductions, the accept /
// reject decision and the next stage input are formed in place.  Finished samples idle.  Completion is polled
// every kPoll iterations.
#include "gncde_internal.h"

namespace gncde {
namespace {

// one workgroup per sample: wide, so its element loops (E = n*h floats, 7 stage buffers) issue many loads at once
constexpr int kAdvThreads = 1024;
// The per-stage element loops run in passes of kAdvU elements per thread (E <= 8192 in one pass); a pass issues
// all of its loads before the first use, so a loop costs about one memory round trip per pass, not per element.
constexpr int kAdvU = 8;
constexpr int kAdvMaxSlices = 16;  // workgroups per sample for an in-attempt stage

struct PidState {
  int phase, st, steps, rejects, evals, status, done, si;
  float t, tn, h, dt, h0, d1, tst;
};

struct PidArgs {
  int B, E, S, max_steps, auto_dt;
  int n, d;     // E = n d: node rows of width d (the norms' canonical order, canon_sumsq)
  float rtol, atol;
  const float* t0;
  const float* t1;
  const float* dt0;
  const float* save_ts;  // [B, S] or nullptr
  PidState* state;      // [B] controller states read by k_pid_advance (and written by k_pid_init)
  PidState* state_out;  // [B] the states it writes (the host swaps the two after every launch: the slices of one
                        // sample never read a state another slice of the same launch has already advanced)
  float* y;     // [B, E]
  float* yt;    // [B, E] stage input (next evaluation)
  float* kk;    // [7, B, E]
  const float* K;  // [B, E] value of the last evaluation
  float* ys;    // output: [B, S, E] (SAVE_TS) or [B, E]
  float* tst;   // [B] time of each sample's next evaluation (written by init / advance)
  float* step_ts;  // [B, step_len] accepted step times (GncdeSolver.step_ts) or nullptr
  int step_len;
  float* vbuf;  // [B, E] the norms' per-element values
  float* rbuf;  // [B, n + ceil(n / 16)] their row and row-block sums
};

// sum of v_e^2 over one sample's [n, d] elements (v in vb, written by this workgroup before the call) in the
// CANONICAL order the persistent solve uses too (gncde_rows.hip group_sumsq): a 4-element chunk of a row is an fma
// chain from 0, a row sums its chunks in order, a 16-row block its rows in order, and the sample its blocks in
// order.  The two controllers therefore see bitwise-equal error norms and take the same accept / reject decisions.
__device__ float canon_sumsq(const float* vb, float* rb, int n, int d, float* red) {
  __syncthreads();  // every element of vb written (global memory, this workgroup)
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float* r = vb + (size_t)i * d;
    float s = 0.f;
    for (int c = 0; c < d; c += 4) {
      float p = 0.f;
      for (int e = c; e < c + 4 && e < d; ++e) p = fmaf(r[e], r[e], p);
      s = c == 0 ? p : s + p;
    }
    rb[i] = s;
  }
  __syncthreads();
  const int nb = (n + 15) / 16;
  for (int q = threadIdx.x; q < nb; q += blockDim.x) {
    float s = rb[16 * q];
    for (int i = 16 * q + 1; i < 16 * q + 16 && i < n; ++i) s += rb[i];
    rb[n + q] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int q = 0; q < nb; ++q) tot += rb[n + q];
    red[0] = tot;
  }
  __syncthreads();
  const float tot = red[0];
  __syncthreads();  // (red and vb are reused by the next call)
  return tot;
}

// initial state: t = t0, saved states at save_ts <= t0, first evaluation f(t0, y0)
__global__ void k_pid_init(PidArgs a, const float* __restrict__ y0) {
  const int b = blockIdx.x;
  const size_t base = (size_t)b * a.E;
  for (int e = threadIdx.x; e < a.E; e += blockDim.x) {
    a.y[base + e] = y0[base + e];
    a.yt[base + e] = y0[base + e];
  }
  const float t0 = a.t0[b];
  int si = 0;
  if (a.S > 0) {
    const float* sts = a.save_ts + (size_t)b * a.S;
    while (si < a.S && sts[si] <= t0) {
      for (int e = threadIdx.x; e < a.E; e += blockDim.x) a.ys[((size_t)b * a.S + si) * a.E + e] = y0[base + e];
      ++si;
    }
  }
  if (threadIdx.x == 0) {
    if (a.step_ts) a.step_ts[(size_t)b * a.step_len] = t0;
    PidState s{};
    s.t = s.tn = s.tst = t0;
    s.dt = a.auto_dt ? 0.f : a.dt0[b];
    s.si = si;
    a.state[b] = s;
    a.tst[b] = s.tst;
  }
}

// grid (slices, B): an in-attempt stage (5 launches in 6) is spread over the sample's slices; every other step of the
// state machine (the attempt end with its error norm, the initial-step heuristic, finishing) runs on slice 0
__global__ void __launch_bounds__(kAdvThreads) k_pid_advance(PidArgs a) {
  __shared__ float red[kAdvThreads / 64];
  __shared__ PidState sh;
  const int b = blockIdx.y, slice = blockIdx.x, NS = gridDim.x;
  const int tid = threadIdx.x;
  const int E = a.E;
  const size_t base = (size_t)b * E;
  const size_t BE = (size_t)a.B * E;
  constexpr int U2 = 2;
  const int stride = NS * kAdvThreads, e0 = slice * kAdvThreads + tid;
  if (tid == 0) sh = a.state[b];
  __syncthreads();
  PidState s = sh;
  if (s.done) {
    if (slice == 0 && tid == 0) a.state_out[b] = s;
    return;
  }
  const bool mid = s.phase == 2 && s.st < 6;
  if (!mid && slice != 0) return;
  const float rtol = a.rtol, atol = a.atol;
  const float t0 = a.t0[b], t1 = a.t1[b];
  const float inv_cnt = 1.0f / (float)E;
  float* y = a.y + base;
  float* yt = a.yt + base;
  const float* K = a.K + base;
  auto kk = [&](int j) { return a.kk + (size_t)j * BE + base; };
  float* vb = a.vbuf + base;
  float* rb = a.rbuf + (size_t)b * (a.n + (a.n + 15) / 16);
  constexpr int U = kAdvU, P = kAdvThreads * kAdvU;
  auto ldu = [&](const float* p, int e0, float(&v)[U]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * kAdvThreads;
      v[u] = e < E ? p[e] : 0.f;
    }
  };
  s.evals++;
  bool start = false;
  if (s.phase == 0) {  // f(t0, y0): FSAL k1 and f0 of the initial-step heuristic
    for (int e = tid; e < E; e += blockDim.x) kk(0)[e] = K[e];
    s.phase = 2;
    if (a.auto_dt) {
      for (int e = tid; e < E; e += blockDim.x) vb[e] = y[e] / fmaf(fabsf(y[e]), rtol, atol);
      const float d0 = sqrtf(canon_sumsq(vb, rb, a.n, a.d, red) * inv_cnt);
      for (int e = tid; e < E; e += blockDim.x) vb[e] = K[e] / fmaf(fabsf(y[e]), rtol, atol);
      const float d1 = sqrtf(canon_sumsq(vb, rb, a.n, a.d, red) * inv_cnt);
      s.d1 = d1;
      s.h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : 0.01f * (d0 / d1);
      for (int e = tid; e < E; e += blockDim.x) yt[e] = fmaf(s.h0, K[e], y[e]);
      s.tst = t0 + s.h0;
      s.phase = 1;
    } else {
      start = true;
    }
  } else if (s.phase == 1) {  // f(t0 + h0, y0 + h0 f0)
    for (int e = tid; e < E; e += blockDim.x) vb[e] = (K[e] - kk(0)[e]) / fmaf(fabsf(y[e]), rtol, atol);
    const float d2 = sqrtf(canon_sumsq(vb, rb, a.n, a.d, red) * inv_cnt) / s.h0;
    const float md = fmaxf(s.d1, d2);
    const float h1 = md <= 1e-15f ? fmaxf(1e-6f, s.h0 * 1e-3f) : powf(0.01f / md, 0.2f);
    s.dt = fminf(100.0f * s.h0, h1);
    s.phase = 2;
    start = true;
  } else {
    float* kst = kk(s.st);
    if (mid) {
      // A stage inside an attempt (e.g. config 5's 255 x 32 over 8 slices): K, y and only the stage buffers the next
      // input reads (j < st + 1, the current one taken from K in registers) in one round trip per pass.
      const int ns1 = s.st + 1;
      float ar[6], cst;
      tsit5_row(ns1, ar, cst);
      for (int ep = e0; ep < E; ep += stride * U2) {
        float kq[U2], yv[U2], kv[6][U2];
#pragma unroll
        for (int u = 0; u < U2; ++u) {
          const int e = ep + u * stride;
          kq[u] = e < E ? K[e] : 0.f;
          yv[u] = e < E ? y[e] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          if (j < ns1 && j != s.st) {  // uniform: a scalar branch around the loads
#pragma unroll
            for (int u = 0; u < U2; ++u) {
              const int e = ep + u * stride;
              kv[j][u] = e < E ? kk(j)[e] : 0.f;
            }
          } else {
#pragma unroll
            for (int u = 0; u < U2; ++u) kv[j][u] = 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U2; ++u) {
          const int e = ep + u * stride;
          float acc = 0.f;  // the memory path's summation order
#pragma unroll
          for (int j = 0; j < 6; ++j) acc = j < ns1 ? fmaf(ar[j], j == s.st ? kq[u] : kv[j][u], acc) : acc;
          if (e < E) {
            kst[e] = kq[u];
            yt[e] = fmaf(s.h, acc, yv[u]);
          }
        }
      }
      s.tst = ns1 == 6 ? s.tn : ns1 == 5 ? __fadd_rn(s.t, s.h) : stage_time(s.t, cst, s.h);  // FSAL stage at the step end
      s.st = ns1;
      if (slice == 0 && tid == 0) {
        a.state_out[b] = s;
        a.tst[b] = s.tst;
      }
      return;
    }
    if (s.st == 6 && E <= P) {
      // Attempt complete, one pass (config 5): the error norm, the dense outputs, the accept copy and the next
      // attempt's stage-1 input all come from ONE round of loads held in registers (this path was 3.3x the
      // in-attempt stage's time when it re-read the stage buffers for each of those steps).  Same arithmetic and
      // summation order as the multi-pass path below.
      float kv[7][U], yv[U], ytv[U];
#pragma unroll
      for (int j = 0; j < 6; ++j) ldu(kk(j), tid, kv[j]);
      ldu(K, tid, kv[6]);
      ldu(y, tid, yv);
      ldu(yt, tid, ytv);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = tid + u * kAdvThreads;
        if (e >= E) break;
        kst[e] = kv[6][u];
        const float err = s.h * (TSIT5_E1 * kv[0][u] + TSIT5_E2 * kv[1][u] + TSIT5_E3 * kv[2][u] + TSIT5_E4 * kv[3][u] +
                                 TSIT5_E5 * kv[4][u] + TSIT5_E6 * kv[5][u] + TSIT5_E7 * kv[6][u]);
        const float sc = fmaf(fmaxf(fabsf(yv[u]), fabsf(ytv[u])), rtol, atol);
        vb[e] = err / sc;
      }
      const float err = sqrtf(canon_sumsq(vb, rb, a.n, a.d, red) * inv_cnt);
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
        if (a.S > 0) {
          const float* sts = a.save_ts + (size_t)b * a.S;
          while (s.si < a.S && sts[s.si] <= s.tn) {  // dense output inside (t, tn]
            float wts[7];
            tsit5_dense((sts[s.si] - s.t) / s.h, wts);
            float* dst = a.ys + ((size_t)b * a.S + s.si) * E;
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int e = tid + u * kAdvThreads;
              if (e >= E) break;
              float acc = 0.f;
#pragma unroll
              for (int j = 0; j < 7; ++j) acc = fmaf(wts[j], kv[j][u], acc);
              dst[e] = fmaf(s.h, acc, yv[u]);
            }
            ++s.si;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = tid + u * kAdvThreads;
          yv[u] = ytv[u];        // y <- y1
          kv[0][u] = kv[6][u];   // kk0 <- f(tn, y1) (FSAL)
          if (e < E) {
            y[e] = yv[u];
            kk(0)[e] = kv[0][u];
          }
        }
        if (a.step_ts && tid == 0 && s.steps + 1 < a.step_len) a.step_ts[(size_t)b * a.step_len + s.steps + 1] = s.tn;
        s.t = s.tn;
        ++s.steps;
      } else {
        ++s.rejects;
      }
      s.dt = factor * s.h;
      s.st = 0;
      bool finish = false;
      if (!(s.t < t1)) {
        finish = true;
      } else if (s.steps + s.rejects >= a.max_steps) {
        s.status = 1;
        finish = true;
      }
      if (finish) {
        if (a.step_ts && s.status == 0 && s.steps + 1 > a.step_len) s.status = 3;  // step record truncated
        for (int q = (a.S == 0 ? -1 : s.si); q < a.S; ++q) {  // SAVE_T1: the final state; SAVE_TS: only on failure
          float* dst = a.S == 0 ? a.ys + base : a.ys + ((size_t)b * a.S + q) * E;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int e = tid + u * kAdvThreads;
            if (e < E) dst[e] = yv[u];
          }
          if (a.S == 0) break;
        }
        if (a.S > 0) s.si = a.S;
        s.done = 1;
        if (tid == 0) a.state_out[b] = s;
        return;
      }
      s.tn = s.t + s.dt;
      if (s.tn > t1 - 1e-6f) s.tn = t1;  // diffrax _clip_to_end
      s.h = s.tn - s.t;
      // stage 1 of the new attempt: y + h a21 kk0 (the multi-pass loop's order: acc = fma(a21, k0, 0))
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = tid + u * kAdvThreads;
        if (e < E) yt[e] = fmaf(s.h, fmaf(TSIT5_A21, kv[0][u], 0.f), yv[u]);
      }
      s.tst = stage_time(s.t, TSIT5_C2, s.h);
      s.st = 1;
      if (tid == 0) {
        a.state_out[b] = s;
        a.tst[b] = s.tst;
      }
      return;
    }
    for (int e0 = tid; e0 < E; e0 += P) {
      float v[U];
      ldu(K, e0, v);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (e0 + u * kAdvThreads < E) kst[e0 + u * kAdvThreads] = v[u];
    }
    if (s.st == 6) {  // attempt complete: yt = y1 candidate, kk6 = f(tn, y1) (= K)
      for (int e0 = tid; e0 < E; e0 += P) {
        float k0[U], k1[U], k2[U], k3[U], k4[U], k5[U], k6[U], yv[U], ytv[U];
        ldu(kk(0), e0, k0);
        ldu(kk(1), e0, k1);
        ldu(kk(2), e0, k2);
        ldu(kk(3), e0, k3);
        ldu(kk(4), e0, k4);
        ldu(kk(5), e0, k5);
        ldu(K, e0, k6);
        ldu(y, e0, yv);
        ldu(yt, e0, ytv);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (e0 + u * kAdvThreads >= E) break;
          const float err = s.h * (TSIT5_E1 * k0[u] + TSIT5_E2 * k1[u] + TSIT5_E3 * k2[u] + TSIT5_E4 * k3[u] +
                                   TSIT5_E5 * k4[u] + TSIT5_E6 * k5[u] + TSIT5_E7 * k6[u]);
          const float sc = fmaf(fmaxf(fabsf(yv[u]), fabsf(ytv[u])), rtol, atol);
          vb[e0 + u * kAdvThreads] = err / sc;
        }
      }
      const float err = sqrtf(canon_sumsq(vb, rb, a.n, a.d, red) * inv_cnt);
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
        if (a.S > 0) {
          const float* sts = a.save_ts + (size_t)b * a.S;
          while (s.si < a.S && sts[s.si] <= s.tn) {  // dense output inside (t, tn]
            float wts[7];
            tsit5_dense((sts[s.si] - s.t) / s.h, wts);
            float* dst = a.ys + ((size_t)b * a.S + s.si) * E;
            for (int e = tid; e < E; e += blockDim.x) {
              float acc = 0.f;
              for (int j = 0; j < 7; ++j) acc = fmaf(wts[j], kk(j)[e], acc);
              dst[e] = fmaf(s.h, acc, y[e]);
            }
            ++s.si;
          }
        }
        __syncthreads();  // every thread has read y / kk before they are overwritten
        for (int e0 = tid; e0 < E; e0 += P) {
          float yv[U], kv[U];
          ldu(yt, e0, yv);
          ldu(K, e0, kv);  // kk6
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int e = e0 + u * kAdvThreads;
            if (e < E) {
              y[e] = yv[u];
              kk(0)[e] = kv[u];
            }
          }
        }
        if (a.step_ts && tid == 0 && s.steps + 1 < a.step_len) a.step_ts[(size_t)b * a.step_len + s.steps + 1] = s.tn;
        s.t = s.tn;
        ++s.steps;
      } else {
        ++s.rejects;
      }
      s.dt = factor * s.h;
      s.st = 0;
      start = true;
    }
  }
  if (start) {  // begin a new attempt (or finish)
    bool finish = false;
    if (!(s.t < t1)) {
      finish = true;
    } else if (s.steps + s.rejects >= a.max_steps) {
      s.status = 1;
      finish = true;
    }
    if (finish) {
      if (a.step_ts && s.status == 0 && s.steps + 1 > a.step_len) s.status = 3;  // step record truncated
      __syncthreads();
      if (a.S == 0) {
        for (int e = tid; e < E; e += blockDim.x) a.ys[base + e] = y[e];
      } else {
        for (; s.si < a.S; ++s.si)  // only on failure
          for (int e = tid; e < E; e += blockDim.x) a.ys[((size_t)b * a.S + s.si) * E + e] = y[e];
      }
      s.done = 1;
      if (tid == 0) a.state_out[b] = s;  // tst keeps its last value: finished samples' evaluations are ignored
      return;
    }
    s.tn = s.t + s.dt;
    if (s.tn > t1 - 1e-6f) s.tn = t1;  // diffrax _clip_to_end
    s.h = s.tn - s.t;
  }
  if (s.phase == 2) {  // next stage input and time
    const int ns1 = s.st + 1;
    float ar[6], cst;
    tsit5_row(ns1, ar, cst);
    __syncthreads();
    for (int e0 = tid; e0 < E; e0 += P) {
      // every stage buffer's loads issued at once (the ones past ns1 are loaded and not used: allocated memory,
      // possibly stale, so they are selected away rather than multiplied by a zero coefficient)
      float kv[6][U], yv[U], acc[U];
#pragma unroll
      for (int j = 0; j < 6; ++j) ldu(kk(j), e0, kv[j]);
      ldu(y, e0, yv);
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = 0.f;
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = j < ns1 ? fmaf(ar[j], kv[j][u], acc[u]) : acc[u];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (e0 + u * kAdvThreads < E) yt[e0 + u * kAdvThreads] = fmaf(s.h, acc[u], yv[u]);
    }
    s.tst = ns1 == 6 ? s.tn : ns1 == 5 ? __fadd_rn(s.t, s.h) : stage_time(s.t, cst, s.h);  // FSAL stage at the step end
    s.st = ns1;
  }
  if (tid == 0) {
    a.state_out[b] = s;
    a.tst[b] = s.tst;
  }
}

__global__ void k_pid_tst(int B, const PidState* __restrict__ st, float* __restrict__ tst, int* __restrict__ active) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  tst[b] = st[b].tst;
  if (!st[b].done) atomicAdd(active, 1);
}

__global__ void k_pid_stats(int B, const PidState* __restrict__ st, const int* __restrict__ fault,
                            int32_t* __restrict__ stats) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  stats[b * 4 + GNCDE_STAT_STEPS] = st[b].steps;
  stats[b * 4 + GNCDE_STAT_REJECTS] = st[b].rejects;
  stats[b * 4 + GNCDE_STAT_EVALS] = st[b].evals;
  stats[b * 4 + GNCDE_STAT_STATUS] = *fault ? 4 : st[b].status;
}

constexpr int kPidPoll = 16;  // controller iterations between completion polls
inline long pid_max_iterations(const GncdeSolver& s) { return 3L + 6L * (long)s.max_steps; }

struct PidRun {
  PidArgs a;  // the controller kernels' argument block
  GncdeProblem p;
  char* ws;
  hipStream_t st;
  float *K, *tst;
  int* active;
  int h_active;  // written by the polling copy; read after the stream is synchronised
  unsigned bars;  // barriers done by one-launch evaluations (generic_vf_eval)
};

}  // namespace

size_t generic_pid_workspace(const GncdeProblem& p) {
  const size_t B = p.B, E = (size_t)p.n * state_dim(p);
  size_t sz = generic_vf_workspace(p);
  sz += 11 * align_up(B * E * 4, 256);                 // y, yt, K, kk[7], the norms' values
  sz += align_up(B * (p.n + (p.n + 15) / 16) * 4, 256);  // their row / row-block sums
  sz += 2 * align_up(B * sizeof(PidState), 256) + 2 * align_up(B * 4, 256) + 256;
  return sz;
}

namespace {

// The PID solve in pieces: pid_begin sets up and launches the init, pid_iterate enqueues one batched evaluation + one
// controller stage, pid_poll_enqueue copies how many samples are still running to the host, pid_end writes the stats.
int pid_begin(PidRun& r, const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys, char* ws,
              hipStream_t st) {
  if (s.method != GNCDE_TSIT5) return GNCDE_ERR_UNSUPPORTED;
  const int B = p.B;
  const size_t E = (size_t)p.n * state_dim(p);
  if (out_dim(p) != state_dim(p)) return GNCDE_ERR_SHAPE;
  char* cur = ws + generic_vf_workspace(p);
  auto take = [&](size_t bytes) {
    char* ptr = cur;
    cur += align_up(bytes, 256);
    return ptr;
  };
  PidArgs& a = r.a;
  a = PidArgs{};
  a.B = B;
  a.E = (int)E;
  a.S = s.save_mode == GNCDE_SAVE_TS ? s.n_save : 0;
  a.max_steps = s.max_steps;
  a.auto_dt = s.dt0 == nullptr;
  a.rtol = s.rtol;
  a.atol = s.atol;
  a.t0 = s.t0;
  a.t1 = s.t1;
  a.dt0 = s.dt0;
  a.save_ts = s.save_ts;
  a.y = reinterpret_cast<float*>(take(B * E * 4));
  a.yt = reinterpret_cast<float*>(take(B * E * 4));
  r.K = reinterpret_cast<float*>(take(B * E * 4));
  a.K = r.K;
  a.kk = reinterpret_cast<float*>(take(7 * B * E * 4));
  a.vbuf = reinterpret_cast<float*>(take(B * E * 4));
  a.rbuf = reinterpret_cast<float*>(take(B * (p.n + (p.n + 15) / 16) * 4));
  a.n = p.n;
  a.d = (int)(E / p.n);
  a.state = reinterpret_cast<PidState*>(take(B * sizeof(PidState)));
  a.state_out = reinterpret_cast<PidState*>(take(B * sizeof(PidState)));
  r.tst = reinterpret_cast<float*>(take(B * 4));
  r.active = reinterpret_cast<int*>(take(B * 4));
  a.ys = ys;
  a.tst = r.tst;
  a.step_ts = s.step_ts;
  a.step_len = s.step_ts_len;
  r.p = p;
  r.ws = ws;
  r.st = st;
  r.h_active = 1;
  r.bars = 0;
  hipLaunchKernelGGL(k_pid_init, dim3(B), dim3(256), 0, st, a, y0);
  generic_vf_prepare(p, ws, st);
  return GNCDE_OK;
}

int pid_iterate(PidRun& r) {
  PidArgs& a = r.a;
  const int rc = generic_vf_eval(r.p, r.tst, a.yt, r.K, r.ws, r.st, true, &r.bars);
  if (rc) return rc;
  const int slices = (a.E + kAdvThreads - 1) / kAdvThreads;
  hipLaunchKernelGGL(k_pid_advance, dim3(slices < kAdvMaxSlices ? slices : kAdvMaxSlices, a.B), dim3(kAdvThreads), 0,
                     r.st, a);
  PidState* t = a.state;  // what this launch wrote is the next one's input
  a.state = a.state_out;
  a.state_out = t;
  return GNCDE_OK;
}

void pid_poll_enqueue(PidRun& r) {
  const PidArgs& a = r.a;
  (void)hipMemsetAsync(r.active, 0, sizeof(int), r.st);
  hipLaunchKernelGGL(k_pid_tst, dim3((a.B + 255) / 256), dim3(256), 0, r.st, a.B, a.state, r.tst, r.active);
  (void)hipMemcpyAsync(&r.h_active, r.active, sizeof(int), hipMemcpyDeviceToHost, r.st);
}

void pid_end(PidRun& r, int32_t* stats) {
  const PidArgs& a = r.a;
  if (stats)
    hipLaunchKernelGGL(k_pid_stats, dim3((a.B + 255) / 256), dim3(256), 0, r.st, a.B, a.state,
                       generic_vf_fault(r.p, r.ws), stats);
}

}  // namespace

int generic_integrate_pid(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys, int32_t* stats,
                          char* ws, hipStream_t st) {
  PidRun r;
  int rc = pid_begin(r, p, s, y0, ys, ws, st);
  if (rc) return rc;
  // each sample needs at most 2 + 6 * max_steps + 1 evaluations
  const long max_iter = pid_max_iterations(s);
  for (long it = 0; it < max_iter; ++it) {
    rc = pid_iterate(r);
    if (rc) return rc;
    if ((it + 1) % kPidPoll == 0) {
      pid_poll_enqueue(r);
      if (hipStreamSynchronize(st) != hipSuccess) return GNCDE_ERR_HIP;
      if (r.h_active == 0) break;
    }
  }
  pid_end(r, stats);
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

}  // namespace gncde
