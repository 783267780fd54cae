// One launch per vector-field evaluation for the generic path's large graphs (BASELINE configs 3 and 5: CDE wrapper,
// n up to 256, one hidden width H in {16, 32, 64}) — the spline, the fusion and every ConvLayer of
// PermEquivGraphVectorField.__call__ (perm_equiv_graph_vector_field.py:85-129; layers.py:36-48,102-160 via the
// factored fusion table) and the CDE contraction (cde_wrapper_vector_field.py:19-26), with no (I + Abar_l) in HBM.
//
// A workgroup owns 16 node rows R of one sample (one MFMA row tile); a sample's ceil(n / 16) workgroups form a group
// that meets at a barrier after every hidden layer (the next layer's product needs every row of Z):
//
//   form     the interval's coefficient rows R and the column strip [:, R] -> A(t), dA/dt(t) of those rows and
//            columns (Horner), kept in registers in the product's A-operand layout; the row / column / diagonal /
//            total reductions as cubics of k_coef_sums' per-plane sums (gncde_generic.hip) -> every layer's rank-1 and
//            diagonal families u_l, w_l, v_l and q_l = (I + Abar_l) 1 in LDS.  The coefficients are read once per
//            evaluation (each element twice: as a row element and as a column element, the second from L2).
//   layer l  Z_l (all n rows: the stage input, or the group's previous layer output) -> LDS, RMSNorm factors;
//            P = (I + Abar_l)[R, :] diag(inv) Z_l on v_mfma_f32_16x16x4f32 with the operand built in registers from
//            the A / dA / A^T / dA^T elements (K split over the four waves, partials summed in LDS in a fixed order);
//            Z_{l+1}[R] = relu(P W'^T + q_l b'^T) (W' = W diag(rms_w), b' = b + W rms_b folded once per solve), stored
//            write-through (sc1) and published by one agent-scope arrival per workgroup; the group's workgroups poll
//            the arrival count (sc1 loads) and read Z_{l+1} with sc1 loads (MI355X_MICROARCH.md, hand-off row 1).
//   output   ODE: dy[R] = tg * (P W'^T + q b'^T).  CDE (de = 8): dy[R, m] = tg sum_{c,j} P[., c] dX[., j] W'[16m+j, c]
//            + tg q sum_j b'[16m + j] dX[., j] (the read-out never materialises the n x 16h matrix).
//
// Residency: every group's workgroups must be co-resident (they wait on each other), so the grid is sized from the
// occupancy query: G groups (at most what fits) loop over the samples g, g + G, ...; every spin is bounded and sets a
// fault word (reported as solver status 4) instead of hanging.  Groups are laid out so a group's workgroups share
// blockIdx % 8 (one XCD under the observed round-robin placement: its coefficient strips and Z re-reads stay in one
// L2) — a speed choice, never needed for correctness.
#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "gncde_internal.h"

namespace gncde {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifdef GNCDE_ROWS_STAMPS
__device__ unsigned long long g_rows_stamps[4096 * 16];
// (solve: the evaluation kStampEval of every workgroup, slot = its ticket)
constexpr int kStampEval = 20;
#define ROWS_STAMP(k) \
  do { if (threadIdx.x == 0 && stamp_on) g_rows_stamps[stamp_slot * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define ROWS_STAMP(k) do {} while (0)
#endif
constexpr int kRB = 16;      // node rows per workgroup
constexpr int kMaxN = 256;   // per wave: four 16-column K chunks (fp32) or two 32-column chunks (bf16)
constexpr int kStrip = 17;   // LDS row stride of the transposed column strip

// The persistent solve's controller inputs and outputs (GncdeSolver, PID controller)
struct SolveArgs {
  int grid_mode;         // 1: GRID controller (grid, nsteps, method, save_steps, rec); 0: PID
  int method, G, save_steps;
  const float* grid;     // [B, G]
  const int32_t* nsteps; // [B]
  float* rec;            // GRID: [B, G-1, S-1, n, H] stage record; PID: [B, R, 5, n, H] (the accepted steps); or nullptr
  float* ckpt;           // PID: [B, R, n, H] accepted steps' starting states (GncdeSolver.pid_ckpt) or nullptr
  float* arec;           // PID: [R, 6, L-1, B, n, H] their stage evaluations' hidden outputs or nullptr
  int R;                 // PID: record slots (GncdeSolver.rec_steps)
  int S, max_steps, auto_dt, step_len;
  float rtol, atol;
  const float* t0;       // [B]
  const float* t1;       // [B]
  const float* dt0;      // [B] (auto_dt = 0)
  const float* save_ts;  // [B, S] (SAVE_TS) or nullptr
  const float* y0;       // [B, n, H]
  float* ys;             // [B, S, n, H] or [B, n, H]
  float* step_ts;        // [B, step_len] or nullptr
  int32_t* stats;        // [B, 4] or nullptr
  float* part;           // [B, 2, nb, 2] the group sums' partials (two buffers, by publication parity)
};

struct RowsArgs {
  int B, n, T, L, G, rounds, nb, big;  // big: floats of the LDS region shared by the strip, Z_l and the partials
  int np;                  // n rounded up to the K chunk (16 fp32, 32 bf16)
  const float* ts;
  const void* coef;        // [B, T-1, 4, n, n] fp32, or bfloat16 (PREC 1 / 2)
  const void* coefT;       // the same planes transposed (generic_vf_prepare, once per solve)
  const float* csum;       // k_coef_sums: [B, T-1, 12 n + 4]
  const float* tcoef;      // [B, T-1, 3, n]
  const float* data_coef;  // [B, T-1, 4, n, 8, 2] (CDE)
  const float* fusion;     // [L, GNCDE_FC]
  const float* wperm;      // W' per layer in the MFMA lane order (permute_linear), back to back
  const uint16_t* wbf;     // bf16 mode: W' per layer as bfloat16 in its natural [d_out, d_in] layout
  const float* bf;         // b' per layer, back to back
  const float* t;          // [B] evaluation times
  const float* y;          // [B, n, H] stage inputs
  float* dy;               // [B, n, H] vector field
  float* zbuf[2];          // [G, n, H] each: the groups' hidden layer outputs, alternating per step
  float* keep;             // optional [L-1, B, n, H]: every sample's hidden layer outputs kept (reverse mode), used
                           // instead of zbuf
  unsigned* zgran;         // solve: [2][B][n H] tagged hand-off granules {value, tag} (zeroed before the solve)
  int poll1;               // solve: a granule wait re-polls only its first stale pair per spin (GNCDE_GRAN_POLL1)
  unsigned* bar;           // [G][kBarStride] arrivals per group (one line each), monotonic within a solve
  unsigned bar0;           // barriers every group completed before this launch
  int* fault;              // set when a barrier wait gives up
  unsigned spin_limit;     // polls before a barrier wait gives up
  unsigned* ticket;        // solve: start-order tickets -> (sample, row block)
  unsigned ticket0;        // tickets taken before this launch
  int b0;                  // solve: the first sample of this launch (the batch runs in resident chunks)
  unsigned* queue;         // solve: samples handed out past the resident groups' first ones (zeroed per solve)
  unsigned* mail;          // solve: [G][kBarStride] each group's latest sample assignment (zeroed per solve)
  int G_all;               // solve: groups of this launch (each starts on sample b0 + its slot)
  SolveArgs s;             // solve only
};

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ floatx4 mfma_bf(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float bf2f(unsigned u, int half) {  // element `half` (0 low, 1 high) of a bf16 pair
  return __builtin_bit_cast(float, half ? (u & 0xffff0000u) : (u << 16));
}
__device__ __forceinline__ float cubic(const float (&c)[4], float f) { return fmaf(f, fmaf(f, fmaf(f, c[0], c[1]), c[2]), c[3]); }
__device__ __forceinline__ float dcubic(const float (&c)[4], float f) {
  return fmaf(f, fmaf(3.0f * f, c[0], 2.0f * c[1]), c[2]);
}

// 8 bf16 at element `e` of a buffer: the 16-byte load at the dword boundary at or below e and the next dword,
// funnel-shifted by one element when e is odd (odd n puts rows at 2-byte boundaries; every load stays dword-aligned)
__device__ __forceinline__ u32x4 load8_bf16(__amdgpu_buffer_rsrc_t r, int e) {
  const int e0 = e & ~1;
  const unsigned sh = (unsigned)(e & 1) * 16u;
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, e0 * 2, 0, 0);
  const unsigned x = __builtin_amdgcn_raw_buffer_load_b32(r, e0 * 2 + 16, 0, 0);
  return u32x4{__builtin_amdgcn_alignbit(v[1], v[0], sh), __builtin_amdgcn_alignbit(v[2], v[1], sh),
               __builtin_amdgcn_alignbit(v[3], v[2], sh), __builtin_amdgcn_alignbit(x, v[3], sh)};
}

// element e of a 16-byte coefficient load as fp32 (fp32: element e; bf16: half e % 2 of dword e / 2)
template <bool BF>
__device__ __forceinline__ float coef_el(u32x4 v, int e) {
  if constexpr (BF) return bf2f(v[e >> 1], e & 1);
  else {
    const unsigned x = v[e];  // (a vector element, not the vector: bit_cast of `v[e]` itself reads element 0)
    return __builtin_bit_cast(float, x);
  }
}

__host__ __device__ constexpr int rows_zs(int H) { return H + 4; }
__host__ __device__ inline int rows_np(int n, bool bf) { return bf ? (n + 31) & ~31 : (n + 15) & ~15; }
// floats of the shared region: the strip [2][NP][17] and the rows block [2][16][NP+4] during the form, then Z_l
// [NP][H+4]; after a layer's product the partials [4][16][H+4] (rows 0 .. 63) and the output tile [16][H+4] (rows
// 64 .. 79: Z_l is consumed by then, and the tile is read before the next form writes the region)
__host__ __device__ inline int rows_big(int n, int H, bool bf) {
  const int np = rows_np(n, bf), z = (np > 80 ? np : 80) * rows_zs(H), s = 2 * np * kStrip + 32 * (np + 4);
  return ((z > s ? z : s) + 3) & ~3;
}
// the bf16-storage solve's per-thread coefficient cache (SOLVE & 8): every thread's raw rows-block and strip loads of
// the current interval, [2][NU = 2][4 planes][256 threads] x 16 bytes
constexpr size_t kCoefCacheBytes = (size_t)2 * 2 * 4 * 256 * 16;
inline size_t rows_smem(int n, int H, int L, bool bf, bool cache = false) {
  const int np = rows_np(n, bf);
  // big | inv [NP] | v_l [L][NP] | w, u, q [3][L][16] | tg [16] | dX [16][17] | red [4][64] x4 | flags [4] | cache
  // (config 5, n = 255 h = 32 L = 4: 77.4 KiB, two workgroups per CU; with the cache 141.4 KiB, one)
  return sizeof(float) * ((size_t)rows_big(n, H, bf) + np + (size_t)L * np + 48 * L + 16 + 16 * kStrip +
                          4 * 64 * 4 + 4) + (cache ? kCoefCacheBytes : 0);
}

// Every buffer in this file is one sample's (or one interval's) block: its base and size are workgroup-uniform.  They
// are taken through readfirstlane so that the descriptor is built in SGPRs even where the compiler cannot prove the
// sample index uniform (the solve's sample queue, values that reach it through LDS or the controller's decisions):
// a descriptor in VGPRs wraps every buffer access in a waterfall loop.
// (Only the adaptive solve needs it — its sample queue and controller decisions — and only it takes it: UNI.)
template <bool UNI = false>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  if constexpr (!UNI) return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  void* q = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// MODE 1: ODE output layer.  MODE 2: CDE read-out (de = 8, cde_hidden = H).  Three workgroups per CU (168 VGPRs)
// for the ODE output, two for the CDE read-out (its weight slice is prefetched into registers).
// PREC 0: fp32.  PREC 1 (GNCDE_COMPUTE_BF16_MFMA): bfloat16 coefficients, and every product — (I + Abar_l) diag(inv) Z,
// the Linears, the read-out — on v_mfma_f32_16x16x32_bf16 with single-plane bf16 operands rounded from the fp32 values
// (fp32 accumulation); the spline, the reductions, RMSNorm and all sums outside the MFMAs stay fp32.  PREC 2
// (GNCDE_COMPUTE_BF16_STORAGE, the persistent solve): bfloat16 coefficients (half the form's coefficient stream and
// its L2 footprint), widened exactly on load, every product fp32: the result is the fp32 computation on the
// bf16-rounded operator, so the adaptive controller sees no per-stage rounding noise.
// SOLVE: 0 one evaluation per launch; the persistent solve with 1 the Tsit5 + PIDController controller, 2 a fixed
// step grid (§ the solve below); + 4: the solve's hand-offs as tagged granules instead of counter barriers; + 8
// (bf16 coefficient storage only): each thread keeps its raw coefficient loads of the current interval in LDS.
template <int H, int MODE, int PREC, int SOLVE>
__global__ void __launch_bounds__(256, MODE == 2 || SOLVE != 0 ? 2 : 3) k_rows(RowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr bool UNI = (SOLVE & 3) == 1 || (SOLVE & 4) != 0;  // uniform buffer descriptors (rsrc): PID, granules
  constexpr bool CBF = PREC != 0;  // bfloat16 coefficients
  constexpr bool BF = PREC == 1;   // bf16 products
  constexpr int ZS = rows_zs(H);
  constexpr int CT = H / 16;           // column tiles of a width-H operand / output
  constexpr int KW = BF ? 32 : 16;     // K chunk of one MFMA step
  constexpr int EL = KW / 4;           // consecutive k per lane per chunk
  constexpr int NJ = kMaxN / (4 * KW);  // chunks per wave
  constexpr int KC = (H + 31) / 32;    // bf16: 32-deep K chunks of a width-H contraction
  const int n = a.n, L = a.L, nb = a.nb, T = a.T;
  const int NP = a.np, nch = NP / KW;
  float* big = sm;
  float* sInv = big + a.big;
  float* sV = sInv + NP;
  float* sRow = sV + (size_t)L * NP;  // w_l [L][16], u_l [L][16], q_l [L][16]
  float* sTg = sRow + 48 * L;
  float* sDx = sTg + 16;
  float* sOut = big + 64 * ZS;  // the output tile [16][ZS] (rows_big)
  floatx4* red = reinterpret_cast<floatx4*>(sDx + 16 * kStrip);
  int* sFlag = reinterpret_cast<int*>(red + 4 * 64);  // [0] barrier gave up, [1] ticket
  // SOLVE & 8: the coefficient cache (thread-private slots: a thread reads back only what it wrote)
  constexpr bool CCACHE = (SOLVE & 8) != 0 && PREC == 2;
  u32x4* ccache = reinterpret_cast<u32x4*>(sFlag + 4);
  int cidx = -1;  // the interval the cache holds (uniform; -1: none, reset for every new sample)

  // ---- which rows of which sample ------------------------------------------------------------------------------
  // One evaluation (k_rows): the grid holds G co-resident groups that loop over the samples in rounds.  Solve: one
  // group per sample.  When every group is resident at once (G = B, a multiple of 8), the groups take the
  // XCD-affine blockIdx layout (a sample's workgroups on one XCD: its coefficients, weights and hand-offs stay in
  // one L2 across the solve's evaluations); otherwise a workgroup takes its (sample, row block) from a ticket in
  // start order, so the workgroups of a group are always ones that have started: a group waits only for members
  // that are already running, and groups of later samples start as earlier solves finish (no co-residency
  // assumption).
  int g, rb;
  if (SOLVE != 0 && a.G > 0 && a.G % 8 == 0) {  // every group resident at once (rows_integrate_pid checked): the XCD-affine layout
    const int x = blockIdx.x;
    g = (x & 7) + 8 * (x / (8 * nb));
    rb = (x >> 3) % nb;
  } else if constexpr (SOLVE != 0) {
    if (threadIdx.x == 0)
      sFlag[1] = (int)(__hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.ticket0);
    __syncthreads();
    // readfirstlane: an LDS value is a vector register to the compiler; as a scalar, every address and buffer
    // descriptor derived from the sample stays in SGPRs (otherwise each buffer access is wrapped in a waterfall loop)
    const int tk = UNI ? __builtin_amdgcn_readfirstlane(sFlag[1]) : sFlag[1];
    g = tk / nb;
    rb = tk % nb;
  } else if (a.G % 8 == 0) {  // a group's workgroups share blockIdx % 8 (bijective for G % 8 == 0)
    const int x = blockIdx.x;
    g = (x & 7) + 8 * (x / (8 * nb));
    rb = (x >> 3) % nb;
  } else {
    g = blockIdx.x / nb;
    rb = blockIdx.x % nb;
  }
  const int gslot = g;  // the group's slot in this launch
  if constexpr (SOLVE != 0) g += a.b0;  // the solve's groups start on samples b0 .. b0 + G - 1 of the batch
  const int r0 = rb * kRB;
  const size_t nn = (size_t)n * n;
  const size_t zgroup = (size_t)n * H;
  unsigned epoch = a.bar0;
  unsigned pub = 0;  // arrivals of this launch (one-evaluation launches: hidden outputs; solve: group sums): parity
  // SOLVE & 4: the persistent solve hands the stage inputs and hidden outputs over as TAGGED GRANULES: element e of the s-th
  // publication of sample b is the 8-byte {value, s + 1} at zgran[((s & 1) B + b) n H + e], two per 16-byte sc1
  // store (MI355X_MICROARCH.md: an 8-byte granule written by one sc1 store, also as half of a 16-byte one, is
  // observed untorn), so no arrival counter and no store drain sit between a producer and its consumers: a consumer
  // polls the data itself until every tag is the current one.  (The group sums keep the counter barrier.)  A
  // publication's buffer is rewritten two publications later, by which time every consumer has read it: a
  // producer of publication s + 2 has consumed s + 1, which every workgroup published after reading s.
  // Measured on config 5 (alternating runs on one box): 6.27 -> 6.74 ms per solve at B = 16, 7.6 -> 8.6 ms at B = 32
  // against the counter hand-offs (sc1 stores + one arrival, the waiters polling the counter), so the default
  // instances keep the counters; GNCDE_SOLVE_GRANULES=1 selects these.
  constexpr bool GRAN = (SOLVE & 4) != 0;
  unsigned hseq = 0;  // solve: granule publications of this group so far
#ifdef GNCDE_ROWS_STAMPS
  bool stamp_on = true;
  const int stamp_slot = SOLVE != 0 ? g * nb + rb : (int)blockIdx.x;
#endif

  auto arrive = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores have reached memory
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(a.bar + (size_t)g * kBarStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ++pub;
  };
  // wait until every workgroup of the group has arrived `epoch` times; a bounded spin: past the limit (or when
  // another workgroup has given up) the fault word is set and the wait returns false in every thread
  auto wait_all = [&]() -> bool {
    ++epoch;
    if (threadIdx.x == 0) {
      const unsigned target = epoch * (unsigned)nb;
      unsigned spins = 0;
      int gave_up = 0;
      while (__hip_atomic_load(a.bar + (size_t)g * kBarStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        ++spins;
        if (spins > a.spin_limit ||
            ((spins & 1023u) == 0 && __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          __hip_atomic_store(a.fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          gave_up = 1;
          break;
        }
      }
      sFlag[0] = gave_up;
    }
    __syncthreads();
    if constexpr (UNI) return __builtin_amdgcn_readfirstlane(sFlag[0]) == 0;  // uniform (see rsrc)
    return sFlag[0] == 0;
  };

  auto gran_rsrc = [&](unsigned s, int bb) {
    return rsrc<UNI>(a.zgran + ((size_t)(s & 1) * a.B + bb) * zgroup * 2, (unsigned)(zgroup * 8));
  };
  // elements e .. e + 3 (one float4 of a row) as two 16-byte {value, tag, value, tag} stores (every vector element
  // copied to a scalar before its bit cast: a bit cast of an ext-vector element reads element 0, see coef_el)
  auto gran_store4 = [&](__amdgpu_buffer_rsrc_t r, int e, const floatx4 v, unsigned tag) {
    const float x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3];
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4{__builtin_bit_cast(unsigned, x0), tag, __builtin_bit_cast(unsigned, x1), tag}, r, e * 8, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4{__builtin_bit_cast(unsigned, x2), tag, __builtin_bit_cast(unsigned, x3), tag}, r, e * 8 + 16, 0, 16);
  };
  // publication s of this sample into Zs [NP][ZS] (rows >= n zero): every granule polled until its tag is s + 1; a
  // bounded wait (past the limit, or when another workgroup gave up, it sets the fault word and returns false)
  auto gran_load = [&](float* Zs, unsigned s) -> bool {
    constexpr int G4 = H / 4, UG = 4;
    const unsigned tag = s + 1;
    const auto r = gran_rsrc(s, g);
    const int tot = a.np * G4, valid = a.n * G4;
    const int tid = threadIdx.x;
    bool good = true;
    for (int e0 = tid; e0 < tot; e0 += 256 * UG) {
      u32x4 p0[UG], p1[UG];
#pragma unroll
      for (int u = 0; u < UG; ++u) {
        const int e = e0 + 256 * u;
        const bool in = e < valid;
        p0[u] = in ? __builtin_amdgcn_raw_buffer_load_b128(r, e * 32, 0, 16) : u32x4{0u, tag, 0u, tag};
        p1[u] = in ? __builtin_amdgcn_raw_buffer_load_b128(r, e * 32 + 16, 0, 16) : u32x4{0u, tag, 0u, tag};
      }
      auto stale = [&]() {
        unsigned m = 0;
#pragma unroll
        for (int u = 0; u < UG; ++u)
          if (p0[u][1] != tag || p0[u][3] != tag || p1[u][1] != tag || p1[u][3] != tag) m |= 1u << u;
        return m;
      };
      unsigned st = stale(), spins = 0;
      while (st) {  // (like wait_all: a wait that has to poll more than spin_limit times gives up)
        if (spins >= a.spin_limit ||
            ((spins & 1023u) == 1023u && __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          __hip_atomic_store(a.fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          good = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        const unsigned want = a.poll1 ? st & (0u - st) : st;  // poll1: the first stale pair only
#pragma unroll
        for (int u = 0; u < UG; ++u)
          if ((want >> u) & 1u) {
            const int e = e0 + 256 * u;
            p0[u] = __builtin_amdgcn_raw_buffer_load_b128(r, e * 32, 0, 16);
            p1[u] = __builtin_amdgcn_raw_buffer_load_b128(r, e * 32 + 16, 0, 16);
          }
        st = stale();
        ++spins;
      }
#pragma unroll
      for (int u = 0; u < UG; ++u) {
        const int e = e0 + 256 * u;
        const unsigned w0 = p0[u][0], w1 = p0[u][2], w2 = p1[u][0], w3 = p1[u][2];
        if (e < tot)
          *reinterpret_cast<floatx4*>(Zs + (e / G4) * ZS + 4 * (e % G4)) =
              floatx4{__builtin_bit_cast(float, w0), __builtin_bit_cast(float, w1), __builtin_bit_cast(float, w2),
                      __builtin_bit_cast(float, w3)};
      }
    }
    return good;
  };

  // the solve's knots, one per lane (T <= 64)
  float ts_lane = SOLVE != 0 && (int)(threadIdx.x & 63) < T ? a.ts[(size_t)g * T + (threadIdx.x & 63)] : 0.f;

  // ---- one vector-field evaluation of sample b at time tb ----------------------------------------------------
  // Layer 0 reads the stage input z0: with plain loads (written before this launch), or, with `handoff`, as a
  // publication of the group (a barrier wait first, sc1 loads).  The output tile dy[R, 0 .. H-1] lands in sOut.
  // Returns false when a barrier wait gave up.
  // kslab: nullptr, or this evaluation's [L-1, B, n, H] slab of kept hidden outputs (the reverse mode's activation
  // record): the hidden hand-offs go through it instead of the group's double buffer
  auto evaluate = [&](const int b, const float tb, const float* z0, const bool handoff, float* kslab)
      __attribute__((always_inline)) -> bool {
    bool ok = true;
    ROWS_STAMP(0);
    // the lane's indices through an opaque move per evaluation: otherwise every per-lane address and bounds mask
    // of the form and the layers is hoisted out of the enclosing loop and held in registers for the whole kernel
    int tid;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
    const int w = tid >> 6, lane = tid & 63, lo = lane & 15, hi = lane >> 4;
    const int ri = r0 + lo;  // this lane's operand row
    const float* tsb = a.ts + (size_t)b * T;
    int idx;
    float f;
    if (SOLVE != 0 && T <= 64) {  // the knots held in registers for the whole solve (no L2 round trip before the form)
      idx = __popcll(__ballot(lane < T && ts_lane < tb)) - 1;
      idx = idx < 0 ? 0 : (idx > T - 2 ? T - 2 : idx);
      f = tb - __shfl(ts_lane, idx);
    } else {
      idx = interval_index_wave(tsb, T, tb);
      f = tb - tsb[idx];
    }
    using CT_ = typename std::conditional<CBF, uint16_t, float>::type;
    const CT_* cb = reinterpret_cast<const CT_*>(a.coef) + ((size_t)b * (T - 1) + idx) * 4 * nn;

    // ---- form -------------------------------------------------------------------------------------------------
    // Both coefficient reads are unconditional coalesced dwordx4 buffer loads from this (sample, interval)'s four
    // planes (the descriptor's range check zero-fills anything past plane a); values outside the matrix are
    // selected to 0 before they reach LDS, so no load sits in a divergent branch.
    const auto crs = rsrc<UNI>(cb, (unsigned)(4 * nn * sizeof(CT_)));
    const int RS = NP + 4;                 // LDS row stride of the rows block
    float* sAr = big + 2 * NP * kStrip;    // rows block A(t)[R, :] [16][RS], then dA/dt [16][RS]
    // 1. issue the rows block (thread = (row tid / 16, columns 4 (tid % 16) + 64 u): 256 coalesced bytes per row
    //    and u), the column strip and every small load of the form (node-vector plane sums, time channel, data
    //    spline) at once: one memory round trip
    const int rr = tid >> 4;
    // fp32: 4 columns per 16-byte load (row rr = tid / 16, columns 4 (tid % 16) + 64 u, u < 4); bf16: 8 per load
    // (columns 8 (tid % 16) + 128 u, u < 2); the strip the same over the transposed planes
    constexpr int CE = CBF ? 8 : 4, NU = CBF ? 2 : 4;
    const int cq = CE * (tid & 15);
    u32x4 rc[NU][4], sc[NU][4];
    // SOLVE & 8: an evaluation on the interval the cache holds reads the raw loads back from LDS (no memory round
    // trip: the adaptive solve stays on one interval for most of its evaluations)
    const bool fresh = !CCACHE || idx != cidx;
    if (fresh) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
          const int e = (int)(q * nn + (size_t)(r0 + rr) * n + cq + 16 * CE * u);
          if constexpr (CBF) rc[u][q] = load8_bf16(crs, e);
          else rc[u][q] = __builtin_amdgcn_raw_buffer_load_b128(crs, e * 4, 0, 0);
        }
      // the column strip [:, R] = rows R of the transposed planes: the same whole-line pattern as the rows block
      const CT_* cbt = reinterpret_cast<const CT_*>(a.coefT) + ((size_t)b * (T - 1) + idx) * 4 * nn;
      const auto crt = rsrc<UNI>(cbt, (unsigned)(4 * nn * sizeof(CT_)));
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
          const int e = (int)(q * nn + (size_t)(r0 + rr) * n + cq + 16 * CE * u);
          if constexpr (CBF) sc[u][q] = load8_bf16(crt, e);
          else sc[u][q] = __builtin_amdgcn_raw_buffer_load_b128(crt, e * 4, 0, 0);
        }
    } else if constexpr (CCACHE) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rc[u][q] = ccache[((0 * NU + u) * 4 + q) * 256 + tid];
          sc[u][q] = ccache[((1 * NU + u) * 4 + q) * 256 + tid];
        }
    }
    const float* cs = a.csum + ((size_t)b * (T - 1) + idx) * ((size_t)12 * n + 4);
    const int nd = tid < n ? tid : n - 1;  // clamped indices + selects: no load inside a divergent branch
    float pv[3][4], pt[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) pv[kd][q] = cs[(q * 3 + kd) * n + nd];
      pt[q] = cs[12 * n + q];
    }
    const int tr = r0 + (tid & 15) < n ? r0 + (tid & 15) : n - 1;
    const float* tc = a.tcoef + ((size_t)b * (T - 1) + idx) * 3 * n + tr;
    const float tcv[3] = {tc[0], tc[n], tc[2 * n]};
    float dcv[3] = {0.f, 0.f, 0.f};
    if constexpr (MODE >= 2) {
      const size_t blk = (size_t)n * 16;
      const int dr = r0 + rr < n ? r0 + rr : n - 1;
      const float* dc = a.data_coef + ((size_t)b * (T - 1) + idx) * 4 * blk + (size_t)dr * 16 + (tid & 15);
      dcv[0] = dc[0];
      dcv[1] = dc[blk];
      dcv[2] = dc[2 * blk];
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int c0 = cq + 16 * CE * u;
      if (c0 < NP)
#pragma unroll
        for (int e = 0; e < CE; ++e) {
          const bool in = r0 + rr < n && c0 + e < n;
          const float cc[4] = {coef_el<CBF>(rc[u][0], e), coef_el<CBF>(rc[u][1], e), coef_el<CBF>(rc[u][2], e),
                               coef_el<CBF>(rc[u][3], e)};
          sAr[rr * RS + c0 + e] = in ? cubic(cc, f) : 0.f;
          sAr[(16 + rr) * RS + c0 + e] = in ? dcubic(cc, f) : 0.f;
        }
    }
    ROWS_STAMP(15);
    if constexpr (CCACHE) {
      if (fresh) {  // keep this interval's raw loads (thread-private slots)
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            ccache[((0 * NU + u) * 4 + q) * 256 + tid] = rc[u][q];
            ccache[((1 * NU + u) * 4 + q) * 256 + tid] = sc[u][q];
          }
        cidx = idx;
      }
    }
    {  // 2. the column strip: Horner of transposed row rr (= column r0 + rr), element kk = node; LDS [node][column]
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int c0 = cq + 16 * CE * u;
        if (c0 < NP)
#pragma unroll
          for (int e = 0; e < CE; ++e) {
            const int kk = c0 + e;
            const bool in = r0 + rr < n && kk < n;
            const float cc[4] = {coef_el<CBF>(sc[u][0], e), coef_el<CBF>(sc[u][1], e), coef_el<CBF>(sc[u][2], e),
                                 coef_el<CBF>(sc[u][3], e)};
            big[kk * kStrip + rr] = in ? cubic(cc, f) : 0.f;
            big[(NP + kk) * kStrip + rr] = in ? dcubic(cc, f) : 0.f;
          }
      }
    }
    // 3. node vectors at t from the per-plane sums (thread = node), the layers' families; tg and dX of the rows
    {
      const bool nin = tid < n;
      const float r = nin ? cubic(pv[0], f) : 0.f, rd = nin ? dcubic(pv[0], f) : 0.f;
      const float c = nin ? cubic(pv[1], f) : 0.f, cd = nin ? dcubic(pv[1], f) : 0.f;
      const float dg = cubic(pv[2], f), dgd = dcubic(pv[2], f);
      const float s = cubic(pt, f), sd = dcubic(pt, f);
      const bool row = tid >= r0 && tid < r0 + kRB && nin;
      for (int l = 0; l < L; ++l) {
        const float* fc = a.fusion + l * GNCDE_FC;
        if (tid < NP)
          sV[l * NP + tid] = fc[GNCDE_FC_VR_A] * r + fc[GNCDE_FC_VR_DA] * rd + fc[GNCDE_FC_VC_A] * c +
                             fc[GNCDE_FC_VC_DA] * cd;
        if (row) {
          const int t = tid - r0;
          const float wv = fc[GNCDE_FC_WR_A] * r + fc[GNCDE_FC_WR_DA] * rd + fc[GNCDE_FC_WC_A] * c +
                           fc[GNCDE_FC_WC_DA] * cd + fc[GNCDE_FC_WS_A] * s + fc[GNCDE_FC_WS_DA] * sd;
          const float uv = fc[GNCDE_FC_IDC] + fc[GNCDE_FC_UD_A] * dg + fc[GNCDE_FC_UD_DA] * dgd + fc[GNCDE_FC_UR_A] * r +
                           fc[GNCDE_FC_UR_DA] * rd + fc[GNCDE_FC_UC_A] * c + fc[GNCDE_FC_UC_DA] * cd +
                           fc[GNCDE_FC_US_A] * s + fc[GNCDE_FC_US_DA] * sd;
          // q_l[i] = sum_k (I + Abar_l)[i][k]: dense terms -> row / column sums, w family n copies, v family
          // sum_k v_k (sum r = sum c = s), the diagonal once
          float qv = fc[GNCDE_FC_E_A] * r + fc[GNCDE_FC_E_DA] * rd + fc[GNCDE_FC_ET_A] * c + fc[GNCDE_FC_ET_DA] * cd;
          qv += (float)n * wv;
          qv += (fc[GNCDE_FC_VR_A] + fc[GNCDE_FC_VC_A]) * s + (fc[GNCDE_FC_VR_DA] + fc[GNCDE_FC_VC_DA]) * sd;
          qv += uv;
          sRow[l * 16 + t] = wv;
          sRow[(L + l) * 16 + t] = uv;
          sRow[(2 * L + l) * 16 + t] = qv;
        }
      }
      if (tid < 16) sTg[tid] = r0 + tid < n ? fmaf(f, fmaf(3.0f * f, tcv[0], 2.0f * tcv[1]), tcv[2]) : 0.f;
      if (MODE >= 2)
        sDx[rr * kStrip + (tid & 15)] = r0 + rr < n ? fmaf(f, fmaf(3.0f * f, dcv[0], 2.0f * dcv[1]), dcv[2]) : 0.f;
    }
    __syncthreads();
    ROWS_STAMP(1);
    // the product's A-operand elements of this lane: (I + Abar)[ri][k] needs A, dA at (ri, k) and at (k, ri), for
    // k = KW kc + EL hi + e, kc = w + 4 j (chunks past the matrix read zeros)
    float Ar[NJ][EL], dAr[NJ][EL], At[NJ][EL], dAt[NJ][EL];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int kc = w + 4 * j, k0 = KW * kc + EL * hi;
      const bool in = kc < nch;
#pragma unroll
      for (int e4 = 0; e4 < EL; e4 += 4) {
        const floatx4 ar = in ? *reinterpret_cast<const floatx4*>(sAr + lo * RS + k0 + e4) : floatx4{0.f, 0.f, 0.f, 0.f};
        const floatx4 dr =
            in ? *reinterpret_cast<const floatx4*>(sAr + (16 + lo) * RS + k0 + e4) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          Ar[j][e4 + e] = ar[e];
          dAr[j][e4 + e] = dr[e];
        }
      }
#pragma unroll
      for (int e = 0; e < EL; ++e) {
        At[j][e] = in ? big[(k0 + e) * kStrip + lo] : 0.f;
        dAt[j][e] = in ? big[(NP + k0 + e) * kStrip + lo] : 0.f;
      }
    }
    __syncthreads();  // the strip's region becomes Z_l
    ROWS_STAMP(2);

    // ---- layers --------------------------------------------------------------------------------------------
    // Z_l -> LDS (a stage input written before this launch with plain loads; a publication of the group with sc1
    // loads after the barrier) and the RMSNorm factors of its rows
    const int zslot = SOLVE != 0 ? b : g;  // the group's hand-off buffers (solve: one group per sample)
    auto load_z = [&](int l) __attribute__((always_inline)) {
      float* Zs = big;
      constexpr int G4 = H / 4, U = 8;
      const int tot = NP * G4, valid = n * G4;
      bool gave = false;
      if (l == 0 && !handoff) {
        const floatx4* Z4 = reinterpret_cast<const floatx4*>(z0);
        for (int e0 = tid; e0 < tot; e0 += 256 * U) {
          floatx4 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int e = e0 + 256 * u;
            v[u] = e < valid ? Z4[e] : floatx4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int e = e0 + 256 * u;
            if (e < tot) *reinterpret_cast<floatx4*>(Zs + (e / G4) * ZS + 4 * (e % G4)) = v[u];
          }
        }
      } else if constexpr (GRAN) {  // the group's latest publication (stage input or hidden output)
        gave = !gran_load(Zs, hseq - 1);
      } else {
        ok = wait_all() && ok;
        // publications alternate buffers, so a buffer is rewritten only after a barrier that every reader of its
        // previous contents has passed
        const float* zin = l == 0 ? z0
                         : kslab ? kslab + ((size_t)(l - 1) * a.B + b) * zgroup
                                          : a.zbuf[(pub - 1) & 1] + (size_t)zslot * zgroup;
        const auto rs = rsrc<UNI>(zin, (unsigned)(zgroup * sizeof(float)));
        for (int e0 = tid; e0 < tot; e0 += 256 * U) {
          floatx4 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int e = e0 + 256 * u;
            v[u] = e < valid ? __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, e * 16, 0, 16))
                             : floatx4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int e = e0 + 256 * u;
            if (e < tot) *reinterpret_cast<floatx4*>(Zs + (e / G4) * ZS + 4 * (e % G4)) = v[u];
          }
        }
      }
      if (__syncthreads_or(gave ? 1 : 0)) ok = false;
      for (int r = tid; r < NP; r += 256) {
        float ss = 0.f;
#pragma unroll
        for (int q = 0; q < G4; ++q) {
          const floatx4 z = *reinterpret_cast<const floatx4*>(Zs + r * ZS + 4 * q);
          ss = fmaf(z.x, z.x, fmaf(z.y, z.y, fmaf(z.z, z.z, fmaf(z.w, z.w, ss))));
        }
        sInv[r] = r < n ? rms_inv(ss, 1.0f / (float)H) : 0.f;
      }
      __syncthreads();
    };
    // P = (I + Abar_l)[R, :] diag(inv) Z_l, the operand built in registers per 16-column chunk; the four K parts
    // land in LDS (aliasing Z_l)
    auto product = [&](int l) __attribute__((always_inline)) {
      const float* Zs = big;
      const float* fc = a.fusion + l * GNCDE_FC;
      const float eA = fc[GNCDE_FC_E_A], edA = fc[GNCDE_FC_E_DA], eTA = fc[GNCDE_FC_ET_A], eTdA = fc[GNCDE_FC_ET_DA];
      const float wl = sRow[l * 16 + lo], ul = sRow[(L + l) * 16 + lo];
      floatx4 acc[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int kc = w + 4 * j;
        if (kc >= nch) break;
        const int k0 = KW * kc + EL * hi;
        float vk[EL], iv[EL];
#pragma unroll
        for (int e4 = 0; e4 < EL; e4 += 4) {
          const floatx4 v4 = *reinterpret_cast<const floatx4*>(sV + l * NP + k0 + e4);
          const floatx4 i4 = *reinterpret_cast<const floatx4*>(sInv + k0 + e4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            vk[e4 + e] = v4[e];
            iv[e4 + e] = i4[e];
          }
        }
        float op[EL];
#pragma unroll
        for (int e = 0; e < EL; ++e) {
          float v = fmaf(eA, Ar[j][e], fmaf(edA, dAr[j][e], fmaf(eTA, At[j][e], fmaf(eTdA, dAt[j][e], wl + vk[e]))));
          if (k0 + e == ri) v += ul;
          op[e] = v * iv[e];
        }
        if constexpr (BF) {
          bf16x8 av;
#pragma unroll
          for (int e = 0; e < 8; ++e) av[e] = (__bf16)op[e];
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            bf16x8 bv;  // Z_l column 16 ct + lo, rows k0 .. k0 + 7
#pragma unroll
            for (int e = 0; e < 8; ++e) bv[e] = (__bf16)Zs[(k0 + e) * ZS + 16 * ct + lo];
            acc[ct] = mfma_bf(av, bv, acc[ct]);
          }
        } else {
          float bz[EL][CT];
#pragma unroll
          for (int e = 0; e < EL; ++e)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) bz[e][ct] = Zs[(k0 + e) * ZS + 16 * ct + lo];
#pragma unroll
          for (int e = 0; e < EL; ++e)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) acc[ct] = mfma4(op[e], bz[e][ct], acc[ct]);
        }
      }
      __syncthreads();  // every Z_l read done: the partials alias it
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) big[(w * 16 + 4 * hi + r) * ZS + 16 * ct + lo] = acc[ct][r];
      __syncthreads();
    };
    // P row lo, columns 16 cc + 4 hi .. + 3: the four K parts in a fixed order
    auto psum4 = [&](int c) -> floatx4 {
      const float* p = big + lo * ZS + c;
      floatx4 v = *reinterpret_cast<const floatx4*>(p);
#pragma unroll
      for (int kp = 1; kp < 4; ++kp) v += *reinterpret_cast<const floatx4*>(p + kp * 16 * ZS);
      return v;
    };
    auto prow = [&](int cc) -> floatx4 { return psum4(16 * cc + 4 * hi); };
    // bf16: P[lo][32 cc + 8 hi .. + 7] (zero past H) as the A operand of a 16x16x32 step
    auto prow8 = [&](int cc, float (&x)[8]) {
      const int c0 = 32 * cc + 8 * hi;
      const bool in = c0 < H;
      const floatx4 p0 = psum4(in ? c0 : 0), p1 = psum4(in ? c0 + 4 : 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = in ? p0[e] : 0.f;
        x[4 + e] = in ? p1[e] : 0.f;
      }
    };
    auto prow_bf = [&](int cc) -> bf16x8 {
      float x[8];
      prow8(cc, x);
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)x[e];
      return v;
    };
    // a bf16 W' operand: row r of the natural [rows, H] layout, columns 32 cc + 8 hi .. + 7 (zero past H)
    auto wrow_bf = [&](const uint16_t* Wl, int r, int cc) -> bf16x8 {
      const int c0 = 32 * cc + 8 * hi;
      u32x4 u = {0u, 0u, 0u, 0u};
      if (c0 < H) u = *reinterpret_cast<const u32x4*>(Wl + (size_t)r * H + c0);
      return __builtin_bit_cast(bf16x8, u);
    };
    // P W'^T + q b'^T for output tile `tile` (rows R, columns 16 tile + lo): acc[r] = row 4 hi + r
    auto linear = [&](int l, int tile) __attribute__((always_inline)) -> floatx4 {
      floatx4 accL = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {
        const uint16_t* Wl = a.wbf + (size_t)l * H * H;
#pragma unroll
        for (int cc = 0; cc < KC; ++cc) accL = mfma_bf(prow_bf(cc), wrow_bf(Wl, 16 * tile + lo, cc), accL);
      } else {
        const floatx4* W4 = reinterpret_cast<const floatx4*>(a.wperm + (size_t)l * H * H);
#pragma unroll
        for (int cc = 0; cc < CT; ++cc) {
          const floatx4 pv = prow(cc), wv = W4[(tile * CT + cc) * 64 + lane];
#pragma unroll
          for (int s = 0; s < 4; ++s) accL = mfma4(pv[s], wv[s], accL);
        }
      }
      const float bc = a.bf[l * H + 16 * tile + lo];
      const float* qrow = sRow + (2 * L + l) * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) accL[r] = fmaf(qrow[4 * hi + r], bc, accL[r]);
      return accL;
    };

    for (int l = 0; l + 1 < L; ++l) {  // hidden layers: Z_{l+1}[R] = relu(P W'^T + q b'^T), published to the group
      load_z(l);
      ROWS_STAMP(3 + 3 * l);
      product(l);
      ROWS_STAMP(4 + 3 * l);
      for (int tile = w; tile < CT; tile += 4) {
        const floatx4 v = linear(l, tile);
#pragma unroll
        for (int r = 0; r < 4; ++r) sOut[(4 * hi + r) * ZS + 16 * tile + lo] = fmaxf(v[r], 0.f);
      }
      __syncthreads();
      constexpr int G4 = H / 4;
      if constexpr (GRAN) {  // the rows as tagged granules (and, recording, as plain floats into the slab)
        const unsigned tag = hseq + 1;
        const auto rg = gran_rsrc(hseq, b);
        const auto rk = rsrc<UNI>(kslab ? kslab + ((size_t)l * a.B + b) * zgroup : a.zbuf[0], (unsigned)(zgroup * 4));
        if (tid < 16 * G4) {
          const int R = tid / G4, q = tid % G4;
          if (r0 + R < n) {
            const floatx4 v = *reinterpret_cast<const floatx4*>(sOut + R * ZS + 4 * q);
            gran_store4(rg, (r0 + R) * H + 4 * q, v, tag);
            if (kslab)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rk, ((r0 + R) * H + 4 * q) * 4, 0, 0);
          }
        }
        ++hseq;
        __syncthreads();  // the output tile is read before the next layer's staging rewrites the region
      } else {
        // (an idle round keeps to its group's own buffers: the sample it recomputes is another group's)
        float* zout = kslab ? kslab + ((size_t)l * a.B + b) * zgroup : a.zbuf[pub & 1] + (size_t)zslot * zgroup;
        const auto rs = rsrc<UNI>(zout, (unsigned)(zgroup * sizeof(float)));
        if (tid < 16 * G4) {  // write-through 16-byte stores of this workgroup's rows, then one arrival
          const int R = tid / G4, q = tid % G4;
          if (r0 + R < n)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(u32x4, *reinterpret_cast<const floatx4*>(sOut + R * ZS + 4 * q)), rs,
                ((r0 + R) * H + 4 * q) * 4, 0, 16);
        }
        arrive();  // its barrier also orders the partials' reuse by the next layer
      }
      ROWS_STAMP(5 + 3 * l);
    }
    {  // the output layer
      const int l = L - 1;
      // CDE: this wave's whole read-out weight slice (16 KB at h = 32) is requested before the barrier wait, the
      // Z load and the product, so the L2 / MALL latency of W' (cold in every launch) hides behind them
      constexpr int KP = MODE == 2 ? 4 / CT : 1, JP = 16 / KP;
      const int ct = w % CT, kp = w / CT, j0 = kp * JP;
      const floatx4* W4 = reinterpret_cast<const floatx4*>(a.wperm + (size_t)l * H * H);
      constexpr bool F32R = MODE == 2 && !BF, BFR = MODE == 2 && BF;
      // (the persistent solve requests its slice after the product instead: held across the barrier wait, its 64
      // VGPRs push the solve's stage values into scratch; its W' is L2-resident across the evaluations)
      constexpr bool PREF = F32R && SOLVE == 0;
      floatx4 wv[F32R ? CT : 1][F32R ? JP : 1];
      // bf16: W'[16 m + j, 32 cc + 8 hi ..], m = 16 ct + lo; at H = 64 the first K chunk (64 VGPRs) is prefetched,
      // the second is requested after the product
      constexpr int KPF = H == 64 ? 1 : KC;
      bf16x8 wb[BFR ? KC : 1][BFR ? JP : 1];
      auto load_wv = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int cc = 0; cc < CT; ++cc)
#pragma unroll
          for (int j = 0; j < JP; ++j) wv[cc][j] = W4[((ct * 16 + j0 + j) * CT + cc) * 64 + lane];
      };
      if constexpr (PREF) load_wv();
      if constexpr (BFR)
#pragma unroll
        for (int cc = 0; cc < KPF; ++cc)
#pragma unroll
          for (int j = 0; j < JP; ++j) wb[cc][j] = wrow_bf(a.wbf + (size_t)l * H * H, 16 * (16 * ct + lo) + j0 + j, cc);
      load_z(l);
      ROWS_STAMP(12);
      product(l);
      if constexpr (F32R && !PREF) load_wv();
      ROWS_STAMP(13);
      if constexpr (MODE == 1) {  // ODE: dy[R] = tg (P W'^T + q b'^T)
        for (int tile = w; tile < CT; tile += 4) {
          const floatx4 v = linear(l, tile);
#pragma unroll
          for (int r = 0; r < 4; ++r) sOut[(4 * hi + r) * ZS + 16 * tile + lo] = v[r] * sTg[4 * hi + r];
        }
      } else {
        // CDE read-out: dy[R, m] = tg (sum_{c, j} P[., c] dX[., j] W'[16 m + j, c] + q sum_j b'[16 m + j] dX[., j])
        const float* bl = a.bf + (size_t)l * H;
        const float* qrow = sRow + (2 * L + l) * 16;
        float dxr[JP];
#pragma unroll
        for (int j = 0; j < JP; ++j) dxr[j] = sDx[lo * kStrip + j0 + j];
        // even / odd j accumulate into two independent chains (the MFMA result latency is not exposed per j)
        floatx4 acc2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        if constexpr (BF) {
#pragma unroll
          for (int cc = KPF; cc < KC; ++cc)
#pragma unroll
            for (int j = 0; j < JP; ++j) wb[cc][j] = wrow_bf(a.wbf + (size_t)l * H * H, 16 * (16 * ct + lo) + j0 + j, cc);
#pragma unroll
          for (int cc = 0; cc < KC; ++cc) {
            float pf[8];
            prow8(cc, pf);
#pragma unroll
            for (int j = 0; j < JP; ++j) {
              bf16x8 av;
#pragma unroll
              for (int e = 0; e < 8; ++e) av[e] = (__bf16)(pf[e] * dxr[j]);
              acc2[j & 1] = mfma_bf(av, wb[cc][j], acc2[j & 1]);
            }
          }
        } else {
#pragma unroll
          for (int cc = 0; cc < CT; ++cc) {
            const floatx4 pv = prow(cc);
#pragma unroll
            for (int j = 0; j < JP; ++j) {
              const floatx4 av = pv * dxr[j];
#pragma unroll
              for (int s = 0; s < 4; ++s) acc2[j & 1] = mfma4(av[s], wv[cc][j][s], acc2[j & 1]);
            }
          }
        }
        floatx4 acc = acc2[0] + acc2[1];
        const int m = 16 * ct + lo;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 4 * hi + r;
          float sb = 0.f;
#pragma unroll
          for (int j = 0; j < JP; ++j) sb = fmaf(bl[16 * m + j0 + j], sDx[R * kStrip + j0 + j], sb);
          acc[r] = fmaf(qrow[R], sb, acc[r]);
        }
        if constexpr (KP > 1) {
          red[w * 64 + lane] = acc;
          __syncthreads();
          if (kp == 0)
#pragma unroll
            for (int p = 1; p < KP; ++p) acc += red[(w + p * CT) * 64 + lane];
        }
        if (kp == 0)
#pragma unroll
          for (int r = 0; r < 4; ++r) sOut[(4 * hi + r) * ZS + m] = sTg[4 * hi + r] * acc[r];
      }
      __syncthreads();  // the output tile is complete; P (aliasing Z_l) and the LDS vectors are free again
      ROWS_STAMP(14);
    }
    return ok;
  };

  if constexpr (SOLVE == 0) {
    for (int it = 0; it < a.rounds; ++it) {
      const int bs = g + it * a.G;
      const bool live = bs < a.B;
      const int b = live ? bs : a.B - 1;  // an idle round computes on a valid sample, keeps its barriers, stores no dy
      evaluate(b, a.t[b], a.y + (size_t)b * zgroup, false, live ? a.keep : nullptr);
      // dy rows R: 16-byte stores of the output tile
      constexpr int G4 = H / 4;
      const int tid = threadIdx.x;
      if (live && tid < 16 * G4) {
        const int R = tid / G4, q = tid % G4;
        if (r0 + R < n)
          *reinterpret_cast<floatx4*>(a.dy + ((size_t)b * n + r0 + R) * H + 4 * q) =
              *reinterpret_cast<const floatx4*>(sOut + R * ZS + 4 * q);
      }
      __syncthreads();  // sOut is rewritten by the next round
    }
  } else {
    // ---- the persistent Tsit5 + PIDController solve of sample g (gncde_pid.hip's k_pid_advance state machine,
    // graph_neural_cde.py:94-104 semantics): every workgroup of the group runs the controller redundantly on
    // identical inputs (the group sums are added in row-block order by everyone), so all take the same decisions.
    // A batch larger than the resident groups runs as ONE launch: a group that finishes its sample takes the next
    // one from a queue (its first workgroup draws it, the others read the group's mailbox), so the batch's cost is
    // its total work over the groups, not the sum of per-chunk maxima (the slowest sample of every chunk).
    for (unsigned asg = 1;; ++asg) {
    const SolveArgs& s = a.s;
    const int b = g;
    const int tid = threadIdx.x;
    // a thread owns 4 consecutive elements of the 16 x H row tile (threads < 4H), kept in registers all solve
    const int orow = (4 * tid) / H, ocol = (4 * tid) % H;
    const bool mine = tid < 4 * H && r0 + orow < n;
    const size_t oel = ((size_t)b * n + r0 + orow) * H + ocol;
    const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
    const float rtol = s.rtol, atol = s.atol;
    constexpr bool GRIDC = (SOLVE & 3) == 2;  // the controller, fixed per instance (one evaluation call site each)
    const float t0 = GRIDC ? 0.f : s.t0[b], t1 = GRIDC ? 0.f : s.t1[b];
    const float inv_cnt = 1.0f / (float)(n * H);
    const size_t E = (size_t)n * H;
    floatx4 y = mine ? *reinterpret_cast<const floatx4*>(s.y0 + oel) : zero;
    floatx4 y1 = zero, kk[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) kk[j] = zero;
    // the stage input of the next evaluation, published to the group as tagged granules
    auto publish = [&](const floatx4 u) {
      if constexpr (GRAN) {
        if (mine) gran_store4(gran_rsrc(hseq, b), (r0 + orow) * H + ocol, u, hseq + 1);
        ++hseq;
        __syncthreads();  // every thread has taken its K from the output tile before the next form rewrites it
      } else {  // sc1 16-byte stores + one arrival
        if (mine)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, u),
                                                 rsrc<UNI>(a.zbuf[pub & 1] + (size_t)b * zgroup, (unsigned)(E * 4)),
                                                 (int)(((r0 + orow) * H + ocol) * 4), 0, 16);
        arrive();
      }
    };
    // (sum of v0, sum of v1) over the group's rows, from each thread's 4-element chunk partials (fma chains from 0)
    // in the CANONICAL order the host-paced controller uses too (gncde_pid.hip canon_sumsq): a row sums its chunks in
    // order, the workgroup its rows in order (published as the row block's partial), and every workgroup adds the nb
    // partials in row-block order — so both controllers take bitwise the same decisions
    float* sr = reinterpret_cast<float*>(red);  // free between evaluations: [2][4H] chunk partials, [2][16] row sums
    auto group_sum2 = [&](float v0, float v1, float& s0, float& s1) -> bool {
      constexpr int CH = H / 4;  // chunks per row
      float* rsum = sr + 8 * H;
      if (tid < 4 * H) {
        sr[tid] = v0;
        sr[4 * H + tid] = v1;
      }
      __syncthreads();
      if (tid < 32) {
        const float* c = sr + (tid >> 4) * 4 * H + (tid & 15) * CH;
        float q = c[0];
#pragma unroll
        for (int j = 1; j < CH; ++j) q += c[j];
        rsum[tid] = q;
      }
      __syncthreads();
      float* part = s.part + (size_t)(2 * b + (pub & 1)) * nb * 2;
      if (tid == 0) {
        const int nr = n - r0 < kRB ? n - r0 : kRB;
        float p0 = rsum[0], p1 = rsum[16];
        for (int r = 1; r < nr; ++r) {
          p0 += rsum[r];
          p1 += rsum[16 + r];
        }
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, floatx2{p0, p1}),
                                              rsrc<UNI>(part, (unsigned)(nb * 8)), rb * 8, 0, 16);
      }
      arrive();
      const bool ok = wait_all();
      const auto rs = rsrc<UNI>(part, (unsigned)(nb * 8));
      float a0 = 0.f, a1 = 0.f;
      for (int q = 0; q < nb; ++q) {
        const floatx2 v = __builtin_bit_cast(floatx2, __builtin_amdgcn_raw_buffer_load_b64(rs, q * 8, 0, 16));
        a0 += v.x;
        a1 += v.y;
      }
      // every lane holds the same sums: as scalars, the controller's decisions (and everything they steer: the hand-off
      // counters, the sample's buffers) stay uniform to the compiler, so no buffer access needs a waterfall loop
      if constexpr (UNI) {
        s0 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, a0)));
        s1 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, a1)));
      } else {
        s0 = a0;
        s1 = a1;
      }
      return ok;
    };
    int steps = 0, rejects = 0, evals = 0, status = 0;
    bool fault = false;
    // ONE evaluation call site (the evaluation body is large: a second inlined copy costs registers); each
    // controller is a step function that takes the evaluation's K, publishes the next stage input and returns
    // false, or returns true when the sample is done.
    floatx4 K = zero;

    // ---- a fixed step grid (GRID controller: RK4, or Tsit5 at ConstantStepSize): the generic path's arithmetic
    // (gncde_generic.hip generic_integrate: k_combo's summation order, stage times), SaveAt(t1) or every step, and
    // the stage record the reverse sweep reads (GncdeSolver.stage_rec)
    const int Gl = s.G;
    const float* gr = GRIDC ? s.grid + (size_t)b * Gl : nullptr;
    int ns = GRIDC ? s.nsteps[b] : 0;
    ns = ns < 0 ? 0 : (ns > Gl - 1 ? Gl - 1 : ns);
    const bool rk4 = s.method == GNCDE_RK4;
    const int S1 = rk4 ? 3 : 5;  // recorded stage inputs per step
    const size_t own = oel - (size_t)b * E;
    auto save_col = [&](int k) {
      if (s.save_steps && mine) *reinterpret_cast<floatx4*>(s.ys + ((size_t)b * Gl + k) * E + own) = y;
    };
    // PID (GncdeSolver.pid_ckpt, ABI 8): the accepted-step record — slot k holds step k's starting state, its stage
    // inputs U_1 .. U_5 and the kept hidden outputs of its six stage evaluations (stage 0 = the FSAL evaluation of
    // step k - 1); an attempt writes the slot of the step it tries, so a rejected attempt's slot is rewritten by the
    // retry; slots >= R are not written (the caller then replays the accepted grid)
    float* kslab = nullptr;  // the next evaluation's kept-output slab
    const size_t aslab = (size_t)(a.L - 1) * a.B * E;
    auto pid_slab = [&](int k, int i) -> float* {
      return !GRIDC && s.arec && k < s.R ? s.arec + ((size_t)k * 6 + i) * aslab : nullptr;
    };
    auto pid_record = [&](int k, int i, const floatx4 u) {  // U_i of step k -> slot (k, i - 1)
      if (!GRIDC && s.rec && mine && k < s.R)
        *reinterpret_cast<floatx4*>(s.rec + (((size_t)b * s.R + k) * 5 + i - 1) * E + own) = u;
    };
    auto pid_ckpt = [&](int k) {
      if (!GRIDC && s.ckpt && mine && k < s.R) *reinterpret_cast<floatx4*>(s.ckpt + ((size_t)b * s.R + k) * E + own) = y;
    };
    auto record = [&](int k, int i, const floatx4 u) {  // stage input U_i of step k -> slot (k, i - 1)
      if (s.rec && mine) *reinterpret_cast<floatx4*>(s.rec + (((size_t)b * (Gl - 1) + k) * S1 + i - 1) * E + own) = u;
    };
    int gk = 0;
    // the PID controller's state (graph_neural_cde.py:94-104 semantics)
    int phase = 0, st = 0, si = 0;
    float t = t0, tn = t0, h = 0.f, dt = 0.f, h0 = 0.f, d1 = 0.f, tst = t0;
    const float* sts = s.S > 0 ? s.save_ts + (size_t)b * s.S : nullptr;

    auto grid_step = [&]() -> bool {
      if (rk4) {
        if (st < 3) {  // k1 .. k3 evaluated: y + h (0.5 k1 | 0.5 k2 | k3)
          const float cf = st < 2 ? 0.5f : 1.0f;
          floatx4 u;
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = fmaf(h, fmaf(cf, K[e], 0.f), y[e]);
          record(gk, st + 1, u);
          publish(u);
          tst = stage_time(t, cf, h);
          ++st;
          return false;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // y + h/6 (k1 + 2 k2 + 2 k3 + k4)
          float acc = fmaf(1.0f / 6.0f, kk[0][e], 0.f);
          acc = fmaf(2.0f / 6.0f, kk[1][e], acc);
          acc = fmaf(2.0f / 6.0f, kk[2][e], acc);
          acc = fmaf(1.0f / 6.0f, kk[3][e], acc);
          y[e] = fmaf(h, acc, y[e]);
        }
        ++gk;
        save_col(gk);
        if (gk >= ns) return true;
        t = gr[gk];
        h = gr[gk + 1] - t;
        tst = t;
        st = 0;
        publish(y);
        return false;
      }
      if (st == 6) {  // y1 accepted; its evaluation is the next step's k1 (FSAL)
        y = y1;
        kk[0] = K;
        ++gk;
        save_col(gk);
        st = 0;
      }
      if (gk >= ns) return true;
      if (st == 0) {
        t = gr[gk];
        h = gr[gk + 1] - t;
      }
      const int ns1 = st + 1;
      float ar[6], cst;
      tsit5_row(ns1, ar, cst);
      floatx4 u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 6; ++j) acc = j < ns1 ? fmaf(ar[j], kk[j][e], acc) : acc;
        u[e] = fmaf(h, acc, y[e]);
      }
      if (ns1 <= 5) record(gk, ns1, u);
      else y1 = u;
      publish(u);
      tst = ns1 == 6 ? gr[gk + 1] : stage_time(t, cst, h);  // the FSAL stage at the step's end knot
      st = ns1;
      return false;
    };

    auto pid_step = [&]() -> bool {
      bool start = false;
      if (phase == 0) {
        kk[0] = K;
        phase = 2;
        if (s.auto_dt) {  // Hairer's initial step (diffrax dt0 = None): d0 = rms(y0 / sc), d1 = rms(f0 / sc)
          float p0 = 0.f, p1 = 0.f;
          if (mine)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float sc = fmaf(fabsf(y[e]), rtol, atol);
              const float u = y[e] / sc, v = K[e] / sc;
              p0 = fmaf(u, u, p0);
              p1 = fmaf(v, v, p1);
            }
          float P0, P1;
          if (!group_sum2(p0, p1, P0, P1)) {
            fault = true;
            return true;
          }
          const float d0 = sqrtf(P0 * inv_cnt);
          d1 = sqrtf(P1 * inv_cnt);
          h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : 0.01f * (d0 / d1);
          floatx4 u;
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = fmaf(h0, K[e], y[e]);
          kslab = nullptr;  // (the heuristic's evaluation is not part of the solve)
          publish(u);
          tst = t0 + h0;
          phase = 1;
          return false;
        }
        start = true;
      } else if (phase == 1) {  // f(t0 + h0, y0 + h0 f0): d2 and the first step
        float p2 = 0.f;
        if (mine)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sc = fmaf(fabsf(y[e]), rtol, atol);
            const float v = (K[e] - kk[0][e]) / sc;
            p2 = fmaf(v, v, p2);
          }
        float P2, unused;
        if (!group_sum2(p2, 0.f, P2, unused)) {
          fault = true;
          return true;
        }
        const float d2 = sqrtf(P2 * inv_cnt) / h0;
        const float md = fmaxf(d1, d2);
        const float h1 = md <= 1e-15f ? fmaxf(1e-6f, h0 * 1e-3f) : powf(0.01f / md, 0.2f);
        dt = fminf(100.0f * h0, h1);
        phase = 2;
        start = true;
      } else if (st < 6) {  // stage st (1 .. 5) of the attempt evaluated: the next stage's input
#pragma unroll
        for (int j = 1; j < 6; ++j)
          if (j == st) kk[j] = K;
        const int ns1 = st + 1;
        float ar[6], cst;
        tsit5_row(ns1, ar, cst);
        floatx4 u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float acc = 0.f;  // k_pid_advance's summation order
#pragma unroll
          for (int j = 0; j < 6; ++j) acc = j < ns1 ? fmaf(ar[j], kk[j][e], acc) : acc;
          u[e] = fmaf(h, acc, y[e]);
        }
        if (ns1 == 6) {
          y1 = u;  // the FSAL stage's input is the step's candidate solution
          kslab = pid_slab(steps + 1, 0);  // its evaluation is stage 0 of the next step, if this one is accepted
        } else {
          pid_record(steps, ns1, u);
          kslab = pid_slab(steps, ns1);
        }
        publish(u);
        tst = ns1 == 6 ? tn : ns1 == 5 ? __fadd_rn(t, h) : stage_time(t, cst, h);  // FSAL stage at the step end
        st = ns1;
        return false;
      } else {  // the attempt is complete: K = f(tn, y1); embedded error, accept / reject, next step size
        float pe = 0.f;
        if (mine)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float err = h * (TSIT5_E1 * kk[0][e] + TSIT5_E2 * kk[1][e] + TSIT5_E3 * kk[2][e] +
                                   TSIT5_E4 * kk[3][e] + TSIT5_E5 * kk[4][e] + TSIT5_E6 * kk[5][e] + TSIT5_E7 * K[e]);
            const float sc = fmaf(fmaxf(fabsf(y[e]), fabsf(y1[e])), rtol, atol);
            const float v = err / sc;
            pe = fmaf(v, v, pe);
          }
        float PE, unused;
        if (!group_sum2(pe, 0.f, PE, unused)) {
          fault = true;
          return true;
        }
        const float err = sqrtf(PE * inv_cnt);
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
          while (si < s.S && sts[si] <= tn) {  // dense output inside (t, tn]
            float wts[7];
            tsit5_dense((sts[si] - t) / h, wts);
            if (mine) {
              floatx4 o;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float acc = 0.f;
#pragma unroll
                for (int j = 0; j < 6; ++j) acc = fmaf(wts[j], kk[j][e], acc);
                acc = fmaf(wts[6], K[e], acc);
                o[e] = fmaf(h, acc, y[e]);
              }
              *reinterpret_cast<floatx4*>(s.ys + ((size_t)b * s.S + si) * E + (oel - (size_t)b * E)) = o;
            }
            ++si;
          }
          y = y1;
          kk[0] = K;  // FSAL
          if (rb == 0 && tid == 0 && s.step_ts && steps + 1 < s.step_len)
            s.step_ts[(size_t)b * s.step_len + steps + 1] = tn;
          t = tn;
          ++steps;
        } else {
          ++rejects;
        }
        dt = factor * h;
        st = 0;
        start = true;
      }
      if (start) {  // begin the next attempt, or finish
        bool finish = false;
        if (!(t < t1)) {
          finish = true;
        } else if (steps + rejects >= s.max_steps) {
          status = 1;
          finish = true;
        }
        if (finish) {
          if (s.step_ts && status == 0 && steps + 1 > s.step_len) status = 3;  // step record truncated
          pid_ckpt(steps);  // the final state
          if (mine) {
            if (s.S == 0) *reinterpret_cast<floatx4*>(s.ys + oel) = y;
            for (int q = si; q < s.S; ++q)  // SAVE_TS: only on failure
              *reinterpret_cast<floatx4*>(s.ys + ((size_t)b * s.S + q) * E + (oel - (size_t)b * E)) = y;
          }
          return true;
        }
        tn = t + dt;
        if (tn > t1 - 1e-6f) tn = t1;  // diffrax _clip_to_end
        h = tn - t;
        floatx4 u;
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = fmaf(h, fmaf(TSIT5_A21, kk[0][e], 0.f), y[e]);
        pid_ckpt(steps);
        pid_record(steps, 1, u);
        kslab = pid_slab(steps, 1);
        publish(u);
        tst = stage_time(t, TSIT5_C2, h);
        st = 1;
      }
      return false;
    };

    if constexpr (GRIDC) {
      save_col(0);
      t = ns > 0 ? gr[0] : gr[ns];
      h = ns > 0 ? gr[1] - gr[0] : 0.f;
      tst = t;
    } else {
      dt = s.auto_dt ? 0.f : s.dt0[b];
      while (si < s.S && sts[si] <= t0) {  // saved states at save_ts <= t0
        if (mine) *reinterpret_cast<floatx4*>(s.ys + ((size_t)b * s.S + si) * E + (oel - (size_t)b * E)) = y;
        ++si;
      }
      if (rb == 0 && tid == 0 && s.step_ts) s.step_ts[(size_t)b * s.step_len] = t0;
    }
    // RK4 on an empty grid evaluates nothing; Tsit5 evaluates its FSAL k0 even then (stats: 1 + 6 ns)
    if (!GRIDC || !rk4 || ns > 0) {
      kslab = pid_slab(0, 0);  // PID: f(t0, y0) is stage 0 of the first step
      publish(y);  // the first evaluation's input: f(t0, y0) (PID: the FSAL k0 and the initial-step heuristic's f0)
      for (;;) {
#ifdef GNCDE_ROWS_STAMPS
        stamp_on = evals == kStampEval;
        if (evals == kStampEval + 1 && threadIdx.x == 0)  // the next evaluation's start: the whole iteration
          g_rows_stamps[stamp_slot * 16 + 15] = __builtin_amdgcn_s_memrealtime();
#endif
        if (!evaluate(b, tst, a.zbuf[(pub - 1) & 1] + (size_t)b * zgroup, true, kslab)) {
          fault = true;
          break;
        }
        K = mine ? *reinterpret_cast<const floatx4*>(sOut + orow * ZS + ocol) : zero;
        ++evals;
        if constexpr (GRIDC) {
#pragma unroll
          for (int j = 0; j < 7; ++j)
            if (j == st) kk[j] = K;
          if (grid_step()) break;
        } else {
          if (pid_step()) break;
        }
      }
    }
    if constexpr (GRIDC) {
      // padded steps (past this sample's grid): every stage input and saved state is the final state
      for (int kp = ns; kp < Gl - 1; ++kp) {
        for (int i = 1; i <= S1; ++i) record(kp, i, y);
        save_col(kp + 1);
      }
      if (!s.save_steps && mine) *reinterpret_cast<floatx4*>(s.ys + oel) = y;
      steps = ns;
    }
    if (rb == 0 && tid == 0 && s.stats) {
      const bool bad = fault || __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int32_t* o = s.stats + (size_t)b * 4;
      o[GNCDE_STAT_STEPS] = steps;
      o[GNCDE_STAT_REJECTS] = rejects;
      o[GNCDE_STAT_EVALS] = evals;
      o[GNCDE_STAT_STATUS] = bad ? 4 : status;
    }
    if (!a.queue || a.B <= a.b0 + a.G_all) break;  // no queue: every sample started on a group of its own
    // the next sample: workgroup 0 of the group draws it and posts (assignment << 20 | sample) to the group's
    // mailbox; every workgroup polls the mailbox until it holds this assignment (a bounded wait, like wait_all)
    if (threadIdx.x == 0) {
      unsigned* mb = a.mail + (size_t)gslot * kBarStride;
      if (rb == 0) {
        const unsigned q = __hip_atomic_fetch_add(a.queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned nx = (unsigned)(a.b0 + a.G_all) + q;
        const bool stop = fault || __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        __hip_atomic_store(mb, (asg << 20) | (!stop && nx < (unsigned)a.B ? nx : (unsigned)a.B), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      unsigned v, spins = 0;
      int next = a.B;
      while (((v = __hip_atomic_load(mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 20) != (asg & 0xFFFu)) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > a.spin_limit ||
            ((spins & 1023u) == 0 && __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          __hip_atomic_store(a.fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v = (asg << 20) | (unsigned)a.B;  // give up: no further sample
          break;
        }
      }
      next = (int)(v & 0xFFFFFu);
      sFlag[1] = fault ? a.B : next;
    }
    __syncthreads();
    const int nx = UNI ? __builtin_amdgcn_readfirstlane(sFlag[1]) : sFlag[1];  // uniform: keeps descriptors scalar
    __syncthreads();  // sFlag is reused by the next sample's barriers
    if (nx >= a.B) break;
    // the group's state for sample nx: its counter line and hand-off buffers start from zero, its knots in registers
    g = nx;
    epoch = a.bar0;
    pub = 0;
    hseq = 0;
    cidx = -1;
    ts_lane = (int)(threadIdx.x & 63) < T ? a.ts[(size_t)g * T + (threadIdx.x & 63)] : 0.f;
    }
  }
}

struct Inst {
  const void* fn;
  void (*launch)(const RowsArgs&, int, size_t, hipStream_t);
};

template <int H, int MODE, int PREC, int SOLVE>
void launch_rows(const RowsArgs& a, int grid, size_t smem, hipStream_t st) {
  hipLaunchKernelGGL((k_rows<H, MODE, PREC, SOLVE>), dim3(grid), dim3(256), smem, st, a);
}

template <int H, int MODE, int PREC, int SOLVE>
Inst inst() {
  return Inst{reinterpret_cast<const void*>(&k_rows<H, MODE, PREC, SOLVE>), &launch_rows<H, MODE, PREC, SOLVE>};
}

template <int PREC, int SOLVE>
bool find_inst_t(int H, int mode, Inst& out) {
  if (mode == 1) {
    if (H == 16) out = inst<16, 1, PREC, SOLVE>();
    else if (H == 32) out = inst<32, 1, PREC, SOLVE>();
    else if (H == 64) out = inst<64, 1, PREC, SOLVE>();
    else return false;
  } else {
    if (H == 16) out = inst<16, 2, PREC, SOLVE>();
    else if (H == 32) out = inst<32, 2, PREC, SOLVE>();
    else if constexpr (PREC == 1 && SOLVE == 0) {  // (fp32: the H = 64 read-out keeps the multi-kernel path)
      if (H == 64) out = inst<64, 2, PREC, SOLVE>();
      else return false;
    } else {
      return false;
    }
  }
  return true;
}
bool find_inst(int H, int mode, bool bf, Inst& out) {
#ifdef GNCDE_EXPERIMENT_BF16_MFMA
  return bf ? find_inst_t<1, 0>(H, mode, out) : find_inst_t<0, 0>(H, mode, out);
#else
  // the single-plane bf16 mode is retired from the product build (round 6: 8-15 % from fp32 on a fixed grid, 12-21x
  // the evaluations under PID, and no BASELINE config uses it); `make experiment` builds its instances
  return !bf && find_inst_t<0, 0>(H, mode, out);
#endif
}

// 256-thread workgroups of one instance resident at this LDS size, x CUs (cached per device): min(occupancy query,
// what the SGPR file admits) per CU.  The occupancy API reports one workgroup per CU too many for kernels with
// 97-112 SGPRs (MI355X_MICROARCH.md, residency): every k_rows instance has 106, and floor(800 / (ceil(sgpr / 16) *
// 16 + 16)) = 6 covers any SGPR count up to 112.  Where the SGPR file binds, one workgroup per CU of margin is kept
// below that bound; where LDS or VGPRs bind (every shape today: 2-3 per CU), the query's answer is exact.
int resident_blocks(const Inst& k, size_t smem) {
  struct Entry {
    int dev;
    const void* fn;
    size_t smem;
    int blocks;
  };
  static std::mutex mu;
  static Entry cache[64];
  static int used = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < used; ++i)
    if (cache[i].dev == dev && cache[i].fn == k.fn && cache[i].smem == smem) return cache[i].blocks;
  int cus = 0, per = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (!ensure_dyn_lds(k.fn, smem)) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k.fn, 256, smem) != hipSuccess) return 0;
  constexpr int kSgprCap = 800 / (112 + 16);
  if (per >= kSgprCap) per = kSgprCap - 1;  // the SGPR file binds: its bound less one workgroup of margin
  const int blocks = per * cus;
  if (used < 64) cache[used++] = Entry{dev, k.fn, smem, blocks};
  return blocks;
}

// compute units of the current device (cached per device)
int cu_count() {
  static std::mutex mu;
  static int cached[64] = {0};
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> lock(mu);
  if (!cached[dev] && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
    cached[dev] = cus;
  return cached[dev];
}

// workgroups per CU the persistent solve places (GNCDE_SOLVE_WG_PER_CU, default 2; at most what is resident)
int solve_wgs_per_cu() {
  const char* e = getenv("GNCDE_SOLVE_WG_PER_CU");
  const int v = e ? atoi(e) : 2;
  return v < 1 ? 1 : (v > 8 ? 8 : v);
}

// polls before a group barrier wait gives up (each poll is an L2 round trip plus s_sleep 1: seconds in all);
// GNCDE_DEBUG_BARRIER_SPINS overrides it so tests can force the fault path
unsigned spin_limit() {
  const char* e = getenv("GNCDE_DEBUG_BARRIER_SPINS");
  return e ? (unsigned)strtoul(e, nullptr, 10) : (1u << 22);
}

bool rows_shape(const GncdeProblem& p, bool bf) {
  if (p.n > kMaxN || p.n < 1) return false;
  const int H = p.dims[0];
  if (H != 16 && H != 32 && H != 64) return false;
  for (int l = 0; l < p.L; ++l)
    if (p.dims[l] != H) return false;
  if (p.cde_hidden > 0) return p.cde_embed == 8 && p.cde_hidden == H && (H <= 32 || bf) && p.dims[p.L] == 16 * H;
  return p.dims[p.L] == H;
}

}  // namespace

int device_cu_count() { return cu_count(); }

bool rows_solve_granules() {
  const char* e = getenv("GNCDE_SOLVE_GRANULES");  // read per call: a test flips it in one process
  return e && atoi(e) != 0;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for launches above 64 KB of LDS, once per (device, kernel, size)
bool ensure_dyn_lds(const void* fn, size_t smem) {
  if (smem <= 64 * 1024) return true;
  struct Entry {
    int dev;
    const void* fn;
    size_t smem;
  };
  static std::mutex mu;
  static Entry done[128];
  static int used = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < used; ++i)
    if (done[i].dev == dev && done[i].fn == fn && done[i].smem >= smem) return true;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess) return false;
  if (used < 128) done[used++] = Entry{dev, fn, smem};
  return true;
}

// The one-launch evaluation's envelope: every hidden width H in {16, 32, 64}, n <= 256, fp32, and an ODE output of
// width H or the de = 8 CDE read-out with cde_hidden = H <= 32.  At H = 64 the CDE read-out weight is 256 KB (n x 16h
// x h): every 16-row workgroup streams all of it and its fp32 MFMA chain dominates the launch (config 3 measured
// 81 us per evaluation against 70 us for the multi-kernel path, whose read-out launch splits 32-row blocks over
// channel halves), so that shape keeps the multi-kernel path.
// GNCDE_COMPUTE_BF16_MFMA runs only here (every shape of the envelope, the H = 64 read-out included: its bf16 MFMA
// chain is an eighth of the fp32 one).
// In fp32 it is also used only when every sample's group is resident at once (one round per launch): with more
// samples than resident groups the rounds serialise their barrier chains, and the multi-kernel path is faster
// (config 5 at B = 64: 42.7 ms per solve on this kernel's two rounds against 36.9 ms multi-kernel).
bool rows_supported(const GncdeProblem& p) {
  const bool bf = p.compute == GNCDE_COMPUTE_BF16_MFMA;
  if (p.compute != GNCDE_COMPUTE_FP32 && !bf) return false;
  if (!rows_shape(p, bf)) return false;
  if (bf) return true;
  Inst k;
  const int H = p.dims[0];
  if (!find_inst(H, p.cde_hidden > 0 ? 2 : 1, false, k)) return false;
  const int nb = (p.n + kRB - 1) / kRB;
  return resident_blocks(k, rows_smem(p.n, H, p.L, false)) / nb >= p.B;
}

bool rows_eval_used(const GncdeProblem& p) { return rows_supported(p); }

#ifdef GNCDE_ROWS_STAMPS
extern "C" int gncde_debug_rows_stamps(unsigned long long* host, int count) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rows_stamps), sizeof(unsigned long long) * count) == hipSuccess ? 0 : -1;
}
#endif

// Launch one evaluation (RowsState: the group layout, fixed per problem, and the barriers done so far).
int rows_vf_eval(const GncdeProblem& p, const float* t, const float* y, float* dy, const float* csum, const void* coefT,
                 const float* wperm, const uint16_t* wbf, const float* bf, float* z0, float* z1, unsigned* bar, int* fault,
                 unsigned& bars_done, hipStream_t st, float* keep) {
  Inst k;
  const int H = p.dims[0], mode = p.cde_hidden > 0 ? 2 : 1;
  const bool bfm = p.compute == GNCDE_COMPUTE_BF16_MFMA;
  if (!find_inst(H, mode, bfm, k)) return GNCDE_ERR_UNSUPPORTED;
  const size_t smem = rows_smem(p.n, H, p.L, bfm);
  const int nb = (p.n + kRB - 1) / kRB;
  const int cap = resident_blocks(k, smem);
  int G = cap / nb;
  if (G < 1) return GNCDE_ERR_UNSUPPORTED;
  if (G >= p.B) {
    G = p.B;
  } else if (G >= 8) {
    G -= G % 8;
  }
  RowsArgs a{};
  a.B = p.B;
  a.n = p.n;
  a.T = p.T;
  a.L = p.L;
  a.G = G;
  a.rounds = (p.B + G - 1) / G;
  a.nb = nb;
  a.big = rows_big(p.n, H, bfm);
  a.np = rows_np(p.n, bfm);
  a.ts = p.ts;
  a.coef = p.coef;
  a.coefT = coefT;
  a.csum = csum;
  a.tcoef = p.tcoef;
  a.data_coef = p.data_coef;
  a.fusion = p.fusion;
  a.wperm = wperm;
  a.wbf = wbf;
  a.bf = bf;
  a.t = t;
  a.y = y;
  a.dy = dy;
  a.zbuf[0] = z0;
  a.zbuf[1] = z1;
  a.keep = keep;
  a.bar = bar;
  a.bar0 = bars_done;
  a.fault = fault;
  a.spin_limit = spin_limit();
  k.launch(a, G * nb, smem, st);
  bars_done += (unsigned)(a.rounds * (p.L - 1));
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

// ---- the persistent solve ------------------------------------------------------------------------------------
// Envelope: the one-launch evaluation's fp32 shapes for any batch (run in chunks of co-resident groups: one group
// must fit); Tsit5 + PID with SaveAt(t1) or SaveAt(ts), or a fixed grid
// (RK4 / Tsit5) with SaveAt(t1) or every step (+ the stage record); the default dispatch (GNCDE_FLAG_GENERIC takes
// the host-paced paths instead).
bool rows_solve_shape(const GncdeProblem& p) {
  Inst k;
  return (p.compute == GNCDE_COMPUTE_FP32 || p.compute == GNCDE_COMPUTE_BF16_STORAGE) && rows_shape(p, false) &&
         find_inst_t<0, 1>(p.dims[0], p.cde_hidden > 0 ? 2 : 1, k);
}

// the persistent solve's instance for this controller (fp32, or bfloat16 coefficient storage: PREC 2), with the
// counter hand-offs or (GNCDE_SOLVE_GRANULES=1) the tagged-granule ones
// The bf16-storage solve keeps its coefficient loads in LDS (SOLVE & 8) when one workgroup per CU holds the whole
// batch (the cache takes 64 KB more LDS per workgroup: one workgroup per CU instead of two); GNCDE_SOLVE_COEF_CACHE=0
// turns it off.
bool solve_coef_cache(const GncdeProblem& p) {
  if (p.compute != GNCDE_COMPUTE_BF16_STORAGE || rows_solve_granules()) return false;
  const char* e = getenv("GNCDE_SOLVE_COEF_CACHE");
  if (e && atoi(e) == 0) return false;
  const int nb = (p.n + kRB - 1) / kRB;
  if (rows_smem(p.n, p.dims[0], p.L, false, true) > 160 * 1024) return false;  // (the LDS a workgroup may take)
  // (caching the form's small loads too — plane sums, totals, time channel, data spline — measured no faster:
  // 5.63 vs 5.62 ms at config 5, B = 16)
  return (long)p.B * nb <= cu_count();
}

bool find_solve_inst(const GncdeProblem& p, const GncdeSolver& s, Inst& k) {
  const int H = p.dims[0], mode = p.cde_hidden > 0 ? 2 : 1;
  const bool grid = s.controller == GNCDE_CTRL_GRID;
  if (solve_coef_cache(p)) return grid ? find_inst_t<2, 10>(H, mode, k) : find_inst_t<2, 9>(H, mode, k);
  if (rows_solve_granules()) {
    if (p.compute == GNCDE_COMPUTE_BF16_STORAGE)
      return grid ? find_inst_t<2, 6>(H, mode, k) : find_inst_t<2, 5>(H, mode, k);
    return grid ? find_inst_t<0, 6>(H, mode, k) : find_inst_t<0, 5>(H, mode, k);
  }
  if (p.compute == GNCDE_COMPUTE_BF16_STORAGE)
    return grid ? find_inst_t<2, 2>(H, mode, k) : find_inst_t<2, 1>(H, mode, k);
  return grid ? find_inst_t<0, 2>(H, mode, k) : find_inst_t<0, 1>(H, mode, k);
}

bool rows_pid_supported(const GncdeProblem& p, const GncdeSolver& s) {
  if (!rows_solve_shape(p) || (s.flags & GNCDE_FLAG_GENERIC)) return false;
  if (s.controller == GNCDE_CTRL_PID) {
    if (s.method != GNCDE_TSIT5 || (s.save_mode != GNCDE_SAVE_T1 && s.save_mode != GNCDE_SAVE_TS)) return false;
  } else if (s.controller == GNCDE_CTRL_GRID) {
    if (s.save_mode != GNCDE_SAVE_T1 && s.save_mode != GNCDE_SAVE_STEPS) return false;
  } else {
    return false;
  }
  Inst k;
  if (!find_solve_inst(p, s, k)) return false;
  const int nb = (p.n + kRB - 1) / kRB;
  return resident_blocks(k, rows_smem(p.n, p.dims[0], p.L, false, solve_coef_cache(p))) >= nb && cu_count() >= nb;
}

size_t rows_pid_scratch(const GncdeProblem& p) {
  const int nb = (p.n + kRB - 1) / kRB;
  return align_up((size_t)p.B * 2 * nb * 2 * sizeof(float), 256);
}

int rows_integrate_pid(const GncdeProblem& p, const GncdeSolver& s, const float* y0, float* ys, int32_t* stats,
                       char* vf_ws, float* part, const float* csum, const void* coefT, const float* wperm,
                       const float* bf, float* z0, float* z1, unsigned* sync, unsigned* zgran, hipStream_t st) {
  Inst k;
  const int H = p.dims[0];
  if (!find_solve_inst(p, s, k)) return GNCDE_ERR_UNSUPPORTED;
  (void)vf_ws;
  const size_t smem = rows_smem(p.n, H, p.L, false, solve_coef_cache(p));
  if (!ensure_dyn_lds(k.fn, smem)) return GNCDE_ERR_HIP;
  const int nb = (p.n + kRB - 1) / kRB;
  RowsArgs a{};
  a.B = p.B;
  a.n = p.n;
  a.T = p.T;
  a.L = p.L;
  a.rounds = 1;
  a.nb = nb;
  a.big = rows_big(p.n, H, false);
  a.np = rows_np(p.n, false);
  a.ts = p.ts;
  a.coef = p.coef;
  a.coefT = coefT;
  a.csum = csum;
  a.tcoef = p.tcoef;
  a.data_coef = p.data_coef;
  a.fusion = p.fusion;
  a.wperm = wperm;
  a.bf = bf;
  a.zbuf[0] = z0;
  a.zbuf[1] = z1;
  a.zgran = zgran;
  {
    const char* e = getenv("GNCDE_GRAN_POLL1");
    a.poll1 = e && atoi(e) != 0;
  }
  a.bar = sync;  // per-sample arrivals, one line each (zeroed by generic_vf_prepare)
  a.fault = reinterpret_cast<int*>(sync + rows_fault_word(p.B));  // the workspace's fault word
  a.ticket = sync + rows_fault_word(p.B) + 1;
  a.queue = sync + rows_fault_word(p.B) + 2;
  a.mail = sync + (size_t)p.B * kBarStride;
  a.ticket0 = 0;
  a.bar0 = 0;
  a.spin_limit = spin_limit();
  SolveArgs& v = a.s;
  v.grid_mode = s.controller == GNCDE_CTRL_GRID;
  v.method = s.method;
  v.G = s.grid_len;
  v.save_steps = s.save_mode == GNCDE_SAVE_STEPS;
  v.grid = s.grid;
  v.nsteps = s.nsteps;
  v.rec = s.controller == GNCDE_CTRL_GRID ? (s.grid_len >= 2 ? s.stage_rec : nullptr) : s.stage_rec;
  v.ckpt = s.controller == GNCDE_CTRL_PID ? s.pid_ckpt : nullptr;
  v.arec = s.controller == GNCDE_CTRL_PID ? s.act_rec : nullptr;
  v.R = s.rec_steps;
  v.S = s.save_mode == GNCDE_SAVE_TS ? s.n_save : 0;
  v.max_steps = s.max_steps;
  v.auto_dt = s.dt0 == nullptr;
  v.step_len = s.step_ts_len;
  v.rtol = s.rtol;
  v.atol = s.atol;
  v.t0 = s.t0;
  v.t1 = s.t1;
  v.dt0 = s.dt0;
  v.save_ts = s.save_ts;
  v.y0 = y0;
  v.ys = ys;
  v.step_ts = s.step_ts;
  v.stats = stats;
  v.part = part;
  // The solve places at most solve_wgs_per_cu() (2) workgroups per CU: cap co-resident groups.  (Round 4: two per CU
  // made every phase 2-3x longer, 93 us per iteration at B = 32 against 29.6 us at B = 16,
  // profiles/r04_config5_solve_stamps*.txt: the groups' arrival counters shared one cache line, so every group's
  // atomics and polls queued on it; with one line per counter (kBarStride) B = 32 takes 7.7 ms in one launch against
  // 12.4 ms as two B = 16 launches, profiles/r05_config5_batch.jsonl, and an iteration 35 us,
  // profiles/r05_config5_solve_stamps_b32.txt.)  A batch past cap runs in the same single launch: each group takes
  // its next sample from the queue when it finishes one (round 5; before, one launch per chunk of cap samples, whose
  // time is the slowest sample of each chunk).  A launch of a multiple of 8 groups takes the XCD-affine layout;
  // otherwise its workgroups take start-order tickets.
  const int cap = std::min(resident_blocks(k, smem), solve_wgs_per_cu() * cu_count()) / nb;
  if (cap < 1) return GNCDE_ERR_UNSUPPORTED;  // no co-resident group (or the device query failed): never loop
  int bc = p.B < cap ? p.B : cap;
  if (bc >= 8) bc &= ~7;
  // The queue pays where samples differ in cost — the adaptive controller's step counts (config 5 B = 64: 17.76 ->
  // 16.37 ms, B = 48: 14.07 -> 13.66 ms, alternating on one box).  A fixed grid gives every sample the same work,
  // and there the chunked launches win when the last chunk is small (B = 48, 100 Tsit5 steps: 40.1 vs 43.2 ms —
  // its 16 samples run one workgroup per CU, while the queue leaves them on CUs still shared two ways): fixed
  // grids keep the chunks.  GNCDE_SOLVE_CHUNKED=1 / 0 forces either (A/B, tests).
  const char* ce = getenv("GNCDE_SOLVE_CHUNKED");
  // (the mailbox packs a sample index into 20 bits: larger batches keep the chunks)
  const bool chunked = (ce ? atoi(ce) != 0 : s.controller != GNCDE_CTRL_PID) || p.B >= (1 << 20);
  if (chunked) {
    a.queue = nullptr;
    unsigned tickets = 0;
    for (int c0 = 0; c0 < p.B; c0 += bc) {
      const int nbc = p.B - c0 < bc ? p.B - c0 : bc;
      a.b0 = c0;
      a.G = nbc % 8 == 0 ? nbc : 0;
      a.G_all = nbc;
      a.ticket0 = tickets;
      if (a.G == 0) tickets += (unsigned)(nbc * nb);
      k.launch(a, nbc * nb, smem, st);
    }
  } else {  // one launch: bc resident groups, the rest of the batch from the sample queue
    a.b0 = 0;
    a.G = bc % 8 == 0 ? bc : 0;
    a.G_all = bc;
    a.ticket0 = 0;
    k.launch(a, bc * nb, smem, st);
  }
  return hipGetLastError() == hipSuccess ? GNCDE_OK : GNCDE_ERR_HIP;
}

void rows_pid_name(const GncdeProblem& p, const GncdeSolver& s, char* buf, size_t len) {
  if (s.controller == GNCDE_CTRL_PID)
    snprintf(buf, len, "rows_pid<%d,%s>", p.dims[0], p.cde_hidden > 0 ? "cde" : "ode");
  else
    snprintf(buf, len, "rows_grid<%d,%s,%s>", p.dims[0], p.cde_hidden > 0 ? "cde" : "ode",
             s.method == GNCDE_RK4 ? "rk4" : "tsit5");
}

}  // namespace gncde
