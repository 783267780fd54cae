// Micro-benchmark of the fp32 MFMA pipe on gfx950 (design input for the fused kernels, not product code):
//   A: one dependent accumulation chain of v_mfma_f32_16x16x4f32 per wave
//   B: four independent chains per wave
//   C: one chain + independent VALU FMAs between the MFMAs (does the VALU hide under the MFMA?)
//   D: VALU FMAs alone (same count as in C)
// Each kernel runs `waves_per_simd` waves per SIMD on every CU; prints cycles per MFMA per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

template <int MODE>
__global__ void probe(float* out, float seed) {
  floatx4 c0 = {seed, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  float a = seed + threadIdx.x, b = seed * 2.f;
  float v0 = a, v1 = b, v2 = a + 1.f, v3 = b + 1.f, v4 = a + 2.f, v5 = b + 2.f, v6 = a + 3.f, v7 = b + 3.f;
  for (int i = 0; i < kIters; ++i) {
    if constexpr (MODE == 0) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
    } else if constexpr (MODE == 1) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    } else if constexpr (MODE == 2) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      v0 = fmaf(v0, a, b); v1 = fmaf(v1, a, b); v2 = fmaf(v2, a, b); v3 = fmaf(v3, a, b);
      v4 = fmaf(v4, a, b); v5 = fmaf(v5, a, b); v6 = fmaf(v6, a, b); v7 = fmaf(v7, a, b);
    } else {
      v0 = fmaf(v0, a, b); v1 = fmaf(v1, a, b); v2 = fmaf(v2, a, b); v3 = fmaf(v3, a, b);
      v4 = fmaf(v4, a, b); v5 = fmaf(v5, a, b); v6 = fmaf(v6, a, b); v7 = fmaf(v7, a, b);
    }
  }
  const float s = c0[0] + c0[1] + c1[2] + c2[3] + c3[0] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
float run(int cus, int wps, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const dim3 grid(cus * wps), block(256);  // 4 waves per block = one per SIMD
  hipLaunchKernelGGL(probe<MODE>, grid, block, 0, 0, out, 1e-3f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<MODE>, grid, block, 0, 0, out, 1e-3f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5.f;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const double ghz = prop.clockRate / 1e6;
  float* out;
  hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
  printf("CUs %d, clock %.2f GHz\n", cus, ghz);
  for (int wps : {1, 2, 4}) {
    const float a = run<0>(cus, wps, out), b = run<1>(cus, wps, out), c = run<2>(cus, wps, out),
                d = run<3>(cus, wps, out);
    // cycles per MFMA per SIMD (wps waves per SIMD, kIters MFMAs each; B issues 4 per iteration)
    const double cyc = ghz * 1e6;  // cycles per ms
    printf("waves/SIMD %d: dep chain %.1f cyc/MFMA | 4 chains %.1f | chain+8 VALU %.1f (per iter) | 8 VALU alone %.1f "
           "(per iter)\n",
           wps, a * cyc / ((double)kIters * wps), b * cyc / (4.0 * kIters * wps), c * cyc / ((double)kIters * wps),
           d * cyc / ((double)kIters * wps));
  }
  hipFree(out);
  return 0;
}
