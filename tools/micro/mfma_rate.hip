// Micro-benchmark: back-to-back issue rate of v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_32x32x8_bf16
// on gfx950 (4 independent accumulators per wave, one wave per SIMD), timed with s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ void kern(float* out, long long* cyc, int iters) {
  f32x16 acc[4] = {};
  bf16x8 a8, b8;
  s16x4 a4, b4;
  for (int e = 0; e < 8; ++e) { a8[e] = (__bf16)(threadIdx.x * 0.001f + e); b8[e] = (__bf16)(e * 0.5f); }
  for (int e = 0; e < 4; ++e) { a4[e] = (short)(threadIdx.x + e); b4[e] = (short)(e + 7); }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (K == 16) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, acc[j], 0, 0, 0);
      else acc[j] = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4, b4, acc[j], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int j = 0; j < 4; ++j) for (int r = 0; r < 16; ++r) s += acc[j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out; long long* cyc;
  hipMalloc(&out, 256 * 256 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(long long));
  long long h[256];
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kern<16>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("32x32x16 bf16: %.1f cycles per MFMA per SIMD\n", (double)h[0] / (iters * 4));
    hipLaunchKernelGGL(kern<8>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("32x32x8  bf16: %.1f cycles per MFMA per SIMD\n", (double)h[0] / (iters * 4));
  }
  hipFree(out); hipFree(cyc);
  return 0;
}
