// Write-rate micro-benchmark for the fused RVQ expansion's z_q_is stream (csrc/rvq.hip
// fused_expand_body): the same store pattern -- per stage i, a (clip, 128-channel block)
// workgroup of 8 waves writes its 128 x T rows of z_q_is[b][i] as 16-B quads of four frames,
// 8 rows x 128 B per wave instruction -- with no loads, no MFMAs, no hand-off waits. Variants:
//   wgs_per_block = 1: one 512-thread workgroup per (clip, block) (the fused launch's shape)
//   wgs_per_block = 2: two workgroups, each half the frame tiles (more workgroups per CU)
// and `dep`: each wave waits for its previous stage's stores before the next stage (vmcnt 0).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/expand_writes.hip -o tools/micro/expand_writes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

__global__ __launch_bounds__(512) void writes(float* zqis, int B, int nq, int T, int split,
                                              int dep) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int blk = blockIdx.x / split, part = blockIdx.x % split;
  const int cb = blk % 8, b = blk / 8;
  const int col = lane & 31, h = lane >> 5;
  const int c0 = cb * 128 + (wave & 3) * 32;
  const int chk = c0 + 4 * h + (lane & 3);
  const int n_ft = (min(128, T) + 31) / 32;
  for (int i = 0; i < nq; ++i) {
    for (int j = 0; j < 2; ++j) {
      const int ft = (wave >> 2) + 2 * j;
      if (ft % split != part || ft >= n_ft) continue;
      int tb = ft * 32;
      if (tb + 32 > T && T >= 32) tb = T - 32;
      const int t = tb + 4 * (col >> 2);
      for (int qd = 0; qd < 4; ++qd) {
        float* row = zqis + (((size_t)b * nq + i) * 1024 + chk + 8 * qd) * T;
        const float v = (float)(i + qd);
        *reinterpret_cast<f4u*>(row + t) = f4u{v, v + 1, v + 2, v + 3};
      }
    }
    if (dep) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

int main() {
  const int B = 32, nq = 8, T = 87;
  const size_t n = (size_t)B * nq * 1024 * T;
  float* d;
  hipMalloc(&d, n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int split : {1, 2, 4}) {
    for (int dep : {0, 1}) {
      const int grid = B * 8 * split;
      for (int w = 0; w < 3; ++w) writes<<<grid, 512>>>(d, B, nq, T, split, dep);
      hipEventRecord(e0);
      const int it = 20;
      for (int w = 0; w < it; ++w) writes<<<grid, 512>>>(d, B, nq, T, split, dep);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / it;
      printf("split %d dep %d: %.1f us per call, %.2f TB/s (z_q_is %.1f MB)\n", split, dep, us,
             n * 4 / us / 1e6, n * 4 / 1e6);
    }
  }
  hipFree(d);
  return 0;
}
