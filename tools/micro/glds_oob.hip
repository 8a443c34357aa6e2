// Probe: does buffer_load_dwordx4 ... lds (LDS-DMA through a raw buffer resource) write zeros
// to LDS for lanes whose offset is out of range (negative voffset, or >= num_records)?
// The x3 conv mainloop's plane staging relies on it for the zero padding of its windows.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void;
__global__ void k(const float* src, int nbytes, float* out) {
  __shared__ __attribute__((aligned(16))) float buf[64 * 4 * 2];
  for (int i = threadIdx.x; i < 512; i += 64) buf[i] = -1.0f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nbytes, 0x00020000);
  int voff = ((int)threadIdx.x - 8) * 16;  // lanes 0..7 negative
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)buf, 16, voff, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(buf + 256), 16, voff + 1024, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = buf[i];
}
int main() {
  const int n = 4096;
  float h[n];
  for (int i = 0; i < n; ++i) h[i] = 1000.0f + i;
  float *d, *o;
  hipMalloc(&d, n * 4);
  hipMalloc(&o, 512 * 4);
  hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
  const int nbytes = 40 * 16;  // valid: 16-B units 0..39
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, nbytes, o);
  float r[512];
  hipMemcpy(r, o, 512 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int lane = 0; lane < 64; ++lane)
    for (int half = 0; half < 2; ++half) {
      const int unit = lane - 8 + half * 64;
      for (int e = 0; e < 4; ++e) {
        const float want = (unit >= 0 && unit < 40) ? 1000.0f + unit * 4 + e : 0.0f;
        const float got = r[half * 256 + lane * 4 + e];
        if (got != want) {
          if (bad < 8) printf("lane %d half %d e %d: got %g want %g\n", lane, half, e, got, want);
          ++bad;
        }
      }
    }
  printf("glds_oob: %s (%d mismatches)\n", bad ? "FAIL" : "PASS: OOB lanes write zeros", bad);
  return bad ? 1 : 0;
}
