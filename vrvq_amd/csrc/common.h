// Shared helpers for the gfx950 VRVQ kernels. Compiled with -ffp-contract=off: every fused
// multiply-add in the product path is written explicitly (fmaf / MFMA) so two kernels that
// must agree bit-for-bit (rvq codes vs expand) evaluate the same expression tree.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/vrvq.h"

#define VRVQ_CHECK_ARG(cond)            \
  do {                                  \
    if (!(cond)) return VRVQ_ERR_ARG;   \
  } while (0)

static inline int vrvq_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

static inline hipStream_t as_stream(vrvq_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Snake activation, models/layers.py:30: x + (alpha + 1e-9)^-1 * sin(alpha * x)^2.
// Evaluated as the reference's op sequence (mul, sin, square, mul, add), one rounding each.
__device__ __forceinline__ float snake_act(float v, float alpha, float inv_alpha) {
  const float s = sinf(alpha * v);
  return v + inv_alpha * (s * s);
}

// 8-term dot product in k order (fmaf chain); used for in_proj/out_proj/codebook distance.
__device__ __forceinline__ float dot8(const float4& a0, const float4& a1, const float4& b0,
                                      const float4& b1) {
  float acc = a0.x * b0.x;
  acc = fmaf(a0.y, b0.y, acc);
  acc = fmaf(a0.z, b0.z, acc);
  acc = fmaf(a0.w, b0.w, acc);
  acc = fmaf(a1.x, b1.x, acc);
  acc = fmaf(a1.y, b1.y, acc);
  acc = fmaf(a1.z, b1.z, acc);
  acc = fmaf(a1.w, b1.w, acc);
  return acc;
}

// out_proj of one frame for one output channel: (W_out[c,:] . zst) + b_out[c]
// (vrvq_rvq_expand's z_q_is).
__device__ __forceinline__ float out_proj1(const float4& w0, const float4& w1, float bias,
                                           const float4& z0, const float4& z1) {
  return dot8(w0, w1, z0, z1) + bias;
}

// LDS-DMA of `nchunks` 1-KiB chunks src -> dst (global_load_lds_dwordx4, 16 B per lane), chunk
// q issued by wave q % nwaves (the calling wave is `wave`). Written as inline asm on purpose:
// the compiler's own LDS-DMA tracking turns later LDS accesses it cannot disambiguate (and
// LDS fences) into vmcnt(0) waits, i.e. it would drain unrelated stores / prefetches. Callers
// wait for completion explicitly (s_waitcnt vmcnt) before the barrier that publishes the data.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; the callers do not use it
__device__ __forceinline__ void vrvq_dma_chunks(const float* src, float* dst, int nchunks,
                                                int wave, int nwaves, int lane) {
  for (int q = wave; q < nchunks; q += nwaves) {
    const float* gp = src + q * 256 + lane * 4;
    const unsigned lds = (unsigned)(size_t)(__attribute__((address_space(3))) float*)(dst + q * 256);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                 :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gp) : "memory", "m0");
  }
}
#pragma clang diagnostic pop
