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

// sin(u)^2 for Snake: Cody-Waite reduction of u by pi (three-term pi, exact with fma for
// |u| < 2^20), then the odd Taylor polynomial of sin to degree 13 on |r| <= pi/2 (truncation
// < 7e-10). sin(u)^2 = sin(r)^2, so the quadrant sign is not needed. 14 VALU instead of the
// ~40 of the general sinf (the mul of the reference's alpha * x is kept as is); max abs error
// of the square 2.2e-7 (sinf: 1e-7) — within the parity tolerance, and the Snake-heavy
// residual units spend most of their VALU here. No range check: see snake_n / sin_sq.
__device__ __forceinline__ float sin_sq_fast(float u) {
  const float k = rintf(u * 0.318309886183790672f);
  float r = fmaf(-k, 3.14159274101257324e+00f, u);
  r = fmaf(-k, -8.74227765734758577e-08f, r);
  r = fmaf(-k, -3.43061790e-15f, r);
  const float r2 = r * r;
  float p = 1.6059043836821614e-10f;            //  1/13!
  p = fmaf(p, r2, -2.5052108385441720e-08f);    // -1/11!
  p = fmaf(p, r2, 2.7557319223985893e-06f);     //  1/9!
  p = fmaf(p, r2, -1.9841269841269841e-04f);    // -1/7!
  p = fmaf(p, r2, 8.3333333333333333e-03f);     //  1/5!
  p = fmaf(p, r2, -1.6666666666666667e-01f);    // -1/3!
  const float s = fmaf(r * r2, p, r);
  return s * s;
}

// Arguments the reduction above does not take: |u| >= 2^20, NaN, Inf. Those go to sinf (ocml:
// Payne-Hanek reduction), which, like the reference's torch.sin, is accurate for any argument.
__device__ __forceinline__ bool snake_arg_big(float u) { return !(fabsf(u) < 0x1p20f); }

__device__ __forceinline__ float sin_sq_exact(float u) {
  const float s = sinf(u);
  return s * s;
}

// Single value with its own range check (an exec-masked branch per element: for the cold
// paths; the hot loops use snake_n).
__device__ __forceinline__ float sin_sq(float u) {
  if (__builtin_expect(snake_arg_big(u), 0)) return sin_sq_exact(u);
  return sin_sq_fast(u);
}

// sin(r) and cos(r) of the reduced argument of u (r = u - k pi, |r| <= pi/2): sin(u) cos(u) =
// sin(r) cos(r) and sin(u)^2 = sin(r)^2 (the (-1)^k signs cancel) -- what Snake's backward
// needs. Same reduction as sin_sq; Taylor polynomials to degree 13 / 14. Same large-argument
// guard as sin_sq (sincosf: the unreduced sin / cos have the same products).
__device__ __forceinline__ void sincos_reduced(float u, float* sr, float* cr) {
  if (__builtin_expect(!(fabsf(u) < 0x1p20f), 0)) {
    sincosf(u, sr, cr);
    return;
  }
  const float k = rintf(u * 0.318309886183790672f);
  float r = fmaf(-k, 3.14159274101257324e+00f, u);
  r = fmaf(-k, -8.74227765734758577e-08f, r);
  r = fmaf(-k, -3.43061790e-15f, r);
  const float r2 = r * r;
  float p = 1.6059043836821614e-10f;
  p = fmaf(p, r2, -2.5052108385441720e-08f);
  p = fmaf(p, r2, 2.7557319223985893e-06f);
  p = fmaf(p, r2, -1.9841269841269841e-04f);
  p = fmaf(p, r2, 8.3333333333333333e-03f);
  p = fmaf(p, r2, -1.6666666666666667e-01f);
  *sr = fmaf(r * r2, p, r);
  float q = -1.1470745597729725e-11f;           // -1/14!
  q = fmaf(q, r2, 2.0876756987868099e-09f);     //  1/12!
  q = fmaf(q, r2, -2.7557319223985891e-07f);    // -1/10!
  q = fmaf(q, r2, 2.4801587301587302e-05f);     //  1/8!
  q = fmaf(q, r2, -1.3888888888888889e-03f);    // -1/6!
  q = fmaf(q, r2, 4.1666666666666667e-02f);     //  1/4!
  q = fmaf(q, r2, -0.5f);                       // -1/2!
  *cr = fmaf(q, r2, 1.0f);
}

// Snake activation, models/layers.py:30: x + (alpha + 1e-9)^-1 * sin(alpha * x)^2.
// The reference's op sequence (mul, sin, square, mul, add); sin^2 from sin_sq.
__device__ __forceinline__ float snake_act(float v, float alpha, float inv_alpha) {
  return v + inv_alpha * sin_sq(alpha * v);
}

// Snake on N values at once (the hot staging / epilogue loops): the fast reduction for all of
// them, and one wave-uniform branch for the group -- taken only when a lane of the wave holds an
// argument past the reduction's range, and then only those elements take sinf. Per element this
// costs one compare (the per-element branch of sin_sq split every element into its own block and
// cost the residual units 5-8 %). Same values as snake_act, element for element.
template <int N>
__device__ __forceinline__ void snake_n(float (&v)[N], const float (&al)[N], const float (&ia)[N]) {
  float u[N], s[N];
  bool big = false;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    u[i] = al[i] * v[i];
    big = big || snake_arg_big(u[i]);
    s[i] = sin_sq_fast(u[i]);
  }
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(big) != 0, 0)) {
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = snake_arg_big(u[i]) ? sin_sq_exact(u[i]) : s[i];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = v[i] + ia[i] * s[i];
}

// ... with one alpha for the whole group
template <int N>
__device__ __forceinline__ void snake_n1(float (&v)[N], float alpha, float inv_alpha) {
  float al[N], ia[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    al[i] = alpha;
    ia[i] = inv_alpha;
  }
  snake_n<N>(v, al, ia);
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
