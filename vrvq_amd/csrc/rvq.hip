// Residual vector quantisation on gfx950: projection GEMM -> 8-dim chain -> HBM expansion.
//
// VBRResidualVectorQuantize.forward (models/quantize.py:328-443) runs, per frame and stage i
// (VectorQuantize.forward / decode_latents, :42-103):
//   z_e(i) = W_in(i) r_i + b_in(i),     r_i = z - sum_{j<i} z_q_j,   z_q_j = W_out(j) zst_j + b_out(j)
//   idx    = argmin_n (sum e^2 - 2 e.cbn_n) + sum cbn_n^2,  e = z_e / max(|z_e|, 1e-12)
//   zst_i  = z_e + (cb[idx] - z_e)                               (straight-through value)
// By linearity z_e(i) = ((P_i + b_in(i)) - Qb_i) - sum_{j<i} M_ij zst_j with P_i = W_in(i) z,
// M_ij = W_in(i) W_out(j) (8x8) and Qb_i = W_in(i) sum_{j<i} b_out(j): the sequential part
// lives in the 8-dim latent space and the 1024-dim work becomes two embarrassingly parallel
// streams. The eval encode's path is ONE launch from the in_proj partials the encoder's last
// conv computes in its epilogue (rvq_pt_kernel: chain parts + expansion workgroups that write
// z_q_is / z_q; conv.hip vrvq_conv1d_proj); on z itself, rvq_fused_kernel (projection units,
// chain parts and expansion in one launch for T <= 96). Both are built from the bodies of the
// three-launch form, which stays as the reference path:
//
//   rvq_project{3,2}_kernel  P partials over 8 channel splits (one workgroup per clip x 96-frame
//                        tile x split, the z slab staged once in LDS; 3: split-bf16 MFMA, 2:
//                        fp32-input v_mfma_f32_16x16x4_f32).
//   rvq_chain_kernel     the chain: <= 16 frames per workgroup, 8 waves; wave w scans its
//                        N/8 codes for all frames at once on the matrix cores (16-code x
//                        16-frame MFMA tiles), then 8 (frame, k) lane groups finish the stage
//                        (cross-wave argmin, raw codeword, loss, projected residual, next z_e)
//                        — two barriers per stage, no global stores until the end.
//   rvq_expand_kernel    z_q_is[b,i,:,:] = W_out(i) zst_i + b_out(i) and the masked sum z_q on
//                        the matrix cores (32-channel x 32-frame tiles): the HBM write stream,
//                        with no LDS and a few VALU per element.
//
// The distance is the reference's fp32 expression (dot in k order, fma(d, -2, e2) + c2, lowest
// index on ties); the projection on the split-bf16 matrix cores (x3) is fp32-accurate but not
// the reference's summation order, so the codes match every golden fixture BY TEST (full
// batches included), not by construction: a near-tie could differ. The fp32-input projection
// (vrvq_rvq_project_variant 2, rvq_project2_kernel) stays available as the exactness fallback.
#include <hip/hip_ext.h>

#include <map>
#include <mutex>
#include <vector>

#include "common.h"
#include "lanes.h"

#ifdef VRVQ_STAMPS
// Fused launch (rvq_fused_kernel), diagnostic build: thread 0 of every workgroup records
// s_memrealtime (100 MHz, one clock for the whole chip) at its phase boundaries into
// stamps[blockIdx][64] (tools/rvq_fused_stamps.py).
#define FSTAMP(buf, slot)                                                                    \
  do {                                                                                     \
    if ((buf) && threadIdx.x == 0)                                                         \
      (buf)[(size_t)blockIdx.x * 64 + (slot)] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
// ... by thread t of the workgroup (the pt expansion's loader wave)
#define FSTAMPT(buf, slot, t)                                                                \
  do {                                                                                     \
    if ((buf) && threadIdx.x == (t))                                                       \
      (buf)[(size_t)blockIdx.x * 64 + (slot)] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#else
#define FSTAMP(buf, slot) do {} while (0)
#define FSTAMPT(buf, slot, t) do {} while (0)
#endif

namespace {

constexpr int RD = 1024;        // latent channels
constexpr int RCD = 8;          // codebook_dim
constexpr int PJ_SPLIT = 8;     // channel splits of the projection GEMM
constexpr int PJ_CPS = RD / PJ_SPLIT;
constexpr int PJ_KC = 32;       // channels per projection K chunk
constexpr int PJ_NC = PJ_CPS / PJ_KC;  // K chunks per split (4)
constexpr int CH_NT = 512;      // chain threads (8 waves)
constexpr int CH_NW = CH_NT / 64;
constexpr int CH_FMAX = 16;     // frames per chain workgroup
constexpr int CH_NQMAX = 32;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr int CPOL_SC1 = 16;    // buffer load / store aux: sc1 (L1 bypass, write-through)
constexpr int RSRC_FLAGS = 0x00020000;  // raw buffer descriptor word 3 (gfx950)

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ------------------------------------------------------------------------------------------
// Prep (once per weight version, like the weight-norm fold):
//   mcol[j][i][k][m] = sum_c W_in(i)[k][c] W_out(j)[c][m] for i > j (else 0)   (this kernel)
//   qb[i][k]         = sum_c W_in(i)[k][c] (sum_{j<i} b_out(j)[c])   (cross_prep_qb_kernel)
// one fmaf chain over c in order per output.
__global__ void cross_prep_kernel(const float* __restrict__ w_in_t,  // [nq][D][8]
                                  const float* __restrict__ w_out,   // [nq][D][8]
                                  const float* __restrict__ b_out,   // [nq][D]
                                  int nq, float* __restrict__ mcol, float* __restrict__ qb) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int nm = nq * nq * 64;
  if (e < nm) {
    const int m = e & 7, k = (e >> 3) & 7, ij = e >> 6;
    const int i = ij % nq, j = ij / nq;
    float acc = 0.0f;
    if (i > j) {
      const float* wi = w_in_t + (size_t)i * RD * RCD + k;
      const float* wo = w_out + (size_t)j * RD * RCD + m;
      for (int c = 0; c < RD; ++c) acc = fmaf(wi[c * RCD], wo[c * RCD], acc);
    }
    mcol[e] = acc;
  }
}

// qb with the bias prefix sums shared: workgroup = stage i; thread c forms
// bs[c] = sum_{j<i} b_out(j)[c] (left to right) into LDS, then 8 lanes run the k-th fmaf chain
// over c in order -- the values of the earlier one-thread-per-output form, which re-summed the
// biases for every channel in each of its nq * 8 threads (O(nq^2 D) serial work: ~1 ms per
// weight version at nq = 28, i.e. every training step).
__global__ __launch_bounds__(RD) void cross_prep_qb_kernel(const float* __restrict__ w_in_t,
                                                           const float* __restrict__ b_out,
                                                           float* __restrict__ qb) {
  __shared__ float bs_s[RD];
  const int i = blockIdx.x, c = threadIdx.x;
  float bs = 0.0f;
  for (int j = 0; j < i; ++j) bs = bs + b_out[(size_t)j * RD + c];
  bs_s[c] = bs;
  __syncthreads();
  if (c < RCD) {
    const float* wi = w_in_t + (size_t)i * RD * RCD + c;
    float acc = 0.0f;
    for (int cc = 0; cc < RD; ++cc) acc = fmaf(wi[cc * RCD], bs_s[cc], acc);
    qb[i * RCD + c] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// Prep: the normalised codebooks in the chain's MFMA A-fragment order, so that every lane loads
// its stage operands as contiguous float4:
//   cbf[i][w][l][t][kh] = cbn[i][w*N/8 + 16 t + (l & 15)][4 kh + (l >> 4)]
// (wave w of the chain owns codes [w N/8, (w+1) N/8) as N/128 tiles of 16 codes).
__global__ void rvq_frag_kernel(const float* __restrict__ cbn, int nq, int N,
                                float* __restrict__ cbf) {
  const size_t total = (size_t)nq * N * RCD;
  const int NT = N / 128;
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total;
       o += (size_t)gridDim.x * blockDim.x) {
    const int kh = (int)(o % 2);
    size_t r = o / 2;
    const int t = (int)(r % NT);
    r /= NT;
    const int l = (int)(r % 64);
    r /= 64;
    const int w = (int)(r % CH_NW);
    const int i = (int)(r / CH_NW);
    const int code = w * (N / CH_NW) + 16 * t + (l & 15);
    cbf[o] = cbn[((size_t)i * N + code) * RCD + 4 * kh + (l >> 4)];
  }
}

// ------------------------------------------------------------------------------------------
// Projection: part[s][n][r] = sum_{c in split s} W_in_t[r/8][c][r%8] z[b][c][t], n = b*T + t,
// r < R = nq*8, fp32-input form (variant 2). One workgroup per (clip, frame tile of <= 96,
// channel split); each wave runs the split's 128 channels in order, 4 per
// v_mfma_f32_16x16x4_f32, from a zero accumulator (an exact fmaf-chain order); a workgroup reads its z slab [128 ch][<= 96 t] from HBM once (row segments, staged in
// LDS in four 32-channel chunks, each consumed as soon as it has landed) and keeps it for every
// 64-row block of stages; the w_in_t operands go straight to registers (32 per lane and block).
// 8 waves: wave w = 16-row tile (w & 3) x three 16-frame column tiles (w >> 2). 256 workgroups
// at configs[1] (32 clips x 8 splits): one per CU, no second round.
constexpr int PJ2_NT = 512;
constexpr int PJ2_TC = 96;                      // frames per tile (6 MFMA column tiles)
constexpr int PJ2_LD = 112;                     // z_s row stride (112 = 48 mod 64: lk groups
                                                // of the B reads land on disjoint bank ranges)
constexpr int PJ2_ZQ = PJ_KC * PJ2_TC / PJ2_NT; // z loads per thread per K chunk (6)

// Where the partials go: plain stores (the three-launch path: the chain reads them after a
// kernel boundary) or, in the fused launch, tagged 8-B granules {partial, tag} written
// through (sc1, 16-B stores = two whole granules): the data is its own flag, the consumer
// checks the tags of what it read (MI355X_MICROARCH.md / cdna_hip_programming.md Guideline 16,
// R2) -- no drain, no flag word.
struct PartSink {
  float* part;
  __amdgpu_buffer_rsrc_t rsrc;  // over the granule buffer (tag != 0)
  unsigned tag;                 // 0: plain floats
  __device__ __forceinline__ void put(size_t off, float4 v) const {
    if (tag) {
      const u32x4 g0 = {__float_as_uint(v.x), tag, __float_as_uint(v.y), tag};
      const u32x4 g1 = {__float_as_uint(v.z), tag, __float_as_uint(v.w), tag};
      __builtin_amdgcn_raw_buffer_store_b128(g0, rsrc, (int)(off * 8), 0, CPOL_SC1);
      __builtin_amdgcn_raw_buffer_store_b128(g1, rsrc, (int)(off * 8 + 16), 0, CPOL_SC1);
    } else {
      *reinterpret_cast<float4*>(part + off) = v;
    }
  }
};

// One (clip b, frame tile tc, channel split s) projection unit; z_s = PJ_CPS * PJ2_LD floats
// of LDS.
__device__ __forceinline__ void project2_body(const float* __restrict__ z, int T, int nq, int tc,
                                              int b, int s, const float* __restrict__ w_in_t,
                                              const PartSink& out, int NF, float* z_s) {
  const int R = nq * RCD;
  const int t0 = tc * PJ2_TC;
  const int ntl = min(PJ2_TC, T - t0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lk = lane >> 4;
  const int rt = wave & 3, ch = wave >> 2;  // row tile, column-tile half
  // A operands of row block rb: row r = 64 rb + 16 rt + lr (stage r / 8, k = r % 8), channels
  // 4 j + lk of the split; rows >= R zeroed (clamped address, mask)
  auto load_w = [&](int rb, float (&av)[PJ_CPS / 4]) {
    const int r = rb * 64 + rt * 16 + lr;
    const unsigned m = 0u - (unsigned)(r < R);
    const float* wp = w_in_t + ((size_t)min(r >> 3, nq - 1) * RD + s * PJ_CPS + lk) * RCD + (r & 7);
#pragma unroll
    for (int j = 0; j < PJ_CPS / 4; ++j)
      av[j] = __uint_as_float(__float_as_uint(wp[(size_t)4 * j * RCD]) & m);
  };
  float av[PJ_CPS / 4];
  load_w(0, av);  // L2-resident weights first, their latency under the z slab's
  const float* zb = z + ((size_t)b * RD + s * PJ_CPS) * T + t0;
  {  // the slab: every load in flight at once
    float zv[PJ_NC][PJ2_ZQ];
#pragma unroll
    for (int kc = 0; kc < PJ_NC; ++kc)
#pragma unroll
      for (int q = 0; q < PJ2_ZQ; ++q) {
        const int e = tid + PJ2_NT * q;
        const int c = e / PJ2_TC, t = e - c * PJ2_TC;
        zv[kc][q] = zb[(size_t)(kc * PJ_KC + c) * T + min(t, ntl - 1)];  // clamped, zeroed below
      }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first wait
#pragma unroll
    for (int kc = 0; kc < PJ_NC; ++kc)
#pragma unroll
      for (int q = 0; q < PJ2_ZQ; ++q) {
        const int e = tid + PJ2_NT * q;
        const int c = e / PJ2_TC, t = e - c * PJ2_TC;
        z_s[(kc * PJ_KC + c) * PJ2_LD + t] =
            __uint_as_float(__float_as_uint(zv[kc][q]) & (0u - (unsigned)(t < ntl)));
      }
  }
  // a use of the weights here keeps their loads ahead of the slab's (issued first, they have
  // landed by now); without it they are sunk below the barrier and waited for one by one
#pragma unroll
  for (int j = 0; j < PJ_CPS / 4; ++j) asm volatile("" ::"v"(av[j]));
  __syncthreads();
  for (int rb = 0; rb * 64 < R; ++rb) {
    float an[PJ_CPS / 4];
    const bool more = (rb + 1) * 64 < R;
    if (more) load_w(rb + 1, an);  // next block's weights under this block's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < PJ_CPS / 4; ++j) {
      const float* zr = z_s + (4 * j + lk) * PJ2_LD + ch * 48 + lr;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], zr[q * 16], acc[q], 0, 0, 0);
    }
    // D layout: lane l, reg q -> row 4 (l >> 4) + q of the tile, frame l & 15
    const int rr = rb * 64 + rt * 16 + 4 * lk;  // rows rr..rr+3 all valid iff rr < R
    if (rr < R) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int t = ch * 48 + q * 16 + lr;
        if (t < ntl) {
          const size_t n = (size_t)b * T + t0 + t;
          out.put(((size_t)s * NF + n) * R + rr,
                  make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]));
        }
      }
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < PJ_CPS / 4; ++j) av[j] = an[j];
    }
  }
}

__global__ __launch_bounds__(PJ2_NT) void rvq_project2_kernel(const float* __restrict__ z, int T,
                                                              int nq, int n_tc,
                                                              const float* __restrict__ w_in_t,
                                                              float* __restrict__ part, int NF) {
  __shared__ __attribute__((aligned(16))) float z_s[PJ_CPS * PJ2_LD];
  PartSink out{part, __builtin_amdgcn_make_buffer_rsrc(part, (short)0, 0, RSRC_FLAGS), 0u};
  project2_body(z, T, nq, blockIdx.x % n_tc, blockIdx.x / n_tc, blockIdx.y, w_in_t, out, NF, z_s);
}

// ------------------------------------------------------------------------------------------
// Projection on the bf16 matrix cores (variant 3): the same unit as rvq_project2_kernel (clip,
// <= 96-frame tile, 128-channel split), with both operands split exactly into three bf16 terms
// and the six products of conv_x3.h (dropped terms <= 2^-23 |ab|: fp32 accuracy) on
// v_mfma_f32_16x16x32_bf16 -- 2.7x the fp32 MFMA rate for the GEMM that bounds the projection
// (64 rows x 128 channels x 96 frames per unit). The z slab goes to LDS transposed, as three
// bf16 planes [plane][frame][channel] (rows of 128 channels + 8 pad: conflict-free 16-B B
// reads); the W_in rows (8 channels per lane, L2) are split in registers.
constexpr int PJ3_LDB = 136;                     // bf16 per frame row (272 B)
constexpr int PJ3_PLANE = PJ2_TC * PJ3_LDB * 2;  // bytes per plane
constexpr int PJ3_LDS = 3 * PJ3_PLANE;           // 78,336 B

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// v = h + m + l exactly (RNE at each step), two values per call (conv_x3.h split3x2)
__device__ __forceinline__ void rvq_split3x2(float v0, float v1, unsigned& h, unsigned& m,
                                             unsigned& l) {
  const f32x2 v = {v0, v1};
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
  const f32x2 hf = {__uint_as_float(hu << 16), __uint_as_float(hu & 0xffff0000u)};
  const f32x2 r = v - hf;
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
  const f32x2 mf = {__uint_as_float(mu << 16), __uint_as_float(mu & 0xffff0000u)};
  const f32x2 s = r - mf;
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(s, bf16x2));
}

__device__ __forceinline__ f32x4 mfma16_bf16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ void project3_body(const float* __restrict__ z, int T, int nq, int tc,
                                              int b, int s, const float* __restrict__ w_in_t,
                                              const PartSink& out, int NF, char* lds,
                                              unsigned long long* stamps = nullptr) {
  constexpr int NIT = (PJ_CPS / 8) * PJ2_TC / PJ2_NT;  // (octet, frame) items per thread: 3
  constexpr int NKS = PJ_CPS / 32;                      // K steps of 32 channels
  const int R = nq * RCD;
  const int t0 = tc * PJ2_TC;
  const int ntl = min(PJ2_TC, T - t0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_rt = (R + 15) / 16;
  const int lr = lane & 15, kg = lane >> 4;
  // A operands of a work item (16-row tile rt): row r = 16 rt + lr, channels 32 ks + 8 kg .. +7
  // of the split (w_in_t[stage][c][k]); rows >= R zeroed
  auto load_w = [&](int rt, float (&w)[NKS][8]) {
    const int r = rt * 16 + lr;
    const unsigned rm = 0u - (unsigned)(r < R);
    const float* wp = w_in_t + ((size_t)min(r >> 3, nq - 1) * RD + s * PJ_CPS + 8 * kg) * RCD + (r & 7);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int u = 0; u < 8; ++u)
        w[ks][u] = __uint_as_float(__float_as_uint(wp[(size_t)(32 * ks + u) * RCD]) & rm);
  };
  float w[NKS][8];
  // the first item's weights (L2) first: their latency runs under the z slab's
  load_w(min(wave, 2 * n_rt - 1) >> 1, w);
  const float* zb = z + ((size_t)b * RD + s * PJ_CPS) * T + t0;
  {  // the slab: every load in flight, then split and stored transposed
    float zv[NIT][8];
#pragma unroll
    for (int q = 0; q < NIT; ++q) {
      const int e = tid + PJ2_NT * q;
      const int o = e / PJ2_TC, t = e - o * PJ2_TC;
#pragma unroll
      for (int u = 0; u < 8; ++u) zv[q][u] = zb[(size_t)(8 * o + u) * T + min(t, ntl - 1)];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < NIT; ++q) {
      const int e = tid + PJ2_NT * q;
      const int o = e / PJ2_TC, t = e - o * PJ2_TC;
      const unsigned m = 0u - (unsigned)(t < ntl);
      unsigned h[4], mm[4], l[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        rvq_split3x2(__uint_as_float(__float_as_uint(zv[q][2 * u]) & m),
                     __uint_as_float(__float_as_uint(zv[q][2 * u + 1]) & m), h[u], mm[u], l[u]);
      char* d = lds + t * (PJ3_LDB * 2) + o * 16;
      *reinterpret_cast<u32x4*>(d) = u32x4{h[0], h[1], h[2], h[3]};
      *reinterpret_cast<u32x4*>(d + PJ3_PLANE) = u32x4{mm[0], mm[1], mm[2], mm[3]};
      *reinterpret_cast<u32x4*>(d + 2 * PJ3_PLANE) = u32x4{l[0], l[1], l[2], l[3]};
    }
  }
  // a use of the weights here keeps their loads ahead of the slab's (else they are sunk below
  // the barrier and waited for one K step at a time)
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int u = 0; u < 8; ++u) asm volatile("" ::"v"(w[ks][u]));
  __syncthreads();
  FSTAMP(stamps, 44);
  // work items (16-row tile rt, half hf = frame tiles 3 hf .. 3 hf + 2) over the 8 waves
  for (int item = wave; item < 2 * n_rt; item += PJ2_NT / 64) {
    const int rt = item >> 1, hf = item & 1;
    if (item != wave) load_w(rt, w);
    f32x4 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      unsigned h[4], mm[4], l[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) rvq_split3x2(w[ks][2 * u], w[ks][2 * u + 1], h[u], mm[u], l[u]);
      const u32x4 ah = {h[0], h[1], h[2], h[3]}, am = {mm[0], mm[1], mm[2], mm[3]},
                  al = {l[0], l[1], l[2], l[3]};
      // the three column tiles' products interleaved (three independent accumulators: the
      // matrix core is not left waiting on a dependent MFMA); per tile the order stays
      // m m, h l, l h, h m, m h, h h
      u32x4 bh[3], bm[3], bl[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const char* bp = lds + ((3 * hf + j) * 16 + lr) * (PJ3_LDB * 2) + (32 * ks + 8 * kg) * 2;
        bh[j] = *reinterpret_cast<const u32x4*>(bp);
        bm[j] = *reinterpret_cast<const u32x4*>(bp + PJ3_PLANE);
        bl[j] = *reinterpret_cast<const u32x4*>(bp + 2 * PJ3_PLANE);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16_bf16(am, bm[j], acc[j]);  // m m
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16_bf16(ah, bl[j], acc[j]);  // h l
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16_bf16(al, bh[j], acc[j]);  // l h
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16_bf16(ah, bm[j], acc[j]);  // h m
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16_bf16(am, bh[j], acc[j]);  // m h
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16_bf16(ah, bh[j], acc[j]);  // h h
      __builtin_amdgcn_sched_barrier(0);  // one K step's operands live at a time
    }
    // D layout: lane l, reg q -> row 4 (l >> 4) + q of the tile, frame l & 15
    const int rr = rt * 16 + 4 * kg;  // rows rr..rr+3 all valid iff rr < R (R = 8 nq)
    if (rr < R) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int t = (3 * hf + j) * 16 + lr;
        if (t < ntl) {
          const size_t n = (size_t)b * T + t0 + t;
          out.put(((size_t)s * NF + n) * R + rr, make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]));
        }
      }
    }
  }
}

__global__ __launch_bounds__(PJ2_NT) void rvq_project3_kernel(const float* __restrict__ z, int T,
                                                              int nq, int n_tc,
                                                              const float* __restrict__ w_in_t,
                                                              float* __restrict__ part, int NF) {
  extern __shared__ __attribute__((aligned(16))) char lds3[];
  PartSink out{part, __builtin_amdgcn_make_buffer_rsrc(part, (short)0, 0, RSRC_FLAGS), 0u};
  project3_body(z, T, nq, blockIdx.x % n_tc, blockIdx.x / n_tc, blockIdx.y, w_in_t, out, NF, lds3);
}

// ------------------------------------------------------------------------------------------
// The chain. Workgroup = frames [n0, n0 + nf) of the flattened (b, t) axis, nf <= 16; 8 waves.
//
// Stage i, S1 (all waves):
//   - deferred U updates: pu[f][ip] -= M_{ip,i-1} zst_{i-1} for ip > i (spread over all threads,
//     issued after the candidate-row gather so they run under its L2 latency; ip = i was done on
//     the critical path in S2 of stage i-1);
//   - distance scan on the matrix cores: wave w owns codes [w N/8, (w+1) N/8) as 16-code tiles;
//     D[code][frame] = cbn . e by two v_mfma_f32_16x16x4_f32 per tile (k = 0..3, then 4..7 on
//     the same accumulator: the k-ordered fma chain of the reference's dot, bitwise), then per
//     lane dist = fma(D, -2, e2) + c2 over its 32 (code, frame) entries in code order, and a
//     lexicographic (dist, code) min across the 4 lanes of each frame -> per-wave candidate;
//   - per wave and frame, the candidate's raw codebook row (gathered from L2 into LDS);
//   - prefetches of stage i+1 (cbn fragments -> registers; c2 slice and M_{.,i+1} ->
//     registers, stored to LDS at the start of stage i+1).
// S2 (lanes (f, k), f < nf, tid = 8 f + k): cross-wave argmin (wave order = code order, lowest
// code on ties), the winner's raw codeword, loss, zst, the next stage's pu[f][i+1] and z_e.
// One workgroup per CU: F = ceil(B*T / 256) frames each (<= 16).
// Two barriers per stage; outputs stay in LDS until the epilogue.
struct ChainArgs {
  const float* part;   // [8][NFS][nq*8]
  int B, T, nq, F, NF;
  int NFS;             // split stride of part in frames (the three-launch path: NF; the fused
                       // launch from the conv's partials: the frames of the whole call)
  const float* b_in;   // [nq][8]
  const float* qb;     // [nq][8]
  const float* mcol;   // [nq][nq][8][8]
  const float* cb;     // [nq][N][8]
  const float* cbf;    // [nq][8][64][N/128][2] normalised codebook, fragment order
  const float* c2;     // [nq][N]
  const float* imp;    // [B][T] or null
  float level;
  int64_t* codes;      // [B][nq][T]
  float* latents;      // [B][nq*8][T]
  float* loss_pf;      // [B][nq][T]
  float* zst;          // [B][nq][T][8]
  float* mask;         // [B][nq][T] or null
  unsigned long long* stamps;  // diagnostic build only (-DVRVQ_STAMPS): [grid][nq + 1][2][8]
};

#ifdef VRVQ_STAMPS
// In-kernel s_memtime stamps (diagnostic build): lanes 0 of waves 0 and 7 record 8 points per
// stage into a buffer nothing else reads.
#define CSTAMP(stage, step)                                                                  \
  do {                                                                                     \
    if (a.stamps && (tid == 0 || tid == 448)) {                                            \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                          \
      a.stamps[(((size_t)blockIdx.x * (a.nq + 1) + (stage)) * 2 + (tid ? 1 : 0)) * 8 +      \
               (step)] = t_;                                                               \
    }                                                                                      \
  } while (0)
#else
#define CSTAMP(stage, step) do {} while (0)
#endif

// LDS carve (floats), shared by the launcher's size computation.
struct ChainLds {
  int e, e2, cd, ci, cr, pu, lat, zs, code, loss, c2, m, total;
  __host__ __device__ ChainLds(int nq, int F, int N) {
    auto al = [](int x) { return (x + 3) & ~3; };
    int o = 0;
    e = o; o += al(CH_FMAX * RCD);
    e2 = o; o += al(CH_FMAX);
    cd = o; o += al(CH_FMAX * CH_NW);
    ci = o; o += al(CH_FMAX * CH_NW);
    cr = o; o += al(CH_FMAX * CH_NW * RCD);
    pu = o; o += al(F * nq * RCD);
    lat = o; o += al(F * nq * RCD);
    zs = o; o += al(F * nq * RCD);
    code = o; o += al(F * nq);
    loss = o; o += al(F * nq);
    c2 = o; o += al(2 * N);
    m = o; o += al(3 * nq * 64);
    total = o;
  }
};

// ------------------------------------------------------------------------------------------
// In-launch hand-offs of the fused path (rvq_fused_kernel): tagged 8-B granules {value, tag},
// each written whole by ONE sc1 store (two per 16-B store) and read with sc1 loads; the reader
// checks the tag of every granule it uses and re-reads until it matches, so the data is its own
// flag (cdna_hip_programming.md Guideline 16, R2; MI355X_MICROARCH.md: granules are observed
// untorn, also as 16-B sc1 halves). Tags: projection partials 64 epoch, stage i zst
// 64 epoch + i + 1; epochs grow per call on a stream, so an older call's granules never match
// (under stream capture the granule area is zeroed by a memset node and the call uses epoch 1).
// The sync block holds only the error word of the bounded waits.
constexpr unsigned SPIN_MAX = 1u << 19;  // bounded spins (~0.5 s); on the bound: *err = code

// A bounded wait that ran out (a hang averted: it cannot happen with the whole grid resident)
// records its code in the stream's sync block (vrvq_rvq_sync_error) and in the process's
// host-mapped error word (system scope: the host reads it without synchronising, and the next
// vrvq_rvq_encode* call / torch op raises on it: vrvq_rvq_pending_error). The workgroup then
// poisons its outputs (codes -1, z_q / z_q_is NaN) instead of publishing garbage as valid data.
__device__ __forceinline__ void report_timeout(unsigned* err, unsigned* err_host, unsigned code) {
  __hip_atomic_store((gu32*)err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (err_host)
    __hip_atomic_store((gu32*)err_host, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load((gu32*)(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct ChainHandoff {              // fused launches only
  unsigned* err;
  unsigned* err_host;              // host-mapped error word (report_timeout) or null
  unsigned spin_max;               // bound of every wait (SPIN_MAX; smaller in the timeout test)
  unsigned epoch;
  __amdgpu_buffer_rsrc_t part;     // the partials' tagged granules, read with sc1 loads
  unsigned long long* zsh;         // this part's stage-0 block of tagged zst granules
  int zsh_stage;                   // granules per stage
  unsigned long long* stamps;      // diagnostic build only
  int dbg;                         // diagnostic build only: FusedArgs::dbg
};

// Where a chain part gets pu = (P + b_in) - Qb of its frames: CH_SPLIT the 8 split partials of
// the three-launch path (plain loads after the projection kernel), CH_GRANULE the tagged
// partial granules of rvq_fused_kernel, CH_PART the 8 split partials the encoder's last conv wrote in its epilogue (vrvq_conv1d_proj;
// plain loads after that kernel's boundary) in rvq_pt_kernel, which publishes every stage.
constexpr int CH_SPLIT = 0, CH_GRANULE = 1, CH_PART = 3;

template <int NM, int MODE>
__device__ __forceinline__ void chain_body(const ChainArgs& a, float* sm, int n0, int nf,
                                           const ChainHandoff& hx) {
  constexpr bool FUSED = MODE != CH_SPLIT;  // in-launch hand-offs: publishes every stage's zst
  constexpr int N = 256 * NM;
  constexpr int NPW = N / CH_NW;   // codes per wave
  constexpr int NT = NPW / 16;     // 16-code MFMA tiles per wave
  const int nq = a.nq, F = a.F;
  const ChainLds L(nq, F, N);
  float* e_s = sm + L.e;
  float* e2_s = sm + L.e2;
  float* cd_s = sm + L.cd;
  int* ci_s = reinterpret_cast<int*>(sm + L.ci);
  float* cr_s = sm + L.cr;      // [16][8 waves][8]: raw codebook row of each wave's candidate
  float* pu_s = sm + L.pu;      // [F][nq][8]: ((P + b_in) - Qb) - U
  float* lat_s = sm + L.lat;    // [F][nq][8]: z_e (output)
  float* zs_s = sm + L.zs;      // [F][nq][8]: zst (output, and the U updates' input)
  int* code_s = reinterpret_cast<int*>(sm + L.code);
  float* loss_s = sm + L.loss;
  float* c2_s = sm + L.c2;      // [2][N]
  float* m_s = sm + L.m;        // [3][nq][8][8]: M_{.,j} for j = i-1, i, i+1 (mod 3)

  const int R = nq * RCD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rf = tid >> 3, rk = tid & 7;  // S2 roles: (frame, k)
  const bool role = rf < nf;
  const int fl = lane & 15, lg = lane >> 4;  // MFMA roles: frame column, k / row group
  const int cw = wave * NPW;
  CSTAMP(nq, 0);

  // stage 0's operands first: they do not depend on the projection (fused: the loads run
  // under the wait for the clip's projection units)
  for (int e = tid; e < CH_FMAX * RCD; e += CH_NT) e_s[e] = 0.0f;
  for (int e = tid; e < CH_FMAX; e += CH_NT) e2_s[e] = 0.0f;
  float av[NT][2];  // cbn fragments of the current stage: code cw + 16 t + fl, k = 4 kh + lg
  auto load_a = [&](int i, float (&dst)[NT][2]) {  // NT / 2 contiguous float4 per lane
    const float* src = a.cbf + (((size_t)i * CH_NW + wave) * 64 + lane) * (2 * NT);
#pragma unroll
    for (int q = 0; q < NT / 2; ++q) {
      const float4 v = ld4(src + 4 * q);
      dst[2 * q][0] = v.x; dst[2 * q][1] = v.y; dst[2 * q + 1][0] = v.z; dst[2 * q + 1][1] = v.w;
    }
  };
  load_a(0, av);
  for (int e = tid; e < N; e += CH_NT) c2_s[e] = a.c2[e];
  if (nq > 1)
    for (int e = tid; e < R * RCD / 4; e += CH_NT)
      reinterpret_cast<float4*>(m_s)[e] = ld4(a.mcol + (size_t)e * 4);
  // ---- prologue: pu = (P + b_in) - Qb (partials summed in split order); stage 0 operands.
  __shared__ int dead_s;  // a bounded wait ran out in this workgroup: outputs poisoned
  if (tid == 0) dead_s = 0;
  if constexpr (MODE == CH_GRANULE) {
    // the clip's 8 partials of this part's frames: tagged granules (16-B sc1 loads, two each),
    // each thread re-reads its item until every tag is this call's (the projection units of
    // the clip run concurrently on other CUs); R = 8 nq: the frames' rows are contiguous
    const unsigned ptag = hx.epoch * 64u;
    for (int e4 = tid; e4 < nf * R / 4; e4 += CH_NT) {
      u32x4 v[PJ_SPLIT][2];
      for (unsigned it = 0;; ++it) {
#pragma unroll
        for (int sp = 0; sp < PJ_SPLIT; ++sp) {
          const int off = (int)((((size_t)sp * a.NF + n0) * R + 4 * e4) * 8);
          v[sp][0] = __builtin_amdgcn_raw_buffer_load_b128(hx.part, off, 0, CPOL_SC1);
          v[sp][1] = __builtin_amdgcn_raw_buffer_load_b128(hx.part, off + 16, 0, CPOL_SC1);
        }
        bool ok = true;
#pragma unroll
        for (int sp = 0; sp < PJ_SPLIT; ++sp)
          ok = ok && v[sp][0][1] == ptag && v[sp][0][3] == ptag && v[sp][1][1] == ptag &&
               v[sp][1][3] == ptag;
        if (ok) break;
        if (it >= hx.spin_max) {
          report_timeout(hx.err, hx.err_host, 1u);
          dead_s = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      FSTAMP(hx.stamps, 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pv = __uint_as_float(v[0][j >> 1][2 * (j & 1)]);
#pragma unroll
        for (int sp = 1; sp < PJ_SPLIT; ++sp) pv = pv + __uint_as_float(v[sp][j >> 1][2 * (j & 1)]);
        const int e = 4 * e4 + j, r = e % R;
        pu_s[e] = (pv + a.b_in[r]) - a.qb[r];
      }
    }
  } else
  // Two (frame, row) items per thread per pass with all 16 partial loads in flight.
  for (int e0 = tid; e0 < nf * R; e0 += 2 * CH_NT) {
    float v[2][PJ_SPLIT];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = e0 + h * CH_NT;
      const size_t base = (size_t)n0 * R + (e < nf * R ? e : 0);
#pragma unroll
      for (int sp = 0; sp < PJ_SPLIT; ++sp) v[h][sp] = a.part[(size_t)sp * a.NFS * R + base];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = e0 + h * CH_NT;
      if (e < nf * R) {
        const int r = e % R;
        float pv = v[h][0];
#pragma unroll
        for (int sp = 1; sp < PJ_SPLIT; ++sp) pv = pv + v[h][sp];
        pu_s[e] = (pv + a.b_in[r]) - a.qb[r];
      }
    }
  }
  __syncthreads();
  float ze = 0.0f;  // S2 lanes: z_e of (rf, rk) at the current stage
  auto set_e = [&](float zv) {  // F.normalize (eps 1e-12) of the 8-lane group's z_e
    ze = zv;
    const float n2 = vrvq::sum8(ze * ze, lane);
    const float e = ze / fmaxf(sqrtf(n2), 1e-12f);
    const float e2 = vrvq::sum8(e * e, lane);
    if (role) {
      e_s[rf * RCD + rk] = e;
      if (rk == 0) e2_s[rf] = e2;
    }
  };
  set_e(role ? pu_s[(rf * nq) * RCD + rk] : 0.0f);
  __syncthreads();
  CSTAMP(nq, 1);
  if constexpr (FUSED) FSTAMP(hx.stamps, 3);

  // next stage's c2 slice / M column: loaded during a stage, stored to LDS at the start of the
  // next (no wait on a load issued in the same stage)
  constexpr int C2W = (NPW + 63) / 64;
  float c2n[C2W];
  float4 mn = make_float4(0.f, 0.f, 0.f, 0.f);
  // fused: waves 0-1 = frames 0..15 x k publish the part's 16-frame block of a stage as tagged
  // 8-B granules {zst, 64 epoch + i + 1} (one sc1 store each: the data is its own flag, no
  // drain, no flag word), k = 2 s + h at slot 4 h + s of the frame (a consumer lane's four k
  // values are 32 contiguous bytes); frames >= nf store 0 with the tag
  auto publish = [&](int st, float v) {
    if (wave < 2) {
      const unsigned long long g =
          ((unsigned long long)(hx.epoch * 64u + (unsigned)st + 1u) << 32) | __float_as_uint(v);
      __hip_atomic_store((gu64*)(hx.zsh + (size_t)st * hx.zsh_stage +
                                 (rf * 8 + (rk & 1) * 4 + (rk >> 1))),
                         g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  for (int i = 0; i < nq; ++i) {
    const bool more = i + 1 < nq;
    // ---- S1 ----
    CSTAMP(i, 0);
    if (i > 0) {
      // stage i operands prefetched during stage i-1: M_{.,i} (read by other waves after
      // barrier 1) and this wave's c2 slice (read by this wave only)
#pragma unroll
      for (int q = 0; q < C2W; ++q)
        if (lane + 64 * q < NPW) c2_s[(i & 1) * N + cw + lane + 64 * q] = c2n[q];
      if (i + 1 < nq && tid * 4 < R * RCD)
        reinterpret_cast<float4*>(m_s + (i % 3) * R * RCD)[tid] = mn;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the c2 slice is in LDS for the scan
    }
    // deferred U updates from stage i-1 for targets ip > i (needed from S2 of this stage on):
    // run after the scan has issued its candidate-row gather, under that L2 latency
    auto deferred_updates = [&]() {
      if (i == 0) return;
      const int nip = nq - 1 - i;
      const float* mj = m_s + ((i - 1) % 3) * R * RCD;
      for (int e = tid; e < nf * nip * RCD; e += CH_NT) {
        const int k = e & 7, q = e >> 3;
        const int f = q / nip, ip = i + 1 + (q - f * nip);
        const float* zr = zs_s + (f * nq + (i - 1)) * RCD;
        const float* mr = mj + (ip * RCD + k) * RCD;
        float* pp = pu_s + (f * nq + ip) * RCD + k;
        *pp = *pp - dot8(ld4(mr), ld4(mr + 4), ld4(zr), ld4(zr + 4));
      }
    };
    CSTAMP(i, 1);
    float an[NT][2];
    CSTAMP(i, 2);
    {
      // distance scan: 16 frames x NT 16-code tiles, K = 8 as two k-quads. All MFMAs first
      // (NT independent accumulators), c2 read before them; then 4 independent argmin chains
      // (one per accumulator row r: codes cw + 16 t + 4 lg + r in increasing t) merged
      // lexicographically (dist, code) -- the same result as one chain in code order.
      const float b0 = e_s[fl * RCD + lg], b1 = e_s[fl * RCD + 4 + lg];
      const float e2 = e2_s[fl];
      const float* c2c = c2_s + (i & 1) * N + cw + 4 * lg;
      float4 cc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) cc[t] = ld4(c2c + t * 16);
      f32x4 d[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        d[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][0], b0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      float bst[4];
      int bix[4];  // 16 t of the best entry (a constant per entry: no per-entry index add)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bst[r] = INFINITY;
        bix[r] = 0;
      }
      const f32x2 m2 = {-2.0f, -2.0f}, e22 = {e2, e2};
      auto amin_tile = [&](int t) {
        // (sum e^2 - 2 e.c) + sum c^2 with the first step as fma(d, -2, e2): 2d is exact,
        // so this is the reference's rounding (models/quantize.py:96-100); two entries per
        // packed fma / add (v_pk_fma_f32, v_pk_add_f32: the same per-element roundings)
        const f32x2 d01 = {d[t][0], d[t][1]}, d23 = {d[t][2], d[t][3]};
        const f32x2 c01 = {cc[t].x, cc[t].y}, c23 = {cc[t].z, cc[t].w};
        const f32x2 s01 = __builtin_elementwise_fma(d01, m2, e22) + c01;
        const f32x2 s23 = __builtin_elementwise_fma(d23, m2, e22) + c23;
        const float dist[4] = {s01.x, s01.y, s23.x, s23.y};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool take = dist[r] < bst[r];  // increasing code index: strict < keeps the first
          bst[r] = take ? dist[r] : bst[r];
          bix[r] = take ? t * 16 : bix[r];
        }
      };
      // the second k-quad of tile t, then the argmin of tile t - 1 (whose MFMAs are done): the
      // compare / select VALU of one tile issues while the matrix core runs the next tile
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        d[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][1], b1, d[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (t > 0) amin_tile(t - 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      amin_tile(NT - 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) bix[r] += cw + 4 * lg + r;
      vrvq::amin(bst[0], bix[0], bst[1], bix[1]);
      vrvq::amin(bst[2], bix[2], bst[3], bix[3]);
      vrvq::amin(bst[0], bix[0], bst[2], bix[2]);
      float best = bst[0];
      int bidx = bix[0];
      vrvq::amin(best, bidx, vrvq::xchg<16>(best, lane), vrvq::xchg<16>(bidx, lane));
      vrvq::amin(best, bidx, vrvq::xchg<32>(best, lane), vrvq::xchg<32>(bidx, lane));
      // the candidate's raw codebook row (L2 gather, models/quantize.py:101-103): only the
      // wave's own candidates, so no per-stage staging of the whole raw codebook (measured: an
      // LDS copy of the stage's codebook, prefetched a stage ahead, is slower -- the gather's
      // latency hides behind the other wave of the SIMD). Issued before the next stage's
      // prefetch, so the wait for it does not cover the prefetch.
      const float* row = a.cb + ((size_t)i * N + (lane < nf ? bidx : 0)) * RCD;
      const float4 r0 = ld4(row), r1 = ld4(row + 4);
      __builtin_amdgcn_sched_barrier(0);  // keep the gather ahead of the prefetch (vmcnt order)
      {  // stage i+1 operands (cbn fragments, c2 slice, M column). Unconditional loads from
         // clamped addresses (the last stage re-reads its own): a branch around them makes the
         // waitcnt pass assume none are outstanding at the join, so the candidate-row wait
         // below would drain the whole prefetch.
        const int in = more ? i + 1 : i;
#ifdef VRVQ_STAMPS
        if (FUSED && (hx.dbg & 2)) {  // timing experiment: no per-stage codebook stream
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            an[t][0] = av[t][0];
            an[t][1] = av[t][1];
          }
        } else
#endif
        load_a(in, an);
#pragma unroll
        for (int q = 0; q < C2W; ++q)
          c2n[q] = a.c2[(size_t)in * N + cw + min(lane + 64 * q, NPW - 1)];
        // M_{.,i+1}: needed from stage i+1 on (stored only when i + 2 < nq)
        mn = ld4(a.mcol + (size_t)min(i + 1, nq - 1) * R * RCD + min(tid * 4, R * RCD - 4));
      }
      deferred_updates();
      if (lane < nf) {
        cd_s[lane * CH_NW + wave] = best;
        ci_s[lane * CH_NW + wave] = bidx;
        float* crw = cr_s + (lane * CH_NW + wave) * RCD;
        *reinterpret_cast<float4*>(crw) = r0;
        *reinterpret_cast<float4*>(crw + 4) = r1;
      }
    }
    CSTAMP(i, 3);
    __syncthreads();  // ------------------------------- candidates, stage i+1's c2 / M ready
    CSTAMP(i, 4);
    // ---- S2 (role lanes) ----
    int bi = 0;
    float zq = 0.0f;
    if (role) {
      const float4 d0 = ld4(cd_s + rf * CH_NW), d1 = ld4(cd_s + rf * CH_NW + 4);
      const int4 i0 = *reinterpret_cast<const int4*>(ci_s + rf * CH_NW);
      const int4 i1 = *reinterpret_cast<const int4*>(ci_s + rf * CH_NW + 4);
      const float dv[CH_NW] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
      const int iv[CH_NW] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
      float bd = dv[0];
      bi = iv[0];
      int bw = 0;
#pragma unroll
      for (int w = 1; w < CH_NW; ++w) {  // wave order = code order: strict < keeps the lowest
        const bool take = dv[w] < bd;
        bd = take ? dv[w] : bd;
        bi = take ? iv[w] : bi;
        bw = take ? w : bw;
      }
      bi = (bi >= 0 && bi < N) ? bi : 0;
      zq = cr_s[(rf * CH_NW + bw) * RCD + rk];  // raw codebook row of the winner
    }
    const float zsv = ze + (zq - ze);  // z_e + (z_q - z_e).detach(), models/quantize.py:73-75
    if constexpr (FUSED) publish(i, zsv);
    const float diff = ze - zq;
    const float l2 = vrvq::sum8(diff * diff, lane);
    if (role) {
      lat_s[(rf * nq + i) * RCD + rk] = ze;
      zs_s[(rf * nq + i) * RCD + rk] = zsv;
      if (rk == 0) {
        code_s[rf * nq + i] = bi;
        loss_s[rf * nq + i] = l2 / 8.0f;  // mse over codebook_dim, models/quantize.py:69-71
      }
    }
    CSTAMP(i, 5);
    if (more) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this group's zst row is in LDS
      float zn = 0.0f;
      if (role) {
        const float* zr = zs_s + (rf * nq + i) * RCD;
        const float* mr = m_s + (i % 3) * R * RCD + ((i + 1) * RCD + rk) * RCD;
        float* pp = pu_s + (rf * nq + i + 1) * RCD + rk;
        zn = *pp - dot8(ld4(mr), ld4(mr + 4), ld4(zr), ld4(zr + 4));
        *pp = zn;
      }
      set_e(zn);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        av[t][0] = an[t][0];
        av[t][1] = an[t][1];
      }
    }
    CSTAMP(i, 6);
    __syncthreads();  // ------------------------------------------------- next stage's e
    CSTAMP(i, 7);
    if constexpr (FUSED) FSTAMP(hx.stamps, 4 + i);
  }
  CSTAMP(nq, 2);

  // ---- epilogue: outputs of every stage (LDS -> HBM); poisoned after a timed-out wait
  const bool dead = FUSED && dead_s != 0;
  for (int e = tid; e < nf * nq * RCD; e += CH_NT) {
    // zst [b][i][t][k] and latents [b][i*8+k][t]
    const int k = e & 7, fi = e >> 3;
    const int i = fi / nf, f = fi - i * nf;
    const int n = n0 + f, b = n / a.T, t = n - b * a.T;
    if (a.zst) a.zst[(((size_t)b * nq + i) * a.T + t) * RCD + k] = zs_s[(f * nq + i) * RCD + k];
    a.latents[(((size_t)b * nq + i) * RCD + k) * a.T + t] =
        dead ? __builtin_nanf("") : lat_s[(f * nq + i) * RCD + k];
  }
  for (int e = tid; e < nf * nq; e += CH_NT) {
    const int i = e / nf, f = e - i * nf;
    const int n = n0 + f, b = n / a.T, t = n - b * a.T;
    const size_t o = ((size_t)b * nq + i) * a.T + t;
    a.codes[o] = dead ? (int64_t)-1 : (int64_t)code_s[f * nq + i];
    a.loss_pf[o] = loss_s[f * nq + i];
    if (a.mask) {
      const float s = a.imp ? (a.imp[n] * a.level) * (float)nq : INFINITY;
      a.mask[o] = (s - (float)i >= 0.0f) ? 1.0f : 0.0f;  // models/utils.py:55-61
    }
  }
  CSTAMP(nq, 3);
  if constexpr (FUSED) FSTAMP(hx.stamps, 36);
}

template <int NM>
__global__ __launch_bounds__(CH_NT) void rvq_chain_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n0 = blockIdx.x * a.F;
  chain_body<NM, CH_SPLIT>(a, sm, n0, min(a.F, a.NF - n0), ChainHandoff{});
}

// ------------------------------------------------------------------------------------------
// Expansion on the matrix cores: z_q_is[b,i,c,t] = (W_out(i)[c,:] . zst[b,i,t,:]) + b_out(i)[c]
// and z_q[b,c,t] = sum_i mask[b,i,t] * z_q_is[b,i,c,t] (stage order, from 0: the masked_sum
// kernel's expression bit for bit). One wave = one (clip, 32-channel, 32-frame) tile over all
// stages; per stage four v_mfma_f32_32x32x2_f32 (K = 8: the out_proj weights x zst, the
// k-ordered fma chain from 0) and the bias as one VALU add -- dot8(W, zst) + bias with the
// reference's roundings (r05: the bias was a 9th k of a fifth MFMA, the same value up to the
// sign of an exact zero). The accumulator layout puts 32 consecutive frames of one channel row
// in each half-wave, so every store instruction writes two 128-B row runs.
struct ExpandArgs {
  const float* zst;    // [B][nq][T][8]
  int B, D, T, nq;
  const float* w_out;  // [nq][D][8]
  const float* b_out;  // [nq][D]
  const float* imp;    // [B][T] or null
  float level;
  const float* mask_in;  // [B][nq][T] or null: explicit mask values (training), replaces imp
  float* z_q_is;       // [B][nq][D][T] or null
  float* z_q;          // [B][D][T]
  float* mask;         // [B][nq][T] or null
  int n_ct, n_tt;      // 32-channel tiles, 32-frame tiles
};

__global__ __launch_bounds__(256) void rvq_expand_kernel(ExpandArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // workgroup = 4 consecutive channel tiles of one (clip, frame tile)
  int bid = blockIdx.x;
  const int ctg = bid % ((a.n_ct + 3) / 4);
  bid /= (a.n_ct + 3) / 4;
  const int tt = bid % a.n_tt;
  const int b = bid / a.n_tt;
  const int ct = ctg * 4 + wave;
  if (ct >= a.n_ct) return;  // no barrier in this kernel
  const int c0 = ct * 32, t0 = tt * 32;
  const int col = lane & 31, h = lane >> 5;
  const int t = t0 + col;
  const bool tv = t < a.T;
  const int tc = tv ? t : a.T - 1;
  const int cr = min(c0 + col, a.D - 1);  // A-operand row of this lane (clamped: D % 32 tail)
  const float s = (a.imp && tv) ? (a.imp[(size_t)b * a.T + t] * a.level) * (float)a.nq : INFINITY;
  const float* zp = a.zst + ((size_t)b * a.nq * a.T + tc) * RCD;
  const size_t zstride = (size_t)a.T * RCD;
  const float* wp = a.w_out + (size_t)cr * RCD;
  const size_t wstride = (size_t)a.D * RCD;
  f32x16 zq;
#pragma unroll
  for (int r = 0; r < 16; ++r) zq[r] = 0.0f;
  // operands of stage i, software-pipelined one stage ahead (the wait for them never covers
  // the previous stage's stores: vmcnt counts stores too)
  // b_out of the accumulator rows c0 + 4 h + (r & 3) + 8 (r >> 2) (clamped at a D % 32 tail:
  // those rows are not stored; D >= 4), loaded for the current stage ahead of the next stage's
  // prefetch
  float4 w0 = ld4(wp), w1 = ld4(wp + 4), z0 = ld4(zp), z1 = ld4(zp + 4);
  for (int i = 0; i < a.nq; ++i) {
    const float4 cw0 = w0, cw1 = w1, cz0 = z0, cz1 = z1;
    float cb[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = ld4(a.b_out + (size_t)i * a.D + min(c0 + 4 * h + 8 * q, a.D - 4));
      cb[4 * q] = v.x; cb[4 * q + 1] = v.y; cb[4 * q + 2] = v.z; cb[4 * q + 3] = v.w;
    }
    if (i + 1 < a.nq) {
      w0 = ld4(wp + (i + 1) * wstride);
      w1 = ld4(wp + (i + 1) * wstride + 4);
      z0 = ld4(zp + (i + 1) * zstride);
      z1 = ld4(zp + (i + 1) * zstride + 4);
    }
    // lane (col, h) supplies k = 2 s + h of step s
    const float wa[4] = {h ? cw0.y : cw0.x, h ? cw0.w : cw0.z, h ? cw1.y : cw1.x, h ? cw1.w : cw1.z};
    const float zb[4] = {h ? cz0.y : cz0.x, h ? cz0.w : cz0.z, h ? cz1.y : cz1.x, h ? cz1.w : cz1.z};
    f32x16 q;
#pragma unroll
    for (int r = 0; r < 16; ++r) q[r] = 0.0f;
#pragma unroll
    for (int st = 0; st < 4; ++st) q = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[st], zb[st], q, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) q[r] = q[r] + cb[r];
    const float m = a.mask_in ? (tv ? a.mask_in[((size_t)b * a.nq + i) * a.T + t] : 0.0f)
                              : ((s - (float)i >= 0.0f) ? 1.0f : 0.0f);  // models/utils.py:45-61
    if (a.mask && ct == 0 && h == 0 && tv) a.mask[((size_t)b * a.nq + i) * a.T + t] = m;
    if (a.z_q_is && tv) {
      float* dst = a.z_q_is + (((size_t)b * a.nq + i) * a.D + c0 + 4 * h) * a.T + t;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2);
        if (c0 + 4 * h + row < a.D) dst[(size_t)row * a.T] = q[r];
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) zq[r] = zq[r] + q[r] * m;
  }
  if (tv) {
    float* dst = a.z_q + ((size_t)b * a.D + c0 + 4 * h) * a.T + t;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2);
      if (c0 + 4 * h + row < a.D) dst[(size_t)row * a.T] = zq[r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// The fused RVQ launches: one kernel instead of projection -> chain -> expansion, every
// workgroup of the grid resident at once (clips per launch from the occupancy query).
//
// rvq_fused_kernel (z [B][D][T], T <= 96): workgroups [0, 8 B) are (clip b, split / part s): the
// projection unit (b, s) (project3_body, partials stored as tagged granules), then chain part s
// of clip b (frames [s F, s F + F), F = ceil(T / 8)), which reads the clip's 8 partials of its
// frames as they land and publishes every stage's zst.
//
// rvq_pt_kernel (below: from the encoder conv's projection partials, any T): workgroups
// [0, B P) are chain parts (clip b, frames [p F, p F + F), F <= 16).
//
// In both, the workgroups after the chain parts are the expansion: (clip b, frame block fb,
// 128-channel block cb) over all stages, each stage once the chain parts of its frames have
// published it, so the z_q_is write stream runs under the chain instead of after it. Same
// expressions as the three launches (tests/test_gpu_parity.py).
constexpr int FU_NP = PJ_SPLIT;     // chain parts per clip of rvq_fused_kernel
constexpr int FU_ROWS = 16;         // frames per part block of the stage hand-off rows (F <= 16)
constexpr int FU_CB = 128;          // channels per expansion workgroup
constexpr int FU_FB = 128;          // frames per expansion workgroup
constexpr int SYNC_ERR = 2048;      // the error word (1 partials wait, 2 stage wait)
constexpr int SYNC_WORDS = 2052;    // used words (x 4 = 8208 B, a multiple of 16)
constexpr int FU_CLIPS_MAX = 32;    // clips per rvq_fused_kernel launch

struct FusedArgs {
  ChainArgs c;                      // part (workspace), B, T, nq, F, NF; outputs
  const float* z;                   // [B][D][T] (rvq_fused_kernel)
  const float* w_in_t;
  const float* w_out;               // [nq][D][8]
  const float* b_out;               // [nq][D]
  float* z_q_is;                    // [B][nq][D][T] or null
  float* z_q;                       // [B][D][T]
  unsigned long long* zsh;          // [B][nq][P][FU_ROWS][8] tagged zst granules
  int zsh_bytes;
  int P;                            // chain parts per clip
  int n_fb;                         // expansion frame blocks per clip
  unsigned* sync;
  unsigned* err_host;               // host-mapped error word (report_timeout) or null
  unsigned spin_max;
  unsigned stall;                   // test knob: chain part 0's start delayed by stall x s_sleep(127)
  unsigned epoch;
  unsigned long long* stamps;       // diagnostic build only
  int dbg;                          // diagnostic build only: bit 0 = expansion skips its MFMAs,
                                    // bit 1 = chain parts skip the next stage's codebook
                                    // fragment loads (outputs wrong; timing only)
  int warm;                         // expansion workgroups pull the stage tables into L2 first
  int poll2;                        // rvq_pt_kernel's loader keeps two looks in flight
};

// The stage tables the chain and the expansion read after stage 0 (normalised / raw codebooks,
// c2, M, W_out, b_out): inside the bench step the encoder's convs have evicted them from L2, and
// the expansion workgroups idle until the chain's first stage anyway. Expansion workgroup e of
// the launch touches slice (e / 8) of every table (workgroups are dealt to the 8 XCDs in turn,
// so each XCD's L2 gets a whole copy); the loaded values feed a sum nothing uses.
__device__ __forceinline__ void warm_tables(const FusedArgs& f, int e, int n_exp, int N,
                                            float* sm) {
  const int slices = max(1, n_exp / 8), k = (e / 8) % slices;
  const size_t nq = (size_t)f.c.nq;
  unsigned acc = 0;
  auto touch = [&](const float* p, size_t n) {  // n floats, a multiple of 4
    const size_t per = ((n / 4 + slices - 1) / slices) * 4;
    const size_t lo = (size_t)k * per, hi = min(n, lo + per);
    for (size_t i = lo + 4 * threadIdx.x; i < hi; i += 4 * blockDim.x) {
      const float4 v = ld4(p + i);
      acc ^= __float_as_uint(v.x) ^ __float_as_uint(v.w);
    }
  };
  touch(f.c.cbf, nq * N * RCD);
  touch(f.c.cb, nq * N * RCD);
  touch(f.c.c2, nq * N);
  touch(f.c.mcol, nq * nq * RCD * RCD);
  touch(f.w_out, nq * RD * RCD);
  touch(f.b_out, nq * RD);
  if (acc == f.spin_max + 0x5a5a5a5au) sm[threadIdx.x] = __uint_as_float(acc);  // never in practice
}

// Expansion workgroup (clip b, frames [128 fb, +128), channels [128 cb, +128)): wave w =
// 32-channel tile (w & 3) x 32-frame tiles {w >> 2, (w >> 2) + 2} of the block; per stage four
// v_mfma_f32_32x32x2_f32 per tile, D[channel][frame] = sum_k W_out[channel][k] zst[frame][k]
// (rvq_expand_kernel's k-ordered products). D leaves the MFMA with one frame per lane and four
// consecutive channels per register quad; a 4 x 4 transpose inside each lane quad (two DPP
// quad_perm exchanges) turns that into four consecutive FRAMES of one channel per register
// quad, so z_q_is / z_q leave as 16-B stores that cover 8 whole 128-B row segments per wave
// instruction (r04's 4-B stores needed 4x the instructions; 16-B stores straight from the
// frame-major D orientation touched 32 rows per instruction and ran slower still:
// profiles/r05i_stamps.log). Bias and mask are then per register (the three-launch kernel's
// expressions, per element).
// The stage's zst rows are tagged granules (the chain's S2 stores). The workgroup reads its
// 128-frame window of them ONCE per stage, 16 B per lane, into an LDS slab (double-buffered,
// one barrier per stage) that every wave takes its B operands from -- r05k's waves each read
// the rows of their own tiles, 4x the workgroup's sc1 reads. A lane loads its slice of stage
// i + 1 (and its W_out row / biases) speculatively BEFORE stage i's stores and checks the tags
// when it gets there -- vmcnt retires in order, so a load issued after the stores would wait
// for them to drain (profiles/r04d_fused_timeline.txt). Slices whose tags are not this call's
// stage yet are re-read until they are (bounded; on the bound the outputs are NaN).
// What bounds a stage is the z_q_is write stream (11.4 MB per stage at B = 32); the same store
// pattern alone writes at 4-5.7 TB/s (tools/micro/expand_writes.hip), next to the chain ~2.7.
struct ExOps {
  float4 w0, w1;
  float bb[4];    // b_out of the lane's four output channels (one per register quad)
};
constexpr int FU_EX_LDS = 2 * FU_FB * RCD * 4;  // the zst slab, two stages

// 4 x 4 transpose inside each lane quad: lane 4 g + k, register 4 qd + u holds E(u, k) on
// entry and E(k, u) on exit (E(row, column) of the quad's 4 x 4 block). Two butterfly steps,
// each swapping one index bit of the register with the same bit of the lane.
__device__ __forceinline__ void quad_transpose(f32x16& q, int lane) {
  const bool o1 = lane & 1, o2 = lane & 2;
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {  // register pairs (0, 1), (2, 3): lanes k ^ 1
      const int r0 = 4 * qd + 2 * p, r1 = r0 + 1;
      const float snd = o1 ? q[r0] : q[r1];
      const float got = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd), 0xB1, 0xF, 0xF, false));
      if (o1) q[r0] = got; else q[r1] = got;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {  // register pairs (0, 2), (1, 3): lanes k ^ 2
      const int r0 = 4 * qd + p, r1 = r0 + 2;
      const float snd = o2 ? q[r0] : q[r1];
      const float got = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd), 0x4E, 0xF, 0xF, false));
      if (o2) q[r0] = got; else q[r1] = got;
    }
  }
}

__device__ __forceinline__ void fused_expand_body(const FusedArgs& f, int e, float* sm) {
  const int nq = f.c.nq, T = f.c.T, F = f.c.F;
  constexpr int NCB = RD / FU_CB;
  const int cb = e % NCB;
  const int fb = (e / NCB) % f.n_fb;
  const int b = e / (NCB * f.n_fb);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = cb * FU_CB + (wave & 3) * 32;
  const int col = lane & 31, h = lane >> 5;
  const int n_ft = (min(FU_FB, T - fb * FU_FB) + 31) / 32;  // frame tiles of this block
  const int ft0 = wave >> 2;
  const bool one = ft0 < n_ft;       // wave-uniform: the wave has a first tile
  const bool two = ft0 + 2 < n_ft;   // ... and a second
  const __amdgpu_buffer_rsrc_t zr =
      __builtin_amdgcn_make_buffer_rsrc(f.zsh, (short)0, f.zsh_bytes, RSRC_FLAGS);
  // after the transpose: lane (g = col >> 2, k = lane & 3, h), register 4 qd + u holds channel
  // c0 + 8 qd + 4 h + k, frame tile_base + 4 g + u
  const int chk = c0 + 4 * h + (lane & 3);  // + 8 qd
  // the slab window: 128 frames from wlo (the last block's window ends at the clip's last frame,
  // so it holds the moved-back last tile); lane tid loads frame wlo + (tid >> 2), dims
  // 2 (tid & 3) + {0, 1} (frames past the clip re-read its last one: loaded, never used)
  const int wlo = T >= FU_FB ? min(fb * FU_FB, T - FU_FB) : 0;
  const int fi = tid >> 2, dp = tid & 3;
  int soff;
  {
    const int t = min(wlo + fi, T - 1);
    const int p = t / F, fr = t - p * F;
    soff = ((((b * nq) * f.P + p) * FU_ROWS + fr) * RCD + 2 * dp) * 8;
  }
  int trow[2];    // the lane's B-operand frame (col) as a slab row
  int tq[2];      // first of the lane's four output frames
  unsigned nact[2];  // per output frame u: the number of active stages (mask = i < n), bytes
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    // the tile's first frame; a clip's last, partial tile is moved back to end at the clip's
    // last frame (it overlaps the tile before it: those frames are computed and written twice,
    // with identical values), so every quad of four frames is whole from T = 32 on
    int tb = fb * FU_FB + (ft0 + 2 * j) * 32;
    if (tb + 32 > T && T >= 32) tb = T - 32;
    trow[j] = min(tb - wlo + col, FU_FB - 1);
    tq[j] = tb + 4 * (col >> 2);
    float sv[4];  // the loads first: one memory latency
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = min(tq[j] + u, T - 1);
      sv[u] = f.c.imp ? (f.c.imp[(size_t)b * T + t] * f.c.level) * (float)nq : INFINITY;
    }
    unsigned w = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // mask[b,i,t] = (s - i >= 0) with s = (imp * level) * nq (models/utils.py:45-61). The
      // fp32 difference rounds monotonically and 0 is exact, so that is s >= i: the first
      // floor(s) + 1 stages (none for NaN or s < 0, all nq for s >= nq - 1 or CBR's inf)
      const int n = sv[u] >= 0.0f ? (int)floorf(fminf(sv[u], (float)(nq - 1))) + 1 : 0;
      w |= (unsigned)n << (8 * u);
    }
    nact[j] = w;
  }
  const int zstage = f.P * FU_ROWS * RCD * 8;  // bytes per stage
  const float* wp = f.w_out + (size_t)(c0 + col) * RCD;  // A operand: channel row c0 + col
  const size_t wstride = (size_t)RD * RCD;
  const unsigned base = f.epoch * 64u;
  auto load_s = [&](int i) {
    return __builtin_amdgcn_raw_buffer_load_b128(zr, soff + i * zstage, 0, CPOL_SC1);
  };
  auto load = [&](int i, ExOps& o) {
    o.w0 = ld4(wp + i * wstride);
    o.w1 = ld4(wp + i * wstride + 4);
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) o.bb[qd] = f.b_out[(size_t)i * RD + chk + 8 * qd];
  };
  auto late = [&](const u32x4& g, int i) -> bool {  // wave-uniform: a slice is not stage i's
    const unsigned tag = base + (unsigned)i + 1u;
    return __builtin_amdgcn_ballot_w64(!(g[1] == tag && g[3] == tag)) != 0;
  };
  // four consecutive frames of one channel: one 16-B store (rows of T floats are dword-
  // aligned); elementwise only where a clip is shorter than a frame tile (T < 32)
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  auto store_quad = [&](float* row, int t, float v0, float v1, float v2, float v3) {
    if (t + 4 <= T) {
      *reinterpret_cast<f4u*>(row + t) = f4u{v0, v1, v2, v3};
    } else {
      if (t < T) row[t] = v0;
      if (t + 1 < T) row[t + 1] = v1;
      if (t + 2 < T) row[t + 2] = v2;
    }
  };
  f32x16 zq[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) zq[j][r] = 0.0f;
  __shared__ int xdead_s;  // some wave's wait ran out (then no wave waits any more)
  if (tid == 0) xdead_s = 0;
  __syncthreads();
  bool dead = false;       // a wait ran out: no more waits (err recorded), outputs NaN
  u32x4 g = load_s(0);
  ExOps cur;
  load(0, cur);
  for (int i = 0; i < nq; ++i) {
    if (!dead && late(g, i)) {
      // stage 0 lands after the chain's first stage: long sleeps between looks
      for (unsigned it = 0;; ++it) {
        if (it >= f.spin_max) {
          if (lane == 0) report_timeout(f.sync + SYNC_ERR, f.err_host, 2u);
          xdead_s = 1;
          dead = true;
          break;
        }
        if (i == 0) __builtin_amdgcn_s_sleep(16); else __builtin_amdgcn_s_sleep(4);
        g = load_s(i);
        if (!late(g, i)) break;
      }
    }
    if (i < 8) FSTAMP(f.stamps, 56 + i);  // the stage's slice seen (diagnostic build)
    float* slab = sm + (i & 1) * (FU_FB * RCD);
    *reinterpret_cast<float2*>(slab + fi * RCD + 2 * dp) =
        make_float2(__uint_as_float(g[0]), __uint_as_float(g[2]));
    __syncthreads();  // the stage's slab is whole; the other buffer is free (stage i - 1 done)
    dead = xdead_s != 0;
    FSTAMP(f.stamps, 1 + i);
    // the next stage's operands ahead of this stage's stores (unconditional, clamped stage: a
    // branch around loads makes the waitcnt pass drain at the join)
    g = load_s(min(i + 1, nq - 1));
    ExOps nxt;
    load(min(i + 1, nq - 1), nxt);
    const float wa[4] = {h ? cur.w0.y : cur.w0.x, h ? cur.w0.w : cur.w0.z,
                         h ? cur.w1.y : cur.w1.x, h ? cur.w1.w : cur.w1.z};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!(j == 0 ? one : two)) break;
      const float4 zb = *reinterpret_cast<const float4*>(slab + trow[j] * RCD + 4 * h);
      f32x16 q;
#pragma unroll
      for (int r = 0; r < 16; ++r) q[r] = 0.0f;
#ifdef VRVQ_STAMPS
      if (!(f.dbg & 1)) {
#endif
      q = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[0], zb.x, q, 0, 0, 0);
      q = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[1], zb.y, q, 0, 0, 0);
      q = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[2], zb.z, q, 0, 0, 0);
      q = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[3], zb.w, q, 0, 0, 0);
#ifdef VRVQ_STAMPS
      }
#endif
      quad_transpose(q, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) q[r] = dead ? __builtin_nanf("") : q[r] + cur.bb[r >> 2];
      if (f.z_q_is) {
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          float* row = f.z_q_is + (((size_t)b * nq + i) * RD + chk + 8 * qd) * T;
          store_quad(row, tq[j], q[4 * qd], q[4 * qd + 1], q[4 * qd + 2], q[4 * qd + 3]);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned n = (nact[j] >> (8 * (r & 3))) & 0xffu;
        const float m = (unsigned)i < n ? 1.0f : 0.0f;  // models/utils.py:45-61
        zq[j][r] = zq[j][r] + q[r] * m;
      }
    }
    if (i < 8) FSTAMP(f.stamps, 48 + i);  // the stage's stores issued (diagnostic build)
    cur = nxt;
  }
  FSTAMP(f.stamps, 40);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (!(j == 0 ? one : two)) break;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      float* row = f.z_q + ((size_t)b * RD + chk + 8 * qd) * T;
      const float d = dead ? __builtin_nanf("") : 0.0f;
      store_quad(row, tq[j], zq[j][4 * qd] + d, zq[j][4 * qd + 1] + d, zq[j][4 * qd + 2] + d,
                 zq[j][4 * qd + 3] + d);
    }
  }
}

__device__ __forceinline__ ChainHandoff fused_handoff(const FusedArgs& f, int b, int p) {
  ChainHandoff hx;
  hx.err = f.sync + SYNC_ERR;
  hx.err_host = f.err_host;
  hx.spin_max = f.spin_max;
  hx.epoch = f.epoch;
  hx.zsh = f.zsh + (size_t)(b * f.c.nq * f.P + p) * FU_ROWS * RCD;
  hx.zsh_stage = f.P * FU_ROWS * RCD;
  hx.stamps = f.stamps;
  hx.dbg = f.dbg;
  return hx;
}

template <int NM, bool PJ3>
__global__ __launch_bounds__(CH_NT, 4) void rvq_fused_kernel(FusedArgs f) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = f.c.B, T = f.c.T, nq = f.c.nq, F = f.c.F;
  const int blk = blockIdx.x;
  FSTAMP(f.stamps, 0);
  if (blk >= B * FU_NP) {
    fused_expand_body(f, blk - B * FU_NP, sm);
    FSTAMP(f.stamps, 41);
    return;
  }
  const int b = blk / FU_NP, s = blk - b * FU_NP;
  const int R = nq * RCD;
  float* part = const_cast<float*>(f.c.part);  // the workspace this launch writes (granules)
  const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
      part, (short)0, (int)((size_t)PJ_SPLIT * f.c.NF * R * 8), RSRC_FLAGS);
  // projection unit (b, s): partials as tagged granules, then straight on to the chain
  PartSink out{part, pr, f.epoch * 64u};
  if (f.stall && blk == 0)  // test knob (vrvq_rvq_debug_stall): a late producer
    for (unsigned k = 0; k < f.stall; ++k) __builtin_amdgcn_s_sleep(127);
  if constexpr (PJ3)
    project3_body(f.z, T, nq, 0, b, s, f.w_in_t, out, f.c.NF, reinterpret_cast<char*>(sm),
                  f.stamps);
  else project2_body(f.z, T, nq, 0, b, s, f.w_in_t, out, f.c.NF, sm);
  FSTAMP(f.stamps, 45);
  __syncthreads();  // the slab's LDS is the chain's from here
  // chain part s of clip b
  const int nf = min(F, T - s * F);
  if (nf <= 0) return;  // no frames (T < 8 F): no expansion lane reads this part's block
  ChainHandoff hx = fused_handoff(f, b, s);
  hx.part = pr;
  chain_body<NM, CH_GRANULE>(f.c, sm, b * T + s * F, nf, hx);
}

// W_in planes of vrvq_conv1d_proj's projection epilogue (conv_core.h proj_epilogue): 16-row
// tiles of the R = 8 nq stage rows
__host__ __device__ inline int pj_nrt(int nq) { return (nq * RCD + 15) / 16; }

// ------------------------------------------------------------------------------------------
// rvq_pt_kernel: the quantizer from the projection partials that the encoder's last conv wrote
// in its epilogue (vrvq_conv1d_proj: part[8][B T][8 nq], rvq_project3_kernel's values bit for
// bit). Neither z nor W_in is read here, and no projection sits in front of the chain.
//   Workgroups [0, B P): chain parts (clip b, frames [p F, p F + F), F <= 16): the 8 partials
// of their frames (plain loads: the conv kernel's boundary orders them) summed in split order
// -- the three-launch chain's expression, so every output equals the three-launch path's bit
// for bit -- then the chain, publishing every stage's zst as tagged granules.
//   Workgroups after: expansion (clip b, 96-frame window fb, 128-channel block cb), 8 waves,
// z_q_is and the masked z_q of the window's 4 x 3 (32-channel, 32-frame) tiles with
// fused_expand_body's expressions (four v_mfma_f32_32x32x2_f32 per tile, DPP quad transpose,
// 16-B stores of four frames of one channel), one channel tile ct = w & 3 per wave (waves w and
// w + 4 share a SIMD: 3 tiles per SIMD): waves 0-2 frame tiles {0, 2}, wave 3 {0, 1}, waves 4-6
// {1}, wave 7 {2}. Wave 7 is also the LOADER: per stage it polls the window's zst granules (6 x
// 16 B per lane, tag-checked, bounded) into one half of a double-buffered LDS slab while every
// wave runs the previous stage out of the other half; one barrier per stage. It issues the poll
// BEFORE its own tile's stores and checks the tags after them: vmcnt retires in order, so the
// check waits for the poll only, not for the stores. r05's expansion polled from every wave,
// and where a look came too early its second look waited behind the wave's whole stage of stores
// (a ~1 us bubble per stage while the chain was ahead). The loader also pulls the stage tables
// into its XCD's L2 while it waits for stage 0 (off by default: VRVQ_RVQ_WARM=1).
constexpr int PT_FB = 96;                          // frames per expansion window (3 tiles)
constexpr int PT_LOADER = 7;                       // the loader wave
constexpr int PT_SLAB = PT_FB * RCD;               // floats per slab half
constexpr int PT_SL = PT_FB * 4 / 64;              // 16-B granule pairs per loader lane (6)
constexpr int PT_NI = 2;                           // tiles per wave, at most
constexpr int PT_ZQ = 2 * PT_SLAB + CH_NT;         // floats: the z_q accumulators
constexpr int PT_NTILE = 12;                       // tiles of a window (4 x 3)
constexpr int PT_EX_FLOATS = PT_ZQ + PT_NTILE * 16 * 64;  // slab, warm-up sink, accumulators

struct PtOps {
  float wa[4];    // W_out[c0 + col][k], k = h, 2 + h, 4 + h, 6 + h (the MFMA steps' A values)
  float bb[4];    // b_out of the lane's four output channels (one per register quad)
};

// first accumulator slot of wave w (its tiles' slots are consecutive; 12 in all)
__device__ __forceinline__ int pt_slot0(int w) { return w < 4 ? 2 * w : 4 + w; }
// frame tile of slot j of wave w (-1: none)
__device__ __forceinline__ int pt_tile(int w, int j) {
  if (w < 3) return j == 0 ? 0 : 2;
  if (w == 3) return j;
  if (w < PT_LOADER) return j == 0 ? 1 : -1;
  return j == 0 ? 2 : -1;
}

__device__ __forceinline__ void pt_expand_body(const FusedArgs& f, int e, int N, float* sm) {
  const int nq = f.c.nq, T = f.c.T, F = f.c.F;
  constexpr int NCB = RD / FU_CB;
  const int cb = e % NCB;
  const int fb = (e / NCB) % f.n_fb;
  const int b = e / (NCB * f.n_fb);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = wave == PT_LOADER;
  const int col = lane & 31, h = lane >> 5;
  const int nfr = min(PT_FB, T - fb * PT_FB);       // frames of this window (>= 1)
  const int n_ft = (nfr + 31) / 32;
  // the slab window: PT_FB frames from wlo (the last window ends at the clip's last frame, so it
  // holds the moved-back last tile). Partial last tiles instead (no frame written twice; 9 of
  // every 96 frames' z_q_is rows are at T = 87) measured slower: 41.75 vs 39.2-40.6 us per
  // launch, each stage's stores 0.3-0.8 us longer (profiles/r06f_stamps.log)
  const int wlo = T >= PT_FB ? min(fb * PT_FB, T - PT_FB) : 0;
  const __amdgpu_buffer_rsrc_t zr =
      __builtin_amdgcn_make_buffer_rsrc(f.zsh, (short)0, f.zsh_bytes, RSRC_FLAGS);
  const int zstage = f.P * FU_ROWS * RCD * 8;  // bytes per stage
  const unsigned base = f.epoch * 64u;
  __shared__ int xdead_s;  // the loader's wait ran out (then no wait any more; outputs NaN)
  if (tid == 0) xdead_s = 0;

  // ---- loader: lane item q = lane + 64 u -> frame wlo + (q >> 2), slots 2 (q & 3) + {0, 1}
  // (frames past the clip re-read its last one: loaded, never used)
  auto soff = [&](int u) {
    const int q = lane + 64 * u;
    const int t = min(wlo + (q >> 2), T - 1);
    const int p = t / F, fr = t - p * F;
    return ((((b * nq) * f.P + p) * FU_ROWS + fr) * RCD + 2 * (q & 3)) * 8;
  };
  // ---- compute state: the wave's channel tile and its frame tiles (wave-uniform activity)
  const int c0 = cb * FU_CB + (wave & 3) * 32;
  const int crow = c0 + col;                  // A-operand row (W_out) of this lane
  const int chk = c0 + 4 * h + (lane & 3);    // after the transpose: channels chk + 8 qd
  const size_t wstride = (size_t)RD * RCD;
  int tbs[PT_NI];  // the tiles' first frames (wave-uniform)
  unsigned nact[PT_NI];
  bool act[PT_NI];
#pragma unroll
  for (int j = 0; j < PT_NI; ++j) {
    const int ft = pt_tile(wave, j);
    act[j] = ft >= 0 && ft < n_ft;
    // the tile's first frame; a clip's last, partial tile is moved back to end at the clip's last
    // frame (it overlaps the tile before it: those frames are written twice, identical values)
    int tb = fb * PT_FB + max(ft, 0) * 32;
    if (tb + 32 > T && T >= 32) tb = T - 32;
    tbs[j] = __builtin_amdgcn_readfirstlane(tb);
    float sv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = min(max(tb + 4 * (col >> 2) + u, 0), T - 1);
      sv[u] = f.c.imp ? (f.c.imp[(size_t)b * T + t] * f.c.level) * (float)nq : INFINITY;
    }
    unsigned w = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // mask[b,i,t] = (s - i >= 0), s = (imp * level) * nq (models/utils.py:45-61): the first
      // floor(s) + 1 stages (none for NaN or s < 0, all nq for s >= nq - 1 or CBR's inf)
      const int n = sv[u] >= 0.0f ? (int)floorf(fminf(sv[u], (float)(nq - 1))) + 1 : 0;
      w |= (unsigned)n << (8 * u);
    }
    nact[j] = w;
  }
  // the lane's B-operand frame (col) as a slab row, and the first of its four output frames
  auto trow = [&](int j) { return min(max(tbs[j] - wlo + col, 0), PT_FB - 1); };
  auto tq = [&](int j) { return tbs[j] + 4 * (col >> 2); };
  auto load_ops = [&](int i, PtOps& o) {
    const float* wp = f.w_out + (size_t)i * wstride + (size_t)crow * RCD + h;
#pragma unroll
    for (int s = 0; s < 4; ++s) o.wa[s] = wp[2 * s];
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) o.bb[qd] = f.b_out[(size_t)i * RD + chk + 8 * qd];
  };
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  auto store_quad = [&](float* row, int t, float v0, float v1, float v2, float v3) {
    if (t + 4 <= T) {
      *reinterpret_cast<f4u*>(row + t) = f4u{v0, v1, v2, v3};
    } else if (t < T) {  // a clip shorter than a frame tile
      row[t] = v0;
      if (t + 1 < T) row[t + 1] = v1;
      if (t + 2 < T) row[t + 2] = v2;
    }
  };
  // the masked z_q accumulators live in LDS ([slot][quad][lane] float4: conflict-free 16-B
  // accesses; in registers they spilled at the 128-VGPR budget with three tiles per wave, and a
  // spill reload would wait behind the stage's stores)
  float4* zacc = reinterpret_cast<float4*>(sm + PT_ZQ) + pt_slot0(wave) * (4 * 64) + lane;
#pragma unroll
  for (int j = 0; j < PT_NI; ++j)
    if (pt_tile(wave, j) >= 0)
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) zacc[(j * 4 + qd) * 64] = make_float4(0.f, 0.f, 0.f, 0.f);
  PtOps cur;
  load_ops(0, cur);
  // idle until stage 0 lands (~6 us): the loader may pull the stage tables into this XCD's L2
  // (fm kernel, r05) before its first poll
  if (loader && f.warm) warm_tables(f, e, (int)gridDim.x - f.c.B * f.P, N, sm + 2 * PT_SLAB);
  __syncthreads();  // xdead_s initialised
  bool dead = false;
  u32x4 g[PT_SL];
  // iteration i: the loader fills slab half (i & 1) with stage i while every wave runs stage
  // i - 1 from the other half
  for (int i = 0; i <= nq; ++i) {
    const bool poll = loader && i < nq && !dead;
    const unsigned tag = base + (unsigned)i + 1u;
    if (poll)  // issued ahead of this wave's stores below
#pragma unroll
      for (int u = 0; u < PT_SL; ++u)
        g[u] = __builtin_amdgcn_raw_buffer_load_b128(zr, soff(u) + i * zstage, 0, CPOL_SC1);
    if (i > 0) {
      const int si = i - 1;  // the stage computed now
      FSTAMP(f.stamps, 1 + si);
      // the next stage's operands ahead of this stage's stores (vmcnt retires in order)
      PtOps nxt;
      load_ops(min(si + 1, nq - 1), nxt);
      const float* slab = sm + (si & 1) * PT_SLAB;
#pragma unroll
      for (int j = 0; j < PT_NI; ++j) {
        if (!act[j]) continue;
        const float4 zb = *reinterpret_cast<const float4*>(slab + trow(j) * RCD + 4 * h);
        f32x16 q;
#pragma unroll
        for (int r = 0; r < 16; ++r) q[r] = 0.0f;
        q = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.wa[0], zb.x, q, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.wa[1], zb.y, q, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.wa[2], zb.z, q, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.wa[3], zb.w, q, 0, 0, 0);
        quad_transpose(q, lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) q[r] = q[r] + cur.bb[r >> 2];
        if (dead)  // wave-uniform (a timed-out wait): poisoned outputs
#pragma unroll
          for (int r = 0; r < 16; ++r) q[r] = __builtin_nanf("");
        if (f.z_q_is) {
#pragma unroll
          for (int qd = 0; qd < 4; ++qd) {
            float* row = f.z_q_is + (((size_t)b * nq + si) * RD + chk + 8 * qd) * T;
            store_quad(row, tq(j), q[4 * qd], q[4 * qd + 1], q[4 * qd + 2], q[4 * qd + 3]);
          }
        }
        float m[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned n = (nact[j] >> (8 * u)) & 0xffu;
          m[u] = (unsigned)si < n ? 1.0f : 0.0f;  // models/utils.py:45-61
        }
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          float4 a = zacc[(j * 4 + qd) * 64];
          a.x = a.x + q[4 * qd] * m[0];
          a.y = a.y + q[4 * qd + 1] * m[1];
          a.z = a.z + q[4 * qd + 2] * m[2];
          a.w = a.w + q[4 * qd + 3] * m[3];
          zacc[(j * 4 + qd) * 64] = a;
        }
        __builtin_amdgcn_sched_barrier(0);  // one tile's 16 values live at a time
      }
      if (si < 8) FSTAMP(f.stamps, 48 + si);  // the stage's stores issued (thread 0)
      cur = nxt;
    }
    if (poll && f.poll2) {
      // two looks in flight: while one look's loads are checked the next one is already on its
      // way, so a stage that lands just after a look is seen half a round trip later instead of
      // a whole one (each sc1 look crosses to the chain part's XCD: ~1-2 us)
      u32x4 h[PT_SL];
      auto look_ok = [&](const u32x4 (&v)[PT_SL]) {
        bool ok = true;
#pragma unroll
        for (int u = 0; u < PT_SL; ++u) ok = ok && v[u][1] == tag && v[u][3] == tag;
        return __builtin_amdgcn_ballot_w64(!ok) == 0;
      };
      bool in_h = false;
      for (unsigned it = 0;; ++it) {
#pragma unroll
        for (int u = 0; u < PT_SL; ++u)
          h[u] = __builtin_amdgcn_raw_buffer_load_b128(zr, soff(u) + i * zstage, 0, CPOL_SC1);
        if (look_ok(g)) break;
        if (it >= f.spin_max) {
          if (lane == 0) {
            report_timeout(f.sync + SYNC_ERR, f.err_host, 2u);
            xdead_s = 1;
          }
          dead = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
#pragma unroll
        for (int u = 0; u < PT_SL; ++u)
          g[u] = __builtin_amdgcn_raw_buffer_load_b128(zr, soff(u) + i * zstage, 0, CPOL_SC1);
        if (look_ok(h)) {
          in_h = true;
          break;
        }
      }
      if (in_h)
#pragma unroll
        for (int u = 0; u < PT_SL; ++u) g[u] = h[u];
    } else if (poll) {  // one look in flight (VRVQ_RVQ_POLL2=0, the A/B)
      for (unsigned it = 0;; ++it) {
        bool ok = true;
#pragma unroll
        for (int u = 0; u < PT_SL; ++u) ok = ok && g[u][1] == tag && g[u][3] == tag;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (it >= f.spin_max) {
          if (lane == 0) {
            report_timeout(f.sync + SYNC_ERR, f.err_host, 2u);
            xdead_s = 1;
          }
          dead = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
#pragma unroll
        for (int u = 0; u < PT_SL; ++u)
          g[u] = __builtin_amdgcn_raw_buffer_load_b128(zr, soff(u) + i * zstage, 0, CPOL_SC1);
      }
    }
    if (poll) {
      if (i < 8) FSTAMPT(f.stamps, 56 + i, 64 * PT_LOADER);  // the stage's rows seen
      float* slab = sm + (i & 1) * PT_SLAB;
#pragma unroll
      for (int u = 0; u < PT_SL; ++u) {
        const int q = lane + 64 * u;
        *reinterpret_cast<float2*>(slab + (q >> 2) * RCD + 2 * (q & 3)) =
            make_float2(__uint_as_float(g[u][0]), __uint_as_float(g[u][2]));
      }
    }
    __syncthreads();  // slab half (i & 1) holds stage i; half ((i - 1) & 1) is free
    dead = xdead_s != 0;
  }
  FSTAMP(f.stamps, 40);
#pragma unroll
  for (int j = 0; j < PT_NI; ++j) {
    if (!act[j]) continue;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      float* row = f.z_q + ((size_t)b * RD + chk + 8 * qd) * T;
      const float d = dead ? __builtin_nanf("") : 0.0f;
      const float4 a = zacc[(j * 4 + qd) * 64];
      store_quad(row, tq(j), a.x + d, a.y + d, a.z + d, a.w + d);
    }
  }
}

template <int NM>
__global__ __launch_bounds__(CH_NT, 4) void rvq_pt_kernel(FusedArgs f) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = f.c.B, T = f.c.T, F = f.c.F;
  const int blk = blockIdx.x;
  FSTAMP(f.stamps, 0);
  if (blk >= B * f.P) {
    pt_expand_body(f, blk - B * f.P, 256 * NM, sm);
    FSTAMP(f.stamps, 41);
    return;
  }
  const int b = blk / f.P, p = blk - b * f.P;
  const int t0 = p * F, nf = min(F, T - t0);
  if (f.stall && blk == 0)  // test knob (vrvq_rvq_debug_stall): a late producer
    for (unsigned k = 0; k < f.stall; ++k) __builtin_amdgcn_s_sleep(127);
  chain_body<NM, CH_PART>(f.c, sm, b * T + t0, nf, fused_handoff(f, b, p));
}

// ------------------------------------------------------------------------------------------
// Projection kernel: 3 = rvq_project3_kernel (split-bf16 matrix cores, default), 2 =
// rvq_project2_kernel (fp32-input MFMA: the exactness fallback, VRVQ_RVQ_PROJECT=2).
int g_project_variant = 0;  // 0: not yet read from the environment

int project_variant() {
  if (g_project_variant == 0) {
    const char* e = getenv("VRVQ_RVQ_PROJECT");
    g_project_variant = (e && e[0] == '2') ? 2 : 3;
  }
  return g_project_variant;
}

int launch_project(const float* z, int batch, int frames, int nq, const float* w_in_t,
                   float* part, hipStream_t st) {
  const long long nf = (long long)batch * frames;
  VRVQ_CHECK_ARG(nf * nq * RCD * PJ_SPLIT < 0x7fffffffLL);
  const int n_tc = (frames + PJ2_TC - 1) / PJ2_TC;
  VRVQ_CHECK_ARG((long long)batch * n_tc < 0x7fffffffLL);
  if (project_variant() == 3) {
    hipError_t e = hipFuncSetAttribute((const void*)rvq_project3_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, PJ3_LDS);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(rvq_project3_kernel, dim3((unsigned)(batch * n_tc), PJ_SPLIT), dim3(PJ2_NT),
                       PJ3_LDS, st, z, frames, nq, n_tc, w_in_t, part, (int)nf);
  } else {
    hipLaunchKernelGGL(rvq_project2_kernel, dim3((unsigned)(batch * n_tc), PJ_SPLIT), dim3(PJ2_NT),
                       0, st, z, frames, nq, n_tc, w_in_t, part, (int)nf);
  }
  return vrvq_launch_status();
}

unsigned long long* g_stamps = nullptr;   // diagnostic build: vrvq_debug_set_stamps
unsigned long long* g_fstamps = nullptr;  // diagnostic build: vrvq_debug_set_fused_stamps
int g_fdbg = 0;                           // diagnostic build: vrvq_debug_set_fused_flags

template <int NM>
int launch_chain_nm(const ChainArgs& a, hipStream_t st, long long nblk) {
  const size_t lds = (size_t)ChainLds(a.nq, a.F, 256 * NM).total * sizeof(float);
  if (lds > 160 * 1024) return VRVQ_ERR_UNSUPPORTED;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)rvq_chain_kernel<NM>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(rvq_chain_kernel<NM>, dim3((unsigned)nblk), dim3(CH_NT), lds, st, a);
  return vrvq_launch_status();
}

int launch_chain(const ChainArgs& a0, int ncode, hipStream_t st) {
  ChainArgs a = a0;
  a.stamps = g_stamps;
  // frames per workgroup: one workgroup per CU (<= 256 in one round) with as few frames each
  // as that allows, at most 16 (one MFMA column tile). The stage time is latency-bound and
  // nearly independent of F (measured: F = 6 at two workgroups per CU was no faster).
  const long long nf = (long long)a.B * a.T;
  long long F = (nf + 255) / 256;
  F = F < 1 ? 1 : (F > CH_FMAX ? CH_FMAX : F);
  a.F = (int)F;
  a.NF = (int)nf;
  a.NFS = a.NFS ? a.NFS : (int)nf;
  const long long nblk = (nf + F - 1) / F;
  VRVQ_CHECK_ARG(nblk < 0x7fffffffLL);
  switch (ncode / 256) {
    case 1: return launch_chain_nm<1>(a, st, nblk);
    case 2: return launch_chain_nm<2>(a, st, nblk);
    case 3: return launch_chain_nm<3>(a, st, nblk);
    default: return launch_chain_nm<4>(a, st, nblk);
  }
}

int launch_expand(const float* zst, int batch, int dim, int frames, int nq, const float* w_out,
                  const float* b_out, const float* imp, float level, float* z_q_is, float* z_q,
                  float* mask, hipStream_t st, const float* mask_in = nullptr) {
  ExpandArgs a{zst, batch, dim, frames, nq, w_out, b_out, imp, level, mask_in, z_q_is, z_q, mask};
  a.n_ct = (dim + 31) / 32;
  a.n_tt = (frames + 31) / 32;
  const long long nblk = (long long)batch * a.n_tt * ((a.n_ct + 3) / 4);
  VRVQ_CHECK_ARG(nblk < 0x7fffffffLL);
  hipLaunchKernelGGL(rvq_expand_kernel, dim3((unsigned)nblk), dim3(256), 0, st, a);
  return vrvq_launch_status();
}

bool rvq_shape_ok(int dim, int cdim, int nq, int ncode) {
  return dim == RD && cdim == RCD && nq <= CH_NQMAX && ncode > 0 && ncode % 256 == 0 &&
         ncode <= 1024;
}

size_t part_floats(long long nf, int nq) { return (size_t)PJ_SPLIT * nf * nq * RCD; }

// zst rows of the three-launch path ([B][nq][T][8] floats) or the fused path's tagged stage
// granules ([B][nq][FU_NP][FU_ROWS][8] x 8 B): the workspace holds the larger
size_t zst_floats(int batch, int frames, int nq) {
  const size_t a = (size_t)batch * frames * nq * RCD;
  const size_t b = (size_t)batch * nq * FU_NP * FU_ROWS * RCD * 2;
  return a > b ? a : b;
}

// ---- fused path, host side -----------------------------------------------------------------
// 1: three launches everywhere; 2: the fused launch where the shape allows (default;
// VRVQ_RVQ_FUSED=0 in the environment or vrvq_rvq_path(1) for the A/B).
int g_rvq_path = 0;

int rvq_path() {
  if (g_rvq_path == 0) {
    const char* e = getenv("VRVQ_RVQ_FUSED");
    g_rvq_path = (e && e[0] == '0') ? 1 : 2;
  }
  return g_rvq_path;
}

// Process-wide state of the fused launches' in-launch hand-offs:
//  * epochs: ONE counter for every call of the process (every stream and device), so tags are
//    unique across streams -- granules a call on another stream left can never match. At
//    EPOCH_RESET the counter restarts at 2 and every library-owned granule area is cleared (on
//    its own stream, ordered after the calls that used it) before a tag can repeat.
//  * granule areas: eager calls hand off through a library-owned area per (device, stream)
//    (hipMalloc, zeroed at allocation, grown on demand), never shared with the caller or the
//    caching allocator: every tag word in it was written by this library (an older epoch). A
//    caller workspace whose previous contents happened to hold 64 * epoch in a tag slot (small
//    integer data does) could otherwise pass a check before the real granule lands.
//  * under stream capture there is no allocation: the call uses the caller's workspace,
//    zeroed by captured memset nodes, and epoch 1 (eager epochs start at 2); the sync block of
//    the stream must exist from an earlier eager call, else the call takes the three launches.
//  * the error word: a per-stream device word (vrvq_rvq_sync_error, synchronising) and one
//    host-mapped word of the process (vrvq_rvq_pending_error, no synchronisation; the torch
//    ops raise on it at their next call).
struct StreamState {
  unsigned* sync = nullptr;  // SYNC_WORDS device words
  void* area = nullptr;      // granules of eager calls
  size_t area_bytes = 0;
};
std::mutex g_fu_mu;
std::map<std::pair<int, hipStream_t>, StreamState> g_fu;
unsigned g_epoch = 1;                 // last epoch handed out (guarded by g_fu_mu)
unsigned* g_err_host = nullptr;       // host-mapped error word
unsigned* g_err_host_dev = nullptr;   // its device address
unsigned g_spin_max = SPIN_MAX;       // vrvq_rvq_debug (timeout test)
int g_pt_cap_limit = 0x7fffffff;      // vrvq_rvq_debug_capacity (fallback test)
unsigned g_stall = 0;
constexpr unsigned EPOCH_RESET = 1u << 24;  // 64 epoch + stage stays below 2^32

struct FusedLaunch {
  unsigned* sync = nullptr;
  unsigned epoch = 0;
  char* area = nullptr;  // granule area of this launch (zeroed by memset nodes under capture)
};

// Sync block, epoch and granule area for one fused launch of `bytes` granules on st; false:
// the fused launch cannot run now (the caller takes another path).
constexpr size_t FU_SYNC_BYTES = (SYNC_WORDS * sizeof(unsigned) + 255) & ~size_t(255);
bool fused_prepare(hipStream_t st, size_t bytes, void* caller_ws, size_t caller_bytes,
                   FusedLaunch* L) {
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return false;
  const bool capturing = cs != hipStreamCaptureStatusNone;
  std::lock_guard<std::mutex> guard(g_fu_mu);
  if (!g_err_host && !capturing) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
      g_err_host = static_cast<unsigned*>(h);
      __atomic_store_n(g_err_host, 0u, __ATOMIC_RELAXED);
      void* d = nullptr;
      if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess) g_err_host_dev = static_cast<unsigned*>(d);
    }
  }
  const size_t sync_bytes = SYNC_WORDS * sizeof(unsigned);
  if (capturing) {
    // no allocation inside a capture (and the capture stream is usually new to us): the sync
    // block and the granule area both come from the caller's workspace, zeroed by memset nodes
    // (the workspace functions count FU_SYNC_BYTES in)
    if (!caller_ws || caller_bytes < bytes + FU_SYNC_BYTES) return false;
    if (hipMemsetAsync(caller_ws, 0, bytes + FU_SYNC_BYTES, st) != hipSuccess) return false;
    L->sync = static_cast<unsigned*>(caller_ws);
    L->area = static_cast<char*>(caller_ws) + FU_SYNC_BYTES;
    L->epoch = 1;
    return true;
  }
  StreamState& ss = g_fu[{device, st}];
  if (!ss.sync) {
    if (hipMalloc(&ss.sync, sync_bytes) != hipSuccess) {
      ss.sync = nullptr;
      return false;
    }
    if (hipMemsetAsync(ss.sync, 0, sync_bytes, st) != hipSuccess) return false;
  }
  {
    if (ss.area_bytes < bytes) {
      if (ss.area) {
        if (hipStreamSynchronize(st) != hipSuccess) return false;
        (void)hipFree(ss.area);
        ss.area = nullptr;
        ss.area_bytes = 0;
      }
      const size_t want = bytes + bytes / 4;
      if (hipMalloc(&ss.area, want) != hipSuccess) {
        ss.area = nullptr;
        return false;
      }
      if (hipMemsetAsync(ss.area, 0, want, st) != hipSuccess) return false;
      ss.area_bytes = want;
    }
    if (++g_epoch >= EPOCH_RESET) {
      g_epoch = 2;
      for (auto& kv : g_fu)
        if (kv.second.area) (void)hipMemsetAsync(kv.second.area, 0, kv.second.area_bytes, kv.first.second);
    }
    L->area = static_cast<char*>(ss.area);
    L->epoch = g_epoch;
  }
  L->sync = ss.sync;
  return true;
}

// Clips per fused launch: every workgroup resident at once, so that no waiting workgroup can
// hold the slot of one it waits for (occupancy query with the launch's dynamic LDS, after the
// attribute that allows it; cached per device, kernel and LDS size).
int fused_clip_capacity(const void* kern, size_t lds, int wg_per_clip) {
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, size_t>, int> cache;
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return 0;
  std::lock_guard<std::mutex> guard(mu);
  const auto key = std::make_tuple(device, kern, lds);
  auto it = cache.find(key);
  int per_cu = 0;
  if (it != cache.end()) {
    per_cu = it->second;
  } else {
    int cus = 0, per = 0;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, CH_NT, lds) != hipSuccess)
      cus = per = 0;
    per_cu = cus * per;  // resident workgroups on the device
    cache[key] = per_cu;
  }
  return per_cu / wg_per_clip;
}

constexpr int FUSED_NA = -1;  // the fused launch does not apply: take the three launches

// Launch timing (vrvq_rvq_timing): while on, every fused launch carries a (start, stop) pair of
// HIP events in its own dispatch packet (hipExtLaunchKernelGGL), so the elapsed time is the
// kernel's own duration on its stream (what rocprofv3 reports for it), with no marker packets
// of their own around it. vrvq_rvq_timing_read averages the recorded pairs.
struct LaunchTimer {
  std::mutex mu;
  bool on = false;
  std::vector<hipEvent_t> pool;  // 2 per recorded launch
  size_t used = 0;
  bool next(hipEvent_t* start, hipEvent_t* stop) {
    std::lock_guard<std::mutex> guard(mu);
    if (!on) return false;
    while (pool.size() < used + 2) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return false;
      pool.push_back(e);
    }
    *start = pool[used];
    *stop = pool[used + 1];
    used += 2;
    return true;
  }
};
LaunchTimer g_timer;

template <typename K>
int launch_timed(K kern, unsigned grid, size_t lds, hipStream_t st, const FusedArgs& f) {
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  if (g_timer.next(&ev0, &ev1))
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(CH_NT), lds, st, ev0, ev1, 0, f);
  else
    hipLaunchKernelGGL(kern, dim3(grid), dim3(CH_NT), lds, st, f);
  return vrvq_launch_status();
}

// Chunk of clips [b0, b0 + bc) of a fused launch: the outputs and inputs offset to it.
void fused_chunk_args(FusedArgs& f, int b0, int bc, int frames, int nq, int F, const float* z,
                      const float* imp, int64_t* codes, float* latents, float* loss_pf,
                      float* z_q_is, float* z_q, float* mask) {
  const size_t DT = (size_t)RD * frames;
  ChainArgs& c = f.c;
  c.B = bc;
  c.T = frames;
  c.nq = nq;
  c.F = F;
  c.NF = bc * frames;
  c.imp = imp ? imp + (size_t)b0 * frames : nullptr;
  c.codes = codes + (size_t)b0 * nq * frames;
  c.latents = latents + (size_t)b0 * nq * RCD * frames;
  c.loss_pf = loss_pf + (size_t)b0 * nq * frames;
  c.zst = nullptr;
  c.mask = mask ? mask + (size_t)b0 * nq * frames : nullptr;
  c.stamps = nullptr;
  f.z = z + b0 * DT;
  f.z_q_is = z_q_is ? z_q_is + (size_t)b0 * nq * DT : nullptr;
  f.z_q = z_q + b0 * DT;
  f.err_host = g_err_host_dev;
  f.spin_max = g_spin_max;
  f.stall = g_stall;
  f.stamps = g_fstamps;
  f.dbg = g_fdbg;
}

size_t zsh_bytes(int bc, int nq, int P) { return (size_t)bc * nq * P * FU_ROWS * RCD * 8; }

template <int NM, bool PJ3>
int launch_fused_nm(const FusedArgs& f0, int batch, int frames, int nq, const float* z,
                    const float* imp, int64_t* codes, float* latents, float* loss_pf,
                    float* z_q_is, float* z_q, float* mask, float* ws, size_t ws_bytes,
                    hipStream_t st) {
  const int F = (frames + FU_NP - 1) / FU_NP;
  size_t lds = (size_t)ChainLds(nq, F, 256 * NM).total * sizeof(float);
  const size_t lds_pj = PJ3 ? (size_t)PJ3_LDS : (size_t)PJ_CPS * PJ2_LD * sizeof(float);
  if (lds < lds_pj) lds = lds_pj;
  if (lds < (size_t)FU_EX_LDS) lds = FU_EX_LDS;
  if (lds > 80 * 1024) return FUSED_NA;
  const void* kern = (const void*)rvq_fused_kernel<NM, PJ3>;
  const int cap = min(FU_CLIPS_MAX, fused_clip_capacity(kern, lds, 2 * FU_NP));
  if (cap < 1) return FUSED_NA;
  const int bc_max = min(batch, cap);
  const size_t part_b = 2 * part_floats((long long)bc_max * frames, nq) * sizeof(float);
  const size_t need = part_b + zsh_bytes(bc_max, nq, FU_NP);
  for (int b0 = 0; b0 < batch; b0 += bc_max) {
    const int bc = min(bc_max, batch - b0);
    FusedArgs f = f0;
    FusedLaunch L;
    if (!fused_prepare(st, need, ws, ws_bytes, &L)) {
      if (b0 == 0) return FUSED_NA;
      return VRVQ_ERR_UNSUPPORTED;  // cannot happen after a first successful chunk
    }
    fused_chunk_args(f, b0, bc, frames, nq, F, z, imp, codes, latents, loss_pf, z_q_is, z_q, mask);
    f.sync = L.sync;
    f.epoch = L.epoch;
    f.c.part = reinterpret_cast<float*>(L.area);  // tagged granules: 2 floats per partial
    f.zsh = reinterpret_cast<unsigned long long*>(L.area + part_b);
    f.zsh_bytes = (int)zsh_bytes(bc, nq, FU_NP);
    f.P = FU_NP;
    f.n_fb = 1;
    const int rc = launch_timed(rvq_fused_kernel<NM, PJ3>, (unsigned)(2 * bc * FU_NP), lds, st, f);
    if (rc) return rc;
  }
  return 0;
}

// Frames per chain part of rvq_pt_kernel: 16, fewer wherever the chain's LDS would not fit twice
// per CU (beside an expansion workgroup).
size_t pt_lds_bytes(int nq, int F, int N) {
  size_t c = (size_t)ChainLds(nq, F, N).total * sizeof(float);
  const size_t ex = (size_t)PT_EX_FLOATS * sizeof(float);  // slab, warm-up sink, one z_q tile
  return c < ex ? ex : c;
}
int pt_frames_per_part(int frames, int nq, int N) {
  static const int f_env = [] {  // VRVQ_RVQ_PT_F: frames per chain part (A/B; 1..16)
    const char* e = getenv("VRVQ_RVQ_PT_F");
    const int v = e ? atoi(e) : 0;
    return v >= 1 && v <= FU_ROWS ? v : 0;
  }();
  // 16 frames per part: fewer, longer chain parts measured fastest at T = 87 (in-step 43.1-43.5
  // us vs 44.2 at F = 11, 44.4-44.8 at 12; profiles/r06g_ab.txt)
  const int F0 = f_env ? min(f_env, frames) : min(FU_ROWS, frames);
  for (int F = F0; F >= 1; --F)
    if (pt_lds_bytes(nq, F, N) <= 80 * 1024) return F;
  return 0;
}
size_t pt_zst_bytes(int batch, int frames, int nq) { return (size_t)batch * nq * frames * RCD * 4; }

// Clips per rvq_pt_kernel launch (every workgroup resident), 0 when not even one clip fits or the
// three launches are selected (vrvq_rvq_path(1)).
template <int NM>
int pt_capacity(int frames, int nq, int* F_out, int* P_out, int* n_fb_out, size_t* lds_out) {
  const int F = pt_frames_per_part(frames, nq, 256 * NM);
  if (F < 1 || rvq_path() == 1) return 0;
  const int P = (frames + F - 1) / F;
  const int n_fb = (frames + PT_FB - 1) / PT_FB;
  const size_t lds = pt_lds_bytes(nq, F, 256 * NM);
  const int wpc = P + (RD / FU_CB) * n_fb;
  *F_out = F;
  *P_out = P;
  *n_fb_out = n_fb;
  *lds_out = lds;
  return min(fused_clip_capacity((const void*)rvq_pt_kernel<NM>, lds, wpc), g_pt_cap_limit);
}

// The quantizer from the conv's partials: rvq_pt_kernel per group of resident clips, or -- the
// shape does not fit (a clip longer than the resident grid) or vrvq_rvq_path(1) -- the chain and
// the expansion as two stream-ordered launches over the same partials (zst through the
// workspace). Both give the same outputs bit for bit.
template <int NM>
int launch_pt_nm(const FusedArgs& f0, int batch, int frames, int nq, const float* part,
                 const float* imp, int64_t* codes, float* latents, float* loss_pf, float* z_q_is,
                 float* z_q, float* mask, void* ws, size_t ws_bytes, hipStream_t st) {
  int F = 0, P = 0, n_fb = 0;
  size_t lds = 0;
  const int cap = pt_capacity<NM>(frames, nq, &F, &P, &n_fb, &lds);
  const int R = nq * RCD;
  if (cap < 1) {
    if (ws_bytes < pt_zst_bytes(batch, frames, nq)) return VRVQ_ERR_ARG;
    float* zst = static_cast<float*>(ws);
    ChainArgs a = f0.c;
    a.part = part; a.B = batch; a.T = frames; a.nq = nq; a.NFS = 0;
    a.imp = imp; a.codes = codes; a.latents = latents; a.loss_pf = loss_pf; a.zst = zst;
    a.mask = mask;
    int rc = launch_chain(a, 256 * NM, st);
    if (rc) return rc;
    return launch_expand(zst, batch, RD, frames, nq, f0.w_out, f0.b_out, imp, f0.c.level, z_q_is,
                         z_q, nullptr, st);
  }
  int bc_max = min(batch, cap);
  while (bc_max > 1 && zsh_bytes(bc_max, nq, P) > 0x7fffffffULL) --bc_max;
  const size_t need = zsh_bytes(bc_max, nq, P);
  const int wpc = P + (RD / FU_CB) * n_fb;
  for (int b0 = 0; b0 < batch; b0 += bc_max) {
    const int bc = min(bc_max, batch - b0);
    FusedArgs f = f0;
    FusedLaunch L;
    if (!fused_prepare(st, need, ws, ws_bytes, &L)) return VRVQ_ERR_UNSUPPORTED;
    fused_chunk_args(f, b0, bc, frames, nq, F, nullptr, imp, codes, latents, loss_pf, z_q_is, z_q,
                     mask);
    f.z = nullptr;
    f.z_q = z_q + (size_t)b0 * RD * frames;
    f.c.part = part + (size_t)b0 * frames * R;  // the chunk's frames within every split
    f.c.NFS = batch * frames;                   // split stride: the call's frames
    f.sync = L.sync;
    f.epoch = L.epoch;
    f.zsh = reinterpret_cast<unsigned long long*>(L.area);
    f.zsh_bytes = (int)zsh_bytes(bc, nq, P);
    f.P = P;
    f.n_fb = n_fb;
    const int rc = launch_timed(rvq_pt_kernel<NM>, (unsigned)(bc * wpc), lds, st, f);
    if (rc) return rc;
  }
  return 0;
}

// W_in planes of the conv projection epilogue in the 16x16x32 A-fragment order: w3in[ks][plane][rt][lane] =
// 8 bf16 of row r = 16 rt + (lane & 15), channels 32 ks + 8 (lane >> 4) .. +7 (zero rows >= R).
__global__ void rvq_pack_w_in_kernel(const float* __restrict__ w_in_t, int nq, u32x4* __restrict__ w3) {
  const int n_rt = pj_nrt(nq), R = nq * RCD;
  const int total = 32 * 3 * n_rt * 64;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int lane = o & 63;
    int q = o >> 6;
    const int rt = q % n_rt;
    q /= n_rt;
    const int plane = q % 3, ks = q / 3;
    const int r = rt * 16 + (lane & 15), c0 = 32 * ks + 8 * (lane >> 4);
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = r < R ? w_in_t[((size_t)(r >> 3) * RD + c0 + u) * RCD + (r & 7)] : 0.0f;
    unsigned h[4], m[4], l[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) rvq_split3x2(v[2 * u], v[2 * u + 1], h[u], m[u], l[u]);
    w3[o] = plane == 0 ? u32x4{h[0], h[1], h[2], h[3]}
          : plane == 1 ? u32x4{m[0], m[1], m[2], m[3]} : u32x4{l[0], l[1], l[2], l[3]};
  }
}

}  // namespace

#ifdef VRVQ_STAMPS
// Diagnostic build only (not in include/vrvq.h): the chain kernel's stamp buffer.
extern "C" int vrvq_debug_set_stamps(unsigned long long* buf) {
  g_stamps = buf;
  return 0;
}
extern "C" int vrvq_debug_set_fused_stamps(unsigned long long* buf) {
  g_fstamps = buf;
  return 0;
}
// bit 0: the expansion workgroups skip their MFMAs (timing experiment; outputs wrong)
extern "C" int vrvq_debug_set_fused_flags(int flags) {
  g_fdbg = flags;
  return 0;
}
#endif

extern "C" int vrvq_rvq_project_variant(int variant) {
  const int prev = project_variant();
  if (variant == 2 || variant == 3) g_project_variant = variant;
  else if (variant != 0) return VRVQ_ERR_ARG;
  return prev;
}

extern "C" int vrvq_rvq_cross_prep(const float* w_in_t, const float* w_out, const float* b_out,
                                   int nq, int dim, int cdim, float* mcol, float* qb,
                                   vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(w_in_t && w_out && b_out && mcol && qb && nq > 0);
  if (dim != RD || cdim != RCD) return VRVQ_ERR_UNSUPPORTED;
  // mcol: one thread per (j, i, k, m) chain; qb: one workgroup per stage (cross_prep_qb_kernel)
  const int total = nq * nq * 64;
  hipLaunchKernelGGL(cross_prep_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     as_stream(stream), w_in_t, w_out, b_out, nq, mcol, qb);
  hipLaunchKernelGGL(cross_prep_qb_kernel, dim3(nq), dim3(RD), 0, as_stream(stream), w_in_t, b_out,
                     qb);
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_frag(const float* cbn, int nq, int ncode, int cdim, float* cbf,
                             vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(cbn && cbf && nq > 0);
  if (!rvq_shape_ok(RD, cdim, nq, ncode)) return VRVQ_ERR_UNSUPPORTED;
  const size_t total = (size_t)nq * ncode * RCD;
  const unsigned grid = (unsigned)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(rvq_frag_kernel, dim3(grid), dim3(256), 0, as_stream(stream), cbn, nq,
                     ncode, cbf);
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_project(const float* z, int batch, int dim, int frames, int nq, int cdim,
                                const float* w_in_t, float* part, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z && w_in_t && part && batch > 0 && frames > 0 && nq > 0);
  if (dim != RD || cdim != RCD) return VRVQ_ERR_UNSUPPORTED;
  return launch_project(z, batch, frames, nq, w_in_t, part, as_stream(stream));
}

extern "C" int vrvq_rvq_chain(const float* part, int batch, int frames, int nq, int ncode,
                              int cdim, const float* b_in, const float* qb, const float* mcol,
                              const float* cb, const float* cbf, const float* c2,
                              const float* imp, float level, int64_t* codes, float* latents,
                              float* loss_pf, float* zst, float* mask, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(part && b_in && qb && mcol && cb && cbf && c2 && codes && latents && loss_pf &&
                 zst);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  if (!rvq_shape_ok(RD, cdim, nq, ncode)) return VRVQ_ERR_UNSUPPORTED;
  ChainArgs a{};
  a.part = part; a.B = batch; a.T = frames; a.nq = nq;
  a.b_in = b_in; a.qb = qb; a.mcol = mcol; a.cb = cb; a.cbf = cbf; a.c2 = c2;
  a.imp = imp; a.level = level;
  a.codes = codes; a.latents = latents; a.loss_pf = loss_pf; a.zst = zst; a.mask = mask;
  return launch_chain(a, ncode, as_stream(stream));
}

extern "C" int vrvq_rvq_expand(const float* zst, int batch, int dim, int frames, int nq, int cdim,
                               const float* w_out, const float* b_out, const float* imp,
                               float level, float* z_q_is, float* z_q, float* mask,
                               vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(zst && w_out && b_out && z_q);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0 && dim >= 4);
  if (cdim != RCD) return VRVQ_ERR_UNSUPPORTED;
  return launch_expand(zst, batch, dim, frames, nq, w_out, b_out, imp, level, z_q_is, z_q, mask,
                       as_stream(stream));
}

extern "C" int vrvq_rvq_expand_masked(const float* zst, int batch, int dim, int frames, int nq,
                                      int cdim, const float* w_out, const float* b_out,
                                      const float* mask, float* z_q_is, float* z_q,
                                      vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(zst && w_out && b_out && mask && z_q);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0 && dim >= 4);
  if (cdim != RCD) return VRVQ_ERR_UNSUPPORTED;
  return launch_expand(zst, batch, dim, frames, nq, w_out, b_out, nullptr, 1.0f, z_q_is, z_q,
                       nullptr, as_stream(stream), mask);
}

extern "C" int vrvq_rvq_workspace(int batch, int frames, int nq, long long* bytes) {
  VRVQ_CHECK_ARG(bytes && batch > 0 && frames > 0 && nq > 0);
  const long long nf = (long long)batch * frames;
  // the fused path's partials are tagged granules (2 floats each)
  *bytes = (long long)(2 * part_floats(nf, nq) + zst_floats(batch, frames, nq)) *
               (long long)sizeof(float) + (long long)FU_SYNC_BYTES;
  return 0;
}

extern "C" int vrvq_rvq_path(int path) {
  const int prev = rvq_path();
  if (path == 1 || path == 2) g_rvq_path = path;
  else if (path != 0) return VRVQ_ERR_ARG;
  return prev;
}

extern "C" int vrvq_rvq_timing(int on) {
  std::lock_guard<std::mutex> guard(g_timer.mu);
  const int prev = g_timer.on ? 1 : 0;
  g_timer.on = on != 0;
  return prev;
}

extern "C" int vrvq_rvq_timing_read(float* mean_ms, int* count) {
  VRVQ_CHECK_ARG(mean_ms && count);
  std::lock_guard<std::mutex> guard(g_timer.mu);
  *mean_ms = 0.0f;
  *count = 0;
  double sum = 0.0;
  for (size_t k = 0; k + 1 < g_timer.used; k += 2) {
    hipError_t e = hipEventSynchronize(g_timer.pool[k + 1]);
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, g_timer.pool[k], g_timer.pool[k + 1]);
    if (e != hipSuccess) return (int)e;
    sum += ms;
    ++*count;
  }
  if (*count) *mean_ms = (float)(sum / *count);
  g_timer.used = 0;
  return 0;
}

extern "C" int vrvq_rvq_sync_error(vrvq_stream_t stream, int* code) {
  VRVQ_CHECK_ARG(code);
  *code = 0;
  hipStream_t st = as_stream(stream);
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return VRVQ_ERR_ARG;
  unsigned* dev = nullptr;
  {
    std::lock_guard<std::mutex> guard(g_fu_mu);
    auto it = g_fu.find({device, st});
    if (it == g_fu.end() || !it->second.sync) return 0;
    dev = it->second.sync;
  }
  unsigned v = 0;
  hipError_t e = hipMemcpyAsync(&v, dev + SYNC_ERR, sizeof(v), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess && v) e = hipMemsetAsync(dev + SYNC_ERR, 0, sizeof(unsigned), st);
  if (e != hipSuccess) return (int)e;
  *code = (int)v;
  if (v && g_err_host) __atomic_store_n(g_err_host, 0u, __ATOMIC_RELAXED);  // reported here
  return 0;
}

extern "C" int vrvq_rvq_pending_error(int* code) {
  VRVQ_CHECK_ARG(code);
  *code = 0;
  std::lock_guard<std::mutex> guard(g_fu_mu);
  if (g_err_host) *code = (int)__atomic_exchange_n(g_err_host, 0u, __ATOMIC_RELAXED);
  return 0;
}

extern "C" int vrvq_rvq_debug(unsigned spin_max, unsigned stall) {
  std::lock_guard<std::mutex> guard(g_fu_mu);
  g_spin_max = spin_max ? spin_max : SPIN_MAX;
  g_stall = stall;
  return 0;
}

extern "C" int vrvq_rvq_encode(const float* z, int batch, int dim, int frames, int nq, int ncode,
                               int cdim, const float* w_in_t, const float* b_in, const float* cb,
                               const float* cbf, const float* c2, const float* w_out,
                               const float* b_out, const float* mcol, const float* qb,
                               const float* imp, float level, int64_t* codes, float* latents,
                               float* loss_pf, float* z_q_is, float* z_q, float* mask,
                               void* workspace, long long workspace_bytes,
                               vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z && w_in_t && b_in && cb && cbf && c2 && w_out && b_out && mcol && qb &&
                 codes && latents && loss_pf && z_q && workspace);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  if (!rvq_shape_ok(dim, cdim, nq, ncode)) return VRVQ_ERR_UNSUPPORTED;
  long long need = 0;
  vrvq_rvq_workspace(batch, frames, nq, &need);
  VRVQ_CHECK_ARG(workspace_bytes >= need);
  VRVQ_CHECK_ARG(((uintptr_t)workspace & 15) == 0);
  const long long nf = (long long)batch * frames;
  float* part = static_cast<float*>(workspace);
  float* zst = part + part_floats(nf, nq);
  hipStream_t st = as_stream(stream);
  if (rvq_path() == 2 && frames <= PJ2_TC && batch <= 0x7fffffff / (2 * FU_NP)) {
    FusedArgs f{};
    ChainArgs& c = f.c;
    c.b_in = b_in; c.qb = qb; c.mcol = mcol; c.cb = cb; c.cbf = cbf; c.c2 = c2;
    c.level = level;
    f.w_in_t = w_in_t;
    f.w_out = w_out;
    f.b_out = b_out;
    int rc = FUSED_NA;
    const bool pj3 = project_variant() == 3;
    const size_t wsb = (size_t)workspace_bytes;
#define VRVQ_FUSED_CASE(NMV)                                                                    \
  rc = pj3 ? launch_fused_nm<NMV, true>(f, batch, frames, nq, z, imp, codes, latents, loss_pf,  \
                                        z_q_is, z_q, mask, part, wsb, st)                     \
           : launch_fused_nm<NMV, false>(f, batch, frames, nq, z, imp, codes, latents, loss_pf, \
                                         z_q_is, z_q, mask, part, wsb, st)
    switch (ncode / 256) {
      case 1: VRVQ_FUSED_CASE(1); break;
      case 2: VRVQ_FUSED_CASE(2); break;
      case 3: VRVQ_FUSED_CASE(3); break;
      default: VRVQ_FUSED_CASE(4); break;
    }
#undef VRVQ_FUSED_CASE
    if (rc != FUSED_NA) return rc;
  }
  int rc = launch_project(z, batch, frames, nq, w_in_t, part, st);
  if (rc) return rc;
  rc = vrvq_rvq_chain(part, batch, frames, nq, ncode, cdim, b_in, qb, mcol, cb, cbf, c2, imp,
                      level, codes, latents, loss_pf, zst, mask, stream);
  if (rc) return rc;
  return launch_expand(zst, batch, dim, frames, nq, w_out, b_out, imp, level, z_q_is, z_q,
                       nullptr, st);
}

extern "C" int vrvq_rvq_w_in_planes_size(int nq, int dim, int cdim, long long* n_u16) {
  VRVQ_CHECK_ARG(n_u16 && nq > 0);
  if (dim != RD || cdim != RCD || nq > CH_NQMAX) return VRVQ_ERR_UNSUPPORTED;
  *n_u16 = 32LL * 3 * pj_nrt(nq) * 64 * 8;
  return 0;
}

extern "C" int vrvq_rvq_pack_w_in(const float* w_in_t, int nq, int dim, int cdim, uint16_t* w3in,
                                  vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(w_in_t && w3in && nq > 0);
  if (dim != RD || cdim != RCD || nq > CH_NQMAX) return VRVQ_ERR_UNSUPPORTED;
  const int total = 32 * 3 * pj_nrt(nq) * 64;
  hipLaunchKernelGGL(rvq_pack_w_in_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     as_stream(stream), w_in_t, nq, reinterpret_cast<u32x4*>(w3in));
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_workspace_part(int batch, int frames, int nq, int ncode, long long* bytes) {
  VRVQ_CHECK_ARG(bytes && batch > 0 && frames > 0 && nq > 0 && ncode > 0);
  if (nq > CH_NQMAX || ncode % 256 != 0 || ncode > 1024) return VRVQ_ERR_UNSUPPORTED;
  // the fused launch's granules under stream capture (+ its sync block), or the two-launch
  // fallback's zst rows: the larger
  long long g = 0;
  const int F = pt_frames_per_part(frames, nq, ncode);
  if (F >= 1) g = (long long)zsh_bytes(batch, nq, (frames + F - 1) / F) + (long long)FU_SYNC_BYTES;
  const long long z = (long long)pt_zst_bytes(batch, frames, nq);
  *bytes = g > z ? g : z;
  return 0;
}

extern "C" int vrvq_rvq_encode_part(const float* part, int batch, int dim, int frames, int nq,
                                    int ncode, int cdim, const float* b_in, const float* cb,
                                    const float* cbf, const float* c2, const float* w_out,
                                    const float* b_out, const float* mcol, const float* qb,
                                    const float* imp, float level, int64_t* codes,
                                    float* latents, float* loss_pf, float* z_q_is, float* z_q,
                                    float* mask, void* workspace, long long workspace_bytes,
                                    vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(part && b_in && cb && cbf && c2 && w_out && b_out && mcol && qb && codes &&
                 latents && loss_pf && z_q && workspace);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  VRVQ_CHECK_ARG(((uintptr_t)workspace & 15) == 0 && ((uintptr_t)part & 15) == 0);
  if (!rvq_shape_ok(dim, cdim, nq, ncode)) return VRVQ_ERR_UNSUPPORTED;
  VRVQ_CHECK_ARG((long long)batch * frames * nq * RCD * PJ_SPLIT < 0x7fffffffLL);
  long long need = 0;
  const int rc0 = vrvq_rvq_workspace_part(batch, frames, nq, ncode, &need);
  if (rc0) return rc0;
  VRVQ_CHECK_ARG(workspace_bytes >= need);
  FusedArgs f{};
  ChainArgs& c = f.c;
  c.b_in = b_in; c.qb = qb; c.mcol = mcol; c.cb = cb; c.cbf = cbf; c.c2 = c2;
  c.level = level;
  f.w_out = w_out;
  f.b_out = b_out;
  // VRVQ_RVQ_WARM=1: the loader warms the stage tables' L2 first (A/B; measured slower here:
  // stage 0 lands at ~6 us, profiles/r06f_ab.txt, r06c_ab.txt)
  static const int warm = [] {
    const char* e = getenv("VRVQ_RVQ_WARM");
    return e ? atoi(e) : 0;
  }();
  f.warm = warm;
  // the loader's two looks in flight (VRVQ_RVQ_POLL2=0: one, the A/B)
  static const int poll2 = [] {
    const char* e = getenv("VRVQ_RVQ_POLL2");
    return e ? atoi(e) : 1;
  }();
  f.poll2 = poll2;
  hipStream_t st = as_stream(stream);
  const size_t wsb = (size_t)workspace_bytes;
  switch (ncode / 256) {
    case 1: return launch_pt_nm<1>(f, batch, frames, nq, part, imp, codes, latents, loss_pf, z_q_is, z_q, mask, workspace, wsb, st);
    case 2: return launch_pt_nm<2>(f, batch, frames, nq, part, imp, codes, latents, loss_pf, z_q_is, z_q, mask, workspace, wsb, st);
    case 3: return launch_pt_nm<3>(f, batch, frames, nq, part, imp, codes, latents, loss_pf, z_q_is, z_q, mask, workspace, wsb, st);
    default: return launch_pt_nm<4>(f, batch, frames, nq, part, imp, codes, latents, loss_pf, z_q_is, z_q, mask, workspace, wsb, st);
  }
}

extern "C" int vrvq_rvq_fused_clips(int frames, int nq, int ncode, int* clips) {
  VRVQ_CHECK_ARG(clips && frames > 0 && nq > 0);
  *clips = 0;
  if (!rvq_shape_ok(RD, RCD, nq, ncode)) return VRVQ_ERR_UNSUPPORTED;
  int F = 0, P = 0, n_fb = 0;
  size_t lds = 0;
  switch (ncode / 256) {
    case 1: *clips = pt_capacity<1>(frames, nq, &F, &P, &n_fb, &lds); break;
    case 2: *clips = pt_capacity<2>(frames, nq, &F, &P, &n_fb, &lds); break;
    case 3: *clips = pt_capacity<3>(frames, nq, &F, &P, &n_fb, &lds); break;
    default: *clips = pt_capacity<4>(frames, nq, &F, &P, &n_fb, &lds); break;
  }
  if (*clips < 0) *clips = 0;
  return 0;
}

extern "C" int vrvq_rvq_debug_capacity(int clips) {
  const int prev = g_pt_cap_limit;
  g_pt_cap_limit = clips >= 0 ? clips : 0x7fffffff;
  return prev;
}
