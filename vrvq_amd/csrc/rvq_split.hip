// Channel-split residual vector quantisation for gfx950: VBRResidualVectorQuantize.forward
// (models/quantize.py:328-443) with the importance gating of models/utils.py:45-61, the same
// outputs as vrvq_rvq_fused, computed by GROUPS of 8 workgroups.
//
// Why split: in the single-workgroup-per-frame-range design (rvq_fused.hip) every CU must pull
// every stage's full weight set (W_in, normalised codebook, W_out: ~100 KB) through its memory
// pipeline for ~11 frames, and its z_q_is stores are 48-byte row pieces; the measured stage
// period is dominated by those two streams, not by arithmetic. Here a group of S = 8
// workgroups shares one frame range (<= 64 frames of one clip); workgroup s owns latent
// channels [128 s, 128 s + 128) and codebook entries [s N/8, (s+1) N/8). Per stage it moves
// only its 1/8 of the weights (~13 KB) and writes its 128 z_q_is rows as contiguous segments
// straight from registers (lane = frame). The price is two tiny exchanges per stage through
// L2: the 8-dim in_proj partial sums (z_e needs all 1024 channels) and the per-slice argmin
// candidates (the nearest codeword needs all N entries).
//
// Workgroup = 4 compute waves + 1 exchange wave (320 threads); lane = frame everywhere.
//   compute wave w: channels 128 s + 32 w + j (j < 32): residual and masked sum in
//                   VGPRs; codebook entries s N/8 + w N/32 + m for the distance scan.
//   exchange wave : publishes / gathers the partials and candidates, z_e, normalisation,
//                   final argmin, raw codeword, loss, codes, mask, latents; LDS-DMA of the
//                   next stage's weight slices. It is the only wave that waits on vmcnt, so
//                   the compute waves' z_q_is stores stay in flight across every barrier.
// Per stage i (4 LDS-only barriers):
//   [P] exchange: sum the 4 waves' in_proj partials, publish, wait for the group, sum the 8
//       slices in a fixed tree order (identical in every workgroup of the group), + b_in ->
//       z_e; L2-normalise; latents
//   [Q] compute : cosine distance over the wave's codebook entries, strict-< argmin
//       exchange: LDS-DMA of stage i+1's weight slices
//   [R] exchange: combine the 4 candidates, publish, wait, combine the 8 slices
//       (lexicographic (dist, index) min = the reference's first-index argmax of -dist),
//       raw codeword (L2 gather), loss, codes, mask, straight-through vector
//   [U] compute : out_proj -> residual update, masked z_q accumulate, z_q_is rows -> HBM;
//       in_proj partials of stage i+1
// Every expression except the in_proj partial-sum order is the one of vrvq_rvq_codes +
// vrvq_rvq_expand, so codes / z_q_is agree with them bit for bit whenever z_e does.
//
// Exchange protocol: per group a monotonically increasing arrival counter in the caller's
// workspace. Publishing = agent-scope relaxed atomic stores of the data, s_waitcnt vmcnt(0)
// (the stores have completed at their coherence point), one atomic add; waiting = agent-scope
// loads of the counter until it reaches S * (number of exchanges so far), then agent-scope
// loads of the data. The 8 workgroups of a group are mapped to one XCD (workgroup w runs on
// XCD w % 8), so the exchange stays inside one L2. Every wait is bounded: on timeout the
// workgroup sets the workspace error word, stops waiting (its outputs are garbage) and still
// runs to the end, so the grid always drains. The last workgroup of a group to leave resets the
// group's counters, so the workspace is zero again after every launch.
// The grid is at most 32 groups (256 workgroups of 320 threads, one per CU: every member of a
// group is resident at once); groups loop over frame ranges.
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int SP_D = 1024;            // latent channels (every conf/*.yml)
constexpr int SP_CD = 8;              // codebook_dim
constexpr int SP_S = 8;               // workgroups per group (channel / codebook slices)
constexpr int SP_CW = SP_D / SP_S;    // channels per workgroup (128)
constexpr int SP_CPW = SP_CW / 4;     // channels per compute wave (32)
constexpr int SP_F = 64;              // frames per range (lane = frame)
constexpr int SP_NT = 320;            // 4 compute waves + 1 exchange wave
constexpr int SP_GMAX = 32;           // groups in the grid at most (default)
constexpr unsigned SP_SPIN = 1u << 20;  // bounded wait (iterations of load + s_sleep)

// workspace layout (bytes)
constexpr size_t WS_HDR = 256;                               // [0] error word
constexpr size_t WS_CNT = 64;                                // per group: [0] arrivals [1] exits
constexpr size_t WS_CNTS = WS_CNT * 64;                      // counters of 64 groups (fixed place)
constexpr size_t WS_XP = (size_t)2 * SP_S * 4 * SP_F * 8;    // per group: [2][S][4 k pairs][64] u64
constexpr size_t WS_XA = (size_t)2 * SP_S * SP_F * 8;        // per group: [2][S][64] u64

typedef float f2 __attribute__((ext_vector_type(2)));

struct SplitArgs {
  const float* z;        // [B][D][T]
  int B, T, nq, N;
  const float* w_in_t;   // [nq][D][8]
  const float* b_in;     // [nq][8]
  const float* cb;       // [nq][N][8]
  const float* cbn;      // [nq][N][8]
  const float* c2;       // [nq][N]
  const float* w_out;    // [nq][D][8]
  const float* b_out;    // [nq][D]
  const float* imp;      // [B][T] or null (CBR: mask = 1)
  float level;
  int64_t* codes;        // [B][nq][T]
  float* latents;        // [B][nq*8][T]
  float* loss_pf;        // [B][nq][T]
  float* z_q_is;         // [B][nq][D][T] or null
  float* z_q;            // [B][D][T]
  float* mask;           // [B][nq][T] or null
  int nr;                // frame ranges per clip
  int items;             // B * nr
  int G;                 // groups in the grid (multiple of 8)
  unsigned char* ws;     // workspace (zero on entry, zero on exit)
  bool sys;              // system-scope exchange (diagnostic knob VRVQ_SPLIT_SYS)
  int dbg;               // diagnostic knob VRVQ_SPLIT_DBG: 1 = z_e from the own slice only
  unsigned long long* stamps;  // diagnostic build only (-DVRVQ_STAMPS): [grid][nq][8]
};

#ifdef VRVQ_STAMPS
#define SSTAMP(step)                                                                  \
  do {                                                                                \
    if (a.stamps && threadIdx.x == 256 && first_item) {                               \
      unsigned long long t_;                                                          \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
      a.stamps[((size_t)blockIdx.x * a.nq + i) * 8 + (step)] = t_;                   \
    }                                                                                 \
  } while (0)
#else
#define SSTAMP(step) do {} while (0)
#endif

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <class T>
__device__ __forceinline__ T* at(T* base, unsigned off) { return base + off; }

// LDS-DMA of nfloat floats (multiple of 4, 16-B aligned) by one wave: 1 KiB per instruction,
// the tail with a lane mask. Completion is waited for by the caller (vmcnt).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; nothing else here uses it
// Wave-uniform source (SGPR pair) + one per-lane 32-bit offset: no 64-bit per-lane addresses.
// `lds` is the destination's LDS byte address.
__device__ __forceinline__ void dma_wave(const float* src, unsigned lds0, int nfloat, int lane) {
  for (int q = 0; q * 256 < nfloat; ++q) {
    if (lane * 4 < nfloat - q * 256) {
      const unsigned lds = lds0 + q * 1024u;
      const float* gp = src + q * 256 + lane * 4;
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                   :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gp) : "memory", "m0");
    }
  }
}
#pragma clang diagnostic pop

// Buffer resources: a wave-uniform 128-bit descriptor + one 32-bit per-lane offset + a uniform
// SGPR offset per row. (Plain pointer arithmetic let the compiler strength-reduce every row's
// address into its own 64-bit per-lane induction variable: > 256 VGPRs and scratch.)
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// (the b32 builtins traffic in uint32: bit casts, not conversions)
__device__ __forceinline__ float ldf(rsrc_t r, unsigned voff, unsigned soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void stf(float v, rsrc_t r, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, 0);
}
constexpr int CP_SC1 = 16;  // device-coherent access (what agent-scope atomics use on gfx950)
typedef unsigned u2 __attribute__((ext_vector_type(2)));
constexpr int CP_SYS = 17;  // sc0 | sc1: system scope (diagnostic knob VRVQ_SPLIT_SYS)
__device__ __forceinline__ void put2(rsrc_t r, unsigned voff, unsigned soff, float lo, float hi,
                                     bool sys) {
  const u2 v = {__float_as_uint(lo), __float_as_uint(hi)};
  if (sys) __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, soff, CP_SYS);
  else __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, soff, CP_SC1);
}
__device__ __forceinline__ u2 get2(rsrc_t r, unsigned voff, unsigned soff, bool sys) {
  if (sys) return __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, CP_SYS);
  return __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, CP_SC1);
}

// Publish (after this wave's exchange stores) and wait until every member of the group has
// published exchange number `n` (1-based). Executed by the exchange wave only.
__device__ __forceinline__ void group_sync(unsigned* cnt, unsigned target, int lane, bool& poisoned,
                                           unsigned* err, bool sys) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // exchange stores (and DMA) complete
  if (lane == 0) {
    if (sys) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (poisoned) return;
  for (unsigned it = 0; it < SP_SPIN; ++it) {
    const unsigned v = __builtin_amdgcn_readfirstlane(
        sys ? __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
            : __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (v >= target) return;
    __builtin_amdgcn_s_sleep(1);
  }
  poisoned = true;
  if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-stage weight slice set ws(i) in LDS: cbn(i), c2(i), W_out(i), b_out(i), W_in(i+1).
template <int NM>
struct WSet {
  static constexpr int NS = 32 * NM;  // codebook entries per workgroup (N / 8)
  float cbn[NS * SP_CD];
  float c2[NS];
  float wout[SP_CW * SP_CD];
  float bout[SP_CW];
  float win[SP_CW * SP_CD];
  // LDS byte offsets of the fields (DMA destinations)
  static constexpr unsigned O_CBN = 0, O_C2 = NS * SP_CD * 4, O_WOUT = O_C2 + NS * 4,
                            O_BOUT = O_WOUT + SP_CW * SP_CD * 4, O_WIN = O_BOUT + SP_CW * 4;
};

template <int NM>
__global__ __launch_bounds__(SP_NT) void rvq_split_kernel(SplitArgs a) {
  constexpr int N = 256 * NM;
  constexpr int NS = N / SP_S;       // entries per workgroup
  constexpr int NPW = NS / 4;        // entries per compute wave (8 NM)
  using W = WSet<NM>;
  constexpr unsigned WSZ = sizeof(W);
  __shared__ __attribute__((aligned(16))) W wsb[2];
  __shared__ __attribute__((aligned(16))) float red[4 * SP_CD * SP_F];  // [w][k][f] in_proj partials
  __shared__ __attribute__((aligned(16))) float ev[SP_CD * SP_F];       // [k][f] normalised z_e
  __shared__ __attribute__((aligned(16))) float e2v[SP_F];              // [f] |e|^2
  __shared__ __attribute__((aligned(16))) float cd[4 * SP_F];           // [w][f] candidate dist
  __shared__ __attribute__((aligned(16))) int ci[4 * SP_F];             // [w][f] candidate index
  __shared__ __attribute__((aligned(16))) float stv[SP_CD * SP_F];      // [k][f] straight-through

  // ---- group / slice: the 8 members of group g run on XCD g % 8 ----
  const int bid = blockIdx.x;
  const int g = ((bid >> 6) << 3) | (bid & 7);
  const int s = (bid >> 3) & 7;
  if (g >= a.items) return;  // whole group idle: every member exits before any barrier

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = a.T, nq = a.nq;

  // The two roles run separate copies of the same barrier sequence
  //   per item: [I] ; per stage: [P] [Q] [R] [U] ; per item: [X]
  // (separate loops, so the register allocator sees each role's live values only).
  if (wave == 4) {
    // =============================== exchange wave ===============================
    unsigned* cnt = reinterpret_cast<unsigned*>(a.ws + WS_HDR + (size_t)g * WS_CNT);
    unsigned* err = reinterpret_cast<unsigned*>(a.ws);
    const rsrc_t xp = rsrc(a.ws + WS_HDR + WS_CNTS + (size_t)g * WS_XP, WS_XP);
    const rsrc_t xa =
        rsrc(a.ws + WS_HDR + WS_CNTS + (size_t)a.G * WS_XP + (size_t)g * WS_XA, WS_XA);
    const unsigned x_off = (unsigned)lane * 8u;  // this lane's u64 in an exchange row
    // LDS byte address of the weight-set buffers (from the __shared__ array itself: a cast of a
    // generic pointer would carry a null check)
    const unsigned wsb_lds = (unsigned)(size_t)(__attribute__((address_space(3))) void*)(wsb);
    unsigned nsync = 0;     // exchanges completed by this group (same in every member)
    bool poisoned = false;  // a wait timed out
    bool first_item = true;
    (void)first_item;
    for (int item = g; item < a.items; item += a.G) {
      const int b = item / a.nr, rg = item - b * a.nr;
      const int t0 = (int)((long long)rg * T / a.nr);
      const int nf = (int)((long long)(rg + 1) * T / a.nr) - t0;  // 1 .. 64
      const bool fvalid = lane < nf;
      const unsigned tl = (unsigned)(t0 + (fvalid ? lane : 0));
      // importance threshold s = (imp * level) * nq of this lane's frame (models/quantize.py:389)
      const float sv = (a.imp && fvalid) ? (a.imp[(size_t)b * T + tl] * a.level) * (float)nq
                                         : INFINITY;
      // W_in(0) -> wsb[1].win (as if ws(-1)), ws(0) -> wsb[0]
      dma_wave(a.w_in_t + (size_t)s * SP_CW * SP_CD, wsb_lds + WSZ + W::O_WIN, SP_CW * SP_CD, lane);
      dma_wave(a.cbn + (size_t)s * NS * SP_CD, wsb_lds + W::O_CBN, NS * SP_CD, lane);
      dma_wave(a.c2 + (size_t)s * NS, wsb_lds + W::O_C2, NS, lane);
      dma_wave(a.w_out + (size_t)s * SP_CW * SP_CD, wsb_lds + W::O_WOUT, SP_CW * SP_CD, lane);
      dma_wave(a.b_out + (size_t)s * SP_CW, wsb_lds + W::O_BOUT, SP_CW, lane);
      if (nq > 1)
        dma_wave(a.w_in_t + ((size_t)SP_D + s * SP_CW) * SP_CD, wsb_lds + W::O_WIN, SP_CW * SP_CD,
                 lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();  // ---------------------------------------------------------------- I
      for (int i = 0; i < nq; ++i) {
        const int par = (nsync >> 1) & 1;  // exchange buffer parity (alternates per stage)
        const int cur = i & 1;
        lds_barrier();  // -------------------------------------------------------------- P
        SSTAMP(0);
        // (1) publish this workgroup's partial, gather the group's, z_e = tree sum + b_in
        {
          float p[SP_CD];
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) {
            const float* rp = red + k * SP_F + lane;
            p[k] = (rp[0] + rp[SP_CD * SP_F]) + (rp[2 * SP_CD * SP_F] + rp[3 * SP_CD * SP_F]);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q)
            put2(xp, x_off, (unsigned)(((par * SP_S + s) * 4 + q) * SP_F * 8), p[2 * q], p[2 * q + 1], a.sys);
        }
        group_sync(cnt, SP_S * (++nsync), lane, poisoned, err, a.sys);
        SSTAMP(1);
        float ze[SP_CD];
        if (a.dbg == 1) {
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) {
            const float* rp = red + k * SP_F + lane;
            ze[k] = (rp[0] + rp[SP_CD * SP_F]) + (rp[2 * SP_CD * SP_F] + rp[3 * SP_CD * SP_F]);
          }
        } else if (a.dbg == 2) {
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) ze[k] = wsb[1].win[k] + 1000.0f * wsb[0].cbn[k];
        } else {
          float ps[SP_S][SP_CD];
#pragma unroll
          for (int t = 0; t < SP_S; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const u2 v = get2(xp, x_off, (unsigned)(((par * SP_S + t) * 4 + q) * SP_F * 8), a.sys);
              ps[t][2 * q] = __uint_as_float(v.x);
              ps[t][2 * q + 1] = __uint_as_float(v.y);
            }
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) {
            const float z = ((ps[0][k] + ps[1][k]) + (ps[2][k] + ps[3][k])) +
                            ((ps[4][k] + ps[5][k]) + (ps[6][k] + ps[7][k]));
            ze[k] = z + a.b_in[i * SP_CD + k];
          }
        }
        // L2 normalisation, models/quantize.py:92-95 (the sum8 butterfly tree of rvq_codes)
        {
          float q2[SP_CD], e[SP_CD];
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) q2[k] = ze[k] * ze[k];
          const float n2 = ((q2[0] + q2[1]) + (q2[2] + q2[3])) + ((q2[4] + q2[5]) + (q2[6] + q2[7]));
          const float den = fmaxf(sqrtf(n2), 1e-12f);
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) e[k] = ze[k] / den;
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) q2[k] = e[k] * e[k];
          const float e2 = ((q2[0] + q2[1]) + (q2[2] + q2[3])) + ((q2[4] + q2[5]) + (q2[6] + q2[7]));
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) ev[k * SP_F + lane] = e[k];
          e2v[lane] = e2;
        }
        if (s == 0 && fvalid) {
          float* lb = a.latents + ((size_t)b * nq + i) * SP_CD * T;
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) lb[(size_t)k * T + tl] = ze[k];
        }
        lds_barrier();  // -------------------------------------------------------------- Q
        SSTAMP(2);
        // (2) next stage's weight slices -> wsb[(i+1)&1] (its last reader, in_proj(i), is done);
        // landed at the vmcnt(0) of the next group_sync
        if (i + 1 < nq) {
          const unsigned nx = wsb_lds + (unsigned)(cur ^ 1) * WSZ;
          const size_t i1 = (size_t)(i + 1);
          dma_wave(a.cbn + (i1 * N + s * NS) * SP_CD, nx + W::O_CBN, NS * SP_CD, lane);
          dma_wave(a.c2 + i1 * N + s * NS, nx + W::O_C2, NS, lane);
          dma_wave(a.w_out + (i1 * SP_D + s * SP_CW) * SP_CD, nx + W::O_WOUT, SP_CW * SP_CD, lane);
          dma_wave(a.b_out + i1 * SP_D + s * SP_CW, nx + W::O_BOUT, SP_CW, lane);
          if (i + 2 < nq)
            dma_wave(a.w_in_t + ((i1 + 1) * SP_D + s * SP_CW) * SP_CD, nx + W::O_WIN,
                     SP_CW * SP_CD, lane);
        }
        lds_barrier();  // -------------------------------------------------------------- R
        SSTAMP(3);
        // (4) workgroup candidate (waves in order), publish, group argmin (slices in order)
        float bd = cd[lane];
        int bx = ci[lane];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const float od = cd[w * SP_F + lane];
          const int oi = ci[w * SP_F + lane];
          const bool take = (od < bd) | ((od == bd) & (oi < bx));
          bd = take ? od : bd;
          bx = take ? oi : bx;
        }
        put2(xa, x_off, (unsigned)((par * SP_S + s) * SP_F * 8), bd, __int_as_float(bx), a.sys);
        group_sync(cnt, SP_S * (++nsync), lane, poisoned, err, a.sys);
        SSTAMP(4);
#pragma unroll
        for (int t = 0; t < SP_S; ++t) {
          const u2 v = get2(xa, x_off, (unsigned)((par * SP_S + t) * SP_F * 8), a.sys);
          const float od = __uint_as_float(v.x);
          const int oi = (int)v.y;
          const bool take = (od < bd) | ((od == bd) & (oi < bx));
          bd = take ? od : bd;
          bx = take ? oi : bx;
        }
        const int ix = (bx >= 0 && bx < N) ? bx : 0;
        // (5) raw codeword (models/quantize.py:102-103), loss, codes, mask, straight-through
        const float* crow = a.cb + ((size_t)i * N + ix) * SP_CD;
        const float4 q0 = *reinterpret_cast<const float4*>(crow);
        const float4 q1 = *reinterpret_cast<const float4*>(crow + 4);
        const float zq[SP_CD] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        float d2[SP_CD];
#pragma unroll
        for (int k = 0; k < SP_CD; ++k) {
          const float diff = ze[k] - zq[k];
          d2[k] = diff * diff;
          stv[k * SP_F + lane] = ze[k] + (zq[k] - ze[k]);  // z_e + (z_q - z_e).detach()
        }
        const float l2 = ((d2[0] + d2[1]) + (d2[2] + d2[3])) + ((d2[4] + d2[5]) + (d2[6] + d2[7]));
        if (s == 0 && fvalid) {
          const size_t fo = ((size_t)b * nq + i) * T;
          a.codes[fo + tl] = (int64_t)bx;
          a.loss_pf[fo + tl] = l2 / 8.0f;
          if (a.mask) a.mask[fo + tl] = (sv - (float)i >= 0.0f) ? 1.0f : 0.0f;
        }
        lds_barrier();  // -------------------------------------------------------------- U
        SSTAMP(5);
      }
      lds_barrier();  // ---------------------------------------------------------------- X
      first_item = false;
    }
    // the last member of the group to leave resets the group's counters (every member adds its
    // exit only after its final wait)
    if (lane == 0) {
      const unsigned old =
          __hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == SP_S - 1) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    // =============================== compute waves ===============================
    const int c0 = s * SP_CW + wave * SP_CPW;  // first channel of this wave
    const int n0 = s * NS + wave * NPW;        // first codebook entry of this wave
    for (int item = g; item < a.items; item += a.G) {
      const int b = item / a.nr, rg = item - b * a.nr;
      const int t0 = (int)((long long)rg * T / a.nr);
      const int nf = (int)((long long)(rg + 1) * T / a.nr) - t0;  // 1 .. 64
      const bool fvalid = lane < nf;
      const float sv = (a.imp && fvalid) ? (a.imp[(size_t)b * T + t0 + lane] * a.level) * (float)nq
                                         : INFINITY;
      // per-lane byte offset of (channel c0, frame t0 + lane) in a [D][T] slab; lanes past the
      // range get an offset beyond every buffer's size (their loads return 0, stores are dropped)
      const unsigned row_off =
          fvalid ? ((unsigned)(c0 * T + t0) + (unsigned)lane) * 4u : 0x80000000u;
      float r[SP_CPW], zacc[SP_CPW];  // residual / masked z_q sum of the wave's channels
      {
        const rsrc_t zr = rsrc(a.z + (size_t)b * SP_D * T, (unsigned)(SP_D * T * 4));
#pragma unroll
        for (int j = 0; j < SP_CPW; ++j) {
          r[j] = ldf(zr, row_off, (unsigned)(j * T * 4));
          zacc[j] = 0.0f;
        }
      }
      // in_proj partials: p[k] = sum_j W_in[k, c_j] r[c_j], j in order (fmaf chain)
      auto in_proj = [&](int wb) __attribute__((always_inline)) {
        float p[SP_CD];
#pragma unroll
        for (int j = 0; j < SP_CPW; ++j) {
          const float* w = wsb[wb].win + (wave * SP_CPW + j) * SP_CD;
          if ((j & 3) == 0) asm volatile("" ::: "memory");  // bound the LDS-load hoisting
          const float4 w0 = *reinterpret_cast<const float4*>(w);
          const float4 w1 = *reinterpret_cast<const float4*>(w + 4);
          const float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int k = 0; k < SP_CD; ++k) p[k] = j == 0 ? wk[k] * r[0] : fmaf(wk[k], r[j], p[k]);
        }
        float* rw = red + wave * SP_CD * SP_F + lane;
#pragma unroll
        for (int k = 0; k < SP_CD; ++k) rw[k * SP_F] = p[k];
      };
      lds_barrier();  // ---------------------------------------------------------------- I
      in_proj(1);
      for (int i = 0; i < nq; ++i) {
        const int cur = i & 1;
        const W& ws = wsb[cur];
        lds_barrier();  // -------------------------------------------------------------- P
        lds_barrier();  // -------------------------------------------------------------- Q
        // (3) nearest codeword over this wave's entries (lowest index on ties):
        // dist = (sum e^2 - 2 e.c) + sum c^2, dot in k order (models/quantize.py:96-100)
        {
          const float4 e0 = make_float4(ev[0 * SP_F + lane], ev[1 * SP_F + lane],
                                        ev[2 * SP_F + lane], ev[3 * SP_F + lane]);
          const float4 e1 = make_float4(ev[4 * SP_F + lane], ev[5 * SP_F + lane],
                                        ev[6 * SP_F + lane], ev[7 * SP_F + lane]);
          const float e2 = e2v[lane];
          float best = INFINITY;
          int bi = 0x7fffffff;
#pragma unroll
          for (int m = 0; m < NPW; ++m) {
            const int nl = wave * NPW + m;  // local entry (uniform)
            if ((m & 3) == 0) asm volatile("" ::: "memory");
            const float4 c0v = *reinterpret_cast<const float4*>(ws.cbn + nl * SP_CD);
            const float4 c1v = *reinterpret_cast<const float4*>(ws.cbn + nl * SP_CD + 4);
            const float dist = (e2 - 2.0f * dot8(e0, e1, c0v, c1v)) + ws.c2[nl];
            const bool t = dist < best;  // entries in increasing order: strict < keeps the first
            best = t ? dist : best;
            bi = t ? n0 + m : bi;
          }
          cd[wave * SP_F + lane] = best;
          ci[wave * SP_F + lane] = bi;
        }
        lds_barrier();  // -------------------------------------------------------------- R
        lds_barrier();  // -------------------------------------------------------------- U
        // (6) out_proj -> residual update, masked z_q accumulate, z_q_is rows
        {
          const float4 zp0 = make_float4(stv[0 * SP_F + lane], stv[1 * SP_F + lane],
                                         stv[2 * SP_F + lane], stv[3 * SP_F + lane]);
          const float4 zp1 = make_float4(stv[4 * SP_F + lane], stv[5 * SP_F + lane],
                                         stv[6 * SP_F + lane], stv[7 * SP_F + lane]);
          const float mf = (sv - (float)i >= 0.0f) ? 1.0f : 0.0f;
          // (z_q_is not materialised: a zero-size buffer, every store dropped)
          const rsrc_t zr = rsrc(a.z_q_is ? a.z_q_is + ((size_t)b * nq + i) * SP_D * T : a.z_q,
                                 a.z_q_is ? (unsigned)(SP_D * T * 4) : 0u);
#pragma unroll
          for (int j = 0; j < SP_CPW; ++j) {
            const int cl = wave * SP_CPW + j;
            if ((j & 3) == 0) asm volatile("" ::: "memory");
            const float4 w0 = *reinterpret_cast<const float4*>(ws.wout + cl * SP_CD);
            const float4 w1 = *reinterpret_cast<const float4*>(ws.wout + cl * SP_CD + 4);
            const float v = out_proj1(w0, w1, ws.bout[cl], zp0, zp1);  // (W_out . st) + b_out
            r[j] = r[j] - v;
            zacc[j] = zacc[j] + v * mf;
            stf(v, zr, row_off, (unsigned)(j * T * 4));
          }
        }
        if (i + 1 < nq) in_proj(cur);
      }
      {
        const rsrc_t zr = rsrc(a.z_q + (size_t)b * SP_D * T, (unsigned)(SP_D * T * 4));
#pragma unroll
        for (int j = 0; j < SP_CPW; ++j)
          stf(zacc[j], zr, row_off, (unsigned)(j * T * 4));
      }
      lds_barrier();  // ---------------------------------------------------------------- X
    }
  }
}

// Groups in the grid: at most 32 (256 workgroups of 5 waves at ~250 VGPRs: one per CU, so every
// member of every group is resident at once on 256 CUs); VRVQ_SPLIT_GMAX (8..64) overrides
// for experiments (beyond 32 it relies on in-order workgroup dispatch for forward progress).
int split_groups(long long items) {
  static const int gmax = [] {
    const char* e = getenv("VRVQ_SPLIT_GMAX");
    const int v = e ? atoi(e) : SP_GMAX;
    return v < 8 ? 8 : (v > 64 ? 64 : v);
  }();
  long long G = items < gmax ? items : gmax;
  return (int)((G + 7) / 8 * 8);
}

}  // namespace

extern "C" int vrvq_rvq_split_workspace(int batch, int frames, long long* bytes) {
  VRVQ_CHECK_ARG(bytes && batch > 0 && frames > 0);
  const long long items = (long long)batch * ((frames + SP_F - 1) / SP_F);
  const int G = split_groups(items);
  *bytes = (long long)(WS_HDR + WS_CNTS + (size_t)G * (WS_XP + WS_XA));
  return VRVQ_OK;
}

extern "C" int vrvq_rvq_split(const float* z, int batch, int dim, int frames, int nq, int ncode,
                              int cdim, const float* w_in_t, const float* b_in, const float* cb,
                              const float* cbn, const float* c2, const float* w_out,
                              const float* b_out, const float* imp, float level, int64_t* codes,
                              float* latents, float* loss_pf, float* z_q_is, float* z_q,
                              float* mask, void* workspace, long long workspace_bytes,
                              vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z && w_in_t && b_in && cb && cbn && c2 && w_out && b_out && codes && latents &&
                 loss_pf && z_q && workspace);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  VRVQ_CHECK_ARG((long long)frames * SP_D < 0x7fffffffLL);  // 32-bit per-row offsets
  if (dim != SP_D || cdim != SP_CD || ncode <= 0 || ncode % 256 != 0 || ncode > 1024)
    return VRVQ_ERR_UNSUPPORTED;
  // LDS-DMA sources must be 16-byte aligned
  const uintptr_t al = (uintptr_t)w_in_t | (uintptr_t)cbn | (uintptr_t)c2 | (uintptr_t)w_out |
                       (uintptr_t)b_out | (uintptr_t)cb | (uintptr_t)workspace;
  VRVQ_CHECK_ARG((al & 15) == 0);
  long long need = 0;
  vrvq_rvq_split_workspace(batch, frames, &need);
  VRVQ_CHECK_ARG(workspace_bytes >= need);
  SplitArgs a{};
  a.z = z; a.B = batch; a.T = frames; a.nq = nq; a.N = ncode;
  a.w_in_t = w_in_t; a.b_in = b_in; a.cb = cb; a.cbn = cbn; a.c2 = c2;
  a.w_out = w_out; a.b_out = b_out; a.imp = imp; a.level = level;
  a.codes = codes; a.latents = latents; a.loss_pf = loss_pf;
  a.z_q_is = z_q_is; a.z_q = z_q; a.mask = mask;
  a.nr = (frames + SP_F - 1) / SP_F;
  const long long items = (long long)batch * a.nr;
  VRVQ_CHECK_ARG(items < 0x7fffffffLL);
  a.items = (int)items;
  a.G = split_groups(items);
  a.ws = static_cast<unsigned char*>(workspace);
  static const bool sys = getenv("VRVQ_SPLIT_SYS") != nullptr;
  a.sys = sys;
  static const int dbg = getenv("VRVQ_SPLIT_DBG") ? atoi(getenv("VRVQ_SPLIT_DBG")) : 0;
  a.dbg = dbg;
  a.stamps = vrvq_g_stamps;
  const dim3 grid((unsigned)(a.G * SP_S));
  hipStream_t st = as_stream(stream);
  switch (ncode / 256) {
    case 1: hipLaunchKernelGGL(rvq_split_kernel<1>, grid, dim3(SP_NT), 0, st, a); break;
    case 2: hipLaunchKernelGGL(rvq_split_kernel<2>, grid, dim3(SP_NT), 0, st, a); break;
    case 3: hipLaunchKernelGGL(rvq_split_kernel<3>, grid, dim3(SP_NT), 0, st, a); break;
    default: hipLaunchKernelGGL(rvq_split_kernel<4>, grid, dim3(SP_NT), 0, st, a); break;
  }
  return vrvq_launch_status();
}
