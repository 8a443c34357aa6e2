// Single-launch residual vector quantisation for gfx950: VBRResidualVectorQuantize.forward
// (models/quantize.py:328-443) with the importance gating of models/utils.py:45-61 — the
// sequential residual chain AND the HBM stream of its outputs (z_q_is, masked z_q, mask,
// codes, latents, per-frame loss) in one kernel.
//
// Why one launch: ~95 % of the algorithmic bytes are the z_q_is rows (nq*D*4 B per frame), and
// each stage's z_q_i is exactly the out_proj value the chain computes for its residual update.
// Writing it from the chain overlaps that HBM stream with the chain's latency instead of
// re-reading the straight-through vectors in a second kernel.
//
// Work unit = one frame range of one clip (<= 12 frames, never straddling clips), so every
// z_q_is row segment a workgroup writes is contiguous; units are mapped XCD-major (consecutive
// units of a clip land on the same XCD / L2, which merges the partial lines of a row).
//
// Thread layout (512 threads = 2 frame groups x 256 channel threads): thread (g, ct) owns latent
// channels c = ct + 256 j (j < 4) of the group's 6 frames — 24 residual VGPRs and 24 masked-sum
// VGPRs; every weight it loads is reused for 6 frames from a register.
//
// Per stage i (two workgroup barriers; every weight is requested at least a phase before use):
//   in_proj (v_pk_fma) -> wave reduce-scatter -> LDS -> vmcnt(0) (stage-i codebook DMA)
//   [A] -> DMA raw codebook(i), W_out(i) ; z_q_is(i-1) tile -> HBM (coalesced row segments) ;
//          z_e, L2-normalise, latents ; cosine-distance scan over this thread's codes, wave
//          argmin -> LDS -> vmcnt (raw / W_out DMA)
//   [B] -> DMA cbn / c2 (i+1), W_in(i+1) -> registers ; final argmin, raw codeword, loss,
//          codes, mask ; out_proj -> residual update, masked z_q accumulate, z_q_i -> LDS tile
// Arithmetic is expression-for-expression the one of vrvq_rvq_codes + vrvq_rvq_expand
// (in_proj partial order aside), so z_q_is is bit-identical to what stage 2 would produce.
#include "common.h"
#include "lanes.h"

namespace {

constexpr int FU_D = 1024;           // latent channels (every conf/*.yml)
constexpr int FU_CD = 8;             // codebook_dim
constexpr int FU_FG = 2;             // frame groups
constexpr int FU_FPG = 6;            // frames per group
constexpr int FU_F = FU_FG * FU_FPG; // frames per workgroup (unit)
constexpr int FU_NT = 256 * FU_FG;   // threads per workgroup (8 waves, 2 per SIMD: 256 VGPRs)
constexpr int FU_NW = FU_NT / 64;
constexpr int FU_CPT = FU_D / 256;   // channels per thread
constexpr int FU_TS = 13;            // LDS tile row stride (odd: conflict-free column access)
constexpr int FU_WV = 56;            // per-wave broadcast slot: [8 k][6 f] vector + [6] extra
constexpr int FU_TR = (FU_D + 4 * FU_NW - 1) / (4 * FU_NW);  // tile row passes (4 rows / wave)

typedef float f2 __attribute__((ext_vector_type(2)));

struct FusedArgs {
  const float* z;        // [B][D][T]
  int B, T, nq;
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
  int units;             // B * nr
  int per_xcd;           // ceil(units / 8)
  int nt_store;          // z_q_is rows stored non-temporal (keep the stage weights L2-resident)
  unsigned long long* stamps;  // diagnostic build only (-DVRVQ_STAMPS): [grid][nq][8]
};

#ifdef VRVQ_STAMPS
#define FSTAMP(step)                                                                  \
  do {                                                                                \
    if (a.stamps && threadIdx.x == 0) {                                               \
      unsigned long long t_;                                                          \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
      a.stamps[((size_t)blockIdx.x * a.nq + i) * 8 + (step)] = t_;                   \
    }                                                                                 \
  } while (0)
#else
#define FSTAMP(step) do {} while (0)
#endif

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// Wave-uniform base + 32-bit per-lane offset: lets the compiler use the SGPR-base (saddr)
// addressing forms instead of a 64-bit VGPR address per access (the host checks that every
// per-row offset fits in 32 bits).
template <class T>
__device__ __forceinline__ T* at(T* base, unsigned off) { return base + off; }

// Workgroup barrier that orders LDS only. __syncthreads() is a workgroup-scope fence on all
// memory, which makes every barrier wait for every outstanding global load / store / LDS-DMA
// (vmcnt(0)); here the outstanding z_q_is stores and next-stage prefetches must stay in flight
// across barriers, and LDS-DMA completion is waited for explicitly where it is needed.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// LDS-DMA of `nchunks` 1-KiB chunks src -> dst, chunk q issued by wave q % FU_NW.
// Written as inline asm on purpose: the compiler's own LDS-DMA tracking turns every later LDS
// access it cannot disambiguate (and every LDS fence) into a vmcnt(0) wait, i.e. it would drain
// the z_q_is store stream and the next-stage prefetches at every barrier. Completion is waited
// for explicitly instead (vmcnt before barriers A and B; see the stage comments).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; nothing else here uses it
__device__ __forceinline__ void dma_chunks(const float* src, float* dst, int nchunks, int wave,
                                           int lane) {
  for (int q = wave; q < nchunks; q += FU_NW) {
    const float* gp = src + q * 256 + lane * 4;
    const unsigned lds = (unsigned)(size_t)(__attribute__((address_space(3))) float*)(dst + q * 256);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                 :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gp) : "memory", "m0");
  }
}
#pragma clang diagnostic pop

template <int NM>
__global__ __launch_bounds__(FU_NT) void rvq_fused_kernel(FusedArgs a) {
  constexpr int N = 256 * NM;  // codebook size
  // LDS: one array per role, so the compiler's LDS-DMA wait tracking can tell the DMA targets
  // (cbn, c2, raw, W_out) from the arrays read while a DMA is in flight (tile, red, wv, ...).
  __shared__ __attribute__((aligned(16))) float cbn_s[N * FU_CD];
  __shared__ __attribute__((aligned(16))) float cand_s[FU_FG * 4 * FU_FPG * FU_CD];  // raw rows
  __shared__ __attribute__((aligned(16))) float wo_s[FU_D * FU_CD];
  __shared__ __attribute__((aligned(16))) float bo_s[FU_D];
  __shared__ __attribute__((aligned(16))) float tile[FU_D * FU_TS];
  __shared__ __attribute__((aligned(16))) float red[FU_FG * 4 * 48];
  __shared__ __attribute__((aligned(16))) float dbs[FU_FG * 32];
  __shared__ __attribute__((aligned(16))) int ibs[FU_FG * 32];
  __shared__ __attribute__((aligned(16))) float wv_all[FU_NW * FU_WV];
  __shared__ __attribute__((aligned(16))) float warm_s[256];  // L2 warm-up DMA sink (never read)
  static_assert((256 + N * FU_CD + FU_FG * 4 * FU_FPG * FU_CD + FU_D * FU_CD + FU_D + FU_D * FU_TS + FU_FG * 4 * 48 + FU_FG * 64 +
                 FU_NW * FU_WV) * 4 <= 160 * 1024, "LDS budget");

  // ---- unit: XCD-major mapping (workgroup w runs on XCD w % 8) ----
  const int bid = blockIdx.x;
  const int u = (bid & 7) * a.per_xcd + (bid >> 3);
  if (u >= a.units) return;  // whole workgroup exits before any barrier
  const int b = u / a.nr, rg = u - b * a.nr;
  const int T = a.T, nq = a.nq;
  const int t0 = (int)((long long)rg * T / a.nr);
  const int nf = (int)((long long)(rg + 1) * T / a.nr) - t0;  // 1 .. 12

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = wave >> 2, wg = wave & 3, ct = tid & 255;
  float* wv = wv_all + wave * FU_WV;
  // (frame, k) lane roles of the per-frame steps: lane = f*8 + k, f < 6 (lanes 48..63 idle)
  const int fl = lane >> 3, kl = lane & 7;
  const bool lrole = lane < 48;
  const bool fvalid = lrole && g * FU_FPG + fl < nf;
  const int tl = t0 + g * FU_FPG + (lrole ? fl : 0);  // this lane's frame

  // importance threshold s = (imp * level) * nq per frame of the group (models/quantize.py:389)
  float sv[FU_FPG];
#pragma unroll
  for (int f = 0; f < FU_FPG; ++f) {
    const int s = g * FU_FPG + f;
    sv[f] = (a.imp && s < nf) ? (a.imp[(size_t)b * T + t0 + s] * a.level) * (float)nq : INFINITY;
  }
  const float s_lane = (a.imp && fvalid) ? (a.imp[(size_t)b * T + tl] * a.level) * (float)nq
                                         : INFINITY;  // this lane's frame (mask output)

  // ---- stage weights ----
  // The normalised codebook and W_out / b_out go HBM/L2 -> LDS by LDS-DMA (no registers):
  //   cbn (i+1)        issued after barrier B(i) (the stage-i distance scans are done),
  //                    landed at the vmcnt(0) before barrier A(i+1);
  //   W_out / b_out(i) issued after barrier A(i) (the stage-(i-1) out_proj reads are done),
  //                    landed at the vmcnt(0) before barrier B(i).
  // Not streamed: |c|^2 is recomputed from the cbn row (codebook_prep's expression), and of the
  // raw codebook only the rows of each wave's argmin candidates are gathered from L2 (below).
  // W_in (i+1) / b_in go to registers after barrier B(i).
  auto dma_cbn = [&](int i) {
    dma_chunks(a.cbn + (size_t)i * N * FU_CD, cbn_s, N * FU_CD / 256, wave, lane);
  };
  auto dma_wo = [&](int i) {
    dma_chunks(a.w_out + (size_t)i * FU_D * FU_CD, wo_s, FU_D * FU_CD / 256, wave, lane);
    dma_chunks(a.b_out + (size_t)i * FU_D, bo_s, FU_D / 256, wave, lane);
  };
  float4 wi[FU_CPT][2];
  auto load_wi = [&](int i) {
    const float* base = a.w_in_t + (size_t)i * FU_D * FU_CD;  // wave-uniform
#pragma unroll
    for (int j = 0; j < FU_CPT; ++j) {
      wi[j][0] = ld4(at(base, (ct + 256 * j) * FU_CD));
      wi[j][1] = ld4(at(base, (ct + 256 * j) * FU_CD + 4));
    }
  };
  // [D][T] row block (columns t0 .. t0+nf) from the LDS tile: 16-lane segments, one row each,
  // 32 rows per pass. Per-lane offsets are loop-invariant single VGPRs; each pass advances the
  // wave-uniform row pointer (SGPRs) and the LDS immediate offset. (Measured: 3 lanes x dwordx4
  // per row issues 5x fewer store instructions but ran 40 % slower — the rows are only
  // dword-aligned, T being odd.)
  const int ss = lane & 15, sub = lane >> 4;
  const unsigned g_off = (unsigned)((wave * 4 + sub) * T + t0 + ss);
  const float* t_lane = tile + (wave * 4 + sub) * FU_TS + ss;
  auto store_tile = [&](float* dst_base, bool nt) {
    if (ss < nf) {
#pragma unroll
      for (int k = 0; k < FU_TR; ++k) {
        if (k == FU_TR - 1 && (wave * 4 + 4 * FU_NW * k) >= FU_D) break;  // wave-uniform
        float* p = at(dst_base + (size_t)(4 * FU_NW * k) * T, g_off);
        const float v = t_lane[4 * FU_NW * k * FU_TS];
        if (nt) __builtin_nontemporal_store(v, p);
        else *p = v;
      }
    }
  };

  dma_cbn(0);
  load_wi(0);
  float bin_nx = a.b_in[kl];
  // L2 warm-up: the workgroups of one XCD (workgroup w runs on XCD w % 8) together touch every
  // stage's weights once (W_in, cbn, W_out, b_out: ~100 KB per stage), each 1/per_xcd of them,
  // as LDS-DMA pieces into a sink that is never read. Every later per-stage DMA / W_in load then
  // hits this XCD's L2 instead of taking a fabric / HBM miss on the chain's critical path. Lands
  // at the vmcnt(0) before barrier A of stage 0.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; nothing else here uses it
  {
    const int xj = bid >> 3;
    auto warm = [&](const float* base, int nchunks) {
      for (int q = xj * FU_NW + wave; q < nchunks; q += a.per_xcd * FU_NW) {
        const float* gp = base + q * 256 + lane * 4;
        const unsigned lds =
            (unsigned)(size_t)(__attribute__((address_space(3))) float*)(warm_s);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                     :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gp) : "memory", "m0");
      }
    };
    warm(a.w_in_t, nq * FU_D * FU_CD / 256);
    warm(a.cbn, nq * N * FU_CD / 256);
    warm(a.w_out, nq * FU_D * FU_CD / 256);
    warm(a.b_out, nq * FU_D / 256);
  }
#pragma clang diagnostic pop

  // ---- residual tile z[b, :, t0 .. t0+nf) -> LDS -> registers ----
  {
    const float* zb = a.z + (size_t)b * FU_D * T;
    float v[FU_TR];
#pragma unroll
    for (int k = 0; k < FU_TR; ++k) {
      const bool row_ok = (wave * 4 + 4 * FU_NW * k) < FU_D;
      v[k] = (ss < nf && row_ok) ? *at(zb + (size_t)(4 * FU_NW * k) * T, g_off) : 0.0f;
    }
    if (ss < FU_F) {
      float* tw = tile + (wave * 4 + sub) * FU_TS + ss;
#pragma unroll
      for (int k = 0; k < FU_TR; ++k)
        if ((wave * 4 + 4 * FU_NW * k) < FU_D) tw[4 * FU_NW * k * FU_TS] = v[k];
    }
  }
  lds_barrier();
  float r[FU_CPT][FU_FPG], zacc[FU_CPT][FU_FPG];
#pragma unroll
  for (int j = 0; j < FU_CPT; ++j)
#pragma unroll
    for (int f = 0; f < FU_FPG; ++f) {
      r[j][f] = tile[(ct + 256 * j) * FU_TS + g * FU_FPG + f];
      zacc[j][f] = 0.0f;
    }
  // (the tile is next written after barrier B of stage 0, when every wave has read it)

  for (int i = 0; i < nq; ++i) {
    const bool more = i + 1 < nq;
    const float bin = bin_nx;
    FSTAMP(0);
    // (1) in_proj partials p[f*8 + k] = sum_j W_in[k, c_j] r[c_j, f]   (packed over k pairs)
    float p[64];
    {
      f2 pp[FU_FPG * 4];
#pragma unroll
      for (int q = 0; q < FU_FPG * 4; ++q) pp[q] = f2{0.0f, 0.0f};
#pragma unroll
      for (int j = 0; j < FU_CPT; ++j) {
        const f2 w01 = {wi[j][0].x, wi[j][0].y}, w23 = {wi[j][0].z, wi[j][0].w};
        const f2 w45 = {wi[j][1].x, wi[j][1].y}, w67 = {wi[j][1].z, wi[j][1].w};
#pragma unroll
        for (int f = 0; f < FU_FPG; ++f) {
          const f2 rr = {r[j][f], r[j][f]};
          pp[f * 4 + 0] = __builtin_elementwise_fma(w01, rr, pp[f * 4 + 0]);
          pp[f * 4 + 1] = __builtin_elementwise_fma(w23, rr, pp[f * 4 + 1]);
          pp[f * 4 + 2] = __builtin_elementwise_fma(w45, rr, pp[f * 4 + 2]);
          pp[f * 4 + 3] = __builtin_elementwise_fma(w67, rr, pp[f * 4 + 3]);
        }
      }
#pragma unroll
      for (int q = 0; q < FU_FPG * 4; ++q) {
        p[2 * q] = pp[q].x;
        p[2 * q + 1] = pp[q].y;
      }
#pragma unroll
      for (int q = FU_FPG * 8; q < 64; ++q) p[q] = 0.0f;
    }
    // (2) wave reduce-scatter: lane l <- wave sum of p[l]
    {
      const float v = vrvq::reduce_scatter64(p, lane);
      if (lrole) red[(g * 4 + wg) * 48 + lane] = v;
    }
    FSTAMP(1);
    // this stage's cbn / c2 DMA and b_in landed (b_in is pinned here: the compiler would
    // otherwise wait for it at its first use, behind the z_q_is stores, with vmcnt(0))
    asm volatile("s_waitcnt vmcnt(0)" :: "v"(bin) : "memory");
    lds_barrier();  // ------------------------------------------------------------------ A
    FSTAMP(2);
    dma_wo(i);
    // z_q_is of the previous stage: tile -> HBM
    const bool tile_out = i > 0 && a.z_q_is;
    if (tile_out) store_tile(a.z_q_is + ((size_t)b * nq + (i - 1)) * FU_D * T, a.nt_store != 0);
    FSTAMP(3);
    // (3) z_e, L2 normalisation (lane = f*8 + k; every wave of the group)
    float ze;
    {
      const float* rp = red + g * 4 * 48 + (lrole ? lane : 0);
      ze = ((rp[0] + rp[48]) + (rp[96] + rp[144])) + bin;
      const float n2 = vrvq::sum8(ze * ze, lane);
      const float e = ze / fmaxf(sqrtf(n2), 1e-12f);
      const float e2 = vrvq::sum8(e * e, lane);
      if (wg == 0 && fvalid)
        *at(a.latents + ((size_t)b * nq + i) * FU_CD * T, kl * T + tl) = ze;
      if (lrole) wv[kl * 6 + fl] = e;
      if (lrole && kl == 0) wv[48 + fl] = e2;
    }
    // (4) nearest codeword over this thread's codes n = ct + 256 m (lowest index on ties)
    float best[8];
    int bidx[8];
    {
      f2 ep[FU_CD][3];
#pragma unroll
      for (int k = 0; k < FU_CD; ++k) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const float2 e = *reinterpret_cast<const float2*>(wv + k * 6 + 2 * q);
          ep[k][q] = f2{e.x, e.y};
        }
      }
      f2 e2p[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const float2 e = *reinterpret_cast<const float2*>(wv + 48 + 2 * q);
        e2p[q] = f2{e.x, e.y};
      }
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        best[f] = INFINITY;
        bidx[f] = 0x7fffffff;
      }
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int n = ct + 256 * m;
        const float4 c0 = *reinterpret_cast<const float4*>(cbn_s + n * FU_CD);
        const float4 c1 = *reinterpret_cast<const float4*>(cbn_s + n * FU_CD + 4);
        const float ck[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        float cc = 0.0f;  // |c|^2 of the normalised row, codebook_prep's fmaf chain
#pragma unroll
        for (int k = 0; k < FU_CD; ++k) cc = fmaf(ck[k], ck[k], cc);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          // dot in k order (mul, then fma chain), then (sum e^2 - 2 e.c) + sum c^2
          // (models/quantize.py:96-100)
          f2 d = ep[0][q] * f2{ck[0], ck[0]};
#pragma unroll
          for (int k = 1; k < FU_CD; ++k) d = __builtin_elementwise_fma(ep[k][q], f2{ck[k], ck[k]}, d);
          const f2 dist = (e2p[q] - 2.0f * d) + f2{cc, cc};
          const bool ta = dist.x < best[2 * q], tb = dist.y < best[2 * q + 1];  // n increasing:
          best[2 * q] = ta ? dist.x : best[2 * q];                              // strict < keeps
          bidx[2 * q] = ta ? n : bidx[2 * q];                                   // the first
          best[2 * q + 1] = tb ? dist.y : best[2 * q + 1];
          bidx[2 * q + 1] = tb ? n : bidx[2 * q + 1];
        }
      }
    }
    vrvq::argmin_scatter8(best, bidx, lane);  // lanes of 8-group f hold the wave argmin of f
    if (kl == 0 && lrole) {
      dbs[(g * 4 + wg) * 8 + fl] = best[0];
      ibs[(g * 4 + wg) * 8 + fl] = bidx[0];
    }
    // raw codebook row of this wave's candidate (the final winner is one of the 4 waves'
    // candidates): an L2 gather of 32 B per frame instead of streaming the 32 KB raw codebook
    if (lrole) {
      const int cix = (bidx[0] >= 0 && bidx[0] < N) ? bidx[0] : 0;
      cand_s[((g * 4 + wg) * FU_FPG + fl) * FU_CD + kl] = a.cb[((size_t)i * N + cix) * FU_CD + kl];
    }
    FSTAMP(4);
    // W_out / b_out DMA of this stage and the candidate rows landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();  // ------------------------------------------------------------------ B
    FSTAMP(5);
    if (more) {
      dma_cbn(i + 1);  // this stage's cbn / c2 reads are done everywhere
      load_wi(i + 1);
      bin_nx = a.b_in[(i + 1) * FU_CD + kl];
    }
    // (5) final argmin, raw codeword, loss, codes, mask, straight-through vector
    {
      float bd = INFINITY;
      int bi = 0, wsel = 0;
      if (lrole) {
        bd = dbs[(g * 4) * 8 + fl];
        bi = ibs[(g * 4) * 8 + fl];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const float od = dbs[(g * 4 + w) * 8 + fl];
          const int oi = ibs[(g * 4 + w) * 8 + fl];
          const bool take = (od < bd) | ((od == bd) & (oi < bi));  // vrvq::amin, + the wave
          bd = take ? od : bd;
          bi = take ? oi : bi;
          wsel = take ? w : wsel;
        }
      }
      const float zq = lrole ? cand_s[((g * 4 + wsel) * FU_FPG + fl) * FU_CD + kl] : 0.0f;
      const float st = ze + (zq - ze);  // z_e + (z_q - z_e).detach(), models/quantize.py:73-75
      const float diff = ze - zq;
      const float l2 = vrvq::sum8(diff * diff, lane);
      if (wg == 0 && fvalid) {
        const size_t fo = ((size_t)b * nq + i) * T;  // wave-uniform row
        if (kl == 0) {
          *at(a.codes + fo, tl) = (int64_t)bi;
          *at(a.loss_pf + fo, tl) = l2 / 8.0f;
        }
        if (kl == 1 && a.mask) *at(a.mask + fo, tl) = (s_lane - (float)i >= 0.0f) ? 1.0f : 0.0f;
      }
      if (lrole) wv[kl * 6 + fl] = st;
    }
    FSTAMP(6);
    // (6) out_proj -> residual update, masked z_q, z_q_i tile
    {
      f2 zp[FU_CD][3];
#pragma unroll
      for (int k = 0; k < FU_CD; ++k) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const float2 z2 = *reinterpret_cast<const float2*>(wv + k * 6 + 2 * q);
          zp[k][q] = f2{z2.x, z2.y};
        }
      }
      float mf[FU_FPG];
#pragma unroll
      for (int f = 0; f < FU_FPG; ++f) mf[f] = (sv[f] - (float)i >= 0.0f) ? 1.0f : 0.0f;
#pragma unroll
      for (int j = 0; j < FU_CPT; ++j) {
        const float4 w0 = *reinterpret_cast<const float4*>(wo_s + (ct + 256 * j) * FU_CD);
        const float4 w1 = *reinterpret_cast<const float4*>(wo_s + (ct + 256 * j) * FU_CD + 4);
        const float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        float* trow = tile + (ct + 256 * j) * FU_TS + g * FU_FPG;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          // out_proj1: (w0*z0, fma chain over k) + bias, packed over frame pairs
          f2 v = f2{wk[0], wk[0]} * zp[0][q];
#pragma unroll
          for (int k = 1; k < FU_CD; ++k) v = __builtin_elementwise_fma(f2{wk[k], wk[k]}, zp[k][q], v);
          const float bj = bo_s[ct + 256 * j];
          v = v + f2{bj, bj};
          r[j][2 * q] = r[j][2 * q] - v.x;
          r[j][2 * q + 1] = r[j][2 * q + 1] - v.y;
          zacc[j][2 * q] = zacc[j][2 * q] + v.x * mf[2 * q];
          zacc[j][2 * q + 1] = zacc[j][2 * q + 1] + v.y * mf[2 * q + 1];
          trow[2 * q] = v.x;
          trow[2 * q + 1] = v.y;
        }
      }
    }
    FSTAMP(7);
  }
  lds_barrier();
  if (a.z_q_is) store_tile(a.z_q_is + ((size_t)b * nq + (nq - 1)) * FU_D * T, a.nt_store != 0);
  lds_barrier();
#pragma unroll
  for (int j = 0; j < FU_CPT; ++j)
#pragma unroll
    for (int f = 0; f < FU_FPG; ++f) tile[(ct + 256 * j) * FU_TS + g * FU_FPG + f] = zacc[j][f];
  lds_barrier();
  store_tile(a.z_q + (size_t)b * FU_D * T, false);  // re-read by the decoder
}

static int rvq_nt_store() {  // tuning override: VRVQ_RVQ_NT=0 (plain stores) | 1 (non-temporal)
  static const int v = [] {
    const char* e = getenv("VRVQ_RVQ_NT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

}  // namespace

extern "C" int vrvq_rvq_fused(const float* z, int batch, int dim, int frames, int nq, int ncode,
                              int cdim, const float* w_in_t, const float* b_in, const float* cb,
                              const float* cbn, const float* c2, const float* w_out,
                              const float* b_out, const float* imp, float level, int64_t* codes,
                              float* latents, float* loss_pf, float* z_q_is, float* z_q,
                              float* mask, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z && w_in_t && b_in && cb && cbn && c2 && w_out && b_out && codes && latents &&
                 loss_pf && z_q);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  VRVQ_CHECK_ARG((long long)frames * FU_D < 0x7fffffffLL);  // 32-bit per-row offsets
  if (dim != FU_D || cdim != FU_CD || ncode <= 0 || ncode % 256 != 0 || ncode > 1024)
    return VRVQ_ERR_UNSUPPORTED;
  FusedArgs a{};
  a.z = z; a.B = batch; a.T = frames; a.nq = nq;
  a.w_in_t = w_in_t; a.b_in = b_in; a.cb = cb; a.cbn = cbn; a.c2 = c2;
  a.w_out = w_out; a.b_out = b_out; a.imp = imp; a.level = level;
  a.codes = codes; a.latents = latents; a.loss_pf = loss_pf;
  a.z_q_is = z_q_is; a.z_q = z_q; a.mask = mask;
  a.nr = (frames + FU_F - 1) / FU_F;
  const long long units = (long long)batch * a.nr;
  VRVQ_CHECK_ARG(units * 8 < 0x7fffffffLL);
  a.units = (int)units;
  a.per_xcd = (int)((units + 7) / 8);
  a.stamps = vrvq_g_stamps;
  a.nt_store = rvq_nt_store();
  const dim3 grid((unsigned)(8 * a.per_xcd));
  hipStream_t st = as_stream(stream);
  switch (ncode / 256) {
    case 1: hipLaunchKernelGGL(rvq_fused_kernel<1>, grid, dim3(FU_NT), 0, st, a); break;
    case 2: hipLaunchKernelGGL(rvq_fused_kernel<2>, grid, dim3(FU_NT), 0, st, a); break;
    case 3: hipLaunchKernelGGL(rvq_fused_kernel<3>, grid, dim3(FU_NT), 0, st, a); break;
    default: hipLaunchKernelGGL(rvq_fused_kernel<4>, grid, dim3(FU_NT), 0, st, a); break;
  }
  return vrvq_launch_status();
}
