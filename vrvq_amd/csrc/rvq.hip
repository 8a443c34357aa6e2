// Residual vector quantisation for gfx950: VBRResidualVectorQuantize.forward
// (models/quantize.py:328-443) split into two launches.
//
//  vrvq_rvq_codes  — the sequential residual chain (in_proj, L2-normalise, cosine-NN argmin
//                    over the codebook, straight-through vector, out_proj, residual update)
//                    for all nq stages in one launch. One workgroup owns F frames; each
//                    thread owns D/256 latent channels x F frames of the residual in VGPRs,
//                    so every weight / codebook value it loads is reused F times from a
//                    register. Weights stream from L2 with coalesced float4 loads.
//  vrvq_rvq_expand — pure HBM streaming: recomputes z_q_is = out_proj(zst) (bit-identical
//                    expression to the chain's), applies the importance mask and writes
//                    z_q_is / z_q / mask as contiguous float4 rows. This is where ~95 % of the
//                    algorithmic bytes go (nq*D*4 B per frame).
#include "common.h"
#include "lanes.h"
#include <stdlib.h>

namespace {

constexpr int RVQ_THREADS = 256;
constexpr int RVQ_D = 1024;     // latent channels (all conf/*.yml)
constexpr int RVQ_CPT = RVQ_D / RVQ_THREADS;
constexpr int RVQ_CD = 8;       // codebook_dim

struct CodesArgs {
  const float* z;
  int B, T, nq, N;
  const float* w_in_t;  // [nq][D][8]
  const float* b_in;    // [nq][8]
  const float* cb;      // [nq][N][8]
  const float* cbn;     // [nq][N][8]
  const float* c2;      // [nq][N]
  const float* w_out;   // [nq][D][8]
  const float* b_out;   // [nq][D]
  int64_t* codes;       // [B][nq][T]
  float* latents;       // [B][nq*8][T]
  float* loss_pf;       // [B][nq][T]
  float* zst;           // [B][nq][T][8]
  unsigned long long* stamps;  // diagnostic build only (-DVRVQ_STAMPS): [blocks][nq][8]
};

#ifdef VRVQ_STAMPS
#define STAMP(step)                                                                   \
  do {                                                                                \
    if (a.stamps && threadIdx.x == 0) {                                               \
      unsigned long long t_;                                                          \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
      a.stamps[((size_t)blockIdx.x * a.nq + i) * 8 + (step)] = t_;                   \
    }                                                                                 \
  } while (0)
#else
#define STAMP(step) do {} while (0)
#endif

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Workgroup = FG frame groups x 4 frames (FG * 256 threads; FG is chosen so that there is about
// one workgroup per CU). Thread (g, t) owns latent channels c = t + 256 j (j < 4) of the 4
// frames of group g: 16 residual VGPRs, and every weight it reads is reused 4 times from a
// register. Stage weights (normalised codebook, c2, W_out, b_out: 72 KB; raw codebook 32 KB,
// double-buffered) are copied to LDS by LDS-DMA, each buffer re-issued for the next stage right
// after its last read, so the copies land during the rest of the stage; W_in comes through
// registers, prefetched one stage ahead. Two workgroup barriers per stage:
//   in_proj (packed FMA) -> wave reduce-scatter (permlane/DPP) -> [A] ->
//   every wave: z_e, L2-normalise, distance scan over its codes n = t + 256 m, argmin
//   reduce-scatter -> [B] -> every wave: final argmin, codeword, loss, straight-through vector,
//   out_proj + residual update.
// Wave-uniform vectors (e, zst of the group's frames) are broadcast through a per-wave LDS slot.
constexpr int RVQ_FPG = 4;  // frames per group
typedef float f2 __attribute__((ext_vector_type(2)));

// LDS-DMA of `nchunks` 1-KiB chunks src -> dst, chunk q issued by wave q % nwaves.
__device__ __forceinline__ void dma_chunks(const float* src, float* dst, int nchunks, int wave,
                                           int nwaves, int lane) {
  for (int q = wave; q < nchunks; q += nwaves)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + q * 256 + lane * 4),
        (__attribute__((address_space(3))) void*)(dst + q * 256), 16, 0, 0);
}

template <int FG, int NM>
__global__ __launch_bounds__(RVQ_THREADS * FG) void rvq_codes_kernel(CodesArgs a) {
  // NM = codes per thread = N / 256 (compile-time: the scan below is branch-free)
  constexpr int F = FG * RVQ_FPG;          // frames per workgroup
  constexpr int NTH = RVQ_THREADS * FG;
  constexpr int NW = NTH / 64;             // waves
  constexpr int N = NM * RVQ_THREADS;      // codebook size
  // LDS (floats). Small arrays first (immediate ds offsets stay < 64 KiB):
  //   red [FG][4][32] | db, ib [FG][4][4] | wv [NW][40] per-wave broadcast slot
  //   cbn [N][8] | c2 [N] | wo [D][8] | bo [D] | raw [2][N][8]
  constexpr int SMALL = FG * 128 + 2 * FG * 16 + NW * 40;
  constexpr int BIG = N * RVQ_CD + N + RVQ_D * RVQ_CD + RVQ_D + 2 * N * RVQ_CD;
  static_assert(BIG >= RVQ_D * F, "residual transpose fits the weight area");
  __shared__ __attribute__((aligned(16))) float smem[SMALL + BIG];
  float* red = smem;
  float* db = red + FG * 128;
  int* ib = reinterpret_cast<int*>(db + FG * 16);
  float* wv_all = reinterpret_cast<float*>(ib + FG * 16);
  float* big = smem + SMALL;
  float* cbn_s = big;
  float* c2_s = cbn_s + N * RVQ_CD;
  float* wo_s = c2_s + N;
  float* bo_s = wo_s + RVQ_D * RVQ_CD;
  float* raw_s = bo_s + RVQ_D;  // [2][N][8]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = wave >> 2;             // frame group
  const int wg = wave & 3;             // wave inside the group
  const int ct = tid & (RVQ_THREADS - 1);
  const int NF = a.B * a.T;
  const int n0 = blockIdx.x * F;
  float* wv = wv_all + wave * 40;      // this wave's broadcast slot: [32] vector + [4] extra

  // ---- residual tile z[b, :, t] through LDS (lanes frame-fastest) ----
  {
    const int f = tid % F;
    const int n = n0 + f;
    const bool valid = n < NF;
    const int b = valid ? n / a.T : 0;
    const int t = valid ? n - b * a.T : 0;
    const float* zb = a.z + (size_t)b * RVQ_D * a.T + t;
    for (int c = tid / F; c < RVQ_D; c += NTH / F)
      big[c * F + f] = valid ? zb[(size_t)c * a.T] : 0.0f;
  }
  __syncthreads();
  float r[RVQ_CPT][RVQ_FPG];
#pragma unroll
  for (int j = 0; j < RVQ_CPT; ++j)
#pragma unroll
    for (int f = 0; f < RVQ_FPG; ++f) r[j][f] = big[(ct + RVQ_THREADS * j) * F + g * RVQ_FPG + f];
  __syncthreads();  // the transpose area becomes the weight buffers

  // stage-0 codebooks (W_out / b_out are fetched inside the stage, after barrier A)
  dma_chunks(a.cbn, cbn_s, N * RVQ_CD / 256, wave, NW, lane);
  dma_chunks(a.c2, c2_s, N / 256, wave, NW, lane);
  dma_chunks(a.cb, raw_s, N * RVQ_CD / 256, wave, NW, lane);

  // per-lane frame/k of the (frame, k) epilogue: lanes l and l^32 mirror each other
  const int ef = (lane >> 3) & 3, ek = lane & 7;
  const int en = n0 + g * RVQ_FPG + ef;
  const bool estore = (wg == 0) && (lane < 32) && en < NF;
  const int eb = en < NF ? en / a.T : 0;
  const int et = en < NF ? en - eb * a.T : 0;

  float4 wi[RVQ_CPT][2];
#pragma unroll
  for (int j = 0; j < RVQ_CPT; ++j) {
    const float* wp = a.w_in_t + (size_t)(ct + RVQ_THREADS * j) * RVQ_CD;
    wi[j][0] = ld4(wp);
    wi[j][1] = ld4(wp + 4);
  }

  for (int i = 0; i < a.nq; ++i) {
    const bool more = i + 1 < a.nq;
    STAMP(0);
    // (1) in_proj partials p[f*8 + k] = sum_j W_in[k, c_j] r[c_j, f]  (v_pk_fma_f32 over k pairs)
    float p[32];
    {
      f2 pp[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) pp[q] = f2{0.0f, 0.0f};
#pragma unroll
      for (int j = 0; j < RVQ_CPT; ++j) {
        const f2 w01 = {wi[j][0].x, wi[j][0].y}, w23 = {wi[j][0].z, wi[j][0].w};
        const f2 w45 = {wi[j][1].x, wi[j][1].y}, w67 = {wi[j][1].z, wi[j][1].w};
#pragma unroll
        for (int f = 0; f < RVQ_FPG; ++f) {
          const f2 rr = {r[j][f], r[j][f]};
          pp[f * 4 + 0] = __builtin_elementwise_fma(w01, rr, pp[f * 4 + 0]);
          pp[f * 4 + 1] = __builtin_elementwise_fma(w23, rr, pp[f * 4 + 1]);
          pp[f * 4 + 2] = __builtin_elementwise_fma(w45, rr, pp[f * 4 + 2]);
          pp[f * 4 + 3] = __builtin_elementwise_fma(w67, rr, pp[f * 4 + 3]);
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        p[2 * q] = pp[q].x;
        p[2 * q + 1] = pp[q].y;
      }
    }
    STAMP(1);
    // (2) wave reduce-scatter: lanes l, l^32 <- wave sum of p[l & 31]
    {
      const float v = vrvq::reduce_scatter32(p, lane);
      if (lane < 32) red[(g * 4 + wg) * 32 + lane] = v;
    }
    const float bin = a.b_in[i * RVQ_CD + ek];
    STAMP(2);
    // this stage's codebook LDS-DMA (issued after barrier B of the previous stage) landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // ---------------------------------------------------------------- A
    STAMP(3);
    // this stage's W_out / b_out (the buffer's last reads, out_proj of stage i-1, precede A)
    dma_chunks(a.w_out + (size_t)i * RVQ_D * RVQ_CD, wo_s, RVQ_D * RVQ_CD / 256, wave, NW, lane);
    dma_chunks(a.b_out + (size_t)i * RVQ_D, bo_s, RVQ_D / 256, wave, NW, lane);
    if (more) {  // next stage's W_in into registers
#pragma unroll
      for (int j = 0; j < RVQ_CPT; ++j) {
        const float* wp = a.w_in_t + ((size_t)(i + 1) * RVQ_D + ct + RVQ_THREADS * j) * RVQ_CD;
        wi[j][0] = ld4(wp);
        wi[j][1] = ld4(wp + 4);
      }
    }
    // (3) z_e and its L2 normalisation, computed by every wave for its group's frames
    //     (lane = f*8 + k; lanes 32..63 mirror 0..31)
    float ze, e, e2;
    {
      const float* rr = red + g * 128 + (lane & 31);
      ze = ((rr[0] + rr[32]) + (rr[64] + rr[96])) + bin;
      const float n2 = vrvq::sum8(ze * ze, lane);
      e = ze / fmaxf(sqrtf(n2), 1e-12f);
      e2 = vrvq::sum8(e * e, lane);
      if (estore) a.latents[((size_t)eb * a.nq * RVQ_CD + i * RVQ_CD + ek) * a.T + et] = ze;
    }
    // broadcast e (k-major, frames interleaved) and e2 through this wave's LDS slot
    if (lane < 32) wv[ek * RVQ_FPG + ef] = e;
    if (lane < 32 && ek == 0) wv[32 + ef] = e2;
    STAMP(4);
    // (4) nearest codeword over this thread's codes (lowest index on ties)
    float best[RVQ_FPG];
    int bidx[RVQ_FPG];
    {
      f2 e01[RVQ_CD], e23[RVQ_CD];
#pragma unroll
      for (int k = 0; k < RVQ_CD; ++k) {
        const float4 ek4 = *reinterpret_cast<const float4*>(wv + k * RVQ_FPG);
        e01[k] = f2{ek4.x, ek4.y};
        e23[k] = f2{ek4.z, ek4.w};
      }
      const float4 e2v = *reinterpret_cast<const float4*>(wv + 32);
      const f2 e2a = {e2v.x, e2v.y}, e2b = {e2v.z, e2v.w};
#pragma unroll
      for (int f = 0; f < RVQ_FPG; ++f) {
        best[f] = INFINITY;
        bidx[f] = 0x7fffffff;
      }
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int n = ct + RVQ_THREADS * m;
        const float4 c0 = *reinterpret_cast<const float4*>(cbn_s + n * RVQ_CD);
        const float4 c1 = *reinterpret_cast<const float4*>(cbn_s + n * RVQ_CD + 4);
        const float ck[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        // dot in k order (mul, then fma chain): bit-identical to dot8 per frame
        f2 da = e01[0] * f2{ck[0], ck[0]}, dbb = e23[0] * f2{ck[0], ck[0]};
#pragma unroll
        for (int k = 1; k < RVQ_CD; ++k) {
          da = __builtin_elementwise_fma(e01[k], f2{ck[k], ck[k]}, da);
          dbb = __builtin_elementwise_fma(e23[k], f2{ck[k], ck[k]}, dbb);
        }
        // (sum e^2 - 2 e.c) + sum c^2   (models/quantize.py:96-100)
        const float cc = c2_s[n];
        const f2 dA = (e2a - 2.0f * da) + f2{cc, cc};
        const f2 dB = (e2b - 2.0f * dbb) + f2{cc, cc};
        const float dv[4] = {dA.x, dA.y, dB.x, dB.y};
#pragma unroll
        for (int f = 0; f < RVQ_FPG; ++f) {
          const bool take = dv[f] < best[f];  // n increasing: strict < keeps the first
          best[f] = take ? dv[f] : best[f];
          bidx[f] = take ? n : bidx[f];
        }
      }
    }
    vrvq::argmin_scatter4(best, bidx, lane);
    if ((lane & 15) == 0) {
      db[(g * 4 + wg) * 4 + (lane >> 4)] = best[0];
      ib[(g * 4 + wg) * 4 + (lane >> 4)] = bidx[0];
    }
    STAMP(5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // W_out / b_out DMA (issued after A) landed
    __syncthreads();  // ---------------------------------------------------------------- B
    STAMP(6);
    if (more) {  // next stage's cbn / c2 / raw codebook (this stage's cbn / c2 reads are done;
                 // the other raw buffer was last read a stage ago)
      dma_chunks(a.cbn + (size_t)(i + 1) * N * RVQ_CD, cbn_s, N * RVQ_CD / 256, wave, NW, lane);
      dma_chunks(a.c2 + (size_t)(i + 1) * N, c2_s, N / 256, wave, NW, lane);
      dma_chunks(a.cb + (size_t)(i + 1) * N * RVQ_CD, raw_s + ((i + 1) & 1) * N * RVQ_CD,
                 N * RVQ_CD / 256, wave, NW, lane);
    }
    // (5) final argmin, codeword, per-frame loss, straight-through vector (every wave)
    {
      float bd = db[(g * 4) * 4 + ef];
      int bi = ib[(g * 4) * 4 + ef];
#pragma unroll
      for (int w = 1; w < 4; ++w) vrvq::amin(bd, bi, db[(g * 4 + w) * 4 + ef], ib[(g * 4 + w) * 4 + ef]);
      const float zq = raw_s[(i & 1) * N * RVQ_CD + bi * RVQ_CD + ek];
      const float st = ze + (zq - ze);  // z_e + (z_q - z_e).detach(), models/quantize.py:73-75
      if (lane < 32) wv[ek * RVQ_FPG + ef] = st;
      if (wg == 0) {
        const float diff = ze - zq;
        const float l2 = vrvq::sum8(diff * diff, lane);
        if (estore) {
          const size_t fo = ((size_t)eb * a.nq + i) * a.T + et;
          a.zst[fo * RVQ_CD + ek] = st;
          if (ek == 0) {
            a.codes[fo] = (int64_t)bi;
            a.loss_pf[fo] = l2 / 8.0f;
          }
        }
      }
    }
    STAMP(7);
    // (6) out_proj + residual update: r[c, f] -= W_out[c, :] . zst[f] + b_out[c]
    {
      float4 wo[RVQ_CPT][2];
      float bo[RVQ_CPT];
#pragma unroll
      for (int j = 0; j < RVQ_CPT; ++j) {
        const int c = ct + RVQ_THREADS * j;
        wo[j][0] = *reinterpret_cast<const float4*>(wo_s + c * RVQ_CD);
        wo[j][1] = *reinterpret_cast<const float4*>(wo_s + c * RVQ_CD + 4);
        bo[j] = bo_s[c];
      }
      f2 z01[RVQ_CD], z23[RVQ_CD];
#pragma unroll
      for (int k = 0; k < RVQ_CD; ++k) {
        const float4 zk = *reinterpret_cast<const float4*>(wv + k * RVQ_FPG);
        z01[k] = f2{zk.x, zk.y};
        z23[k] = f2{zk.z, zk.w};
      }
#pragma unroll
      for (int j = 0; j < RVQ_CPT; ++j) {
        const float wk[8] = {wo[j][0].x, wo[j][0].y, wo[j][0].z, wo[j][0].w,
                             wo[j][1].x, wo[j][1].y, wo[j][1].z, wo[j][1].w};
        // out_proj1 per frame: (w0*z0, fma chain over k) + bias -- packed over frame pairs
        f2 qa = f2{wk[0], wk[0]} * z01[0], qb = f2{wk[0], wk[0]} * z23[0];
#pragma unroll
        for (int k = 1; k < RVQ_CD; ++k) {
          qa = __builtin_elementwise_fma(f2{wk[k], wk[k]}, z01[k], qa);
          qb = __builtin_elementwise_fma(f2{wk[k], wk[k]}, z23[k], qb);
        }
        qa = qa + f2{bo[j], bo[j]};
        qb = qb + f2{bo[j], bo[j]};
        r[j][0] = r[j][0] - qa.x;
        r[j][1] = r[j][1] - qa.y;
        r[j][2] = r[j][2] - qb.x;
        r[j][3] = r[j][3] - qb.y;
      }
    }
    // LDS hazards: red (written before A of the next stage) was last read before B here; db/ib
    // (written before B) were last read before A; wv is wave-private.
  }
}

// ------------------------------------------------------------------------------------------
// Expansion: lane = frame (flattened b*T + t, 256 per workgroup), workgroup also owns CB
// latent channels. For each stage the lane loads its frame's 8-float straight-through vector
// once; each channel's W_out row is wave-uniform and comes through the scalar cache. Every
// store instruction writes 64 consecutive frames of one channel row (256 B), so the z_q_is
// stream is written at full coalescing; z_q accumulates the masked sum in registers in stage
// order (models/quantize.py:420-421).
struct ExpandArgs {
  const float* zst;     // [B][nq][T][8]
  int B, D, T, nq;
  const float* w_out;   // [nq][D][8]
  const float* b_out;   // [nq][D]
  const float* imp;     // [B][T] or null (CBR: mask = 1)
  float level;
  float* z_q_is;        // [B][nq][D][T] or null
  float* z_q;           // [B][D][T]
  float* mask;          // [B][nq][T] or null
  int n_cc;             // channel chunks
};

constexpr int EXP_THREADS = 256;
constexpr int EXP_CB = 16;  // channels per workgroup

__global__ __launch_bounds__(EXP_THREADS) void rvq_expand_kernel(
    ExpandArgs a, const float* __restrict__ zst_g, const float* __restrict__ w_out,
    const float* __restrict__ b_out, const float* __restrict__ imp_g, float* __restrict__ z_q_is,
    float* __restrict__ z_q, float* __restrict__ mask) {
  // All pointers are distinct buffers (restrict): lets the compiler keep the wave-uniform
  // weight loads on the scalar path ahead of the stores.
  const int cc = blockIdx.x % a.n_cc;
  const int fc = blockIdx.x / a.n_cc;
  const int c0 = cc * EXP_CB;
  const int NF = a.B * a.T;
  const int n = fc * EXP_THREADS + threadIdx.x;
  const bool valid = n < NF;
  const int b = valid ? n / a.T : 0;
  const int t = valid ? n - b * a.T : 0;
  const float s = (imp_g && valid) ? (imp_g[n] * a.level) * (float)a.nq : INFINITY;

  // This workgroup's W_out rows / biases for every stage: [nq][CB][8] then [nq][CB].
  extern __shared__ __attribute__((aligned(16))) float w_s[];
  for (int e = threadIdx.x; e < a.nq * EXP_CB * 2; e += EXP_THREADS) {
    const int i = e / (EXP_CB * 2), r = e - i * (EXP_CB * 2);
    reinterpret_cast<float4*>(w_s)[e] =
        *reinterpret_cast<const float4*>(w_out + ((size_t)i * a.D + c0) * RVQ_CD + r * 4);
  }
  for (int e = threadIdx.x; e < a.nq * EXP_CB; e += EXP_THREADS) {
    const int i = e / EXP_CB, q = e - i * EXP_CB;
    w_s[a.nq * EXP_CB * RVQ_CD + e] = b_out[(size_t)i * a.D + c0 + q];
  }
  __syncthreads();

  float acc[EXP_CB];
#pragma unroll
  for (int q = 0; q < EXP_CB; ++q) acc[q] = 0.0f;

  for (int i = 0; i < a.nq; ++i) {
    float4 z0 = make_float4(0.f, 0.f, 0.f, 0.f), z1 = z0;
    if (valid) {
      const float* zp = zst_g + (((size_t)b * a.nq + i) * a.T + t) * RVQ_CD;
      z0 = ld4(zp);
      z1 = ld4(zp + 4);
    }
    const float m = (s - (float)i >= 0.0f) ? 1.0f : 0.0f;  // models/utils.py:45-61
    if (mask && cc == 0 && valid) mask[((size_t)b * a.nq + i) * a.T + t] = m;
    float* dst = z_q_is ? z_q_is + (((size_t)b * a.nq + i) * a.D + c0) * a.T + t : nullptr;
    // Wave-uniform weight rows: LDS broadcast reads.
    const float* wrow = w_s + i * EXP_CB * RVQ_CD;
    const float* brow = w_s + a.nq * EXP_CB * RVQ_CD + i * EXP_CB;
    float v[EXP_CB];
#pragma unroll
    for (int q = 0; q < EXP_CB; ++q) {
      const float4 w0 = *reinterpret_cast<const float4*>(wrow + q * RVQ_CD);
      const float4 w1 = *reinterpret_cast<const float4*>(wrow + q * RVQ_CD + 4);
      v[q] = out_proj1(w0, w1, brow[q], z0, z1);
      acc[q] = acc[q] + v[q] * m;
    }
    if (dst && valid) {
#pragma unroll
      for (int q = 0; q < EXP_CB; ++q) dst[(size_t)q * a.T] = v[q];
    }
  }
  if (valid) {
    float* zq = z_q + ((size_t)b * a.D + c0) * a.T + t;
#pragma unroll
    for (int q = 0; q < EXP_CB; ++q) zq[(size_t)q * a.T] = acc[q];
  }
}

}  // namespace

unsigned long long* vrvq_g_stamps = nullptr;  // shared with rvq_fused.hip (common.h)

// Diagnostic hook (stamped builds only): per-block per-stage s_memtime stamps of the codes kernel.
extern "C" int vrvq_debug_set_stamps(unsigned long long* buf) {
  vrvq_g_stamps = buf;
  return 0;
}

extern "C" int vrvq_rvq_codes(const float* z, int batch, int dim, int frames, int nq, int ncode,
                              int cdim, const float* w_in_t, const float* b_in, const float* cb,
                              const float* cbn, const float* c2, const float* w_out,
                              const float* b_out, int64_t* codes, float* latents,
                              float* loss_pf, float* zst, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z && w_in_t && b_in && cb && cbn && c2 && w_out && b_out && codes && latents &&
                 loss_pf && zst);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  if (dim != RVQ_D || cdim != RVQ_CD || ncode <= 0 || ncode % RVQ_THREADS != 0 ||
      ncode > 1024)
    return VRVQ_ERR_UNSUPPORTED;
  CodesArgs a{z, batch, frames, nq, ncode, w_in_t, b_in, cb, cbn, c2, w_out, b_out,
              codes, latents, loss_pf, zst, vrvq_g_stamps};
  // Frame groups per workgroup: aim at one workgroup per CU (256 CUs), at most 3 groups
  // (768 threads, 3 waves/SIMD).
  const long long nf = (long long)batch * frames;
  int fg = (int)((nf + RVQ_FPG * 256 - 1) / (RVQ_FPG * 256));
  fg = fg < 1 ? 1 : (fg > 3 ? 3 : fg);
  static const int fg_env = [] {  // tuning override: VRVQ_RVQ_FG=1|2|3
    const char* e = getenv("VRVQ_RVQ_FG");
    return e ? atoi(e) : 0;
  }();
  if (fg_env >= 1 && fg_env <= 3) fg = fg_env;
  const long long nblk = (nf + fg * RVQ_FPG - 1) / (fg * RVQ_FPG);
  VRVQ_CHECK_ARG(nblk < 0x7fffffffLL);
  hipStream_t st = as_stream(stream);
  const int nm = ncode / RVQ_THREADS;
#define VRVQ_CODES_LAUNCH(FGV, NMV) \
  hipLaunchKernelGGL((rvq_codes_kernel<FGV, NMV>), dim3((unsigned)nblk), dim3(RVQ_THREADS * FGV), 0, st, a)
#define VRVQ_CODES_NM(FGV)                      \
  switch (nm) {                                 \
    case 1: VRVQ_CODES_LAUNCH(FGV, 1); break;   \
    case 2: VRVQ_CODES_LAUNCH(FGV, 2); break;   \
    case 3: VRVQ_CODES_LAUNCH(FGV, 3); break;   \
    default: VRVQ_CODES_LAUNCH(FGV, 4); break;  \
  }
  if (fg == 1) { VRVQ_CODES_NM(1) }
  else if (fg == 2) { VRVQ_CODES_NM(2) }
  else { VRVQ_CODES_NM(3) }
#undef VRVQ_CODES_NM
#undef VRVQ_CODES_LAUNCH
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_expand(const float* zst, int batch, int dim, int frames, int nq, int cdim,
                               const float* w_out, const float* b_out, const float* imp,
                               float level, float* z_q_is, float* z_q, float* mask,
                               vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(zst && w_out && b_out && z_q);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0 && dim > 0);
  if (cdim != RVQ_CD || dim % EXP_CB != 0) return VRVQ_ERR_UNSUPPORTED;
  ExpandArgs a{zst, batch, dim, frames, nq, w_out, b_out, imp, level, z_q_is, z_q, mask,
               dim / EXP_CB};
  const long long nf = (long long)batch * frames;
  const long long nblk = (nf + EXP_THREADS - 1) / EXP_THREADS * a.n_cc;
  VRVQ_CHECK_ARG(nblk < 0x7fffffffLL);
  const size_t lds = (size_t)nq * EXP_CB * (RVQ_CD + 1) * sizeof(float);
  if (lds > 64 * 1024) return VRVQ_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(rvq_expand_kernel, dim3((unsigned)nblk), dim3(EXP_THREADS), lds,
                     as_stream(stream), a, zst, w_out, b_out, imp, z_q_is, z_q, mask);
  return vrvq_launch_status();
}
