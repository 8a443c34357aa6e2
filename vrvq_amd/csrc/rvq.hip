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
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Wave-wide reduce-scatter of 64 per-lane values: afterwards lane l holds sum over all 64
// lanes of v[l]. 63 shuffles + adds instead of 64 * 6 for a plain butterfly per value.
__device__ __forceinline__ float wave_reduce_scatter64(float (&v)[64], int lane) {
#pragma unroll
  for (int h = 32; h >= 1; h >>= 1) {
    // Value selects via bit masks: a plain `up ? v[a] : v[b]` is folded by the optimiser
    // into a dynamically indexed load, which sends the whole array to scratch memory.
    const unsigned m = (lane & h) ? 0xffffffffu : 0u;
#pragma unroll
    for (int q = 0; q < h; ++q) {
      const unsigned lo = __float_as_uint(v[q]), hi = __float_as_uint(v[q + h]);
      const float keep = __uint_as_float((lo & ~m) | (hi & m));
      const float send = __uint_as_float((hi & ~m) | (lo & m));
      v[q] = keep + __shfl_xor(send, h);
    }
  }
  return v[0];
}

template <int F>
__global__ __launch_bounds__(RVQ_THREADS) void rvq_codes_kernel(CodesArgs a) {
  static_assert(F * RVQ_CD == 64, "reduce-scatter maps (frame, k) onto the 64 lanes");
  __shared__ __attribute__((aligned(16))) float zs[RVQ_D * F];        // residual load transpose
  __shared__ float red[4][64];
  __shared__ __attribute__((aligned(16))) float e_s[F][RVQ_CD];
  __shared__ float e2_s[F];
  __shared__ float dbest[4][F];
  __shared__ int ibest[4][F];
  __shared__ __attribute__((aligned(16))) float zst_s[F][RVQ_CD];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NF = a.B * a.T;
  const int n0 = blockIdx.x * F;

  // ---- load the residual tile z[b, :, t] for the block's frames through LDS ----
  // Each lane reads one (channel, frame): lanes f-fastest -> F contiguous floats per row.
  {
    const int f = tid % F;
    const int n = n0 + f;
    const bool valid = n < NF;
    const int b = valid ? n / a.T : 0;
    const int t = valid ? n - b * a.T : 0;
    const float* zb = a.z + (size_t)b * RVQ_D * a.T + t;
    for (int c = tid / F; c < RVQ_D; c += RVQ_THREADS / F)
      zs[c * F + f] = valid ? zb[(size_t)c * a.T] : 0.0f;
  }
  __syncthreads();
  float r[RVQ_CPT][F];
#pragma unroll
  for (int j = 0; j < RVQ_CPT; ++j)
#pragma unroll
    for (int f = 0; f < F; ++f) r[j][f] = zs[(tid + RVQ_THREADS * j) * F + f];

  // Frame owned by lane (frame-stage epilogue runs on wave 0: lane = f*8 + k).
  const int ef = lane >> 3, ek = lane & 7;
  const int en = n0 + ef;
  const bool evalid = en < NF;
  const int eb = evalid ? en / a.T : 0;
  const int et = evalid ? en - eb * a.T : 0;

  for (int i = 0; i < a.nq; ++i) {
    // ---- in_proj partials: p[f][k] = sum_j W_in[k, c_j] * r[c_j, f] ----
    float p[64];
#pragma unroll
    for (int q = 0; q < 64; ++q) p[q] = 0.0f;
#pragma unroll
    for (int j = 0; j < RVQ_CPT; ++j) {
      const float* wp = a.w_in_t + ((size_t)i * RVQ_D + tid + RVQ_THREADS * j) * RVQ_CD;
      const float4 w0 = ld4(wp), w1 = ld4(wp + 4);
      const float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int f = 0; f < F; ++f)
#pragma unroll
        for (int k = 0; k < RVQ_CD; ++k) p[f * RVQ_CD + k] = fmaf(wk[k], r[j][f], p[f * RVQ_CD + k]);
    }
    red[wave][lane] = wave_reduce_scatter64(p, lane);
    __syncthreads();

    // ---- z_e, L2 normalisation (wave 0; lane = f*8 + k) ----
    float ze = 0.0f;
    if (wave == 0) {
      ze = ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) + a.b_in[i * RVQ_CD + ek];
      float n2 = ze * ze;
      n2 += __shfl_xor(n2, 1);
      n2 += __shfl_xor(n2, 2);
      n2 += __shfl_xor(n2, 4);
      const float e = ze / fmaxf(sqrtf(n2), 1e-12f);
      float e2 = e * e;
      e2 += __shfl_xor(e2, 1);
      e2 += __shfl_xor(e2, 2);
      e2 += __shfl_xor(e2, 4);
      e_s[ef][ek] = e;
      if (ek == 0) e2_s[ef] = e2;
      if (evalid)
        a.latents[((size_t)eb * a.nq * RVQ_CD + i * RVQ_CD + ek) * a.T + et] = ze;
    }
    __syncthreads();

    // ---- nearest codeword: thread scans n = tid + 256*m (increasing) ----
    float best[F];
    int bidx[F];
#pragma unroll
    for (int f = 0; f < F; ++f) {
      best[f] = INFINITY;
      bidx[f] = 0x7fffffff;
    }
    for (int n = tid; n < a.N; n += RVQ_THREADS) {
      const float* cp = a.cbn + ((size_t)i * a.N + n) * RVQ_CD;
      const float4 c0 = ld4(cp), c1 = ld4(cp + 4);
      const float cc2 = a.c2[(size_t)i * a.N + n];
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const float4 e0 = *reinterpret_cast<const float4*>(&e_s[f][0]);
        const float4 e1 = *reinterpret_cast<const float4*>(&e_s[f][4]);
        // (sum e^2 - 2 e.c) + sum c^2, models/quantize.py:96-100
        const float d = (e2_s[f] - 2.0f * dot8(e0, e1, c0, c1)) + cc2;
        if (d < best[f]) {
          best[f] = d;
          bidx[f] = n;
        }
      }
    }
    // wave argmin (lowest index on ties: torch max(1) first-occurrence semantics)
#pragma unroll
    for (int f = 0; f < F; ++f) {
#pragma unroll
      for (int h = 32; h >= 1; h >>= 1) {
        const float od = __shfl_xor(best[f], h);
        const int oi = __shfl_xor(bidx[f], h);
        if (od < best[f] || (od == best[f] && oi < bidx[f])) {
          best[f] = od;
          bidx[f] = oi;
        }
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int f = 0; f < F; ++f) {
        dbest[wave][f] = best[f];
        ibest[wave][f] = bidx[f];
      }
    }
    __syncthreads();

    // ---- codeword gather, per-frame loss, straight-through vector (wave 0) ----
    if (wave == 0) {
      float bd = dbest[0][ef];
      int bi = ibest[0][ef];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const float od = dbest[w][ef];
        const int oi = ibest[w][ef];
        if (od < bd || (od == bd && oi < bi)) {
          bd = od;
          bi = oi;
        }
      }
      const float zq = a.cb[((size_t)i * a.N + bi) * RVQ_CD + ek];
      const float diff = ze - zq;
      float l2 = diff * diff;
      l2 += __shfl_xor(l2, 1);
      l2 += __shfl_xor(l2, 2);
      l2 += __shfl_xor(l2, 4);
      const float st = ze + (zq - ze);  // z_e + (z_q - z_e).detach(), models/quantize.py:73-75
      zst_s[ef][ek] = st;
      if (evalid) {
        const size_t fo = ((size_t)eb * a.nq + i) * a.T + et;
        a.zst[fo * RVQ_CD + ek] = st;
        if (ek == 0) {
          a.codes[fo] = (int64_t)bi;
          a.loss_pf[fo] = l2 / 8.0f;
        }
      }
    }
    __syncthreads();

    // ---- out_proj + residual update: r[c, f] -= W_out[c, :] . zst[f] + b_out[c] ----
#pragma unroll
    for (int j = 0; j < RVQ_CPT; ++j) {
      const int c = tid + RVQ_THREADS * j;
      const float* wp = a.w_out + ((size_t)i * RVQ_D + c) * RVQ_CD;
      const float4 w0 = ld4(wp), w1 = ld4(wp + 4);
      const float bo = a.b_out[(size_t)i * RVQ_D + c];
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const float4 z0 = *reinterpret_cast<const float4*>(&zst_s[f][0]);
        const float4 z1 = *reinterpret_cast<const float4*>(&zst_s[f][4]);
        r[j][f] = r[j][f] - out_proj1(w0, w1, bo, z0, z1);
      }
    }
    // zst_s / e_s are rewritten only after the next stage's first barrier: no WAR hazard.
  }
}

// ------------------------------------------------------------------------------------------
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
  int CB;               // channels per workgroup
  int n_cb;             // D / CB
};

constexpr int EXP_THREADS = 256;
constexpr int EXP_MAXV = 4;  // float4 outputs per thread per stage (CB*T <= 4096)

__global__ __launch_bounds__(EXP_THREADS) void rvq_expand_kernel(ExpandArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* zq_s = sm;                       // [T][8]
  float* wo_s = zq_s + a.T * RVQ_CD;      // [CB][8]
  float* bo_s = wo_s + a.CB * RVQ_CD;     // [CB]
  float* s_s = bo_s + a.CB;               // [T] scaled importance

  const int b = blockIdx.x / a.n_cb;
  const int c0 = (blockIdx.x - b * a.n_cb) * a.CB;
  const int tid = threadIdx.x;
  const int E4 = a.CB * a.T / 4;

  for (int t = tid; t < a.T; t += EXP_THREADS)
    s_s[t] = a.imp ? (a.imp[(size_t)b * a.T + t] * a.level) * (float)a.nq : INFINITY;

  float4 acc[EXP_MAXV];
#pragma unroll
  for (int v = 0; v < EXP_MAXV; ++v) acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);

  for (int i = 0; i < a.nq; ++i) {
    const float* zsrc = a.zst + ((size_t)b * a.nq + i) * a.T * RVQ_CD;
    for (int q = tid; q < a.T * RVQ_CD / 4; q += EXP_THREADS)
      reinterpret_cast<float4*>(zq_s)[q] = reinterpret_cast<const float4*>(zsrc)[q];
    const float* wsrc = a.w_out + ((size_t)i * a.D + c0) * RVQ_CD;
    for (int q = tid; q < a.CB * RVQ_CD / 4; q += EXP_THREADS)
      reinterpret_cast<float4*>(wo_s)[q] = reinterpret_cast<const float4*>(wsrc)[q];
    for (int q = tid; q < a.CB; q += EXP_THREADS) bo_s[q] = a.b_out[(size_t)i * a.D + c0 + q];
    __syncthreads();

    if (a.mask && c0 == 0) {
      for (int t = tid; t < a.T; t += EXP_THREADS)
        a.mask[((size_t)b * a.nq + i) * a.T + t] = (s_s[t] - (float)i >= 0.0f) ? 1.0f : 0.0f;
    }
    float* dst = a.z_q_is ? a.z_q_is + (((size_t)b * a.nq + i) * a.D + c0) * a.T : nullptr;
#pragma unroll
    for (int v = 0; v < EXP_MAXV; ++v) {
      const int e4 = tid + v * EXP_THREADS;
      if (e4 >= E4) break;
      float out[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = e4 * 4 + q;
        const int cl = e / a.T;
        const int t = e - cl * a.T;
        const float4 w0 = *reinterpret_cast<const float4*>(wo_s + cl * RVQ_CD);
        const float4 w1 = *reinterpret_cast<const float4*>(wo_s + cl * RVQ_CD + 4);
        const float4 z0 = *reinterpret_cast<const float4*>(zq_s + t * RVQ_CD);
        const float4 z1 = *reinterpret_cast<const float4*>(zq_s + t * RVQ_CD + 4);
        const float val = out_proj1(w0, w1, bo_s[cl], z0, z1);
        const float m = (s_s[t] - (float)i >= 0.0f) ? 1.0f : 0.0f;
        out[q] = val;
        // z_q = sum_i z_q_is * mask (models/quantize.py:421), accumulated in stage order
        (&acc[v].x)[q] = (&acc[v].x)[q] + val * m;
      }
      if (dst) {
        reinterpret_cast<float4*>(dst)[e4] = make_float4(out[0], out[1], out[2], out[3]);
      }
    }
    __syncthreads();
  }
  float* zdst = a.z_q + ((size_t)b * a.D + c0) * a.T;
#pragma unroll
  for (int v = 0; v < EXP_MAXV; ++v) {
    const int e4 = tid + v * EXP_THREADS;
    if (e4 >= E4) break;
    reinterpret_cast<float4*>(zdst)[e4] = acc[v];
  }
}

}  // namespace

extern "C" int vrvq_rvq_codes(const float* z, int batch, int dim, int frames, int nq, int ncode,
                              int cdim, const float* w_in_t, const float* b_in, const float* cb,
                              const float* cbn, const float* c2, const float* w_out,
                              const float* b_out, int64_t* codes, float* latents,
                              float* loss_pf, float* zst, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z && w_in_t && b_in && cb && cbn && c2 && w_out && b_out && codes && latents &&
                 loss_pf && zst);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  if (dim != RVQ_D || cdim != RVQ_CD || ncode <= 0 || ncode % RVQ_THREADS != 0)
    return VRVQ_ERR_UNSUPPORTED;
  CodesArgs a{z, batch, frames, nq, ncode, w_in_t, b_in, cb, cbn, c2, w_out, b_out,
              codes, latents, loss_pf, zst};
  constexpr int F = 8;
  const long long nf = (long long)batch * frames;
  const long long nblk = (nf + F - 1) / F;
  VRVQ_CHECK_ARG(nblk < 0x7fffffffLL);
  hipLaunchKernelGGL(rvq_codes_kernel<F>, dim3((unsigned)nblk), dim3(RVQ_THREADS), 0,
                     as_stream(stream), a);
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_expand(const float* zst, int batch, int dim, int frames, int nq, int cdim,
                               const float* w_out, const float* b_out, const float* imp,
                               float level, float* z_q_is, float* z_q, float* mask,
                               vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(zst && w_out && b_out && z_q);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0 && dim > 0);
  if (cdim != RVQ_CD) return VRVQ_ERR_UNSUPPORTED;
  // Channels per workgroup: largest power of two with CB*T <= 4096 (>= 4), dividing D.
  int cb = 4;
  while (cb * 2 <= dim && cb * 2 * frames <= EXP_THREADS * EXP_MAXV * 4) cb *= 2;
  if (cb * frames > EXP_THREADS * EXP_MAXV * 4 || dim % cb != 0) return VRVQ_ERR_UNSUPPORTED;
  ExpandArgs a{zst, batch, dim, frames, nq, w_out, b_out, imp, level, z_q_is, z_q, mask,
               cb, dim / cb};
  const size_t lds = (size_t)(frames * RVQ_CD + cb * RVQ_CD + cb + frames) * sizeof(float);
  if (lds > 64 * 1024) return VRVQ_ERR_UNSUPPORTED;
  const long long nblk = (long long)batch * a.n_cb;
  VRVQ_CHECK_ARG(nblk < 0x7fffffffLL);
  hipLaunchKernelGGL(rvq_expand_kernel, dim3((unsigned)nblk), dim3(EXP_THREADS), lds,
                     as_stream(stream), a);
  return vrvq_launch_status();
}
