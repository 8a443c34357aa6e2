// Residual vector quantisation as projection + 8-dim chain + HBM expansion (gfx950).
//
// VBRResidualVectorQuantize.forward (models/quantize.py:353-365) runs, per frame and stage i,
//   z_e(i) = W_in(i) r_i + b_in(i),   r_i = z - sum_{j<i} (W_out(j) zst_j + b_out(j)),
// i.e. every stage streams both 8x1024 projections past the 1024-dim residual. By linearity
//   z_e(i) = ((P_i + b_in(i)) - Qb_i) - sum_{j<i} M_ij zst_j,
//   P_i = W_in(i) z,  M_ij = W_in(i) W_out(j)  (8x8),  Qb_i = W_in(i) sum_{j<i} b_out(j),
// so the chain needs only the 8-dim P_i (one GEMM over z for all stages), nq(nq-1)/2 tiny 8x8
// matrices and the codebooks: no 1024-dim residual, no per-stage weight stream. z_q_is =
// W_out(i) zst_i + b_out(i) is then a pure HBM stream (vrvq_rvq_expand, rvq.hip), computed with
// the reference's expression. Same fp32 data, different rounding path for z_e only: the codes of
// every golden fixture (nq 8 / 28 / 32, stress sets) are reproduced bit for bit.
//
//   vrvq_rvq_cross_prep  M (stored per source stage j: mcol[j][i][8][8], zero for i <= j) and
//                        Qb — once per weight version (like the weight-norm fold)
//   vrvq_rvq_project     P partials: part[s][n][i*8+k] over 8 channel splits (fp32 packed FMA)
//   vrvq_rvq_chain       the 8-dim chain over all stages: codes, latents (z_e), per-frame
//                        loss, straight-through vectors, importance mask
#include "common.h"
#include "lanes.h"

namespace {

constexpr int CH_D = 1024;        // latent channels
constexpr int CH_CD = 8;          // codebook_dim
constexpr int PJ_SPLIT = 8;       // channel splits of the projection GEMM
constexpr int PJ_CPS = CH_D / PJ_SPLIT;
constexpr int CH_F = 16;          // frame slots per chain workgroup (a unit never straddles clips)
constexpr int CH_NT = 512;        // chain threads: 8 waves (two per SIMD), 2 frames each
constexpr int CH_NW = CH_NT / 64;
constexpr int CH_FPW = CH_F / CH_NW;
constexpr int CH_NQMAX = 32;

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ------------------------------------------------------------------------------------------
// Prep: mcol[j][i][k][m] = sum_c W_in(i)[k][c] W_out(j)[c][m] for i > j (else 0);
//       qb[i][k]        = sum_c W_in(i)[k][c] (sum_{j<i} b_out(j)[c]) (bias sum in stage order).
// One thread per output, fmaf chain over c (prep only; not on the timed path).
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
      const float* wi = w_in_t + (size_t)i * CH_D * CH_CD + k;
      const float* wo = w_out + (size_t)j * CH_D * CH_CD + m;
      for (int c = 0; c < CH_D; ++c) acc = fmaf(wi[c * CH_CD], wo[c * CH_CD], acc);
    }
    mcol[e] = acc;
  } else if (e < nm + nq * CH_CD) {
    const int q = e - nm, i = q / CH_CD, k = q % CH_CD;
    const float* wi = w_in_t + (size_t)i * CH_D * CH_CD + k;
    float acc = 0.0f;
    for (int c = 0; c < CH_D; ++c) {
      float bs = 0.0f;
      for (int j = 0; j < i; ++j) bs = bs + b_out[(size_t)j * CH_D + c];
      acc = fmaf(wi[c * CH_CD], bs, acc);
    }
    qb[q] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// Projection GEMM: part[s][n][r] = sum_{c in split s} W_in_t[r/8][c][r%8] z[b][c][t],
// n = b*T + t, r < R = nq*8. Workgroup = 64 frames x 64 rows (8 stages) x one 128-channel
// split; both operand tiles are staged in LDS first with every load of a thread in flight
// (z rows 256-B coalesced, W_in rows contiguous float4). Then lane = frame, wave = 16 rows
// (8 packed row pairs): per channel one LDS read of x and four broadcast b128 reads of W.
// 64 KiB of LDS: two workgroups per CU.
__global__ __launch_bounds__(256) void rvq_project_kernel(const float* __restrict__ z, int B,
                                                          int T, int nq,
                                                          const float* __restrict__ w_in_t,
                                                          float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float z_s[PJ_CPS * 64];  // [c][frame]
  __shared__ __attribute__((aligned(16))) float w_s[PJ_CPS * 64];  // [c][row]
  const int NF = B * T, R = nq * CH_CD;
  const int ft = blockIdx.x, s = blockIdx.y, rc = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = ft * 64 + lane;
  const bool valid = n < NF;
  const int nc = valid ? n : NF - 1;  // clamped: loads stay unconditional
  const int b = nc / T, t = nc - b * T;
  {
    const float* zp = z + ((size_t)b * CH_D + s * PJ_CPS + wave) * T + t;
    float v[PJ_CPS / 4];
#pragma unroll
    for (int q = 0; q < PJ_CPS / 4; ++q) v[q] = zp[(size_t)(4 * q) * T];
    // W tile: float4 e = tid + 256 q -> stage sl = e / (2*PJ_CPS), channel c, half h
    float4 w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 256 * q;
      const int sl = e / (2 * PJ_CPS), rem = e - sl * (2 * PJ_CPS);
      const int st = rc * 8 + sl;
      w[q] = st < nq ? ld4(w_in_t + ((size_t)st * CH_D + s * PJ_CPS) * CH_CD + rem * 4)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < PJ_CPS / 4; ++q) z_s[(wave + 4 * q) * 64 + lane] = v[q];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 256 * q;
      const int sl = e / (2 * PJ_CPS), rem = e - sl * (2 * PJ_CPS);
      const int c = rem >> 1, h = rem & 1;
      *reinterpret_cast<float4*>(w_s + c * 64 + sl * 8 + h * 4) = w[q];
    }
  }
  __syncthreads();
  const int r0 = rc * 64 + wave * 16;  // this wave's first row (a multiple of 8: 2 stages)
  if (r0 >= R) return;                 // wave-uniform, after the only barrier
  const bool two = r0 + 8 < R;
  f2 acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = f2{0.0f, 0.0f};
#pragma unroll 8
  for (int c = 0; c < PJ_CPS; ++c) {
    const float x = z_s[c * 64 + lane];
    const f2 xx = {x, x};
    const float* wr = w_s + c * 64 + wave * 16;
    const float4 a0 = ld4(wr), a1 = ld4(wr + 4), b0 = ld4(wr + 8), b1 = ld4(wr + 12);
    acc[0] = __builtin_elementwise_fma(f2{a0.x, a0.y}, xx, acc[0]);
    acc[1] = __builtin_elementwise_fma(f2{a0.z, a0.w}, xx, acc[1]);
    acc[2] = __builtin_elementwise_fma(f2{a1.x, a1.y}, xx, acc[2]);
    acc[3] = __builtin_elementwise_fma(f2{a1.z, a1.w}, xx, acc[3]);
    acc[4] = __builtin_elementwise_fma(f2{b0.x, b0.y}, xx, acc[4]);
    acc[5] = __builtin_elementwise_fma(f2{b0.z, b0.w}, xx, acc[5]);
    acc[6] = __builtin_elementwise_fma(f2{b1.x, b1.y}, xx, acc[6]);
    acc[7] = __builtin_elementwise_fma(f2{b1.z, b1.w}, xx, acc[7]);
  }
  if (!valid) return;
  float* dst = part + ((size_t)s * NF + n) * R + r0;
  *reinterpret_cast<float4*>(dst) = make_float4(acc[0].x, acc[0].y, acc[1].x, acc[1].y);
  *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[2].x, acc[2].y, acc[3].x, acc[3].y);
  if (two) {
    *reinterpret_cast<float4*>(dst + 8) = make_float4(acc[4].x, acc[4].y, acc[5].x, acc[5].y);
    *reinterpret_cast<float4*>(dst + 12) = make_float4(acc[6].x, acc[6].y, acc[7].x, acc[7].y);
  }
}

// ------------------------------------------------------------------------------------------
// The 8-dim chain. Unit = one frame range (<= 16 frames) of one clip; 512 threads = 8 waves
// (two per SIMD), and each WAVE owns 2 frames end to end: z_e, normalisation, the
// cosine-distance scan over ALL codes (lane l: codes l + 64 m, packed over code pairs), the
// argmin (wave all-reduce: min distance, then the lowest index attaining it — torch's
// first-index rule), the raw codeword (an L2 gather of the winning row), loss, stores and the
// running projected residual
//   U[f][i'][k] = sum_{j<i'} (M_{i'j} zst_j)[k],   z_e(i) = ((P_i + b_in) - Qb_i) - U[f][i].
// No cross-wave data exchange: the one barrier per stage guards the double-buffered stage
// codebook (normalised rows, squared norms) and the M block, which LDS-DMA brings in a stage
// ahead. Global stores of a stage are issued after that barrier so no wait covers them.
struct ChainArgs {
  const float* part;   // [8][B*T][nq*8]
  int B, T, nq;
  const float* b_in;   // [nq][8]
  const float* qb;     // [nq][8]
  const float* mcol;   // [nq][nq][8][8]
  const float* cb;     // [nq][N][8]
  const float* cbn;    // [nq][N][8]
  const float* c2;     // [nq][N]
  const float* imp;    // [B][T] or null
  float level;
  int64_t* codes;      // [B][nq][T]
  float* latents;      // [B][nq*8][T]
  float* loss_pf;      // [B][nq][T]
  float* zst;          // [B][nq][T][8]
  float* mask;         // [B][nq][T] or null
  int nr, units, per_xcd;
  unsigned long long* stamps;  // diagnostic build only (-DVRVQ_STAMPS): [grid][nq][8]
};

#ifdef VRVQ_STAMPS
#define CSTAMP(step)                                                                  \
  do {                                                                                \
    if (a.stamps && threadIdx.x == 0) {                                               \
      unsigned long long t_;                                                          \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
      a.stamps[((size_t)blockIdx.x * a.nq + i) * 8 + (step)] = t_;                   \
    }                                                                                 \
  } while (0)
#else
#define CSTAMP(step) do {} while (0)
#endif

template <int NM>
__global__ __launch_bounds__(CH_NT) void rvq_chain_kernel(ChainArgs a) {
  constexpr int N = 256 * NM;
  constexpr int CPL = N / 64;  // codes per lane (4 .. 16), scanned as CPL/2 pairs
  __shared__ __attribute__((aligned(16))) float cbn_s[2][N * CH_CD];
  __shared__ __attribute__((aligned(16))) float c2_s[2][N];
  __shared__ __attribute__((aligned(16))) float m_s[CH_NQMAX * 64];              // M_{.,i}
  __shared__ __attribute__((aligned(16))) float u_s[CH_F * CH_NQMAX * CH_CD];    // [f][i][k]
  __shared__ __attribute__((aligned(16))) float wv_s[CH_NW][32];  // per wave [2 f][8 k] + [2]

  const int bid = blockIdx.x;
  const int u = (bid & 7) * a.per_xcd + (bid >> 3);
  if (u >= a.units) return;
  const int b = u / a.nr, rg = u - b * a.nr;
  const int T = a.T, nq = a.nq, R = nq * CH_CD;
  const int t0 = (int)((long long)rg * T / a.nr);
  const int nf = (int)((long long)(rg + 1) * T / a.nr) - t0;
  const int NF = a.B * T;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* wv = wv_s[wave];
  // (frame, k) roles: lane = fl*8 + k, fl < 2 (lanes 16..63 carry no frame)
  const int fl = (lane >> 3) & 1, k = lane & 7;
  const int f = wave * CH_FPW + fl;  // frame slot in the unit
  const bool role = lane < CH_FPW * CH_CD;
  const bool fvalid = role && f < nf;
  const int tl = t0 + (fvalid ? f : 0);
  const size_t n_f = (size_t)b * T + tl;
  const float s_imp = (a.imp && fvalid) ? (a.imp[(size_t)b * T + tl] * a.level) * (float)nq
                                        : INFINITY;

  auto dma_stage = [&](int i, int buf) {  // codebook of stage i -> buffer buf (all waves)
    vrvq_dma_chunks(a.cbn + (size_t)i * N * CH_CD, cbn_s[buf], N * CH_CD / 256, wave, CH_NW,
                    lane);
    vrvq_dma_chunks(a.c2 + (size_t)i * N, c2_s[buf], N / 256, wave, CH_NW, lane);
  };
  // M block of source stage i (nq*64 floats, in whole 1-KiB chunks: only blocks i <= nq-2 are
  // ever fetched, so the rounded-up tail stays inside the mcol allocation)
  auto dma_m = [&](int i) {
    vrvq_dma_chunks(a.mcol + (size_t)i * R * CH_CD, m_s, (R * CH_CD + 255) / 256, wave, CH_NW,
                    lane);
  };
  // ((P + b_in) - Qb) of stage i for this lane's (frame, k); P = the projection partials
  // summed in split order
  auto load_p = [&](int i) {
    float v[PJ_SPLIT];
#pragma unroll
    for (int sp = 0; sp < PJ_SPLIT; ++sp)
      v[sp] = a.part[((size_t)sp * NF + n_f) * R + i * CH_CD + k];
    float pv = v[0];
#pragma unroll
    for (int sp = 1; sp < PJ_SPLIT; ++sp) pv = pv + v[sp];
    return (pv + a.b_in[i * CH_CD + k]) - a.qb[i * CH_CD + k];
  };

  dma_stage(0, 0);
  if (nq > 1) dma_m(0);
  if (role)
    for (int i = 0; i < nq; ++i) u_s[(f * CH_NQMAX + i) * CH_CD + k] = 0.0f;
  float p_nx = role ? load_p(0) : 0.0f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nq > 1) dma_stage(1, 1);

  for (int i = 0; i < nq; ++i) {
    const bool more = i + 1 < nq;
    const int buf = i & 1;
    CSTAMP(0);
    const float pc = p_nx;
    if (more && role) p_nx = load_p(i + 1);  // a stage of latency to hide
    // (1) z_e = ((P + b_in) - Qb) - U, L2 normalisation; broadcast e / e2 through the wave slot
    float ze = 0.0f;
    if (role) ze = pc - u_s[(f * CH_NQMAX + i) * CH_CD + k];
    {
      const float n2 = vrvq::sum8(ze * ze, lane);
      const float e = ze / fmaxf(sqrtf(n2), 1e-12f);
      const float e2 = vrvq::sum8(e * e, lane);
      if (role) wv[fl * CH_CD + k] = e;
      if (role && k == 0) wv[16 + fl] = e2;
    }
    CSTAMP(1);
    // (2) distance scan over this lane's codes n = lane + 64 m, packed over code pairs
    float best[CH_FPW];
    int bidx[CH_FPW];
    {
      float ev[CH_FPW][CH_CD], e2v[CH_FPW];
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) {
        const float4 x0 = *reinterpret_cast<const float4*>(wv + q * CH_CD);
        const float4 x1 = *reinterpret_cast<const float4*>(wv + q * CH_CD + 4);
        ev[q][0] = x0.x; ev[q][1] = x0.y; ev[q][2] = x0.z; ev[q][3] = x0.w;
        ev[q][4] = x1.x; ev[q][5] = x1.y; ev[q][6] = x1.z; ev[q][7] = x1.w;
        e2v[q] = wv[16 + q];
        best[q] = INFINITY;
        bidx[q] = 0x7fffffff;
      }
      const float* cbs = cbn_s[buf];
      const float* c2b = c2_s[buf];
#pragma unroll
      for (int m = 0; m < CPL; m += 2) {
        const int n0 = lane + 64 * m, n1 = n0 + 64;
        const float4 a0 = *reinterpret_cast<const float4*>(cbs + n0 * CH_CD);
        const float4 a1 = *reinterpret_cast<const float4*>(cbs + n0 * CH_CD + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(cbs + n1 * CH_CD);
        const float4 b1 = *reinterpret_cast<const float4*>(cbs + n1 * CH_CD + 4);
        const f2 c[8] = {f2{a0.x, b0.x}, f2{a0.y, b0.y}, f2{a0.z, b0.z}, f2{a0.w, b0.w},
                         f2{a1.x, b1.x}, f2{a1.y, b1.y}, f2{a1.z, b1.z}, f2{a1.w, b1.w}};
        const f2 cc = {c2b[n0], c2b[n1]};
#pragma unroll
        for (int q = 0; q < CH_FPW; ++q) {
          // dot in k order (mul, then fma chain); (sum e^2 - 2 e.c) + sum c^2 with the first
          // step as fma(d, -2, e2): 2d is exact, so this is the reference's rounding
          // (models/quantize.py:96-100)
          f2 d = f2{ev[q][0], ev[q][0]} * c[0];
#pragma unroll
          for (int kk = 1; kk < CH_CD; ++kk)
            d = __builtin_elementwise_fma(f2{ev[q][kk], ev[q][kk]}, c[kk], d);
          const f2 dist = __builtin_elementwise_fma(d, f2{-2.0f, -2.0f}, f2{e2v[q], e2v[q]}) + cc;
          // codes of a lane in increasing n: strict < keeps the first
          const bool t0k = dist.x < best[q];
          best[q] = t0k ? dist.x : best[q];
          bidx[q] = t0k ? n0 : bidx[q];
          const bool t1k = dist.y < best[q];
          best[q] = t1k ? dist.y : best[q];
          bidx[q] = t1k ? n1 : bidx[q];
        }
      }
    }
    CSTAMP(2);
    // (3) wave argmin per frame: min distance, then the lowest index attaining it
    int bi;
    {
      float dm[CH_FPW];
      int im[CH_FPW];
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) dm[q] = best[q];
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) dm[q] = fminf(dm[q], vrvq::xchg<1>(dm[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) dm[q] = fminf(dm[q], vrvq::xchg<2>(dm[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) dm[q] = fminf(dm[q], vrvq::xchg<4>(dm[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) dm[q] = fminf(dm[q], vrvq::xchg<8>(dm[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) dm[q] = fminf(dm[q], vrvq::xchg<16>(dm[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) dm[q] = fminf(dm[q], vrvq::xchg<32>(dm[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) im[q] = best[q] == dm[q] ? bidx[q] : 0x7fffffff;
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) im[q] = min(im[q], vrvq::xchg<1>(im[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) im[q] = min(im[q], vrvq::xchg<2>(im[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) im[q] = min(im[q], vrvq::xchg<4>(im[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) im[q] = min(im[q], vrvq::xchg<8>(im[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) im[q] = min(im[q], vrvq::xchg<16>(im[q], lane));
#pragma unroll
      for (int q = 0; q < CH_FPW; ++q) im[q] = min(im[q], vrvq::xchg<32>(im[q], lane));
      bi = fl == 0 ? im[0] : im[1];
      bi = (bi >= 0 && bi < N) ? bi : 0;  // NaN distances: stay in range
    }
    CSTAMP(3);
    // (4) raw codeword (L2 gather of the winning row), loss, straight-through vector
    const float zq = a.cb[((size_t)i * N + bi) * CH_CD + k];
    const float zs = ze + (zq - ze);  // z_e + (z_q - z_e).detach(), models/quantize.py:73-75
    const float diff = ze - zq;
    const float l2 = vrvq::sum8(diff * diff, lane);
    if (role) wv[fl * CH_CD + k] = zs;
    CSTAMP(4);
    if (more) {
      // (5) running projected residual: U[f][i'][k] += (M_{i' i} zst_i)[k] for i' > i
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // M_{.,i} (DMA'd a stage ago) landed
      if (role && i + 1 < nq) {
        const float4 z0 = *reinterpret_cast<const float4*>(wv + fl * CH_CD);
        const float4 z1 = *reinterpret_cast<const float4*>(wv + fl * CH_CD + 4);
#pragma unroll 4
        for (int ip = i + 1; ip < nq; ++ip) {
          const float4 w0 = *reinterpret_cast<const float4*>(m_s + (ip * CH_CD + k) * CH_CD);
          const float4 w1 = *reinterpret_cast<const float4*>(m_s + (ip * CH_CD + k) * CH_CD + 4);
          const int o = (f * CH_NQMAX + ip) * CH_CD + k;
          u_s[o] = u_s[o] + dot8(w0, w1, z0, z1);
        }
      }
      CSTAMP(5);
      __syncthreads();  // -------------------- stage i+1's codebook landed (vmcnt(0) above)
      // buffer `buf` (this stage's codebook) and m_s are free everywhere now
      if (i + 2 < nq) {
        dma_m(i + 1);
        dma_stage(i + 2, buf);
      }
    }
    // (6) this stage's global stores, after the barrier: no wait above covers them
    if (fvalid) {
      const size_t fo = ((size_t)b * nq + i) * T + tl;
      a.latents[(((size_t)b * nq + i) * CH_CD + k) * T + tl] = ze;
      a.zst[fo * CH_CD + k] = zs;
      if (k == 0) {
        a.codes[fo] = (int64_t)bi;
        a.loss_pf[fo] = l2 / 8.0f;
      }
      if (k == 1 && a.mask) a.mask[fo] = (s_imp - (float)i >= 0.0f) ? 1.0f : 0.0f;
    }
    CSTAMP(6);
  }
}

}  // namespace

extern "C" int vrvq_rvq_cross_prep(const float* w_in_t, const float* w_out, const float* b_out,
                                   int nq, int dim, int cdim, float* mcol, float* qb,
                                   vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(w_in_t && w_out && b_out && mcol && qb && nq > 0);
  if (dim != CH_D || cdim != CH_CD) return VRVQ_ERR_UNSUPPORTED;
  const int total = nq * nq * 64 + nq * CH_CD;
  hipLaunchKernelGGL(cross_prep_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     as_stream(stream), w_in_t, w_out, b_out, nq, mcol, qb);
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_project(const float* z, int batch, int dim, int frames, int nq, int cdim,
                                const float* w_in_t, float* part, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z && w_in_t && part && batch > 0 && frames > 0 && nq > 0);
  if (dim != CH_D || cdim != CH_CD) return VRVQ_ERR_UNSUPPORTED;
  const long long nf = (long long)batch * frames;
  VRVQ_CHECK_ARG(nf * nq * CH_CD * PJ_SPLIT < 0x7fffffffLL);
  const int R = nq * CH_CD;
  const dim3 grid((unsigned)((nf + 63) / 64), PJ_SPLIT, (unsigned)((R + 63) / 64));
  hipLaunchKernelGGL(rvq_project_kernel, grid, dim3(256), 0, as_stream(stream), z, batch,
                     frames, nq, w_in_t, part);
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_chain(const float* part, int batch, int frames, int nq, int ncode,
                              int cdim, const float* b_in, const float* qb, const float* mcol,
                              const float* cb, const float* cbn, const float* c2,
                              const float* imp, float level, int64_t* codes, float* latents,
                              float* loss_pf, float* zst, float* mask, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(part && b_in && qb && mcol && cb && cbn && c2 && codes && latents && loss_pf &&
                 zst);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0);
  if (cdim != CH_CD || nq > CH_NQMAX || ncode <= 0 || ncode % 256 != 0 || ncode > 1024)
    return VRVQ_ERR_UNSUPPORTED;
  ChainArgs a{};
  a.part = part; a.B = batch; a.T = frames; a.nq = nq;
  a.b_in = b_in; a.qb = qb; a.mcol = mcol; a.cb = cb; a.cbn = cbn; a.c2 = c2;
  a.imp = imp; a.level = level;
  a.codes = codes; a.latents = latents; a.loss_pf = loss_pf; a.zst = zst; a.mask = mask;
  a.nr = (frames + CH_F - 1) / CH_F;
  const long long units = (long long)batch * a.nr;
  VRVQ_CHECK_ARG(units * 8 < 0x7fffffffLL);
  a.units = (int)units;
  a.per_xcd = (int)((units + 7) / 8);
  a.stamps = vrvq_g_stamps;
  const dim3 grid((unsigned)(8 * a.per_xcd));
  hipStream_t st = as_stream(stream);
  switch (ncode / 256) {
    case 1: hipLaunchKernelGGL(rvq_chain_kernel<1>, grid, dim3(CH_NT), 0, st, a); break;
    case 2: hipLaunchKernelGGL(rvq_chain_kernel<2>, grid, dim3(CH_NT), 0, st, a); break;
    case 3: hipLaunchKernelGGL(rvq_chain_kernel<3>, grid, dim3(CH_NT), 0, st, a); break;
    default: hipLaunchKernelGGL(rvq_chain_kernel<4>, grid, dim3(CH_NT), 0, st, a); break;
  }
  return vrvq_launch_status();
}
