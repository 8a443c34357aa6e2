// Snake-fused 1-D convolution and polyphase transposed convolution for gfx950.
//
// Implicit GEMM:  Y[M x N] = W[M x K] * Xs[K x N]
//   M = output channels (or phase-channels for the transposed conv), N = output time,
//   K = Cin * taps, Xs = im2col(snake(x)) never materialised: each workgroup stages a
//   [CK channels x (BN*stride + halo)] window of snake(x) in LDS once per K-chunk and the
//   B-operand of every tap is read from that window at offset (j*stride + tap*dil).
// MFMA: v_mfma_f32_32x32x2_f32 (exact fp32, k-ordered fmaf chain, 64 cyc/SIMD issue).
//   A (32x2):  lane l holds W[m = l&31][k = l>>5]
//   B (2x32):  lane l holds Xs[k = l>>5][n = l&31]
//   D (32x32): lane l, reg r holds Y[row = (r&3) + 8*(r>>2) + 4*(l>>5)][col = l&31]
// So each store instruction writes 32 consecutive time steps (128 B) per row.
//
// Reference semantics: models/layers.py:17-41 (WNConv1d, WNConvTranspose1d, snake),
// :52-110 (ResidualUnit skip, EncoderBlock, DecoderBlock), models/dac_vrvq.py:19-80,
// models/importance_subnet.py:38-45.
#include "common.h"
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

struct ConvArgs {
  const float* x;          // [B][cin][tin]
  const float* alpha;      // [cin] or null
  const float* inv_alpha;  // [cin]
  const float* w;          // [cin][KS][m_pad]
  const float* bias;       // [cout] or null
  const float* res;        // [B][cout][ylen] or null
  float* y;                // [B][cout][ylen] or null
  const float* alpha_o;    // [cout] snake of the NEXT layer, applied in the epilogue, or null
  const float* inv_alpha_o;
  float* ys;               // [B][cout][ylen] snake_o(y), or null
  int cin, tin;
  int M;                   // GEMM rows: cout (normal) or cout*up (transposed)
  int m_pad;
  int cout;
  int stride, pad, dil;
  int ssh;                 // log2(stride) for a power-of-two stride >= 2 (phase-split window), else 0
  int ng;                  // GEMM columns (output positions of the GEMM)
  int up, up_pad;          // transposed conv: upsample factor and its padding (0 = normal)
  int ylen;                // output row length
  int epi;
  int n_mt, n_nt;          // M tiles, N tiles
};

template <int KS, int BM>
struct ChunkCfg {
  // Input channels per K-chunk: CK*KS ~ 32..64 rows of W per stage (half for 192-row tiles,
  // so two double-buffered stages still fit twice per CU).
  static constexpr int CK0 = KS == 1 ? 32 : KS <= 4 ? 16 : KS <= 8 ? 8 : 4;
  static constexpr int CK = (BM > 128 && CK0 >= 8) ? CK0 / 2 : CK0;
};

__device__ __forceinline__ float apply_epi(float v, int epi) {
  if (epi == VRVQ_EPI_TANH) return tanhf(v);
  if (epi == VRVQ_EPI_SIGMOID) return 1.0f / (1.0f + expf(-v));
  return v;
}

// Largest input window a thread stages per K-chunk: stride <= KS/2 for the strided (k = 2s)
// encoder convs, dilation <= 9 for the k = 7 residual-unit convs.
template <int KS, int BN>
struct WinCfg {
  static constexpr int SMAX = (KS == 4 || KS == 8 || KS == 16) ? KS / 2 : 1;
  static constexpr int DMAX = KS == 7 ? 9 : 1;
  static constexpr int XW_MAX = (BN - 1) * SMAX + (KS - 1) * DMAX + 1;
  static constexpr int PER_ROW = (XW_MAX + 63) / 64;  // positions per lane per row
};

// Epilogue column passes: the accumulator tile goes through LDS in BM x (BN / EPASS) pieces of
// at most 64 KiB, EPASS dividing the wave-column count.
template <int BM, int BN, int WN>
struct EpiCfg {
  static constexpr int need = (BM * BN * 4 + 65535) / 65536;
  static constexpr int EPASS = need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : 8;
  static_assert(WN % EPASS == 0 || EPASS == 1, "epilogue passes must split the wave columns");
  static constexpr int BNP = BN / EPASS;
};

template <int BM, int BN, int WM, int NW, int KS>
__global__ __launch_bounds__(64 * NW) void conv_mfma_kernel(ConvArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int WN = NW / WM;
  constexpr int TM = BM / WM;
  constexpr int TN = BN / WN;
  constexpr int RM = TM / 32;
  constexpr int RN = TN / 32;
  constexpr int CK = ChunkCfg<KS, BM>::CK;
  constexpr int KROWS = CK * KS;
  constexpr int WQ4 = KROWS * BM / 4;               // float4 of W per chunk
  constexpr int WQ = (WQ4 + NT - 1) / NT;           // ... per thread
  constexpr int XROWS = (CK + NW - 1) / NW;         // x rows per wave per chunk
  constexpr int XPR = WinCfg<KS, BN>::PER_ROW;
  constexpr int EPASS = EpiCfg<BM, BN, WN>::EPASS;
  constexpr int BNP = EpiCfg<BM, BN, WN>::BNP;
  static_assert(NW * 64 == NT && WM * WN == NW, "waves");
  static_assert(RM >= 1 && RN >= 1 && TM % 32 == 0 && TN % 32 == 0, "tile");
  static_assert(CK % 2 == 0, "chunk shape");

  // Two LDS stages: [W chunk | x window] x 2. The next chunk is prefetched into registers
  // while the current one feeds the MFMAs, then written to the other stage: one barrier per
  // K-chunk.
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int XW = (BN - 1) * a.stride + (KS - 1) * a.dil + 1;
  // Strided convs store the window phase-split, [phase][position / stride], so the B-operand
  // read of every tap is unit-stride across lanes (no LDS bank conflicts).
  const int XP = a.ssh ? (XW + a.stride - 1) >> a.ssh : XW;
  const int XWP = a.ssh ? ((XP << a.ssh) + 3) & ~3 : (XW + 3) & ~3;
  const int STG = KROWS * BM + CK * XWP;

  int bid = blockIdx.x;
  const int mt = bid % a.n_mt;
  bid /= a.n_mt;
  const int nt = bid % a.n_nt;
  const int b = bid / a.n_nt;
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int lr = lane & 31;
  const int lh = lane >> 5;

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const float* xb = a.x + (size_t)b * a.cin * a.tin;
  const int xbase = n0 * a.stride - a.pad;
  // Wave-uniform fast paths: every chunk holds CK real channels, and the window lies inside
  // [0, tin) (no zero padding): the loads then need no per-lane predicates.
  const bool cin_full = a.cin % CK == 0;
  const bool interior = cin_full && xbase >= 0 && xbase + XW <= a.tin;

  float4 wreg[WQ];
  float xreg[XROWS][XPR];

  auto load_chunk = [&](int ci0) {
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int idx = tid + q * NT;
      const int rr = idx / (BM / 4);
      const int cc = (idx - rr * (BM / 4)) * 4;
      const float4* src = reinterpret_cast<const float4*>(a.w + (size_t)(ci0 * KS + rr) * a.m_pad + m0 + cc);
      if (WQ4 % NT == 0 && cin_full) wreg[q] = *src;
      else wreg[q] = (idx < WQ4 && ci0 + rr / KS < a.cin) ? *src : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (interior) {
#pragma unroll
      for (int rw = 0; rw < XROWS; ++rw) {
        const int cl = wave + NW * rw;
        const float* xr = xb + (size_t)(ci0 + cl) * a.tin + xbase;
#pragma unroll
        for (int u = 0; u < XPR; ++u) {
          const int p = lane + 64 * u;
          xreg[rw][u] = (cl < CK && p < XW) ? xr[p] : 0.0f;
        }
      }
    } else {
#pragma unroll
      for (int rw = 0; rw < XROWS; ++rw) {
        const int cl = wave + NW * rw;
        const int ci = ci0 + cl;
        const float* xr = xb + (size_t)ci * a.tin;
#pragma unroll
        for (int u = 0; u < XPR; ++u) {
          const int p = lane + 64 * u;
          const int t = xbase + p;
          xreg[rw][u] = (cl < CK && ci < a.cin && p < XW && t >= 0 && t < a.tin) ? xr[t] : 0.0f;
        }
      }
    }
  };
  auto store_chunk = [&](float* stg, int ci0) {
    float* ws = stg;
    float* xs = stg + KROWS * BM;
#pragma unroll
    for (int q = 0; q < WQ; ++q)
      if (WQ4 % NT == 0 || tid + q * NT < WQ4) reinterpret_cast<float4*>(ws)[tid + q * NT] = wreg[q];
#pragma unroll
    for (int rw = 0; rw < XROWS; ++rw) {
      const int cl = wave + NW * rw;
      if (cl >= CK) continue;
      const int ci = ci0 + cl;
      const bool sn = a.alpha != nullptr && ci < a.cin;
      const float al = sn ? a.alpha[ci] : 0.f, ia = sn ? a.inv_alpha[ci] : 0.f;
#pragma unroll
      for (int u = 0; u < XPR; ++u) {
        const int p = lane + 64 * u;
        float v = xreg[rw][u];
        if (sn) v = snake_act(v, al, ia);  // snake(0) = 0: zero padding commutes with Snake
        if (a.ssh) {
          if (p < XW) xs[cl * XWP + (p & (a.stride - 1)) * XP + (p >> a.ssh)] = v;
        } else if (p < XWP) {
          xs[cl * XWP + p] = v;
        }
      }
    }
  };

  int cur = 0;
  load_chunk(0);
  store_chunk(smem, 0);
  __syncthreads();
  for (int ci0 = 0; ci0 < a.cin; ci0 += CK) {
    const bool more = ci0 + CK < a.cin;
    if (more) load_chunk(ci0 + CK);  // global loads in flight during the MFMAs below
    const float* ws = smem + cur * STG;
    const float* xs = ws + KROWS * BM;
    // ---- MFMA over the chunk: K order = (tap, channel pair) ----
    // Software-pipelined: the LDS operands of step s+1 are read before the MFMAs of step s
    // are issued, so the ds_read latency hides behind the MFMAs instead of stalling every
    // step on lgkmcnt(0).
    constexpr int CP = CK / 2;
    constexpr int NSTEP = KS * CP;
    const int col = wn * TN + lr;
    auto rd = [&](int st, float (&av)[RM], float (&bv)[RN]) {
      const int k = st / CP, kr = (st % CP) * 2 + lh;
#pragma unroll
      for (int i = 0; i < RM; ++i) av[i] = ws[(kr * KS + k) * BM + wm * TM + i * 32 + lr];
      const int xo = a.ssh ? kr * XWP + (k & (a.stride - 1)) * XP + col + (k >> a.ssh)
                           : kr * XWP + col + k * a.dil;
#pragma unroll
      for (int j = 0; j < RN; ++j) bv[j] = xs[xo + j * 32];
    };
    auto mma = [&](const float (&av)[RM], const float (&bv)[RN]) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    };
    {
      float a0[RM], b0[RN], a1[RM], b1[RN];
      rd(0, a0, b0);
#pragma unroll
      for (int st = 0; st < NSTEP; st += 2) {
        // sched_barrier(0): keep each read group ahead of the MFMAs it overlaps (the
        // scheduler otherwise sinks the reads to the MFMAs that consume them).
        if (st + 1 < NSTEP) rd(st + 1, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        if (st + 2 < NSTEP) rd(st + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        if (st + 1 < NSTEP) mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (more) store_chunk(smem + (cur ^ 1) * STG, ci0 + CK);
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue through LDS (every stage buffer is free after the loop's last barrier) ----
  // The accumulator tile is transposed to row-major [BM][BNP] (EPASS column passes) so that
  // each wave then handles 64 consecutive output positions of one row: residual loads and
  // y / snake(y) stores are 256-B coalesced, and the per-element Snake of the next layer runs
  // in a rolled loop.
  float* ct = smem;
  const int mrows = min(BM, a.M - m0);
#pragma unroll
  for (int pass = 0; pass < EPASS; ++pass) {
    if (pass > 0) __syncthreads();
    if (wn / (WN / EPASS) == pass) {
      const int cbase = wn * TN - pass * BNP;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            ct[(wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * BNP + cbase + j * 32 + lr] =
                acc[i][j][r];
    }
    __syncthreads();
    const int p0 = n0 + pass * BNP;  // first GEMM column of this pass
    if (a.up == 0) {
      // Each thread owns 4 consecutive columns per step; U steps are loaded (accumulator
      // tile, bias, residual, next-layer alpha) before anything is stored, so the global
      // loads of a step group are in flight together.
      constexpr int NV = BNP / 4;
      constexpr int ITER = (BM * NV + NT - 1) / NT;
      constexpr int U = ITER >= 4 ? 4 : ITER;
      const int ncols = min(BNP, a.ng - p0);
      const bool vec = (a.ylen & 3) == 0;
      for (int it0 = 0; it0 < ITER; it0 += U) {
        float v[U][4], sa[U], si[U];
        size_t ob[U];
        int nl[U];
        bool ok[U], full[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = tid + NT * (it0 + u);
          const int ml = e / NV;
          nl[u] = (e - ml * NV) * 4;
          ok[u] = it0 + u < ITER && ml < mrows && nl[u] < ncols;
          full[u] = vec && nl[u] + 4 <= ncols;
          const int m = ok[u] ? m0 + ml : m0;
          const float4 c = ok[u] ? *reinterpret_cast<const float4*>(ct + ml * BNP + nl[u])
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
          const float bb = (a.bias && ok[u]) ? a.bias[m] : 0.0f;
          v[u][0] = c.x + bb; v[u][1] = c.y + bb; v[u][2] = c.z + bb; v[u][3] = c.w + bb;
          ob[u] = ((size_t)b * a.cout + m) * a.ylen + p0 + nl[u];
          sa[u] = (a.ys && ok[u]) ? a.alpha_o[m] : 0.0f;
          si[u] = (a.ys && ok[u]) ? a.inv_alpha_o[m] : 0.0f;
          if (a.res && ok[u]) {
            if (full[u]) {
              const float4 r = *reinterpret_cast<const float4*>(a.res + ob[u]);
              v[u][0] = r.x + v[u][0]; v[u][1] = r.y + v[u][1];
              v[u][2] = r.z + v[u][2]; v[u][3] = r.w + v[u][3];
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q)
                if (nl[u] + q < ncols) v[u][q] = a.res[ob[u] + q] + v[u][q];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[u][q] = apply_epi(v[u][q], a.epi);
          if (a.y && ok[u]) {
            if (full[u]) {
              *reinterpret_cast<float4*>(a.y + ob[u]) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q)
                if (nl[u] + q < ncols) a.y[ob[u] + q] = v[u][q];
            }
          }
        }
        if (a.ys) {
          for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            float sv[4];
            for (int q = 0; q < 4; ++q) sv[q] = snake_act(v[u][q], sa[u], si[u]);
            if (full[u]) {
              *reinterpret_cast<float4*>(a.ys + ob[u]) = make_float4(sv[0], sv[1], sv[2], sv[3]);
            } else {
              for (int q = 0; q < 4; ++q)
                if (nl[u] + q < ncols) a.ys[ob[u] + q] = sv[q];
            }
          }
        }
      }
    } else {
      // transposed conv: GEMM row m = co*up + phase, column n -> t = n*up + phase - up_pad.
      // Walk (channel, t) so consecutive lanes store consecutive t.
      const int up = a.up, tl_n = BNP * up;
      const int co0 = m0 / up, nco = min(BM / up, a.cout - co0);
      for (int e = tid; e < BM * BNP; e += NT) {
        const int cl = e / tl_n, tl = e - cl * tl_n;
        const int nl = tl / up, ph = tl - nl * up;
        const int t = (p0 + nl) * up + ph - a.up_pad;
        if (cl < nco && p0 + nl < a.ng && t >= 0 && t < a.ylen) {
          const int co = co0 + cl;
          float v = ct[(cl * up + ph) * BNP + nl];
          if (a.bias) v = v + a.bias[co];
          const size_t o = ((size_t)b * a.cout + co) * a.ylen + t;
          if (a.y) a.y[o] = v;
          if (a.ys) a.ys[o] = snake_act(v, a.alpha_o[co], a.inv_alpha_o[co]);
        }
      }
    }
  }
}

// Small-Cout conv (Cout <= 8, stride 1): the decoder's 96->1 k7 + Tanh output layer and the
// importance subnet's 32->8 / 8->1 k3 tail. An MFMA tile would be >= 75 % padding and the layer
// is HBM-bound on reading x, so: one thread per output sample, snake(x) rows of SC channels
// staged in LDS per step (window 256 + (k-1)*dil), every output channel accumulated in VGPRs.
constexpr int SMALL_BT = 256;
constexpr int SMALL_SC = 16;
constexpr int SMALL_COUT = 8;
constexpr int SMALL_WMAX = 2048;  // cin * k * cout weights staged in LDS

template <int COUT>
__global__ __launch_bounds__(256) void conv_small_cout_kernel(ConvArgs a, int ks) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* w_s = sm;                      // [cin][k][COUT]
  float* xs = sm + SMALL_WMAX;          // [SMALL_SC][XW]
  const int XW = SMALL_BT + (ks - 1) * a.dil;
  const int n_t = (a.ng + SMALL_BT - 1) / SMALL_BT;
  const int b = blockIdx.x / n_t;
  const int t0 = (blockIdx.x - b * n_t) * SMALL_BT;
  const int tid = threadIdx.x;
  const float* xb = a.x + (size_t)b * a.cin * a.tin;
  for (int e = tid; e < a.cin * ks * COUT; e += 256) {
    const int c = e % COUT, rk = e / COUT;
    w_s[e] = a.w[(size_t)rk * a.m_pad + c];
  }
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = 0.0f;

  for (int ci0 = 0; ci0 < a.cin; ci0 += SMALL_SC) {
    const int nc = min(SMALL_SC, a.cin - ci0);
    for (int e = tid; e < nc * XW; e += 256) {
      const int cl = e / XW, p = e - cl * XW;
      const int ci = ci0 + cl;
      const int t = t0 - a.pad + p;
      float v = 0.0f;
      if (t >= 0 && t < a.tin) {
        v = xb[(size_t)ci * a.tin + t];
        if (a.alpha) v = snake_act(v, a.alpha[ci], a.inv_alpha[ci]);
      }
      xs[cl * XW + p] = v;
    }
    __syncthreads();
    for (int cl = 0; cl < nc; ++cl) {
      const float* wr = w_s + (size_t)(ci0 + cl) * ks * COUT;
      const float* xr = xs + cl * XW + tid;
      for (int k = 0; k < ks; ++k) {
        const float xv = xr[k * a.dil];
#pragma unroll
        for (int c = 0; c < COUT; ++c) acc[c] = fmaf(wr[k * COUT + c], xv, acc[c]);
      }
    }
    __syncthreads();
  }
  const int t = t0 + tid;
  if (t < a.ng) {
#pragma unroll
    for (int c = 0; c < COUT; ++c) {
      if (c < a.M) {
        float v = acc[c];
        if (a.bias) v = v + a.bias[c];
        const size_t o = ((size_t)b * a.cout + c) * a.ylen + t;
        if (a.res) v = a.res[o] + v;
        v = apply_epi(v, a.epi);
        if (a.y) a.y[o] = v;
        if (a.ys) a.ys[o] = snake_act(v, a.alpha_o[c], a.inv_alpha_o[c]);
      }
    }
  }
}

int launch_small(const ConvArgs& a, int batch, int ks, hipStream_t st) {
  if (a.cin * ks * (a.M == 1 ? 1 : SMALL_COUT) > SMALL_WMAX) return VRVQ_ERR_UNSUPPORTED;
  const size_t lds = (size_t)(SMALL_WMAX + SMALL_SC * (SMALL_BT + (ks - 1) * a.dil)) * sizeof(float);
  if (lds > 64 * 1024) return VRVQ_ERR_UNSUPPORTED;
  const long long nblk = (long long)batch * ((a.ng + SMALL_BT - 1) / SMALL_BT);
  if (nblk <= 0 || nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
  if (a.M == 1)
    hipLaunchKernelGGL(conv_small_cout_kernel<1>, dim3((unsigned)nblk), dim3(256), lds, st, a, ks);
  else
    hipLaunchKernelGGL(conv_small_cout_kernel<SMALL_COUT>, dim3((unsigned)nblk), dim3(256), lds, st, a, ks);
  return vrvq_launch_status();
}

template <int BM, int BN, int WM, int NW, int KS>
int launch_cfg(const ConvArgs& a0, int batch, hipStream_t st) {
  ConvArgs a = a0;
  a.n_mt = (a.M + BM - 1) / BM;
  a.n_nt = (a.ng + BN - 1) / BN;
  if (a.m_pad < a.n_mt * BM) return VRVQ_ERR_ARG;
  constexpr int CK = ChunkCfg<KS, BM>::CK;
  const int XW = (BN - 1) * a.stride + (KS - 1) * a.dil + 1;
  const int XP = a.ssh ? (XW + a.stride - 1) >> a.ssh : XW;
  const int XWP = a.ssh ? ((XP << a.ssh) + 3) & ~3 : (XW + 3) & ~3;
  if (XW > 64 * WinCfg<KS, BN>::PER_ROW) return VRVQ_ERR_UNSUPPORTED;  // window > staged lanes
  size_t lds = 2 * (size_t)(CK * KS * BM + CK * XWP) * sizeof(float);
  const size_t epi = (size_t)BM * EpiCfg<BM, BN, NW / WM>::BNP * sizeof(float);
  if (lds < epi) lds = epi;  // epilogue tile
  if (lds > 160 * 1024) return VRVQ_ERR_UNSUPPORTED;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_mfma_kernel<BM, BN, WM, NW, KS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  const long long nblk = (long long)a.n_mt * a.n_nt * batch;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
  hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, NW, KS>), dim3((unsigned)nblk), dim3(64 * NW),
                     lds, st, a);
  return vrvq_launch_status();
}

static int conv_variant() {  // tuning override: VRVQ_CONV_VARIANT=0 (4-wave) | 1 (8-wave wide)
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// Tile choice: BM from the GEMM row count, BN minimising padded columns (prefer wide).
template <int KS>
int dispatch_tiles(const ConvArgs& a, int batch, hipStream_t st) {
  auto waste = [&](int bn) { return ((a.ng + bn - 1) / bn) * bn - a.ng; };
  int bn;
  if (a.ng <= 32) bn = 32;
  else if (a.ng <= 96) {
    // T = 87 / 88 layers: one 96-wide tile per clip when that still gives >= 1.5 workgroups
    // per CU, otherwise three 32-wide tiles (more workgroups for the deep-K, narrow-N GEMMs).
    const long long blocks96 = (long long)((a.M + 127) / 128) * batch;
    bn = blocks96 >= 384 ? 96 : 32;
  }
  else if (a.ng < 4096 && waste(64) * 10 < waste(128) * 7) bn = 64;
  else bn = 128;
  if (a.M <= 32) return launch_cfg<32, 128, 1, 4, KS>(a, batch, st);
  if (bn == 32) return launch_cfg<128, 32, 4, 4, KS>(a, batch, st);
  if (bn == 96) return launch_cfg<128, 96, 4, 4, KS>(a, batch, st);
  constexpr bool kWide = KS == 1 || KS == 2 || KS == 3 || KS == 7;  // register budget at 512 threads
  const bool wide = kWide && conv_variant() == 1 && bn == 128 && a.ng >= 4096;
  if (a.M <= 64) {
    if (bn == 64) return launch_cfg<64, 64, 2, 4, KS>(a, batch, st);
    if constexpr (kWide) if (wide) return launch_cfg<64, 256, 2, 8, KS>(a, batch, st);
    return launch_cfg<64, 128, 2, 4, KS>(a, batch, st);
  }
  // 96- and 192-row tiles: no padded rows for the C = 96 / 192 decoder blocks
  if (a.M <= 96) {
    if constexpr (kWide) if (wide) return launch_cfg<96, 256, 1, 8, KS>(a, batch, st);
    return launch_cfg<96, 128, 1, 4, KS>(a, batch, st);
  }
  if (KS >= 3 && a.M % 128 != 0 && a.M % 192 == 0) {
    if constexpr (kWide) if (wide) return launch_cfg<192, 256, 2, 8, KS>(a, batch, st);
    return launch_cfg<192, 128, 2, 4, KS>(a, batch, st);
  }
  if (bn == 64) return launch_cfg<128, 64, 2, 4, KS>(a, batch, st);
  if constexpr (kWide) if (wide) return launch_cfg<128, 256, 2, 8, KS>(a, batch, st);
  return launch_cfg<128, 128, 2, 4, KS>(a, batch, st);
}

int dispatch_ks(int ks, const ConvArgs& a, int batch, hipStream_t st) {
  switch (ks) {
    case 1: return dispatch_tiles<1>(a, batch, st);
    case 2: return dispatch_tiles<2>(a, batch, st);
    case 3: return dispatch_tiles<3>(a, batch, st);
    case 4: return dispatch_tiles<4>(a, batch, st);
    case 7: return dispatch_tiles<7>(a, batch, st);
    case 8: return dispatch_tiles<8>(a, batch, st);
    case 16: return dispatch_tiles<16>(a, batch, st);
    default: return VRVQ_ERR_UNSUPPORTED;
  }
}

__global__ void pack_conv1d_kernel(const float* __restrict__ w, int cout, int cin, int k,
                                   int cout_pad, float* __restrict__ wp) {
  const size_t total = (size_t)cin * k * cout_pad;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int co = (int)(i % cout_pad);
    const size_t rk = i / cout_pad;
    const int kk = (int)(rk % k);
    const int ci = (int)(rk / k);
    wp[i] = co < cout ? w[((size_t)co * cin + ci) * k + kk] : 0.0f;
  }
}

// Polyphase layout: wp[ci][tap][co*s + r]; tap 1 <-> x[m] (kernel index r),
// tap 0 <-> x[m-1] (kernel index r + s).
__global__ void pack_convt1d_kernel(const float* __restrict__ w, int cin, int cout, int s,
                                    int cout_pad, float* __restrict__ wp) {
  const size_t total = (size_t)cin * 2 * cout_pad;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int mm = (int)(i % cout_pad);
    const size_t rk = i / cout_pad;
    const int tap = (int)(rk % 2);
    const int ci = (int)(rk / 2);
    float v = 0.0f;
    if (mm < cout * s) {
      const int co = mm / s, r = mm - co * s;
      const int kk = tap == 1 ? r : r + s;
      v = w[((size_t)ci * cout + co) * (2 * s) + kk];
    }
    wp[i] = v;
  }
}

}  // namespace

extern "C" int vrvq_conv1d(const float* x, int batch, int cin, int tin, const float* alpha,
                           const float* inv_alpha, const float* w_packed, int cout,
                           int cout_pad, int k, int stride, int pad, int dil, const float* bias,
                           const float* residual, int epilogue, float* y, int tout,
                           const float* alpha_out, const float* inv_alpha_out, float* y_snake,
                           vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && w_packed && (y || y_snake));
  VRVQ_CHECK_ARG(y_snake == nullptr || (alpha_out && inv_alpha_out));
  VRVQ_CHECK_ARG(batch > 0 && cin > 0 && tin > 0 && cout > 0 && k > 0 && stride > 0 &&
                 dil > 0 && pad >= 0 && tout > 0);
  VRVQ_CHECK_ARG(cout_pad >= cout && cout_pad % 128 == 0);
  VRVQ_CHECK_ARG(alpha == nullptr || inv_alpha != nullptr);
  VRVQ_CHECK_ARG(epilogue >= 0 && epilogue <= 2);
  const long long expect = ((long long)tin + 2LL * pad - (long long)dil * (k - 1) - 1) / stride + 1;
  VRVQ_CHECK_ARG(expect == tout);
  ConvArgs a{};
  a.x = x; a.alpha = alpha; a.inv_alpha = inv_alpha; a.w = w_packed; a.bias = bias;
  a.res = residual; a.y = y;
  a.alpha_o = alpha_out; a.inv_alpha_o = inv_alpha_out; a.ys = y_snake;
  a.cin = cin; a.tin = tin; a.M = cout; a.m_pad = cout_pad; a.cout = cout;
  a.stride = stride; a.pad = pad; a.dil = dil; a.ng = tout; a.up = 0; a.up_pad = 0;
  a.ssh = 0;
  if (stride > 1 && (stride & (stride - 1)) == 0)
    while ((1 << a.ssh) < stride) ++a.ssh;
  a.ylen = tout; a.epi = epilogue;
  if (cout <= SMALL_COUT && stride == 1 && cin * k * (cout == 1 ? 1 : SMALL_COUT) <= SMALL_WMAX)
    return launch_small(a, batch, k, as_stream(stream));
  return dispatch_ks(k, a, batch, as_stream(stream));
}

extern "C" int vrvq_conv_transpose1d(const float* x, int batch, int cin, int tin,
                                     const float* alpha, const float* inv_alpha,
                                     const float* w_packed, int cout, int cout_pad, int stride,
                                     const float* bias, float* y, const float* alpha_out,
                                     const float* inv_alpha_out, float* y_snake,
                                     vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && w_packed && (y || y_snake));
  VRVQ_CHECK_ARG(y_snake == nullptr || (alpha_out && inv_alpha_out));
  VRVQ_CHECK_ARG(batch > 0 && cin > 0 && tin > 0 && cout > 0 && stride > 0);
  VRVQ_CHECK_ARG(cout_pad >= cout * stride && cout_pad % 128 == 0);
  VRVQ_CHECK_ARG(alpha == nullptr || inv_alpha != nullptr);
  const int p = (stride + 1) / 2;  // math.ceil(stride / 2), models/layers.py:102
  ConvArgs a{};
  a.x = x; a.alpha = alpha; a.inv_alpha = inv_alpha; a.w = w_packed; a.bias = bias;
  a.res = nullptr; a.y = y;
  a.alpha_o = alpha_out; a.inv_alpha_o = inv_alpha_out; a.ys = y_snake;
  a.cin = cin; a.tin = tin; a.M = cout * stride; a.m_pad = cout_pad; a.cout = cout;
  a.stride = 1; a.pad = 1; a.dil = 1; a.ng = tin + 1; a.up = stride; a.up_pad = p;
  a.ylen = (tin - 1) * stride - 2 * p + 2 * stride;
  a.epi = VRVQ_EPI_NONE;
  return dispatch_ks(2, a, batch, as_stream(stream));
}

extern "C" int vrvq_pack_conv1d_weight(const float* w, int cout, int cin, int k, int cout_pad,
                                       float* w_packed, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(w && w_packed && cout > 0 && cin > 0 && k > 0 && cout_pad >= cout);
  const size_t total = (size_t)cin * k * cout_pad;
  const unsigned grid = (unsigned)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(pack_conv1d_kernel, dim3(grid), dim3(256), 0, as_stream(stream), w, cout,
                     cin, k, cout_pad, w_packed);
  return vrvq_launch_status();
}

extern "C" int vrvq_pack_convt1d_weight(const float* w, int cin, int cout, int stride,
                                        int cout_pad, float* w_packed, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(w && w_packed && cout > 0 && cin > 0 && stride > 0 && cout_pad >= cout * stride);
  const size_t total = (size_t)cin * 2 * cout_pad;
  const unsigned grid = (unsigned)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(pack_convt1d_kernel, dim3(grid), dim3(256), 0, as_stream(stream), w, cin,
                     cout, stride, cout_pad, w_packed);
  return vrvq_launch_status();
}
