// Shared building blocks of the MFMA implicit-GEMM convolutions (conv.hip) and the fused
// ResidualUnit (conv_ru.hip): argument block, tile configuration, the K-chunk mainloop and the
// LDS-transposed epilogue. See conv.hip for the GEMM mapping and the MFMA operand layouts.
#pragma once
#include "common.h"
#include <type_traits>

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace vrvq_conv {

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
  const unsigned* w3;      // pre-split bf16 weight planes (conv_x3.h) or null: fp32 MFMA path
  // Strided conv (k = 2s, s = 2^psh) on the x3 loop as a stride-1 k = 2 conv over the
  // phase-split view xv[c*s + r][m] = x[c][m*s + r - ppad] (conv_x3.h): cin / tin above are the
  // view's (pcin * s, tout + 1), x is [B][pcin][ptin]. psh = 0: no view.
  int psh, ppad, pcin, ptin;
  // in_proj of every RVQ stage in the epilogue (vrvq_conv1d_proj, 128-row tiles of the
  // 1024-channel z): pj_part[s][b * ng + n][8 pj_nq] over the tile's channel split s = m0 / 128,
  // W_in as bf16 planes in the 16x16x32 A-fragment order (vrvq_rvq_pack_w_in); null: none
  const unsigned* pj_w3;
  float* pj_part;
  int pj_nq;
  int pj_nf;               // frames of the whole call (B * ng): the partials' split stride
  // split-K over the channel chunks (the deep-K, narrow-N T <= 96 layers, vrvq_conv1d_ws):
  // workgroup (tile, s) sums chunks [s per, (s + 1) per) of its tile into ks_part (fragment
  // order), conv_splitk_epilogue_kernel adds the ks_split partials in s order and runs the
  // epilogue. ks_split <= 1: none.
  int ks_split;
  float* ks_part;
};

// v = h + m + l exactly (RNE at each step; conv_x3.h split3x2), two values per call
__device__ __forceinline__ void split3x2_core(float v0, float v1, unsigned& h, unsigned& m,
                                              unsigned& l) {
  typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
  typedef float f32x2_ __attribute__((ext_vector_type(2)));
  const f32x2_ v = {v0, v1};
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_));
  const f32x2_ hf = {__uint_as_float(hu << 16), __uint_as_float(hu & 0xffff0000u)};
  const f32x2_ r = v - hf;
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2_));
  const f32x2_ mf = {__uint_as_float(mu << 16), __uint_as_float(mu & 0xffff0000u)};
  const f32x2_ s = r - mf;
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(s, bf16x2_));
}

template <int KS, int BM, int BN>
struct ChunkCfg {
  // Input channels per K-chunk: CK*KS ~ 32..64 rows of W per stage (half for 192-row tiles,
  // so two double-buffered stages still fit twice per CU).
  // The strided encoder convs (KS = 2 s in {4, 8, 16}) take half of that: with their wide
  // input windows a full chunk needs ~99 KB for the two stages, one workgroup per CU, and
  // their short K then leaves every prologue / epilogue exposed (measured at B = 32:
  // 64->128 s2 877 -> 680 us, 128->256 s4 1279 -> 1072, 512->1024 s8 at BN 32 888 -> 696;
  // but 256->512 s8 at BN 128 1319 -> 1606, so k16 keeps 4 channels on 128-wide tiles).
  static constexpr int CK0 = KS == 1 ? 32 : KS <= 3 ? 16 : KS == 4 ? 8 : KS == 7 ? 8
                             : KS == 8 ? 4 : BN > 32 ? 4 : 2;
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


// Tile geometry shared by the mainloop / epilogue of one <BM, BN, WM, NW> configuration.
template <int BM, int BN, int WM, int NW>
struct TileCfg {
  static constexpr int NT = 64 * NW;
  static constexpr int WN = NW / WM;
  static constexpr int TM = BM / WM;
  static constexpr int TN = BN / WN;
  static constexpr int RM = TM / 32;
  static constexpr int RN = TN / 32;
};

// K loop over a.cin in chunks of CK input channels x KS taps: two LDS stages [W chunk | x
// window], the next chunk prefetched into registers while the current one feeds the MFMAs, one
// barrier per chunk. acc must be zero on entry. Ends with a barrier (every stage buffer free).
template <int BM, int BN, int WM, int NW, int KS>
__device__ __forceinline__ void conv_mainloop(
    const ConvArgs& a, float* smem,
    f32x16 (&acc)[TileCfg<BM, BN, WM, NW>::RM][TileCfg<BM, BN, WM, NW>::RN], int b, int m0,
    int n0) {
  constexpr int NT = 64 * NW;
  constexpr int WN = NW / WM;
  constexpr int TM = BM / WM;
  constexpr int TN = BN / WN;
  constexpr int RM = TM / 32;
  constexpr int RN = TN / 32;
  constexpr int CK = ChunkCfg<KS, BM, BN>::CK;
  constexpr int KROWS = CK * KS;
  constexpr int WQ4 = KROWS * BM / 4;               // float4 of W per chunk
  constexpr int WQ = (WQ4 + NT - 1) / NT;           // ... per thread
  constexpr int XROWS = (CK + NW - 1) / NW;         // x rows per wave per chunk
  constexpr int XPR = WinCfg<KS, BN>::PER_ROW;
  static_assert(NW * 64 == NT && WM * WN == NW, "waves");
  static_assert(RM >= 1 && RN >= 1 && TM % 32 == 0 && TN % 32 == 0, "tile");
  static_assert(CK % 2 == 0, "chunk shape");

  const int XW = (BN - 1) * a.stride + (KS - 1) * a.dil + 1;
  const int XP = a.ssh ? (XW + a.stride - 1) >> a.ssh : XW;
  const int XWP = a.ssh ? ((XP << a.ssh) + 3) & ~3 : (XW + 3) & ~3;
  const int STG = KROWS * BM + CK * XWP;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int lr = lane & 31;
  const int lh = lane >> 5;

  const float* xb = a.x + (size_t)b * a.cin * a.tin;
  const int xbase = n0 * a.stride - a.pad;
  // Wave-uniform fast paths: every chunk holds CK real channels, and the window lies inside
  // [0, tin) (no zero padding): the loads then need no per-lane predicates.
  const bool cin_full = a.cin % CK == 0;
  const bool interior = cin_full && xbase >= 0 && xbase + XW <= a.tin;

  float4 wreg[WQ];
  float xreg[XROWS][XPR];

  // Loads are branch-free, from clamped addresses; the zeroing of out-of-range values (rows
  // past cin, window positions outside [0, tin)) happens in store_chunk. A conditional load
  // compiles to an exec-masked branch, and the wait at its join drains every load in flight:
  // the W loads of the next chunk were waited for before its x loads were even issued.
  const int wrows = a.cin * KS;  // rows of the packed weight
  auto load_chunk = [&](int ci0) {
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int idx = (WQ4 % NT == 0) ? tid + q * NT : min(tid + q * NT, WQ4 - 1);
      const int rr = idx / (BM / 4);
      const int cc = (idx - rr * (BM / 4)) * 4;
      const int row = min(ci0 * KS + rr, wrows - 1);
      wreg[q] = *reinterpret_cast<const float4*>(a.w + (size_t)row * a.m_pad + m0 + cc);
    }
    if (interior) {
#pragma unroll
      for (int rw = 0; rw < XROWS; ++rw) {
        const int cl = min(wave + NW * rw, CK - 1);
        const float* xr = xb + (size_t)(ci0 + cl) * a.tin + xbase;
#pragma unroll
        for (int u = 0; u < XPR; ++u) xreg[rw][u] = xr[min(lane + 64 * u, XW - 1)];
      }
    } else {
#pragma unroll
      for (int rw = 0; rw < XROWS; ++rw) {
        const int ci = min(ci0 + min(wave + NW * rw, CK - 1), a.cin - 1);
        const float* xr = xb + (size_t)ci * a.tin;
#pragma unroll
        for (int u = 0; u < XPR; ++u)
          xreg[rw][u] = xr[min(max(xbase + lane + 64 * u, 0), a.tin - 1)];
      }
    }
  };
  auto store_chunk = [&](float* stg, int ci0) {
    float* ws = stg;
    float* xs = stg + KROWS * BM;
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int idx = tid + q * NT;
      if (WQ4 % NT == 0 || idx < WQ4) {
        const int rr = idx / (BM / 4);
        reinterpret_cast<float4*>(ws)[idx] =
            (cin_full || ci0 + rr / KS < a.cin) ? wreg[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
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
        const int t = xbase + p;
        const bool ok = ci < a.cin && p < XW && (interior || (t >= 0 && t < a.tin));
        float v = ok ? xreg[rw][u] : 0.0f;
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
  const int last = ((a.cin - 1) / CK) * CK;
  for (int ci0 = 0; ci0 < a.cin; ci0 += CK) {
    // next chunk's loads in flight during the MFMAs below; unconditional (the last chunk
    // reloads itself into the idle stage) so the compiler cannot sink them past the MFMAs
    const int cn = min(ci0 + CK, last);
    load_chunk(cn);
    __builtin_amdgcn_sched_barrier(0);
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
    store_chunk(smem + (cur ^ 1) * STG, cn);
    __syncthreads();
    cur ^= 1;
  }

}

// ---- in_proj of the RVQ stages in the epilogue of the encoder's last conv (vrvq_conv1d_proj).
// For the tile's 128 output channels (latent split s = m0 / 128) and its frames:
//   part[s][b * ng + n][r] = sum_{c in split s} W_in[r][c] z[c][n],  z = acc + bias,  r < 8 nq
// -- rvq_project3_kernel's unit (csrc/rvq.hip, project3_body) bit for bit: z and W_in split
// exactly into three bf16 planes; per 16-row x 16-frame tile the split's four 32-channel k-steps
// in order, each k-step's six products m m, h l, l h, h m, m h, h h on v_mfma_f32_16x16x32_bf16
// from a zero accumulator (each output column depends on its own frame only, so the tile width
// does not change a bit). The chain then sums the eight splits in order, as the three-launch
// path does: the quantizer's input never goes back to HBM as z and is not re-read from it.
// z crosses LDS as three planes [plane][frame][channel] (rows of 128 + 8 channels: conflict-free
// 16-B B reads), 32 frames per pass.
constexpr int PJE_LDB = 136;                      // bf16 per frame row
constexpr int PJE_FR = 32;                        // frames per pass
constexpr int PJE_PLANE = PJE_FR * PJE_LDB * 2;   // bytes per plane (8,704)
constexpr int PJE_LDS = 3 * PJE_PLANE;            // 26,112 B

template <int BM, int BN, int WM, int NW>
__device__ __forceinline__ void proj_epilogue(
    const ConvArgs& a, float* smem,
    const f32x16 (&acc)[TileCfg<BM, BN, WM, NW>::RM][TileCfg<BM, BN, WM, NW>::RN], int b,
    int m0, int n0) {
  static_assert(BM == 128, "one latent split (128 channels) per tile");
  typedef unsigned pj_u32x4 __attribute__((ext_vector_type(4)));
  typedef float pj_f32x4 __attribute__((ext_vector_type(4)));
  typedef __bf16 pj_bf16x8 __attribute__((ext_vector_type(8)));
  using TC = TileCfg<BM, BN, WM, NW>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  const int fr = lane & 15, kg = lane >> 4;  // 16x16x32 roles: frame / row, k group
  const int s = m0 / BM;
  const int R = a.pj_nq * 8, n_rt = (R + 15) / 16;
  const pj_u32x4* w3 = reinterpret_cast<const pj_u32x4*>(a.pj_w3);
  char* lds = reinterpret_cast<char*>(smem);
  auto mfma = [](pj_u32x4 x, pj_u32x4 y, pj_f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(pj_bf16x8, x),
                                                   __builtin_bit_cast(pj_bf16x8, y), c, 0, 0, 0);
  };
  // A planes of one item (row tile rt): the split's 4 k-steps x 3 planes, L2 -> registers
  auto load_a = [&](int rt, pj_u32x4 (&av)[4][3]) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        av[kk][p] = w3[((size_t)((4 * s + kk) * 3 + p) * n_rt + rt) * 64 + lane];
  };
  const int n_items = 2 * n_rt;  // (row tile, 16-frame half of the pass)
  for (int p0 = 0; p0 < BN; p0 += PJE_FR) {
    if (n0 + p0 >= a.ng) break;  // block-uniform
    pj_u32x4 av[4][3];
    if (wave < n_items) load_a(wave >> 1, av);  // the first item's weights under the staging
    __syncthreads();  // the previous pass's planes are no longer read
    // z of this pass's 32 columns (one 32-column accumulator block of one wave column) -> planes
#pragma unroll
    for (int j = 0; j < TC::RN; ++j) {
      if (wn * TC::TN + j * 32 != p0) continue;
#pragma unroll
      for (int i = 0; i < TC::RM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ml = wm * TC::TM + i * 32 + 8 * q + 4 * lh;  // channels ml .. ml + 3
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            v[u] = a.bias ? acc[i][j][4 * q + u] + a.bias[m0 + ml + u] : acc[i][j][4 * q + u];
          unsigned h[2], mm[2], l[2];
          split3x2_core(v[0], v[1], h[0], mm[0], l[0]);
          split3x2_core(v[2], v[3], h[1], mm[1], l[1]);
          char* d = lds + lr * (PJE_LDB * 2) + ml * 2;
          *reinterpret_cast<uint2*>(d) = make_uint2(h[0], h[1]);
          *reinterpret_cast<uint2*>(d + PJE_PLANE) = make_uint2(mm[0], mm[1]);
          *reinterpret_cast<uint2*>(d + 2 * PJE_PLANE) = make_uint2(l[0], l[1]);
        }
    }
    __syncthreads();
    for (int it = wave; it < n_items; it += NW) {
      const int rt = it >> 1, ct = it & 1;
      if (it != wave) load_a(rt, av);
      pj_f32x4 d4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const char* bp = lds + (ct * 16 + fr) * (PJE_LDB * 2) + (32 * kk + 8 * kg) * 2;
        const pj_u32x4 bh = *reinterpret_cast<const pj_u32x4*>(bp);
        const pj_u32x4 bm = *reinterpret_cast<const pj_u32x4*>(bp + PJE_PLANE);
        const pj_u32x4 bl = *reinterpret_cast<const pj_u32x4*>(bp + 2 * PJE_PLANE);
        d4 = mfma(av[kk][1], bm, d4);  // m m
        d4 = mfma(av[kk][0], bl, d4);  // h l
        d4 = mfma(av[kk][2], bh, d4);  // l h
        d4 = mfma(av[kk][0], bm, d4);  // h m
        d4 = mfma(av[kk][1], bh, d4);  // m h
        d4 = mfma(av[kk][0], bh, d4);  // h h
      }
      // D: lane l, reg q -> row 16 rt + 4 (l >> 4) + q, frame l & 15
      const int rr = rt * 16 + 4 * kg;  // rows rr .. rr + 3 all valid iff rr < R (R = 8 nq)
      const int n = n0 + p0 + ct * 16 + fr;
      if (rr < R && n < a.ng)
        *reinterpret_cast<float4*>(a.pj_part + ((size_t)s * a.pj_nf + (size_t)b * a.ng + n) * R + rr) =
            make_float4(d4[0], d4[1], d4[2], d4[3]);
    }
  }
  __syncthreads();  // every LDS buffer free again for the epilogue below
}

// Epilogue through LDS: the accumulator tile is transposed to row-major [BM][BNP] so each wave
// stores 64 consecutive output positions of one row (bias, residual, Tanh/Sigmoid, y and the
// next layer's Snake). Expects every LDS buffer free (after a barrier).
template <int BM, int BN, int WM, int NW>
__device__ __forceinline__ void conv_epilogue(
    const ConvArgs& a, float* smem,
    f32x16 (&acc)[TileCfg<BM, BN, WM, NW>::RM][TileCfg<BM, BN, WM, NW>::RN], int b, int m0,
    int n0) {
  constexpr int NT = 64 * NW;
  constexpr int WN = NW / WM;
  constexpr int TM = BM / WM;
  constexpr int TN = BN / WN;
  constexpr int RM = TM / 32;
  constexpr int RN = TN / 32;
  constexpr int EPASS = EpiCfg<BM, BN, WN>::EPASS;
  constexpr int BNP = EpiCfg<BM, BN, WN>::BNP;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int lr = lane & 31;
  const int lh = lane >> 5;

  if constexpr (BM == 128) {
    if (a.pj_part) {
      proj_epilogue<BM, BN, WM, NW>(a, smem, acc, b, m0, n0);
      if (!a.y && !a.ys) return;  // z itself not wanted: the partials are its use
    }
  }
  // ---- epilogue through LDS (every stage buffer is free after the loop's last barrier) ----
  // The accumulator tile is transposed to row-major [BM][BNP] (EPASS column passes) so that
  // each wave then handles 64 consecutive output positions of one row: residual loads and
  // y / snake(y) stores are 256-B coalesced, and the per-element Snake of the next layer runs
  // in a rolled loop.
  float* ct = smem;
  const int mrows = min(BM, a.M - m0);
  for (int pass = 0; pass < EPASS; ++pass) {  // (unrolled by the compiler where it fits)
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
            float sv[4] = {v[u][0], v[u][1], v[u][2], v[u][3]};
            snake_n1<4>(sv, sa[u], si[u]);
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
      // Walk (channel, t) so consecutive lanes store consecutive t. The decoder's strides
      // (2, 4, 8) get compile-time index arithmetic (shifts instead of integer divisions).
      auto walk = [&](auto up_c) {
        constexpr int UPC = decltype(up_c)::value;
        const int up = UPC ? UPC : a.up, tl_n = BNP * up;
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
      };
      // Strides 2 / 4 / 8: each thread owns 4 consecutive output samples of one channel and
      // stores them as one 16-B vector (dword-aligned: t0 = p0*up + 4q - up_pad).
      auto walk4 = [&](auto up_c) {
        constexpr int UP = decltype(up_c)::value;
        constexpr int QN = BNP * UP / 4;  // quads per channel row of the tile
        const int co0 = m0 / UP, nco = min(BM / UP, a.cout - co0);
        for (int q = tid; q < (BM / UP) * QN; q += NT) {
          const int cl = q / QN, tl0 = (q - cl * QN) * 4;
          const int t0 = p0 * UP + tl0 - a.up_pad;
          if (cl >= nco) continue;
          const int co = co0 + cl;
          const float bb = a.bias ? a.bias[co] : 0.0f;
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int tl = tl0 + u, nl = tl / UP, ph = tl - nl * UP;
            v[u] = ct[(cl * UP + ph) * BNP + nl];
            if (a.bias) v[u] = v[u] + bb;
          }
          const size_t o = ((size_t)b * a.cout + co) * a.ylen + t0;
          const bool full = p0 + (tl0 + 3) / UP < a.ng && t0 >= 0 && t0 + 3 < a.ylen;
          float sv[4] = {v[0], v[1], v[2], v[3]};
          if (a.ys) snake_n1<4>(sv, a.alpha_o[co], a.inv_alpha_o[co]);
          if (full) {
            typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
            if (a.y) *reinterpret_cast<f4u*>(a.y + o) = f4u{v[0], v[1], v[2], v[3]};
            if (a.ys) *reinterpret_cast<f4u*>(a.ys + o) = f4u{sv[0], sv[1], sv[2], sv[3]};
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int t = t0 + u;
              if (p0 + (tl0 + u) / UP < a.ng && t >= 0 && t < a.ylen) {
                if (a.y) a.y[o + u] = v[u];
                if (a.ys) a.ys[o + u] = sv[u];
              }
            }
          }
        }
      };
      if (a.up == 8 && BM % 8 == 0) walk4(std::integral_constant<int, 8>{});
      else if (a.up == 4 && BM % 4 == 0) walk4(std::integral_constant<int, 4>{});
      else if (a.up == 2) walk4(std::integral_constant<int, 2>{});
      else walk(std::integral_constant<int, 0>{});
    }
  }
}

}  // namespace vrvq_conv
