// fp32 convolution on the bf16 matrix cores: the "x3" mainloop.
//
// gfx950 runs v_mfma_f32_32x32x16_bf16 at 16x the FLOP rate of the fp32-input
// v_mfma_f32_32x32x2_f32 (32 vs 64 cycles for 8x the K). Every fp32 operand is split exactly
// into three bf16 terms, v = h + m + l (round-to-nearest at each step: |m| <= 2^-8 |v|,
// |l| <= 2^-16 |v|, and l is exact because a float has 24 significant bits), and a product
// a*b is accumulated as the six terms whose size is >= 2^-16 |ab|:
//     a_h b_h  +  (a_m b_m + a_h b_l + a_l b_h + a_h b_m + a_m b_h)
// in fp32 (bf16 x bf16 products are exact in fp32). The dropped terms a_m b_l + a_l b_m +
// a_l b_l are <= 2^-23 |ab|, the size of one fp32 rounding, so the result carries fp32
// accuracy (tests compare it with the fp32 path and fp64). 6 bf16 MFMAs per 16 K
// (192 cycles) replace 8 fp32 MFMAs (512 cycles): 2.7x the MFMA ceiling.
//
// Operand layouts (32x32x16 bf16: lane l, r = l & 31, h = l >> 5 holds A[row r][k = 8h + e]
// and B[k = 8h + e][col r], e = 0..7): K is ordered in "octets" of 8 consecutive input
// channels at one tap; a K-chunk of CK channels has NO = KS * CK / 8 octets (tap-major),
// padded to an even NO2 with zero weights, and MFMA step q takes octets (2q, 2q + 1) on the
// two lane halves. Both operands are 16-byte LDS reads of one octet per plane:
//     W stage  [plane][octet][BM rows][8]       (pre-split in HBM: vrvq_pack_x3_weight)
//     X stage  [plane][CK/8][XWP positions][8]  (snake(x) split while staging)
// The next K-chunk's W planes and x window are loaded into registers during the current
// chunk's MFMAs (x: eight channels per position, split into three 16-byte planes at the store).
#pragma once
#include "conv_core.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace vrvq_conv {

// LDS stages of the x3 K loop. 1 (default): one stage, refilled between two barriers after
// the chunk's MFMAs; half the LDS and no prefetch registers let two workgroups share a CU,
// and each one's MFMAs cover the other's loads, barriers and epilogue. 2: double-buffered
// with the next chunk prefetched into registers during the MFMAs, one workgroup per CU for
// the larger tiles.
// Tiles up to 128 x 128 take 1 (two workgroups per CU), the 192-row x 128 tiles 2 (their
// registers allow one wave per SIMD, so the prefetch has to hide the loads).
template <int BM, int BN>
constexpr int x3_stages() { return BM * BN <= 128 * 128 ? 1 : 2; }

// 64 x 256 k7 tiles ("pair" chunks): a K-chunk of 16 channels, two channel octets per tap, so
// the 7 taps fill 14 octet slots = 7 MFMA steps with no zero octet (an 8-channel k7 chunk pads
// its 7 octets to 8: 1/8 of its MFMAs multiply zero weights), 168 MFMAs per wave between two
// barriers instead of 96. The weight planes stay in the 8-channel packing (two packed chunks
// per K-chunk, pad octets skipped while staging): 43 KB W + <= 30 KB x per stage, two
// workgroups per CU.
// A pair tile needs Cin to be a multiple of the K-chunk (launch_cfg falls back otherwise). The
// k1 + skip GEMMs on the same construction (128 x 64 tiles, two 32-channel packed chunks per
// K-chunk) measured slower: profiles/r03_x3_pair_ab.txt.
// The same pairing for the 2-tap GEMMs (the strided encoder convs through the phase-split view
// and the polyphase ConvTranspose): 32-channel K-chunks of 8 octets = 4 MFMA steps (the
// 16-channel chunk has 2), on the 128- and 32-wide tiles up to 128 rows (one LDS stage, two
// workgroups per CU). Measured per layer at B = 32 (profiles/r04d_layer_table.txt vs
// r03f_layer_table.txt): 128 x 128 tiles 5-13 % faster (64->128 s2, 128->256 s4, ConvT 384->192
// s4), 128 x 32 10 % (512->1024 s8 at T = 87); 128 x 64 and 128 x 96 4-14 % slower (the doubled
// weight stage costs the 128 x 64 tile its third workgroup per CU): those keep 16-channel chunks.
template <int KS, int BM, int BN>
constexpr bool x3_pair() {
  return (KS == 7 && BM == 64 && BN == 256) ||
         (KS == 2 && BM <= 128 && (BN == 128 || BN == 32));
}

template <int KS, bool PAIR = false>
struct X3Cfg {  // PAIR = false: also the HBM packing of the weight planes (vrvq_pack_x3_weight)
  static constexpr int CK = (PAIR ? 2 : 1) * (KS == 1 ? 32 : KS <= 3 ? 16 : 8);  // channels per K-chunk
  static constexpr int NC8 = CK / 8;                        // channel octets per tap
  static constexpr int NO = KS * NC8;                       // octets per chunk
  static constexpr int NO2 = (NO + 1) & ~1;                 // padded to MFMA steps
  static constexpr int NSTEP = NO2 / 2;
};

// Three planes of two floats (RNE at each step): v = h + m + l exactly.
__device__ __forceinline__ void split3x2(float v0, float v1, unsigned& h, unsigned& m,
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

__device__ __forceinline__ f32x16 mfma_bf16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// LDS bytes of one pipeline stage.
template <int KS, int BM, bool PAIR>
__host__ __device__ constexpr int x3_stage_w_bytes() {
  return PAIR ? 2 * 3 * X3Cfg<KS>::NO * BM * 16 : 3 * X3Cfg<KS>::NO2 * BM * 16;
}
__host__ __device__ inline int x3_xwp(int xw) { return (xw + 3) & ~3; }

// W chunk staging through registers: uint4 u = tid + r*NT of the stage holds
// (plane, octet, row) = (u / BM) -> w3[((chunk*3 + plane)*NO2 + octet)*m_pad + m0 + row].
// Plain global loads (not LDS-DMA): the compiler then places the wait for them right before
// the ds_write after the chunk's MFMAs; with LDS-DMA in inline asm it cannot see the loads and
// its conservative waits at the next global load exposed their whole latency every chunk.
template <int KS, int BM, bool PAIR, int NT>
struct X3W {
  static constexpr int TOTAL = x3_stage_w_bytes<KS, BM, PAIR>() / 16;  // uint4 per stage
  static constexpr int WQ = (TOTAL + NT - 1) / NT;                   // per thread
};

// K loop of the implicit GEMM on the split operands. Same contract as conv_mainloop (acc zero
// on entry, holds W * Xs of the tile on exit, ends after a barrier with every LDS stage free);
// stride-1 windows only (a.ssh == 0), a.w3 = the pre-split weight.
// PH: the phase-split view of a strided conv (ConvArgs::psh > 0; compile-time, so the stride-1
// instantiations keep their plain window addressing).
// SB: single-buffered LDS operand reads in the chunk's MFMA loop (one step's operands live
// instead of two: fewer registers, so more workgroups per CU where the registers were the limit)
// XPF (single-stage loop only): the next chunk's x window is loaded into registers BEFORE the
// chunk's MFMAs (raw fp32, zeroed / Snake / split at the store as before), so only the weight
// planes' L2 round trip stays between the two barriers of the refill.
template <int BM, int BN, int WM, int NW, int KS, bool PH = false,
          bool PAIR = x3_pair<KS, BM, BN>(), bool SB = false, bool XPF = false>
__device__ __forceinline__ void conv_mainloop_x3(
    const ConvArgs& a, float* smem,
    f32x16 (&acc)[TileCfg<BM, BN, WM, NW>::RM][TileCfg<BM, BN, WM, NW>::RN], int b, int m0,
    int n0, int kc0 = 0, int kc1 = 0x7fffffff) {
  using TC = TileCfg<BM, BN, WM, NW>;
  static_assert(!PAIR || ((KS == 7 || KS == 1) && !PH) || KS == 2,
                "pair chunks: k7 / k1 stride-1 windows, the 2-tap GEMMs");
  using XC = X3Cfg<KS, PAIR>;
  constexpr int NO2P = X3Cfg<KS>::NO2;  // octet slots per packed (HBM) chunk
  constexpr int NOP = X3Cfg<KS>::NO;    // ... of them real (k7: 7 taps; k1: 4 channel octets)
  constexpr int NC8P = X3Cfg<KS>::NC8;  // channel octets per packed chunk
  static_assert(!PAIR || X3Cfg<KS, true>::NSTEP == NOP, "pair step q = packed octet q");
  constexpr int NT = TC::NT, RM = TC::RM, RN = TC::RN, TM = TC::TM, TN = TC::TN;
  constexpr int CK = XC::CK, NC8 = XC::NC8, NO = XC::NO, NO2 = XC::NO2, NSTEP = XC::NSTEP;
  constexpr int XW_MAX = (BN - 1) + (KS - 1) * (KS == 7 ? 9 : 1) + 1;
  constexpr int XI = (NC8 * XW_MAX + NT - 1) / NT;  // x items (octet, position) per thread
  constexpr int WB = x3_stage_w_bytes<KS, BM, PAIR>();

  const int XW = (BN - 1) + (KS - 1) * a.dil + 1;
  const int XWP = x3_xwp(XW);
  const int STG = WB + 3 * NC8 * XWP * 16;  // bytes per stage
  constexpr int X3_STAGES = x3_stages<BM, BN>();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  const u32x4* w3 = reinterpret_cast<const u32x4*>(a.w3);
  // phase-split view (strided convs, a.psh > 0): view channel cv = c*s + r, position m reads
  // x[c][m*s + r - ppad]; with psh = 0 the same expressions reduce to x[cv][m]
  const int psh = PH ? a.psh : 0, pmask = (1 << psh) - 1, ppad = PH ? a.ppad : 0;
  const int ptin = PH ? a.ptin : a.tin;
  const float* xb = a.x + (size_t)b * (PH ? (size_t)a.pcin * a.ptin : (size_t)a.cin * a.tin);
  const int xbase = n0 - a.pad;
  const int nitems = NC8 * XW;
  char* sbase = reinterpret_cast<char*>(smem);


  constexpr int WQ = X3W<KS, BM, PAIR, NT>::WQ, WTOT = X3W<KS, BM, PAIR, NT>::TOTAL;
  u32x4 wr[WQ];
  auto load_w = [&](int chunk) {
#pragma unroll
    for (int r = 0; r < WQ; ++r) {
      const int u = min(tid + r * NT, WTOT - 1);  // clamped: no conditional load
      if constexpr (PAIR) {
        // stage entry ((half * 3 + plane) * NOP + po) * BM + row <- octet po of packed chunk
        // 2 chunk + half
        const int hp = u / (NOP * BM), r2 = u - hp * (NOP * BM);
        const int po = r2 / BM, row = r2 - po * BM;
        const int half = hp / 3, pl = hp - half * 3;
        wr[r] = w3[(((size_t)(2 * chunk + half) * 3 + pl) * NO2P + po) * a.m_pad + m0 + row];
      } else {
        const int po = u / BM, row = u - po * BM;
        wr[r] = w3[((size_t)chunk * 3 * NO2 + po) * a.m_pad + m0 + row];
      }
    }
  };
  auto store_w = [&](char* stg) {
    u32x4* ws = reinterpret_cast<u32x4*>(stg);
#pragma unroll
    for (int r = 0; r < WQ; ++r)
      if (WTOT % NT == 0 || tid + r * NT < WTOT) ws[tid + r * NT] = wr[r];
  };
  float xr[XI][8];
  // Branch-free loads from clamped addresses, kept raw: the zeroing select outside the window
  // / input runs in store_x, after the MFMAs. (A select here makes the wave wait for the
  // load before the chunk's MFMAs, and vmcnt retires in order, so that wait also covers the
  // W DMA issued before it: the whole memory latency exposed once per chunk.)
  // pair tiles: every input channel's Snake parameters in LDS behind the stage (their 16 per
  // chunk do not fit the scalar registers); the phase-split view: per real channel (cv >> psh)
  float* snl = reinterpret_cast<float*>(sbase + X3_STAGES * STG);  // after every stage
  auto load_x = [&](int ci0) {
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int e = tid + it * NT;
      const int c8 = NC8 == 1 ? 0 : e / XW, pos = e - c8 * XW;
      const int tc = min(max(xbase + pos, 0), a.tin - 1);
      const int cb = ci0 + (e < nitems ? c8 : 0) * 8;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int cv = min(cb + u, a.cin - 1);
        if constexpr (PH) {
          const int tp = min(max((tc << psh) + (cv & pmask) - ppad, 0), ptin - 1);
          xr[it][u] = xb[(size_t)(cv >> psh) * ptin + tp];
        } else {
          xr[it][u] = xb[(size_t)cv * a.tin + tc];
        }
      }
    }
  };
  auto store_x = [&](char* stg, int ci0) {
    u32x4* xs = reinterpret_cast<u32x4*>(stg + WB);
    // the chunk's channels are workgroup-uniform: their Snake parameters are loaded once per
    // chunk outside the (divergent) item loop -- scalar loads, no vector-memory round trip
    // between the chunk's barriers -- and selected per item by its channel octet
    const bool sn = a.alpha != nullptr;
    constexpr int NU = NC8 == 1 ? 8 : 1;
    float alu[NU], iau[NU];
    if constexpr (NC8 == 1) {
      if (sn) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int ci = PH ? min(ci0 + u, a.cin - 1) >> psh : min(ci0 + u, a.cin - 1);
          alu[u] = a.alpha[ci];
          iau[u] = a.inv_alpha[ci];
        }
      }
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
      const int e = tid + it * NT;
      if (e >= nitems) continue;
      const int c8 = NC8 == 1 ? 0 : e / XW, pos = e - c8 * XW;
      const int t = xbase + pos;
      const bool okp = t >= 0 && t < a.tin;
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int cv = ci0 + c8 * 8 + u;
        bool ok = okp && cv < a.cin;
        if constexpr (PH) {
          const int tp = (t << psh) + (cv & pmask) - ppad;
          ok = ok && tp >= 0 && tp < ptin;
        }
        v[u] = ok ? xr[it][u] : 0.0f;
      }
      if (sn) {
        float al[8], ia[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if constexpr (NC8 == 1) {
            al[u] = alu[u];
            ia[u] = iau[u];
          } else if constexpr (PAIR) {  // from the LDS table (prologue)
            const int ci = min(ci0 + c8 * 8 + u, a.cin - 1) >> psh;
            al[u] = snl[ci];
            ia[u] = snl[(a.cin >> psh) + ci];
          } else {
            const int ci = PH ? min(ci0 + c8 * 8 + u, a.cin - 1) >> psh : min(ci0 + c8 * 8 + u, a.cin - 1);
            al[u] = a.alpha[ci];
            ia[u] = a.inv_alpha[ci];
          }
        }
        snake_n<8>(v, al, ia);  // snake(0) = 0
      }
      unsigned h[4], m[4], l[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) split3x2(v[2 * u], v[2 * u + 1], h[u], m[u], l[u]);
      xs[(0 * NC8 + c8) * XWP + pos] = u32x4{h[0], h[1], h[2], h[3]};
      xs[(1 * NC8 + c8) * XWP + pos] = u32x4{m[0], m[1], m[2], m[3]};
      xs[(2 * NC8 + c8) * XWP + pos] = u32x4{l[0], l[1], l[2], l[3]};
    }
  };

  // channel chunks [kc0, kc1) of the K loop (split-K: one part of them)
  const int nchunks = min((a.cin + CK - 1) / CK, kc1);
  const int col = wn * TN + lr;
  auto rd_at = [&](const u32x4* ws, const u32x4* xs, int q, u32x4 (&av)[3][RM], u32x4 (&bv)[3][RN]) {
    // octet slot o = 2 q + lh: (tap, channel octet) in tap-major order; a pair chunk's slot
    // (q, lh) is octet q of its packed chunk lh: tap q / NC8P, channel octet
    // lh * NC8P + q % NC8P of the staged window
    const int o = 2 * q + lh;
    const int tap = PAIR ? q / NC8P : o < NO ? o / NC8 : 0;  // padded octet: zero weights, any valid x
    const int c8 = PAIR ? lh * NC8P + q % NC8P : o - (o / NC8) * NC8;
    const int wo = PAIR ? lh * 3 * NOP + q : o;  // + plane * (PAIR ? NOP : NO2)
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < RM; ++i)
        av[p][i] = ws[(p * (PAIR ? NOP : NO2) + wo) * BM + wm * TM + i * 32 + lr];
    const int xo = c8 * XWP + col + tap * a.dil;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < RN; ++j) bv[p][j] = xs[p * NC8 * XWP + xo + j * 32];
  };
  auto mma_at = [&](const u32x4 (&av)[3][RM], const u32x4 (&bv)[3][RN]) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        f32x16 t = acc[i][j];
        t = mfma_bf16(av[1][i], bv[1][j], t);  // m m
        t = mfma_bf16(av[0][i], bv[2][j], t);  // h l
        t = mfma_bf16(av[2][i], bv[0][j], t);  // l h
        t = mfma_bf16(av[0][i], bv[1][j], t);  // h m
        t = mfma_bf16(av[1][i], bv[0][j], t);  // m h
        acc[i][j] = mfma_bf16(av[0][i], bv[0][j], t);  // h h
      }
  };
  auto chunk_mma = [&](const u32x4* ws, const u32x4* xs) {
    if constexpr (SB) {
#pragma unroll
      for (int q = 0; q < NSTEP; ++q) {
        u32x4 a0[3][RM], b0[3][RN];
        rd_at(ws, xs, q, a0, b0);
        mma_at(a0, b0);
      }
      return;
    }
    u32x4 a0[3][RM], b0[3][RN], a1[3][RM], b1[3][RN];
    rd_at(ws, xs, 0, a0, b0);
#pragma unroll
    for (int q = 0; q < NSTEP; q += 2) {
      if (q + 1 < NSTEP) rd_at(ws, xs, q + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma_at(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 2 < NSTEP) rd_at(ws, xs, q + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < NSTEP) mma_at(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if constexpr (PAIR) {
    if (a.alpha != nullptr) {
      const int nsc = a.cin >> psh;  // real channels
      for (int c = tid; c < nsc; c += NT) {
        snl[c] = a.alpha[c];
        snl[nsc + c] = a.inv_alpha[c];
      }
      __syncthreads();
    }
  }
  int cur = 0;
  load_w(kc0);
  load_x(kc0 * CK);
  store_w(sbase);
  store_x(sbase, kc0 * CK);
  __syncthreads();
  for (int c = kc0; c < nchunks; ++c) {
    // Next chunk's loads in flight during this chunk's MFMAs. Unconditional (the last chunk
    // reloads itself into the idle stage): under `if (more)` the compiler sinks the loads past
    // the MFMAs into the store block, their only user.
    const int cn = min(c + 1, nchunks - 1);
    char* nxt = sbase + (cur ^ (X3_STAGES - 1)) * STG;
    if constexpr (X3_STAGES == 2) {
      load_w(cn);
      load_x(cn * CK);
      __builtin_amdgcn_sched_barrier(0);
    } else if constexpr (XPF) {
      load_x(cn * CK);  // unconditional (the last chunk reloads itself): see above
      __builtin_amdgcn_sched_barrier(0);
    }
    chunk_mma(reinterpret_cast<const u32x4*>(sbase + cur * STG),
              reinterpret_cast<const u32x4*>(sbase + cur * STG + WB));
    if constexpr (X3_STAGES == 1) {
      // Single stage: the refill is not prefetched (its registers would coexist with the
      // MFMA operands and spill); the other workgroup on the CU runs its MFMAs meanwhile.
      // Measured on the k = 1 tiles, where the prefetch registers do fit (r04p,
      // profiles/r04p_k1_prefetch_ab.txt): 2-23 % slower per layer -- the 128 x 64 tile drops
      // from three workgroups per CU to two, the 128 x 128 one gains nothing.
      __syncthreads();  // every wave done with the stage
      if (c + 1 < nchunks) {
        load_w(cn);
        if constexpr (!XPF) load_x(cn * CK);
        // every load of the refill in flight before the first store waits on one (else the
        // x loads are issued only after the W stores: two memory round trips per chunk)
        __builtin_amdgcn_sched_barrier(0);
        store_w(nxt);
        store_x(nxt, cn * CK);
      }
    } else {
      store_w(nxt);
      store_x(nxt, cn * CK);
    }
    __syncthreads();
    cur ^= X3_STAGES - 1;
  }
}

// LDS bytes the x3 mainloop needs for a window of XW positions.
template <int KS, int BM, int BN, bool PAIR = x3_pair<KS, BM, BN>()>
inline size_t x3_lds_bytes(int xw, int cin) {
  const size_t xb = 3 * (size_t)X3Cfg<KS, PAIR>::NC8 * x3_xwp(xw) * 16;
  const size_t snake = PAIR ? 2 * (size_t)cin * sizeof(float) : 0;
  return x3_stages<BM, BN>() * ((size_t)x3_stage_w_bytes<KS, BM, PAIR>() + xb) + snake;
}

}  // namespace vrvq_conv
