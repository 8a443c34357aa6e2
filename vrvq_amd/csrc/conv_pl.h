// The k7 "planes" mainloop: the x3 pair-chunk k7 GEMM (conv_x3.h, 64 x 256 tiles, 16-channel
// K-chunks, 168 MFMAs per wave per chunk) fed entirely by LDS-DMA from operands that are already
// split into bf16 planes in HBM: the weight planes (vrvq_pack_x3_weight) and the input
// snake(x) planes xp[B][3][C/8][T][8] that the producing epilogue wrote (ConvArgs::ysp). No
// register staging and no split on the consumer side: each K-chunk's stage is 72 one-KB
// `buffer_load_dwordx4 ... lds` pieces (42 weight pieces [half][plane][octet][64 rows], 30 window
// pieces [plane][channel octet][64 positions]) + 4 dummies, 19 per wave, issued one chunk AHEAD into the
// second of two LDS stages while the current chunk's MFMAs run (counted vmcnt, raw barriers,
// cdna_hip_programming.md §5 "Pipelining across barriers"). Window positions outside [0, T)
// come back as zeros from the buffer resource's range check (one resource per clip; such a
// position's offset is set past num_records: tools/micro/glds_oob.hip checks the zeros), which
// is the conv's zero padding (snake(0) = 0). One workgroup of 4 waves per CU (2 x 76 KB of LDS).
//
// The MFMA sequence (operand reads, the six products per step, their order) is
// conv_mainloop_x3's for the same tile, so the outputs are bit-identical to the register-staged
// pair tile on the same input values (the planes hold the split the staging would make).
#pragma once
#include "conv_x3.h"

namespace vrvq_conv {

typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int PL_BM = 64, PL_BN = 256, PL_NW = 4;
constexpr int PL_XWP = ((PL_BN - 1) + 6 * 9 + 1 + 63) / 64 * 64;  // window row: 320 positions
// A stage is 1-KB slots: 44 weight slots (42 pieces [half][plane][octet][64 rows] + 2 unused
// dummy slots) then 32 window slots (30 pieces [plane][channel octet][5 x 64 positions] + 2
// dummies), so piece j of wave w always goes to slot 4 j + w: 19 pieces per wave, the same
// kinds in the same order on every wave (no per-wave branch), LDS offsets linear in j.
constexpr int PL_NWP = 2 * 3 * X3Cfg<7>::NO;  // weight pieces per chunk (42)
constexpr int PL_WS = 44;                     // weight slots
constexpr int PL_NXP = 3 * 2 * (PL_XWP / 64); // window pieces per chunk (30)
constexpr int PL_XS = 32;                     // window slots
constexpr int PL_PER_WAVE = (PL_WS + PL_XS) / PL_NW;  // 19
constexpr int PL_WJ = PL_WS / PL_NW;          // the first 11 pieces of a wave are weight pieces
constexpr int PL_STG = (PL_WS + PL_XS) * 1024;        // 77,824 B
constexpr int PL_LDS = 2 * PL_STG;                    // 155,648 B: one workgroup per CU
static_assert(PL_WS >= PL_NWP && PL_XS >= PL_NXP && (PL_WS + PL_XS) % PL_NW == 0 &&
              PL_WS % PL_NW == 0, "slots");

template <int BM, int BN, int WM, int NW>
__device__ __forceinline__ void conv_mainloop_pl(
    const ConvArgs& a, float* smem,
    f32x16 (&acc)[TileCfg<BM, BN, WM, NW>::RM][TileCfg<BM, BN, WM, NW>::RN], int b, int m0,
    int n0) {
  static_assert(BM == PL_BM && BN == PL_BN && NW == PL_NW, "the planes tile");
  using TC = TileCfg<BM, BN, WM, NW>;
  constexpr int RM = TC::RM, RN = TC::RN, TM = TC::TM, TN = TC::TN;
  constexpr int NOP = X3Cfg<7>::NO;    // 7 octet slots per packed chunk (one per tap)
  constexpr int NO2P = X3Cfg<7>::NO2;  // 8 (HBM packing pads to an even count)
  constexpr int NC8 = 2, NSTEP = 7;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;
  char* sbase = reinterpret_cast<char*>(smem);
  const int nchunks = a.cin / 16;
  const int c8n = a.cin >> 3;
  const int xbase = n0 - a.pad;
  // this clip's planes [3][cin / 8][tin][8] under ONE buffer resource, the weight planes under
  // another; a window position outside [0, tin) gets an offset >= 2^31 (past num_records:
  // zeros), so rows never bleed into each other. Per-lane offsets of chunk 0 are fixed for the
  // whole K loop (+ the chunk's stride).
  const size_t clip_elems = (size_t)3 * c8n * a.tin * 8;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.x) + (b * clip_elems) / 2, (short)0, (int)(clip_elems * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned*>(a.w3), (short)0, 0x7fffffff, 0x00020000);
  const unsigned wchunk = (unsigned)(2 * 3 * NO2P) * a.m_pad * 16;  // bytes per K-chunk
  const unsigned xchunk = (unsigned)(2 * a.tin * 16);               // two channel octets
  unsigned voff[PL_PER_WAVE];
#pragma unroll
  for (int j = 0; j < PL_PER_WAVE; ++j) {
    if (j < PL_WJ) {
      const int k = min(PL_NW * j + wave, PL_NWP - 1);  // the dummies reload the last piece
      const int half = k / (3 * NOP), pl = (k / NOP) % 3, po = k % NOP;
      voff[j] = (unsigned)((((half * 3 + pl) * NO2P + po) * a.m_pad + m0 + lane) * 16);
    } else {
      const int q = min(PL_NW * (j - PL_WJ) + wave, PL_NXP - 1);
      const int row = q / (PL_XWP / 64), seg = q % (PL_XWP / 64);
      const int pl = row >> 1, c8 = row & 1;
      const int t = xbase + seg * 64 + lane;
      voff[j] = (t >= 0 && t < a.tin) ? (unsigned)(((pl * c8n + c8) * a.tin + t) * 16)
                                      : 0xC0000000u;
    }
  }
  auto issue = [&](int c, int st) {
    char* slot0 = sbase + st * PL_STG + wave * 1024;
#pragma unroll
    for (int j = 0; j < PL_PER_WAVE; ++j) {
      if (j < PL_WJ)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void_t*)(slot0 + j * PL_NW * 1024), 16,
                                                 voff[j] + c * wchunk, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void_t*)(slot0 + j * PL_NW * 1024), 16,
                                                 voff[j] + c * xchunk, 0, 0, 0);
    }
  };

  const int col = wn * TN + lr;
  auto rd_at = [&](const u32x4* ws, const u32x4* xs, int q, u32x4 (&av)[3][RM],
                   u32x4 (&bv)[3][RN]) {
    // step q: tap q, channel octet lh of the 16-channel chunk (conv_mainloop_x3's pair slots)
    const int tap = q, c8 = lh;
    const int wo = lh * 3 * NOP + q;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < RM; ++i) av[p][i] = ws[(p * NOP + wo) * BM + wm * TM + i * 32 + lr];
    const int xo = c8 * PL_XWP + col + tap * a.dil;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < RN; ++j) bv[p][j] = xs[p * NC8 * PL_XWP + xo + j * 32];
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

  issue(0, 0);
  for (int c = 0; c < nchunks; ++c) {
    const int cur = c & 1;
    if (c + 1 < nchunks) {
      issue(c + 1, cur ^ 1);  // stage cur ^ 1 was freed by the barrier ending chunk c - 1
      // chunk c's pieces have landed (FIFO); chunk c + 1's stay in flight
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PL_PER_WAVE) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's pieces of chunk c are in LDS
    const u32x4* ws = reinterpret_cast<const u32x4*>(sbase + cur * PL_STG);
    const u32x4* xs = reinterpret_cast<const u32x4*>(sbase + cur * PL_STG + PL_WS * 1024);
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage cur free for chunk c + 2's pieces
  }
}

}  // namespace vrvq_conv
