// Fused ResidualUnit for gfx950 (models/layers.py:52-68):
//   y = x + conv1(snake2(conv7_dil(snake1(x)))),  snake1(x) given (producer-side Snake)
// in one launch per (clip, time tile), all C channels in the workgroup:
//   phase 1  h = W7 * window(x_snk) + b7         the conv.hip mainloop (K = 7C, MFMA)
//   mid      hs = snake2(h) -> LDS tile [C][BN]  never written to HBM
//   phase 2  acc = W1 * hs                        K = C; B operand straight from the LDS tile,
//                                                 A operand (W1, L2-resident) register-
//                                                 prefetched a group of steps ahead, no barriers
//   out      y = acc + b1 + x (y optional) and snake_next(y)   the conv.hip epilogue
// Versus the two-launch form this removes the write + re-read of snake2(h) (2 C*T*4 bytes per
// unit and clip) and the separate k=1 launch. Every epilogue expression and the phase-2 K order
// are those of the two launches; the phase-1 K order too wherever the two-launch k7 uses the
// same tile height (C <= 192), so there the output is bit-identical to them.
// Instantiated for C in {64, 96, 128, 192, 256} (the long-time-axis blocks). Measured and
// dropped: C = 384 (an 8-wave 384x64 tile ran 8 % slower than the two launches); the 512 /
// 768-channel units (T = 696) use the two-launch form.
#include "common.h"
#include "conv_core.h"
#include "conv_x3.h"
#include <stdlib.h>

namespace {

using namespace vrvq_conv;

struct RuArgs {
  ConvArgs p1;         // phase 1 (x = snake1(x), w = W7 packed, no Snake prologue)
  ConvArgs p2;         // epilogue (bias b1, residual x, y / ys / next Snake)
  const float* b7;     // [C]
  const float* alpha2; // [C]  Snake between the two convs
  const float* inv_alpha2;
  const float* w1;     // [C][1][m_pad]  packed k=1 weight
  const u32x4* w1x3;   // pre-split W1 (vrvq_pack_x3_weight, k = 1) or null
  int C;
  int p2h;             // ru_p2x3h tiles: phase 2 on the split MFMA in two K-halves (else fp32)
};

// Phase 2 on the split bf16 MFMA when its three hs planes (6 B per element) fit in the LDS
// the kernel already holds: C = 64 / 96 / 192 (C = 128 at BN = 128 would need 96 KiB and
// drop to one workgroup per CU: it runs phase 2 in two K-halves, ru_p2x3h).
template <int BM, int BN>
constexpr bool ru_p2x3() { return BM * BN * 6 <= 80 * 1024; }
// ... else in two K-halves (half the planes + the other half parked as fp32) where that fits:
// C = 128 at BN = 128 (rows split over two wave rows)
template <int BM, int BN, int WM>
constexpr bool ru_p2x3h() {
  return !ru_p2x3<BM, BN>() && WM == 2 && BM % 32 == 0 && BM * BN * 5 <= 80 * 1024;
}

template <int BM, int BN, int WM, int NW, bool X3>
__global__ __launch_bounds__(64 * NW)
__attribute__((amdgpu_waves_per_eu(X3 && x3_stages<BM, BN>() == 1 ? 2 : 1)))
void ru_fused_kernel(RuArgs ra) {
  using TC = TileCfg<BM, BN, WM, NW>;
  constexpr int RM = TC::RM, RN = TC::RN, TM = TC::TM, TN = TC::TN;
  constexpr int NS = BM / 2;   // phase-2 MFMA steps (k = 2 channels per step)
  constexpr int PF = 8;        // steps per prefetch group
  static_assert(NS % PF == 0, "phase-2 steps per group");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const ConvArgs& a = ra.p1;
  const int nt = blockIdx.x % a.n_nt;
  const int b = blockIdx.x / a.n_nt;
  const int n0 = nt * BN;
  const int C = ra.C;

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  // phase 1 on the bf16x3 split path when a pre-split W7 is given (conv_x3.h)
  // single-buffered operand reads in phase 1 (conv_x3.h): C = 96 / 128 / 192 units 2-4 %
  // faster (profiles/r04q_sb_ab.txt; C = 96 drops to 164 VGPRs: three workgroups per CU)
#ifdef VRVQ_X3_SB_ALL  // A/B build
  constexpr bool SB = true;
#else
  constexpr bool SB = BM == 96 || BM == 192 || BM == 128;
#endif
  if constexpr (X3) conv_mainloop_x3<BM, BN, WM, NW, 7, false, x3_pair<7, BM, BN>(), SB>(a, smem, acc, b, 0, n0);
  else conv_mainloop<BM, BN, WM, NW, 7>(a, smem, acc, b, 0, n0);  // ends with a barrier

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int lr = lane & 31, lh = lane >> 5;

  if constexpr (X3 && ru_p2x3<BM, BN>()) {
    if (ra.w1x3 != nullptr) {
      // ---- mid: hs = snake2(h + b7) split into three bf16 planes [plane][C/8][BN][8]: the
      // lane's 4 consecutive rows of each accumulator group are half of one channel octet
      constexpr int NC8 = BM / 8;
      char* hsb = reinterpret_cast<char*>(smem);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row0 = wm * TM + i * 32 + 8 * g + 4 * lh;
          float bb[4], al[4], ia[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool ok = row0 + u < C;
            bb[u] = ok ? ra.b7[row0 + u] : 0.0f;
            al[u] = ok ? ra.alpha2[row0 + u] : 0.0f;
            ia[u] = ok ? ra.inv_alpha2[row0 + u] : 0.0f;
          }
          const int c8 = (wm * TM + i * 32 + 8 * g) / 8;
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = acc[i][j][4 * g + u] + bb[u];
            snake_n<4>(v, al, ia);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = row0 + u < C ? v[u] : 0.0f;
            unsigned h[2], m[2], l[2];
            split3x2(v[0], v[1], h[0], m[0], l[0]);
            split3x2(v[2], v[3], h[1], m[1], l[1]);
            const int col = wn * TN + j * 32 + lr;
            const size_t off = ((size_t)c8 * BN + col) * 16 + lh * 8;
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u32x2*>(hsb + off) = u32x2{h[0], h[1]};
            *reinterpret_cast<u32x2*>(hsb + (size_t)NC8 * BN * 16 + off) = u32x2{m[0], m[1]};
            *reinterpret_cast<u32x2*>(hsb + 2 * (size_t)NC8 * BN * 16 + off) = u32x2{l[0], l[1]};
          }
        }
      __syncthreads();
      // ---- phase 2: acc = W1 * hs, K = C in steps of 16 channels (octets 2q | 2q + 1 on the
      // lane halves: the K order of the x3 k = 1 conv, so the fused unit and the two launches
      // agree bit for bit). W1 planes from L2, one step ahead.
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
      constexpr int NQ = BM / 16;
      const u32x4* hs = reinterpret_cast<const u32x4*>(hsb);
      auto lda = [&](int q, u32x4 (&av)[3][RM]) {
        const int o = 2 * q + lh;  // global octet; k = 1 packing: chunks of 4 octets
        const int ch = o >> 2, oo = o & 3;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int i = 0; i < RM; ++i)
            av[p][i] = ra.w1x3[((size_t)(ch * 3 + p) * 4 + oo) * a.m_pad + wm * TM + i * 32 + lr];
      };
      u32x4 an[3][RM];
      lda(0, an);
#pragma unroll 2
      for (int q = 0; q < NQ; ++q) {
        u32x4 ac[3][RM], bv[3][RN];
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int i = 0; i < RM; ++i) ac[p][i] = an[p][i];
        lda(min(q + 1, NQ - 1), an);
        const int o = 2 * q + lh;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int j = 0; j < RN; ++j) bv[p][j] = hs[((size_t)p * NC8 + o) * BN + wn * TN + j * 32 + lr];
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            f32x16 t = acc[i][j];
            t = mfma_bf16(ac[1][i], bv[1][j], t);  // m m
            t = mfma_bf16(ac[0][i], bv[2][j], t);  // h l
            t = mfma_bf16(ac[2][i], bv[0][j], t);  // l h
            t = mfma_bf16(ac[0][i], bv[1][j], t);  // h m
            t = mfma_bf16(ac[1][i], bv[0][j], t);  // m h
            acc[i][j] = mfma_bf16(ac[0][i], bv[0][j], t);  // h h
          }
      }
      __syncthreads();  // hs reads done: the epilogue reuses the LDS
      conv_epilogue<BM, BN, WM, NW>(ra.p2, smem, acc, b, 0, n0);
      return;
    }
  }

  if constexpr (X3 && ru_p2x3h<BM, BN, WM>()) {
    if (ra.w1x3 != nullptr && ra.p2h) {
      // ---- phase 2 on the split bf16 MFMA in two K-halves (C = 128 at BN = 128: the three
      // planes of all 128 channels would take 96 KB). The wm = 0 waves hold rows [0, 64): they
      // write them as half 0's planes [plane][8 octets][BN][8] (48 KB); the wm = 1 waves park
      // rows [64, 128) as fp32 snake2(h + b7) [64][BN] behind them (32 KB): 80 KB, still two
      // workgroups per CU. Half 0's eight K-steps run, the parked rows are split into the same
      // planes, half 1's run: the octet order of the x3 k = 1 conv, so the unit is bit-identical
      // to the two launches, as for C = 64 / 96 / 192.
      constexpr int HC8 = BM / 16;  // channel octets per half
      constexpr int HQ = BM / 32;   // K-steps (16 channels) per half
      char* hsb = reinterpret_cast<char*>(smem);
      float* park = reinterpret_cast<float*>(hsb + (size_t)3 * HC8 * BN * 16);
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row0 = wm * TM + i * 32 + 8 * g + 4 * lh;
          float bb[4], al[4], ia[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool ok = row0 + u < C;
            bb[u] = ok ? ra.b7[row0 + u] : 0.0f;
            al[u] = ok ? ra.alpha2[row0 + u] : 0.0f;
            ia[u] = ok ? ra.inv_alpha2[row0 + u] : 0.0f;
          }
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = acc[i][j][4 * g + u] + bb[u];
            snake_n<4>(v, al, ia);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = row0 + u < C ? v[u] : 0.0f;
            const int col = wn * TN + j * 32 + lr;
            if (row0 < BM / 2) {  // wave-uniform (wm)
              unsigned h[2], m[2], l[2];
              split3x2(v[0], v[1], h[0], m[0], l[0]);
              split3x2(v[2], v[3], h[1], m[1], l[1]);
              const size_t off = ((size_t)(row0 >> 3) * BN + col) * 16 + lh * 8;
              *reinterpret_cast<u32x2*>(hsb + off) = u32x2{h[0], h[1]};
              *reinterpret_cast<u32x2*>(hsb + (size_t)HC8 * BN * 16 + off) = u32x2{m[0], m[1]};
              *reinterpret_cast<u32x2*>(hsb + 2 * (size_t)HC8 * BN * 16 + off) = u32x2{l[0], l[1]};
            } else {
#pragma unroll
              for (int u = 0; u < 4; ++u) park[(row0 - BM / 2 + u) * BN + col] = v[u];
            }
          }
        }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
      const u32x4* hs = reinterpret_cast<const u32x4*>(hsb);
      auto lda = [&](int q, u32x4 (&av)[3][RM]) {
        const int o = 2 * q + lh;  // global octet; k = 1 packing: chunks of 4 octets
        const int ch = o >> 2, oo = o & 3;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int i = 0; i < RM; ++i)
            av[p][i] = ra.w1x3[((size_t)(ch * 3 + p) * 4 + oo) * a.m_pad + wm * TM + i * 32 + lr];
      };
      u32x4 an[3][RM];
      lda(0, an);
      auto steps = [&](int q0) {  // K-steps q0 .. q0 + HQ - 1 against the half in the planes
#pragma unroll 2
        for (int q = q0; q < q0 + HQ; ++q) {
          u32x4 ac[3][RM], bv[3][RN];
#pragma unroll
          for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int i = 0; i < RM; ++i) ac[p][i] = an[p][i];
          lda(min(q + 1, 2 * HQ - 1), an);
          const int o = 2 * (q - q0) + lh;
#pragma unroll
          for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int j = 0; j < RN; ++j)
              bv[p][j] = hs[((size_t)p * HC8 + o) * BN + wn * TN + j * 32 + lr];
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j) {
              f32x16 t = acc[i][j];
              t = mfma_bf16(ac[1][i], bv[1][j], t);  // m m
              t = mfma_bf16(ac[0][i], bv[2][j], t);  // h l
              t = mfma_bf16(ac[2][i], bv[0][j], t);  // l h
              t = mfma_bf16(ac[0][i], bv[1][j], t);  // h m
              t = mfma_bf16(ac[1][i], bv[0][j], t);  // m h
              acc[i][j] = mfma_bf16(ac[0][i], bv[0][j], t);  // h h
            }
        }
      };
      steps(0);
      __syncthreads();  // half 0's planes no longer read
      for (int e = tid; e < HC8 * BN; e += 64 * NW) {  // the parked rows -> half 1's planes
        const int c8 = e / BN, col = e - c8 * BN;
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = park[(c8 * 8 + u) * BN + col];
        unsigned h[4], m[4], l[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) split3x2(v[2 * u], v[2 * u + 1], h[u], m[u], l[u]);
        u32x4* dst = reinterpret_cast<u32x4*>(hsb) + (size_t)c8 * BN + col;
        dst[0] = u32x4{h[0], h[1], h[2], h[3]};
        dst[(size_t)HC8 * BN] = u32x4{m[0], m[1], m[2], m[3]};
        dst[2 * (size_t)HC8 * BN] = u32x4{l[0], l[1], l[2], l[3]};
      }
      __syncthreads();
      steps(HQ);
      __syncthreads();  // hs reads done: the epilogue reuses the LDS
      conv_epilogue<BM, BN, WM, NW>(ra.p2, smem, acc, b, 0, n0);
      return;
    }
  }

  // ---- mid: hs[row][col] = snake2(h + b7) in the MFMA D layout (rows >= C: zero) ----
  float* hs = smem;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const bool ok = row < C;
      const float bb = ok ? ra.b7[row] : 0.0f;
      const float al = ok ? ra.alpha2[row] : 0.0f, ia = ok ? ra.inv_alpha2[row] : 0.0f;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const float v = acc[i][j][r] + bb;  // conv.hip epilogue: c + bias
        hs[row * BN + wn * TN + j * 32 + lr] = ok ? snake_act(v, al, ia) : 0.0f;
      }
    }
  __syncthreads();

  // ---- phase 2: acc = W1 * hs over K = C in channel pairs (the k=1 launch's K order) ----
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  const float* wa = ra.w1 + (size_t)lh * a.m_pad + wm * TM + lr;  // + 2 s m_pad + i 32
  const float* hb = hs + lh * BN + wn * TN + lr;                  // + 2 s BN + j 32
  float an[PF][RM];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int i = 0; i < RM; ++i) an[p][i] = wa[(size_t)(2 * p) * a.m_pad + i * 32];
  for (int g = 0; g < NS; g += PF) {
    float ac[PF][RM];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int i = 0; i < RM; ++i) ac[p][i] = an[p][i];
    if (g + PF < NS) {  // next group's W1 values in flight during this group's MFMAs
#pragma unroll
      for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int i = 0; i < RM; ++i) an[p][i] = wa[(size_t)(2 * (g + PF + p)) * a.m_pad + i * 32];
    }
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      float bv[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) bv[j] = hb[(2 * (g + p)) * BN + j * 32];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[p][i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // hs reads done: the epilogue reuses the LDS
  conv_epilogue<BM, BN, WM, NW>(ra.p2, smem, acc, b, 0, n0);
}

// x3 phase 1 for every C <= 192 (C = 256: its 256-row weight stage leaves room for one
// workgroup per CU; it keeps the fp32 path). Measured at B = 32 with the single-stage x3
// loop: RU 96 2.12 -> 1.77 ms, RU 192 4.00 -> 3.15 ms, RU 128 1.97 -> 1.35 ms per unit
// (profiles/r02zg_layer_table.txt). VRVQ_RU_X3=0: never, 1: C = 64 / 128 only, 2: all.
static bool ru_x3_ok(int C) {
  static const int v = [] {
    const char* e = getenv("VRVQ_RU_X3");
    return e ? atoi(e) : 2;
  }();
  return v == 2 ? true : v == 1 ? (C == 64 || C == 128) : false;
}

// tuning override: VRVQ_RU_BN64=1 runs the C = 64 / 128 units on 64-wide time tiles (more
// workgroups per CU; C = 128 then fits phase 2 on the x3 MFMA) | 0 (default: 128-wide)
static bool ru_bn64() {
  static const bool v = [] {
    const char* e = getenv("VRVQ_RU_BN64");
    return e && atoi(e) != 0;
  }();
  return v;
}

// tuning override: VRVQ_RU_P2H=0 keeps the C = 128 unit's phase 2 on the fp32 MFMA (A/B)
static bool ru_p2_halves() {
  static const bool v = [] {
    const char* e = getenv("VRVQ_RU_P2H");
    return !e || atoi(e) != 0;
  }();
  return v;
}

template <int BM, int BN, int WM, int NW>
int launch_ru(RuArgs ra, int batch, hipStream_t st) {
  ra.p2h = ru_p2_halves() ? 1 : 0;
  constexpr int CK = ChunkCfg<7, BM, BN>::CK;
  ConvArgs& a = ra.p1;
  a.n_mt = 1;
  a.n_nt = (a.ng + BN - 1) / BN;
  ra.p2.n_mt = 1;
  ra.p2.n_nt = a.n_nt;
  if (a.m_pad < BM || ra.C > BM) return VRVQ_ERR_ARG;
  const int XW = (BN - 1) + 6 * a.dil + 1;
  const int XWP = (XW + 3) & ~3;
  if (XW > 64 * WinCfg<7, BN>::PER_ROW) return VRVQ_ERR_UNSUPPORTED;
  size_t lds = 2 * (size_t)(CK * 7 * BM + CK * XWP) * sizeof(float);
  const size_t hsz = (size_t)BM * BN * sizeof(float);
  const size_t epi = (size_t)BM * EpiCfg<BM, BN, NW / WM>::BNP * sizeof(float);
  if (lds < hsz) lds = hsz;
  if (lds < epi) lds = epi;
  const long long nblk = (long long)a.n_nt * batch;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
  if constexpr (BM <= 192) {
    size_t lx = x3_lds_bytes<7, BM, BN>(XW, a.cin);
    if (lx < hsz) lx = hsz;
    if (ru_p2x3<BM, BN>() && ra.w1x3 != nullptr && lx < (size_t)BM * BN * 6) lx = (size_t)BM * BN * 6;
    if (ru_p2x3h<BM, BN, WM>() && ra.w1x3 != nullptr && ru_p2_halves() &&
        lx < (size_t)BM * BN * 5)
      lx = (size_t)BM * BN * 5;
    if (lx < epi) lx = epi;
    if (a.w3 != nullptr && XW <= (BN - 1) + 6 * 9 + 1 && lx <= 160 * 1024 && ru_x3_ok(BM)) {
      if (lx > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)ru_fused_kernel<BM, BN, WM, NW, true>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lx);
        if (e != hipSuccess) return (int)e;
      }
      hipLaunchKernelGGL((ru_fused_kernel<BM, BN, WM, NW, true>), dim3((unsigned)nblk),
                         dim3(64 * NW), lx, st, ra);
      return vrvq_launch_status();
    }
  }
  if (lds > 160 * 1024) return VRVQ_ERR_UNSUPPORTED;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)ru_fused_kernel<BM, BN, WM, NW, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((ru_fused_kernel<BM, BN, WM, NW, false>), dim3((unsigned)nblk),
                     dim3(64 * NW), lds, st, ra);
  return vrvq_launch_status();
}

}  // namespace

extern "C" int vrvq_residual_unit(const float* x, const float* x_snk, int batch, int channels,
                                  int frames, int dil, const float* w7_packed,
                                  const uint16_t* w7_x3, const uint16_t* w1_x3,
                                  const float* b7,
                                  const float* alpha2, const float* inv_alpha2,
                                  const float* w1_packed, const float* b1, int cout_pad,
                                  float* y, const float* alpha_out, const float* inv_alpha_out,
                                  float* y_snake, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && x_snk && w7_packed && b7 && alpha2 && inv_alpha2 && w1_packed && b1);
  VRVQ_CHECK_ARG(y || y_snake);
  VRVQ_CHECK_ARG(y_snake == nullptr || (alpha_out && inv_alpha_out));
  VRVQ_CHECK_ARG(batch > 0 && channels > 0 && frames > 0 && dil >= 1 && dil <= 9);
  VRVQ_CHECK_ARG(cout_pad >= channels && cout_pad % 128 == 0);
  RuArgs ra{};
  ConvArgs& p = ra.p1;
  p.x = x_snk; p.alpha = nullptr; p.inv_alpha = nullptr; p.w = w7_packed; p.bias = nullptr;
  p.res = nullptr; p.y = nullptr; p.alpha_o = nullptr; p.inv_alpha_o = nullptr; p.ys = nullptr;
  p.cin = channels; p.tin = frames; p.M = channels; p.m_pad = cout_pad; p.cout = channels;
  p.stride = 1; p.pad = 3 * dil; p.dil = dil; p.ssh = 0; p.ng = frames; p.up = 0; p.up_pad = 0;
  p.ylen = frames; p.epi = VRVQ_EPI_NONE;
  p.w3 = reinterpret_cast<const unsigned*>(w7_x3);
  ConvArgs& q = ra.p2;
  q = p;
  q.bias = b1; q.res = x; q.y = y; q.alpha_o = alpha_out; q.inv_alpha_o = inv_alpha_out;
  q.ys = y_snake;
  ra.b7 = b7; ra.alpha2 = alpha2; ra.inv_alpha2 = inv_alpha2; ra.w1 = w1_packed;
  ra.w1x3 = w7_x3 != nullptr ? reinterpret_cast<const u32x4*>(w1_x3) : nullptr;
  ra.C = channels;
  hipStream_t st = as_stream(stream);
  switch (channels) {
    case 64:
      if (ru_bn64()) return launch_ru<64, 64, 2, 4>(ra, batch, st);
      return launch_ru<64, 128, 2, 4>(ra, batch, st);
    case 96: return launch_ru<96, 128, 1, 4>(ra, batch, st);
    case 128:
      if (ru_bn64()) return launch_ru<128, 64, 2, 4>(ra, batch, st);
      return launch_ru<128, 128, 2, 4>(ra, batch, st);
    case 192: return launch_ru<192, 64, 2, 4>(ra, batch, st);
    case 256: return launch_ru<256, 64, 2, 4>(ra, batch, st);
    default: return VRVQ_ERR_UNSUPPORTED;
  }
}
