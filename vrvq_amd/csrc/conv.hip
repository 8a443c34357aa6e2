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
#include "conv_core.h"
#include "conv_x3.h"
#include <stdlib.h>

namespace {

using namespace vrvq_conv;

template <int BM, int BN, int WM, int NW, int KS, bool X3, bool PH = false,
          bool PAIR = x3_pair<KS, BM, BN>(), bool SPLIT = false, bool XPF = false>
__global__ __launch_bounds__(64 * NW)
__attribute__((amdgpu_waves_per_eu(X3 && x3_stages<BM, BN>() == 1 ? 2 : 1)))
void conv_mfma_kernel(ConvArgs a) {
  using TC = TileCfg<BM, BN, WM, NW>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int bid = blockIdx.x;
  int ks = 0;  // split-K part (SPLIT: the a.ks_split K parts of a tile are adjacent workgroups)
  if (SPLIT) {
    ks = bid % a.ks_split;
    bid /= a.ks_split;
  }
  // M tile fastest (an M-tile-slowest order, all CUs on one weight tile for L2 reuse, measured
  // no faster in r02: the weight tiles are not what limits)
  const int mt = bid % a.n_mt;
  bid /= a.n_mt;
  const int nt = bid % a.n_nt;
  const int b = bid / a.n_nt;
  const int m0 = mt * BM;
  const int n0 = nt * BN;
  f32x16 acc[TC::RM][TC::RN];
#pragma unroll
  for (int i = 0; i < TC::RM; ++i)
#pragma unroll
    for (int j = 0; j < TC::RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  // single-buffered operand reads (conv_x3.h) on the k1 and 128-wide 2-tap tiles: 2-6 % per
  // k1 layer, +1.7 % end to end with the ResidualUnit rule (profiles/r04q_sb_ab.txt)
#ifdef VRVQ_X3_SB_ALL  // A/B build
  constexpr bool SB = true;
#else
  // (XPF: the x prefetch registers take the place of the second operand set)
  constexpr bool SB = KS == 1 || (KS == 2 && BN == 128) || XPF;
#endif
  if constexpr (X3) {
    if constexpr (SPLIT) {
      // split-K: this part's chunks, the raw sums to ks_part in fragment order (the tile's
      // 64 NW threads x RM RN 16 floats, lane-contiguous: 256-B stores), no epilogue here
      constexpr int CK = X3Cfg<KS, PAIR>::CK;
      const int nch = (a.cin + CK - 1) / CK, per = (nch + a.ks_split - 1) / a.ks_split;
      if (ks * per < nch)  // (a forced part count can leave the last part empty: zero sums)
        conv_mainloop_x3<BM, BN, WM, NW, KS, PH, PAIR, SB>(a, smem, acc, b, m0, n0, ks * per,
                                                            min(nch, (ks + 1) * per));
      constexpr int NR = TC::RM * TC::RN * 16;
      const size_t tile = ((size_t)b * a.n_nt + nt) * a.n_mt + mt;
      const size_t ntile = (size_t)gridDim.x / a.ks_split;
      float* dst = a.ks_part + ((size_t)ks * ntile + tile) * (size_t)NR * 64 * NW +
                   (threadIdx.x >> 6) * NR * 64 + (threadIdx.x & 63);
#pragma unroll
      for (int i = 0; i < TC::RM; ++i)
#pragma unroll
        for (int j = 0; j < TC::RN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[((i * TC::RN + j) * 16 + r) * 64] = acc[i][j][r];
      return;
    }
    conv_mainloop_x3<BM, BN, WM, NW, KS, PH, PAIR, SB, XPF>(a, smem, acc, b, m0, n0);
  } else {
    conv_mainloop<BM, BN, WM, NW, KS>(a, smem, acc, b, m0, n0);
  }
  conv_epilogue<BM, BN, WM, NW>(a, smem, acc, b, m0, n0);
}

// Split-K epilogue: one workgroup per tile (the block order of conv_mfma_kernel without its K
// parts) adds the a.ks_split partial accumulators in part order -- a fixed order that depends on
// the layer only, not on the batch -- and runs the tile's epilogue (bias, residual, activation,
// next Snake) exactly as the unsplit kernel does.
template <int BM, int BN, int WM, int NW>
__global__ __launch_bounds__(64 * NW) void conv_splitk_epilogue_kernel(ConvArgs a) {
  using TC = TileCfg<BM, BN, WM, NW>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int bid = blockIdx.x;
  const int mt = bid % a.n_mt;
  bid /= a.n_mt;
  const int nt = bid % a.n_nt;
  const int b = bid / a.n_nt;
  constexpr int NR = TC::RM * TC::RN * 16;
  const size_t tile = blockIdx.x;  // ((b n_nt + nt) n_mt + mt): the split kernel's order
  const size_t pstride = (size_t)gridDim.x * NR * 64 * NW;
  const float* src = a.ks_part + tile * (size_t)NR * 64 * NW + (threadIdx.x >> 6) * NR * 64 +
                     (threadIdx.x & 63);
  f32x16 acc[TC::RM][TC::RN];
#pragma unroll
  for (int i = 0; i < TC::RM; ++i)
#pragma unroll
    for (int j = 0; j < TC::RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = src[((i * TC::RN + j) * 16 + r) * 64];
  for (int s = 1; s < a.ks_split; ++s)
#pragma unroll
    for (int i = 0; i < TC::RM; ++i)
#pragma unroll
      for (int j = 0; j < TC::RN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          acc[i][j][r] = acc[i][j][r] + src[s * pstride + ((i * TC::RN + j) * 16 + r) * 64];
  conv_epilogue<BM, BN, WM, NW>(a, smem, acc, b, mt * BM, nt * BN);
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

  // staged positions: the window of this block's output positions only (short rows: T = 87)
  const int pmax = min(XW, a.ng - t0 + (ks - 1) * a.dil);
  for (int ci0 = 0; ci0 < a.cin; ci0 += SMALL_SC) {
    const int nc = min(SMALL_SC, a.cin - ci0);
    const int total = nc * pmax;
    // eight loads in flight per thread from clamped addresses, then the zeroing / Snake / LDS
    // stores (a load under the range branch made every iteration wait for its own load)
    for (int e0 = tid; e0 < total; e0 += 8 * 256) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = min(e0 + u * 256, total - 1);
        const int cl = e / pmax, p = e - cl * pmax;
        const int tc = min(max(t0 - a.pad + p, 0), a.tin - 1);
        v[u] = xb[(size_t)(ci0 + cl) * a.tin + tc];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 256;
        if (e < total) {
          const int cl = e / pmax, p = e - cl * pmax;
          const int ci = ci0 + cl;
          const int t = t0 - a.pad + p;
          float x = 0.0f;
          if (t >= 0 && t < a.tin) {
            x = v[u];
            if (a.alpha) x = snake_act(x, a.alpha[ci], a.inv_alpha[ci]);
          }
          xs[cl * XW + p] = x;
        }
      }
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

// Cout = 1 as a stream (the decoder's 96->1 k7 + Tanh, HBM-bound on reading x): no LDS, no
// barriers; each thread owns 4 consecutive outputs and per input channel reads the 12-sample
// window t0-4 .. t0+7 as three 16-B loads (covers pad <= 4 and k-1-pad <= 4 at dilation 1),
// channels unrolled by 8 so their loads are in flight together (measured at B = 32, 96 -> 1 k7:
// 364 us for the LDS-staged kernel, 277 us at 8 outputs x 4 channels per thread, 235 us at
// 4 x 8, 163 us (3.4 TB/s) with the window / Snake branches hoisted out of the channel loop). Accumulation order per output:
// channel, then tap -- conv_small_cout_kernel's fmaf chain, so the two agree bit for bit.
constexpr int C1_T = 4;
constexpr int C1_W = 12;  // window samples per channel
template <int KS, int PAD, bool SNK>
__global__ __launch_bounds__(256) void conv_cout1_stream_kernel(ConvArgs a) {
  static_assert(PAD <= 4 && 4 - PAD + KS - 1 + C1_T - 1 < C1_W, "window t0-4 .. t0+7");
  constexpr int SH = 4 - PAD;  // window index of tap 0 for output t0
  const int n_t = (a.ng + 256 * C1_T - 1) / (256 * C1_T);
  const int b = blockIdx.x / n_t;
  const int t0 = ((blockIdx.x - b * n_t) * 256 + (int)threadIdx.x) * C1_T;
  if (t0 >= a.ng) return;  // no barrier in this kernel
  const float* xb = a.x + (size_t)b * a.cin * a.tin;
  const bool interior = t0 - 4 >= 0 && t0 - 4 + C1_W <= a.tin;
  float acc[C1_T];
#pragma unroll
  for (int u = 0; u < C1_T; ++u) acc[u] = 0.0f;
  // the window path and the Snake flag are decided once, outside the channel loop: a branch
  // per channel would drain each channel's loads before the next are issued
  auto run = [&](auto interior_c, auto snake_c) {
    constexpr bool INTERIOR = decltype(interior_c)::value, SNAKE = decltype(snake_c)::value;
    auto load_win = [&](int c, float (&xv)[C1_W]) {
      const float* xr = xb + (size_t)c * a.tin + t0 - 4;
      if constexpr (INTERIOR) {
#pragma unroll
        for (int q = 0; q < C1_W / 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(xr + 4 * q);
          xv[4 * q] = v.x; xv[4 * q + 1] = v.y; xv[4 * q + 2] = v.z; xv[4 * q + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < C1_W; ++j) {
          const int t = t0 - 4 + j;
          const float v = xb[(size_t)c * a.tin + min(max(t, 0), a.tin - 1)];
          xv[j] = __uint_as_float(__float_as_uint(v) & (0u - (unsigned)(t >= 0 && t < a.tin)));
        }
      }
    };
    auto accum = [&](int c, float (&xv)[C1_W]) {
      if constexpr (SNAKE) snake_n1<C1_W>(xv, a.alpha[c], a.inv_alpha[c]);  // snake(0) = 0
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const float wv = a.w[(size_t)(c * KS + k) * a.m_pad];
#pragma unroll
        for (int u = 0; u < C1_T; ++u) acc[u] = fmaf(wv, xv[SH + k + u], acc[u]);
      }
    };
    constexpr int CU = 8;
    int c = 0;
    for (; c + CU <= a.cin; c += CU) {
      float xv[CU][C1_W];
#pragma unroll
      for (int i = 0; i < CU; ++i) load_win(c + i, xv[i]);
#pragma unroll
      for (int i = 0; i < CU; ++i) accum(c + i, xv[i]);
    }
    for (; c < a.cin; ++c) {
      float xv[C1_W];
      load_win(c, xv);
      accum(c, xv);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (interior) {
    run(T_{}, std::integral_constant<bool, SNK>{});
  } else {
    run(F_{}, std::integral_constant<bool, SNK>{});
  }
#pragma unroll
  for (int u = 0; u < C1_T; ++u) {
    const int t = t0 + u;
    if (t < a.ng) {
      float v = acc[u];
      if (a.bias) v = v + a.bias[0];
      const size_t o = (size_t)b * a.ylen + t;
      if (a.res) v = a.res[o] + v;
      v = apply_epi(v, a.epi);
      if (a.y) a.y[o] = v;
      if (a.ys) a.ys[o] = snake_act(v, a.alpha_o[0], a.inv_alpha_o[0]);
    }
  }
}

// Cin = 1 conv (the encoder's 1 -> 64 k7 input conv, models/dac_vrvq.py:27): no MFMA tile
// (K = 7), HBM-bound on writing y and snake(y) (2 x 64 x 4 B per sample). Thread = 4
// consecutive output samples x CI1_CG channels; its 4 + KS - 1 input samples once, per channel
// the k-ordered fmaf chain from 0, then conv_epilogue's expressions (bias, residual, act, the
// next layer's Snake) and one 16-B store per output row: a wave writes 1 KB runs per channel.
constexpr int CI1_T = 4;
constexpr int CI1_CG = 16;
template <int KS>
__global__ __launch_bounds__(256) void conv_cin1_stream_kernel(ConvArgs a) {
  const int n_t = (a.ng + 256 * CI1_T - 1) / (256 * CI1_T);
  const int n_cg = a.M / CI1_CG;
  int blk = blockIdx.x;
  const int cg = blk % n_cg;
  blk /= n_cg;
  const int tt = blk % n_t, b = blk / n_t;
  const int t0 = (tt * 256 + (int)threadIdx.x) * CI1_T;
  if (t0 >= a.ng) return;  // no barrier in this kernel
  const float* xb = a.x + (size_t)b * a.tin;
  constexpr int W = CI1_T + KS - 1;
  float xv[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {  // clamped address, zeroed outside [0, tin) (zero padding)
    const int t = t0 - a.pad + j;
    const float v = xb[min(max(t, 0), a.tin - 1)];
    xv[j] = __uint_as_float(__float_as_uint(v) & (0u - (unsigned)(t >= 0 && t < a.tin)));
  }
  const bool full = t0 + CI1_T <= a.ng;
#pragma unroll 4
  for (int c = 0; c < CI1_CG; ++c) {
    const int co = cg * CI1_CG + c;
    float v[CI1_T];
#pragma unroll
    for (int u = 0; u < CI1_T; ++u) v[u] = 0.0f;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const float wv = a.w[(size_t)k * a.m_pad + co];
#pragma unroll
      for (int u = 0; u < CI1_T; ++u) v[u] = fmaf(wv, xv[k + u], v[u]);
    }
    const float bb = a.bias ? a.bias[co] : 0.0f;
    const size_t o = ((size_t)b * a.cout + co) * a.ylen + t0;
#pragma unroll
    for (int u = 0; u < CI1_T; ++u) v[u] = v[u] + bb;
    if (a.res) {
#pragma unroll
      for (int u = 0; u < CI1_T; ++u)
        if (full || t0 + u < a.ng) v[u] = a.res[o + u] + v[u];
    }
#pragma unroll
    for (int u = 0; u < CI1_T; ++u) v[u] = apply_epi(v[u], a.epi);
    if (a.y) {
      if (full) *reinterpret_cast<float4*>(a.y + o) = make_float4(v[0], v[1], v[2], v[3]);
      else
        for (int u = 0; u < CI1_T; ++u)
          if (t0 + u < a.ng) a.y[o + u] = v[u];
    }
    if (a.ys) {
      snake_n1<CI1_T>(v, a.alpha_o[co], a.inv_alpha_o[co]);
      if (full) *reinterpret_cast<float4*>(a.ys + o) = make_float4(v[0], v[1], v[2], v[3]);
      else
        for (int u = 0; u < CI1_T; ++u)
          if (t0 + u < a.ng) a.ys[o + u] = v[u];
    }
  }
}

int launch_small(const ConvArgs& a, int batch, int ks, hipStream_t st) {
  if (a.M == 1 && a.cout == 1 && a.stride == 1 && a.dil == 1 && a.tin % 4 == 0 &&
      ((ks == 7 && a.pad == 3) || (ks == 3 && a.pad == 1))) {
    const long long nblk = (long long)batch * ((a.ng + 256 * C1_T - 1) / (256 * C1_T));
    if (nblk <= 0 || nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
    // the consumer-side Snake variant is its own kernel: its registers do not set the plain
    // variant's occupancy
    if (ks == 7 && a.alpha)
      hipLaunchKernelGGL((conv_cout1_stream_kernel<7, 3, true>), dim3((unsigned)nblk), dim3(256), 0, st, a);
    else if (ks == 7)
      hipLaunchKernelGGL((conv_cout1_stream_kernel<7, 3, false>), dim3((unsigned)nblk), dim3(256), 0, st, a);
    else if (a.alpha)
      hipLaunchKernelGGL((conv_cout1_stream_kernel<3, 1, true>), dim3((unsigned)nblk), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((conv_cout1_stream_kernel<3, 1, false>), dim3((unsigned)nblk), dim3(256), 0, st, a);
    return vrvq_launch_status();
  }
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

// x3 ConvTranspose with M a multiple of 96 (not of 128): 96-row pair tiles (default) |
// VRVQ_CONV_CONVT96=0: the 192 x 128 two-stage tile
static int convt_96() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_CONVT96");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// The 64 x 256 pair k7 tiles with the next chunk's x window prefetched into registers during the
// MFMAs (conv_x3.h XPF; profiles/r06x_xpf_layers.txt: 1-3.5 % per layer). Tuning override
// VRVQ_CONV_XPF=0 | 1.
static int conv_x3_xpf() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_XPF");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// Cin = 1 convs on conv_cin1_stream_kernel (default) | VRVQ_CONV_CIN1=0: the fp32 MFMA tile
static int cin1_stream() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_CIN1");
    return e ? atoi(e) : 1;
  }();
  return v;
}



// The x3 launch of a tile (PAIR: its K-chunk form); VRVQ_ERR_UNSUPPORTED when its LDS does not
// fit (the caller then takes the fp32-input loop).
template <int BM, int BN, int WM, int NW, int KS, bool PAIR, bool SPLIT = false, bool XPF = false>
int launch_x3(const ConvArgs& a, int XW, size_t epi, long long nblk, hipStream_t st) {
  // the pair tiles' Snake table only when the staging applies a Snake (the producer-side
  // snake(x) inputs of the k7 layers need none: 3-6 KB of LDS back)
  size_t lx = x3_lds_bytes<KS, BM, BN, PAIR>(XW, a.alpha ? (a.psh ? a.cin >> a.psh : a.cin) : 0);
  if (lx < epi) lx = epi;
  if (lx > 160 * 1024) return VRVQ_ERR_UNSUPPORTED;
  if constexpr (KS == 2) {
    if (a.psh) {  // strided conv through the phase-split view
      if (lx > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(
            (const void*)conv_mfma_kernel<BM, BN, WM, NW, KS, true, true, PAIR, SPLIT, XPF>,
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lx);
        if (e != hipSuccess) return (int)e;
      }
      hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, NW, KS, true, true, PAIR, SPLIT, XPF>),
                         dim3((unsigned)nblk), dim3(64 * NW), lx, st, a);
      return vrvq_launch_status();
    }
  }
  if (a.psh) return VRVQ_ERR_ARG;
  if (lx > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(
        (const void*)conv_mfma_kernel<BM, BN, WM, NW, KS, true, false, PAIR, SPLIT, XPF>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lx);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, NW, KS, true, false, PAIR, SPLIT, XPF>),
                     dim3((unsigned)nblk), dim3(64 * NW), lx, st, a);
  return vrvq_launch_status();
}

template <int BM, int BN, int WM, int NW, int KS>
int launch_cfg(const ConvArgs& a0, int batch, hipStream_t st) {
  ConvArgs a = a0;
  a.n_mt = (a.M + BM - 1) / BM;
  a.n_nt = (a.ng + BN - 1) / BN;
  if (a.m_pad < a.n_mt * BM) return VRVQ_ERR_ARG;
  // transposed conv: a tile must hold whole output channels (rows co*up .. co*up + up-1), the
  // epilogue maps rows back with co0 = m0 / up
  if (a.up > 0 && BM % a.up != 0) return VRVQ_ERR_UNSUPPORTED;
  constexpr int CK = ChunkCfg<KS, BM, BN>::CK;
  const int XW = (BN - 1) * a.stride + (KS - 1) * a.dil + 1;
  const int XP = a.ssh ? (XW + a.stride - 1) >> a.ssh : XW;
  const int XWP = a.ssh ? ((XP << a.ssh) + 3) & ~3 : (XW + 3) & ~3;
  size_t epi = (size_t)BM * EpiCfg<BM, BN, NW / WM>::BNP * sizeof(float);
  if (a.pj_part) {  // RVQ in_proj epilogue: one latent split per tile, its z planes in LDS
    if (BM != 128) return VRVQ_ERR_UNSUPPORTED;
    if (epi < (size_t)PJE_LDS) epi = PJE_LDS;
  }
  const long long nblk = (long long)a.n_mt * a.n_nt * batch;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
  // bf16x3 split path (conv_x3.h): stride-1 windows, a pre-split weight, the stage in LDS
  if constexpr (NW == 4 && BM <= 192 && (KS == 1 || KS == 2 || KS == 3 || KS == 7)) {
    constexpr int XW_MAX = (BN - 1) + (KS - 1) * (KS == 7 ? 9 : 1) + 1;
    if (a.w3 != nullptr && a.stride == 1 && a.ssh == 0 && XW <= XW_MAX) {
      // pair tiles (conv_x3.h) need whole K-chunks: other Cin run the tile on plain chunks
      int rc = VRVQ_ERR_UNSUPPORTED;
      if (x3_pair<KS, BM, BN>() && a.cin % X3Cfg<KS, true>::CK == 0) {
        constexpr bool kXpf = KS == 7 && x3_pair<KS, BM, BN>();  // the 64 x 256 pair k7 tile
        if (kXpf && conv_x3_xpf())
          rc = launch_x3<BM, BN, WM, NW, KS, x3_pair<KS, BM, BN>(), false, kXpf>(a, XW, epi, nblk, st);
        else
          rc = launch_x3<BM, BN, WM, NW, KS, x3_pair<KS, BM, BN>()>(a, XW, epi, nblk, st);
      }
      else
        rc = launch_x3<BM, BN, WM, NW, KS, false>(a, XW, epi, nblk, st);
      if (rc != VRVQ_ERR_UNSUPPORTED) return rc;
    }
  }
  if (a.psh) return VRVQ_ERR_UNSUPPORTED;  // the phase-split view exists on the x3 loop only
  if (XW > 64 * WinCfg<KS, BN>::PER_ROW) return VRVQ_ERR_UNSUPPORTED;  // window > staged lanes
  size_t lds = 2 * (size_t)(CK * KS * BM + CK * XWP) * sizeof(float);
  if (lds < epi) lds = epi;  // epilogue tile
  if (lds > 160 * 1024) return VRVQ_ERR_UNSUPPORTED;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_mfma_kernel<BM, BN, WM, NW, KS, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, NW, KS, false>), dim3((unsigned)nblk),
                     dim3(64 * NW), lds, st, a);
  return vrvq_launch_status();
}



// Measured (profiles/r01j_conv_k1_ab.txt): 768 x 768 k1 + skip at T = 696, 485 -> 386 us with
// 192-row tiles (384: 930 -> 922 us); 256-row tiles for 512 / 768 were slower (248 / 473 us).
static int conv_k1_192() {  // tuning override: VRVQ_CONV_K1_192=0 (128-row) | 1 (192-row, default)
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_K1_192");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// Measured (profiles/r01j_conv_k7_ab.txt): 768 x 768 k7 at T = 696, 2150 -> 1795 us with
// 192-row x 64-col tiles (K chunk 4 channels), 427 -> 434 audio-sec/s end to end.
static int conv_k7_192() {  // tuning override: VRVQ_CONV_K7_192=0 | 1 (192-row k7 tiles at BN 64,
  static const int v = [] {  // default) | 2 (also at BN 128)
    const char* e = getenv("VRVQ_CONV_K7_192");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// Measured (profiles/r01k_convt_ab.txt): ConvT 768->384 s8 2443 -> 2345 us, 384->192 s4
// 2887 -> 2660 us with 192-row tiles; 432 -> 434 audio-sec/s.
static int conv_t_192() {  // tuning override: VRVQ_CONVT_192=0 | 1 (192-row ConvT tiles, default)
  static const int v = [] {
    const char* e = getenv("VRVQ_CONVT_192");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// T = 87 layers: the 96-wide tile (one per clip) when it gives at least this many workgroups,
// else three 32-wide tiles (tuning override VRVQ_CONV_BN96_MIN; each N tile re-streams its M
// tile's whole weight block, so the narrow tiles triple the weight traffic)
static long long conv_bn96_min() {
  static const long long v = [] {
    const char* e = getenv("VRVQ_CONV_BN96_MIN");
    return e ? atoll(e) : 384LL;
  }();
  return v;
}

// The phase-split strided convs at T <= 96 (512 -> 1024 s8 at T = 87): tile width, fixed per
// layer type (batch-invariant sums). Tuning override VRVQ_CONV_PH_T87=32 (default) | 96.
// Measured (profiles/r05zf_t87_tiles_ab.txt): 96-wide 691 -> 629 us for that layer, bench
// within the spread; the k3 layers at 96 (VRVQ_CONV_BN96_MIN=0) no faster. The layer is bound
// by its 128-chunk serial K loop per workgroup, not by the weight re-streaming alone.
static int conv_ph_t87() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_PH_T87");
    return e && atoi(e) == 96 ? 96 : 32;
  }();
  return v;
}

// x3 k7 layers over long rows (M a multiple of 64 and >= 128, Cin a multiple of 16): 64 x 256
// tiles on 16-channel "pair" K-chunks (conv_x3.h: no zero octet, 168 MFMAs per wave between
// barriers). 384 x 384 k7 at T = 5568, B = 32: 2027 -> 755-796 us (0.43 -> 0.50 of the x3
// ceiling), 256 x 256: 934 -> 781-785 us (profiles/r03_x3_pair_ab.txt).
// 768 x 768 / 512 x 512 k7 at T = 696: 1125 -> 962 / 514 -> 407 us despite 72 of every 768
// columns padded. Tuning override VRVQ_CONV_X3_WIDE=0 (128- / 192-row tiles, 8-channel
// chunks) | 1 (pair tiles for T >= 4096) | 2 (pair tiles for T >= 640, default).
static int conv_x3_wide() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_X3_WIDE");
    return e ? atoi(e) : 2;
  }();
  return v;
}

// 2-tap GEMMs at T < 4096 that the padding rule sends to 64-wide tiles run 128-wide pair tiles
// (half the weight re-streaming, 32-channel K chunks): 256 -> 512 s8 at T = 696 940 -> 878 us,
// ConvT 768 -> 384 s8 1388 -> 1296 us (profiles/r04ze_ph128_ab.txt). Tuning override
// VRVQ_CONV_PH128=1 (the strided encoder convs only) | 0 (64-wide) | 2 (default: also the
// ConvTranspose layers)
static int conv_ph128() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_PH128");
    return e ? atoi(e) : 2;
  }();
  return v;
}

static int conv_k1x3_192() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_K1X3_192");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// Split-K for the deep-K, narrow-N layers at T <= 96 (the encoder's 512 -> 1024 s8 conv, the
// importance subnet's k3 convs, the decoder's 1024 -> 1536 k7 at T = 87): their 32-wide tiles
// re-streamed every M tile's whole weight block per 32 columns (50 MB of planes x 87 column
// tiles for the s8 conv), and one 96-wide tile per clip gives too few workgroups to hide a
// 128-chunk serial K loop. Here: 128 x 96 tiles (one per clip: the weight block read once per
// clip) with the channel chunks cut into S = 4 parts (at least 8 chunks a part) -- a function of
// the layer only, so a clip's sums do not change with the batch. Per layer at B = 32
// (profiles/r06ks_splitk_sweep.txt, S = none / 2 / 3 / 4 / 6 / 8): 512 -> 1024 s8 645 / 441 /
// 469 / 445 / 462 / 455 us, 1024 -> 1024 k3 182 / 140 / 169 / 143 / 155 / 159, 1024 -> 512 k3
// 124 / 95 / 91 / 79 / 94 / 85, 512 -> 128 k3 48 -> 38 (S <= 4: 32 chunks), 1024 -> 1536 k7
// 518 / 525 / 530 / 467 / 496 / 479: S = 4 is within 1 % of the best everywhere.
// Tuning override VRVQ_CONV_SPLITK=0 (off) | S (forced part count).
static int conv_splitk_env() {
  static const int v = [] {
    const char* e = getenv("VRVQ_CONV_SPLITK");
    return e ? atoi(e) : -1;
  }();
  return v;
}

// K parts of a layer (0: none). ks = the GEMM's taps (2 for the phase-split view), cin = the
// GEMM's channels (the view's for a strided conv). The same for vrvq_conv1d_proj (the encoder's
// last conv, whose shape the ImportanceSubnet's first conv shares): its projection epilogue then
// runs in the split-K epilogue launch, on the same z bits as the plain conv's.
int splitk_parts(int M, int cin, int ng, int ks, bool psh, bool up, bool x3) {
  const int env = conv_splitk_env();
  if (env == 0 || !x3 || up || ng > 96 || M % 128 != 0) return 0;
  if (!(ks == 3 || ks == 7 || (ks == 2 && psh))) return 0;
  const int ck = ks == 2 ? X3Cfg<2, true>::CK : ks == 3 ? X3Cfg<3>::CK : X3Cfg<7>::CK;
  if (ks == 2 && cin % ck != 0) return 0;
  const int nch = (cin + ck - 1) / ck;
  int S = env > 0 ? env : 4;
  if (S > nch / 8) S = nch / 8;
  return S >= 2 ? S : 0;
}

size_t splitk_bytes(int S, int M, int ng, int batch) {
  return S ? (size_t)S * batch * (M / 128) * ((ng + 95) / 96) * 128 * 96 * sizeof(float) : 0;
}

template <int KS>
int launch_splitk(const ConvArgs& a0, int batch, int S, hipStream_t st) {
  if constexpr (KS == 2 || KS == 3 || KS == 7) {
    ConvArgs a = a0;
    a.ks_split = S;
    a.n_mt = a.M / 128;
    a.n_nt = (a.ng + 95) / 96;
      if (a.m_pad < a.n_mt * 128) return VRVQ_ERR_ARG;
    const int XW = 95 + (KS - 1) * a.dil + 1;
    constexpr int XW_MAX = 95 + (KS - 1) * (KS == 7 ? 9 : 1) + 1;
    if (XW > XW_MAX) return VRVQ_ERR_UNSUPPORTED;
    size_t epi = (size_t)128 * EpiCfg<128, 96, 1>::BNP * sizeof(float);
    if (a.pj_part && epi < (size_t)PJE_LDS) epi = PJE_LDS;
    const long long tiles = (long long)a.n_mt * a.n_nt * batch;
    if (tiles * S > 0x7fffffffLL) return VRVQ_ERR_ARG;
    const int rc = launch_x3<128, 96, 4, 4, KS, KS == 2, true>(a, XW, epi, tiles * S, st);
    if (rc) return rc;
    hipLaunchKernelGGL((conv_splitk_epilogue_kernel<128, 96, 4, 4>), dim3((unsigned)tiles),
                       dim3(256), epi, st, a);
    return vrvq_launch_status();
  } else {
    (void)a0; (void)batch; (void)S; (void)st;
    return VRVQ_ERR_UNSUPPORTED;
  }
}

// Tile choice: BM from the GEMM row count, BN minimising padded columns (prefer wide).
template <int KS>
int dispatch_tiles(const ConvArgs& a, int batch, hipStream_t st) {
  if (a.ks_part != nullptr) {
    const int S = splitk_parts(a.M, a.cin, a.ng, KS, a.psh > 0, a.up > 0, a.w3 != nullptr);
    if (S > 0) {
      const int rc = launch_splitk<KS>(a, batch, S, st);
      if (rc != VRVQ_ERR_UNSUPPORTED) return rc;
    }
  }
  auto waste = [&](int bn) { return ((a.ng + bn - 1) / bn) * bn - a.ng; };
  int bn;
  if (a.ng <= 32) bn = 32;
  else if (a.ng <= 96) {
    // T = 87 / 88 layers: one 96-wide tile per clip when that still gives >= 1.5 workgroups
    // per CU, otherwise three 32-wide tiles (more workgroups for the deep-K, narrow-N GEMMs).
    const long long blocks96 = (long long)((a.M + 127) / 128) * batch;
    bn = blocks96 >= conv_bn96_min() ? 96 : 32;
    // 2-tap x3 GEMMs: the 32-wide tile pairs its K octets (conv_x3.h x3_pair) and the 96-wide
    // one does not, so a clip's sums would change order with the batch. Their width is fixed
    // instead (batch-invariant outputs, tests/test_gpu_parity.py test_batch_invariance_*): the
    // polyphase ConvTranspose (up > 0) 96-wide, the phase-split strided convs 32-wide -- what
    // configs[1] (B = 32) ran before.
    if (KS == 2 && a.w3 != nullptr) bn = a.up > 0 ? 96 : conv_ph_t87();
  }
  // k = 16 (the stride-8 encoder convs): the 8 MB weight block does not fit in L2, so the
  // 128-wide tile's halved weight re-streaming beats its padding (1490 -> 1323 us at T = 696,
  // profiles/r02u_conv_ab.txt)
  else if (a.ng < 4096 && KS != 16 && waste(64) * 10 < waste(128) * 7)
    bn = 64;
  else bn = 128;
  if (KS == 2 && bn == 64 && a.w3 != nullptr &&
      ((a.psh > 0 && conv_ph128() >= 1) || (a.up > 0 && conv_ph128() >= 2)))
    bn = 128;
  if (KS == 2 && a.up > 0 && 128 % a.up != 0) {
    // polyphase ConvTranspose1d with a stride that does not divide 128 (3, 6): 192-row tiles,
    // which hold whole output channels; other strides (5, 7, ...) are rejected by launch_cfg
    if (bn <= 96 && bn != 64) bn = 64;
    if (bn == 64) return launch_cfg<192, 64, 2, 4, KS>(a, batch, st);
    return launch_cfg<192, 128, 2, 4, KS>(a, batch, st);
  }
  if (a.M <= 32) return launch_cfg<32, 128, 1, 4, KS>(a, batch, st);
  if constexpr (KS == 7) {
    const int wide = conv_x3_wide();
    if (a.w3 != nullptr && a.stride == 1 && a.up == 0 && a.M >= 128 && a.M % 64 == 0 &&
        a.cin % 16 == 0 && ((wide >= 1 && a.ng >= 4096) || (wide == 2 && a.ng >= 640))) {
      return launch_cfg<64, 256, 1, 4, KS>(a, batch, st);
    }
  }
  if (bn == 32) return launch_cfg<128, 32, 4, 4, KS>(a, batch, st);
  if (bn == 96) return launch_cfg<128, 96, 4, 4, KS>(a, batch, st);
  if (a.M <= 64) {
    if (bn == 64) return launch_cfg<64, 64, 2, 4, KS>(a, batch, st);
    return launch_cfg<64, 128, 2, 4, KS>(a, batch, st);
  }
  // 96- and 192-row tiles: no padded rows for the C = 96 / 192 decoder blocks
  if (a.M <= 96) {
    return launch_cfg<96, 128, 1, 4, KS>(a, batch, st);
  }
  if (KS == 7 && conv_k7_192() && a.M % 192 == 0) {
    if (bn == 64) return launch_cfg<192, 64, 2, 4, KS>(a, batch, st);
    if (conv_k7_192() == 2) return launch_cfg<192, 128, 2, 4, KS>(a, batch, st);
  }
  // (the 192-row k1 / ConvT tiles are fp32-path choices: with the x3 weights the 128-row
  // tiles, two workgroups per CU, are faster — 638 -> 649 audio-sec/s at B = 32,
  // profiles/r02zh_tile_ab.txt)
  if (KS == 2 && a.up > 0 && conv_t_192() && a.w3 == nullptr && a.M % 192 == 0) {
    // polyphase ConvTranspose1d with M = Cout * stride phase rows a multiple of 192
    if (bn == 64) return launch_cfg<192, 64, 2, 4, KS>(a, batch, st);
    return launch_cfg<192, 128, 2, 4, KS>(a, batch, st);
  }
  if (KS == 2 && a.up > 0 && a.w3 != nullptr && a.M % 96 == 0 && a.M % 128 != 0 &&
      convt_96()) {
    // x3 polyphase ConvTranspose1d with 96-row multiples (192 -> 96 s2: M = 192): 96-row
    // tiles on the pair chunks (two workgroups per CU) instead of the two-stage 192 x 128 tile
    // (single-stage 192 x 64 tiles, x read once: 981-988 vs 942-954 us, r06t_convt_layers.txt)
    return launch_cfg<96, 128, 1, 4, KS>(a, batch, st);
  }
  if ((KS >= 3 || (KS == 2 && a.up > 0)) && a.M % 128 != 0 && a.M % 192 == 0) {
    // (KS == 2 with up > 0: the polyphase ConvTranspose1d 192->96 s2, M = 192 phase rows)
    return launch_cfg<192, 128, 2, 4, KS>(a, batch, st);
  }
  if constexpr (KS == 1) {
    // x3 k1 GEMMs with M a multiple of 192 on 192 x 64 single-buffered tiles (154 VGPRs, three
    // workgroups per CU; each x column block read 2x / 4x instead of 3x / 6x): 384 x 384 at
    // T = 5568 602 -> 541 us, 768 x 768 at T = 696 253 -> 249 (profiles/r04x_k1_192_ab.txt).
    // Tuning override VRVQ_CONV_K1X3_192=0 (128-row tiles) | 1 (default)
    if (conv_k1x3_192() && a.w3 != nullptr && a.M % 192 == 0)
      return launch_cfg<192, 64, 2, 4, KS>(a, batch, st);
    // k = 1 GEMMs with M a multiple of 192 (the 384 / 768-channel ResidualUnit k1 + skip):
    // 192-row tiles read each x column block 2x / 4x instead of 3x / 6x (tuning knob)
    if (conv_k1_192() && a.w3 == nullptr && a.M % 192 == 0 && a.M % 128 == 0) {
      if (bn == 64) return launch_cfg<192, 64, 2, 4, KS>(a, batch, st);
      return launch_cfg<192, 128, 2, 4, KS>(a, batch, st);
    }
  }
  if (bn == 64) return launch_cfg<128, 64, 2, 4, KS>(a, batch, st);
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

// Pre-split weight for the x3 mainloop (conv_x3.h): from the fp32 packed layout
// wp[ci][tap][m_pad] (WNConv1d; the polyphase ConvTranspose1d layout is the same with 2 taps)
// to w3[chunk][plane][octet][m_pad][8] bf16, octet o = tap * CK/8 + channel octet (zero for
// the padding octet and channels >= cin).
template <int KS>
__global__ void pack_x3_kernel(const float* __restrict__ wp, int cin, int m_pad,
                               u32x4* __restrict__ w3, size_t total) {
  using XC = X3Cfg<KS>;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(i % m_pad);
    size_t r = i / m_pad;
    const int o = (int)(r % XC::NO2);
    r /= XC::NO2;
    const int plane = (int)(r % 3);
    const int chunk = (int)(r / 3);
    const int tap = o / XC::NC8, c8 = o - tap * XC::NC8;
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ci = chunk * XC::CK + c8 * 8 + u;
      v[u] = (o < XC::NO && ci < cin) ? wp[((size_t)ci * KS + tap) * m_pad + m] : 0.0f;
    }
    unsigned h[4], mm[4], l[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) split3x2(v[2 * u], v[2 * u + 1], h[u], mm[u], l[u]);
    w3[i] = plane == 0 ? u32x4{h[0], h[1], h[2], h[3]}
          : plane == 1 ? u32x4{mm[0], mm[1], mm[2], mm[3]} : u32x4{l[0], l[1], l[2], l[3]};
  }
}

static long long x3_size_u16(int cin, int k, int m_pad) {
  auto sz = [&](int ck, int no2) {
    return (long long)((cin + ck - 1) / ck) * 3 * no2 * m_pad * 8;
  };
  switch (k) {
    case 1: return sz(X3Cfg<1>::CK, X3Cfg<1>::NO2);
    case 2: return sz(X3Cfg<2>::CK, X3Cfg<2>::NO2);
    case 3: return sz(X3Cfg<3>::CK, X3Cfg<3>::NO2);
    case 7: return sz(X3Cfg<7>::CK, X3Cfg<7>::NO2);
    default: return -1;
  }
}

}  // namespace

extern "C" int vrvq_x3_weight_size(int cin, int k, int cout_pad, long long* n_u16) {
  VRVQ_CHECK_ARG(n_u16 && cin > 0 && cout_pad > 0);
  const long long n = x3_size_u16(cin, k, cout_pad);
  if (n < 0) return VRVQ_ERR_UNSUPPORTED;
  *n_u16 = n;
  return 0;
}

extern "C" int vrvq_pack_x3_weight(const float* w_packed, int cin, int k, int cout_pad,
                                   uint16_t* w_x3, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(w_packed && w_x3 && cin > 0 && cout_pad > 0);
  const long long n = x3_size_u16(cin, k, cout_pad);
  if (n < 0) return VRVQ_ERR_UNSUPPORTED;
  const size_t total = (size_t)n / 8;
  const unsigned grid = (unsigned)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  u32x4* out = reinterpret_cast<u32x4*>(w_x3);
  hipStream_t st = as_stream(stream);
  switch (k) {
    case 1: hipLaunchKernelGGL(pack_x3_kernel<1>, dim3(grid), dim3(256), 0, st, w_packed, cin, cout_pad, out, total); break;
    case 2: hipLaunchKernelGGL(pack_x3_kernel<2>, dim3(grid), dim3(256), 0, st, w_packed, cin, cout_pad, out, total); break;
    case 3: hipLaunchKernelGGL(pack_x3_kernel<3>, dim3(grid), dim3(256), 0, st, w_packed, cin, cout_pad, out, total); break;
    default: hipLaunchKernelGGL(pack_x3_kernel<7>, dim3(grid), dim3(256), 0, st, w_packed, cin, cout_pad, out, total); break;
  }
  return vrvq_launch_status();
}

extern "C" int vrvq_conv1d(const float* x, int batch, int cin, int tin, const float* alpha,
                           const float* inv_alpha, const float* w_packed,
                           const uint16_t* w_x3, int cout,
                           int cout_pad, int k, int stride, int pad, int dil, const float* bias,
                           const float* residual, int epilogue, float* y, int tout,
                           const float* alpha_out, const float* inv_alpha_out, float* y_snake,
                           vrvq_stream_t stream) {
  return vrvq_conv1d_ws(x, batch, cin, tin, alpha, inv_alpha, w_packed, w_x3, cout, cout_pad, k,
                        stride, pad, dil, bias, residual, epilogue, y, tout, alpha_out,
                        inv_alpha_out, y_snake, nullptr, 0, stream);
}

extern "C" int vrvq_conv1d_workspace(int batch, int cin, int tin, int cout, int k, int stride,
                                     int pad, int dil, int x3, long long* bytes) {
  VRVQ_CHECK_ARG(bytes && batch > 0 && cin > 0 && tin > 0 && cout > 0 && k > 0 && stride > 0 &&
                 dil > 0 && pad >= 0);
  const long long tout = ((long long)tin + 2LL * pad - (long long)dil * (k - 1) - 1) / stride + 1;
  VRVQ_CHECK_ARG(tout > 0);
  int S = 0;
  if (stride > 1) {  // the phase-split view (vrvq_conv1d: k = 2 stride, power-of-two stride)
    if (x3 && k == 2 * stride && (stride & (stride - 1)) == 0 && pad < stride)
      S = splitk_parts(cout, cin * stride, (int)tout, 2, true, false, true);
  } else {
    S = splitk_parts(cout, cin, (int)tout, k, false, false, x3 != 0);
  }
  *bytes = (long long)splitk_bytes(S, cout, (int)tout, batch);
  return 0;
}

extern "C" int vrvq_conv1d_ws(const float* x, int batch, int cin, int tin, const float* alpha,
                              const float* inv_alpha, const float* w_packed,
                              const uint16_t* w_x3, int cout, int cout_pad, int k, int stride,
                              int pad, int dil, const float* bias, const float* residual,
                              int epilogue, float* y, int tout, const float* alpha_out,
                              const float* inv_alpha_out, float* y_snake, void* workspace,
                              long long ws_bytes, vrvq_stream_t stream) {
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
  a.x = x; a.alpha = alpha; a.inv_alpha = inv_alpha; a.w = w_packed;
  a.bias = bias; a.res = residual; a.y = y;
  a.alpha_o = alpha_out; a.inv_alpha_o = inv_alpha_out; a.ys = y_snake;
  a.cin = cin; a.tin = tin; a.M = cout; a.m_pad = cout_pad; a.cout = cout;
  a.stride = stride; a.pad = pad; a.dil = dil; a.ng = tout; a.up = 0; a.up_pad = 0;
  a.ssh = 0;
  if (stride > 1 && (stride & (stride - 1)) == 0)
    while ((1 << a.ssh) < stride) ++a.ssh;
  a.ylen = tout; a.epi = epilogue;
  a.w3 = reinterpret_cast<const unsigned*>(w_x3);
  if (workspace != nullptr) {
    long long need = 0;
    const int rc = vrvq_conv1d_workspace(batch, cin, tin, cout, k, stride, pad, dil,
                                         w_x3 != nullptr, &need);
    if (rc) return rc;
    VRVQ_CHECK_ARG(ws_bytes >= need);
    if (need > 0) a.ks_part = static_cast<float*>(workspace);
  }
  if (w_x3 != nullptr && stride > 1) {
    // strided conv on the x3 loop: a stride-1 k = 2 conv over the phase-split view of x
    // (conv_core.h ConvArgs::psh); w_x3 holds the planes of W'[co][c*s + r][j] = W[co][c][j*s + r]
    if (k != 2 * stride || a.ssh == 0 || pad >= stride) return VRVQ_ERR_UNSUPPORTED;
    a.psh = a.ssh; a.ppad = pad; a.pcin = cin; a.ptin = tin;
    a.cin = cin * stride; a.tin = tout + 1;
    a.stride = 1; a.pad = 0; a.dil = 1; a.ssh = 0;
    return dispatch_ks(2, a, batch, as_stream(stream));
  }
  if (cout <= SMALL_COUT && stride == 1 && cin * k * (cout == 1 ? 1 : SMALL_COUT) <= SMALL_WMAX)
    return launch_small(a, batch, k, as_stream(stream));
  if (cin == 1 && k == 7 && stride == 1 && dil == 1 && !alpha && cout % CI1_CG == 0 &&
      tout % 4 == 0 && cin1_stream()) {
    const long long nblk =
        (long long)batch * ((tout + 256 * CI1_T - 1) / (256 * CI1_T)) * (cout / CI1_CG);
    if (nblk <= 0 || nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
    hipLaunchKernelGGL(conv_cin1_stream_kernel<7>, dim3((unsigned)nblk), dim3(256), 0,
                       as_stream(stream), a);
    return vrvq_launch_status();
  }
  return dispatch_ks(k, a, batch, as_stream(stream));
}

extern "C" int vrvq_conv1d_proj(const float* x, int batch, int cin, int tin, const float* alpha,
                                const float* inv_alpha, const float* w_packed,
                                const uint16_t* w_x3, int cout, int cout_pad, int k, int pad,
                                int dil, const float* bias, float* y, int tout,
                                const uint16_t* w3in, int nq, float* part, void* workspace,
                                long long ws_bytes, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && w_packed && w3in && part);
  VRVQ_CHECK_ARG(batch > 0 && cin > 0 && tin > 0 && cout > 0 && k > 0 && dil > 0 && pad >= 0 &&
                 tout > 0 && nq > 0);
  VRVQ_CHECK_ARG(cout_pad >= cout && cout_pad % 128 == 0);
  VRVQ_CHECK_ARG(alpha == nullptr || inv_alpha != nullptr);
  VRVQ_CHECK_ARG(((uintptr_t)part & 15) == 0 && ((uintptr_t)w3in & 15) == 0);
  if (cout != 1024 || nq > 32) return VRVQ_ERR_UNSUPPORTED;  // the latent (RD) / CH_NQMAX
  const long long expect = (long long)tin + 2LL * pad - (long long)dil * (k - 1);
  VRVQ_CHECK_ARG(expect == tout);
  VRVQ_CHECK_ARG((long long)batch * tout * nq * 8 * 8 < 0x7fffffffLL);
  ConvArgs a{};
  a.x = x; a.alpha = alpha; a.inv_alpha = inv_alpha; a.w = w_packed; a.bias = bias; a.y = y;
  a.cin = cin; a.tin = tin; a.M = cout; a.m_pad = cout_pad; a.cout = cout;
  a.stride = 1; a.pad = pad; a.dil = dil; a.ng = tout; a.up = 0; a.up_pad = 0; a.ssh = 0;
  a.ylen = tout; a.epi = VRVQ_EPI_NONE;
  a.w3 = reinterpret_cast<const unsigned*>(w_x3);
  a.pj_w3 = reinterpret_cast<const unsigned*>(w3in);
  a.pj_part = part;
  a.pj_nq = nq;
  a.pj_nf = batch * tout;
  if (workspace != nullptr) {  // split-K as vrvq_conv1d_ws (same shape, same parts)
    long long need = 0;
    const int rc = vrvq_conv1d_workspace(batch, cin, tin, cout, k, 1, pad, dil, w_x3 != nullptr,
                                         &need);
    if (rc) return rc;
    VRVQ_CHECK_ARG(ws_bytes >= need);
    if (need > 0) a.ks_part = static_cast<float*>(workspace);
  }
  // the MFMA tiles only (their epilogue owns the projection); every 1024-row tile is 128 rows
  return dispatch_ks(k, a, batch, as_stream(stream));
}

extern "C" int vrvq_conv_transpose1d(const float* x, int batch, int cin, int tin,
                                     const float* alpha, const float* inv_alpha,
                                     const float* w_packed, int cout, int cout_pad, int stride,
                                     const float* bias, float* y, const float* alpha_out,
                                     const float* inv_alpha_out, float* y_snake,
                                     vrvq_stream_t stream) {
  // math.ceil(stride / 2), models/layers.py:102
  return vrvq_conv_transpose1d_pad(x, batch, cin, tin, alpha, inv_alpha, w_packed, nullptr,
                                   cout, cout_pad, stride, (stride + 1) / 2, bias, y, alpha_out,
                                   inv_alpha_out, y_snake, stream);
}

extern "C" int vrvq_conv_transpose1d_pad(const float* x, int batch, int cin, int tin,
                                         const float* alpha, const float* inv_alpha,
                                         const float* w_packed, const uint16_t* w_x3,
                                         int cout, int cout_pad,
                                         int stride, int pad, const float* bias, float* y,
                                         const float* alpha_out, const float* inv_alpha_out,
                                         float* y_snake, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && w_packed && (y || y_snake));
  VRVQ_CHECK_ARG(y_snake == nullptr || (alpha_out && inv_alpha_out));
  VRVQ_CHECK_ARG(batch > 0 && cin > 0 && tin > 0 && cout > 0 && stride > 0);
  // pad 0 = the padding=False windows of the chunked codec (models/dac_base.py:72-82)
  VRVQ_CHECK_ARG(pad >= 0 && pad < stride);
  VRVQ_CHECK_ARG(cout_pad >= cout * stride && cout_pad % 64 == 0);
  VRVQ_CHECK_ARG(alpha == nullptr || inv_alpha != nullptr);
  const int p = pad;
  ConvArgs a{};
  a.x = x; a.alpha = alpha; a.inv_alpha = inv_alpha; a.w = w_packed; a.bias = bias;
  a.res = nullptr; a.y = y;
  a.alpha_o = alpha_out; a.inv_alpha_o = inv_alpha_out; a.ys = y_snake;
  a.cin = cin; a.tin = tin; a.M = cout * stride; a.m_pad = cout_pad; a.cout = cout;
  a.stride = 1; a.pad = 1; a.dil = 1; a.ng = tin + 1; a.up = stride; a.up_pad = p;
  a.ylen = (tin - 1) * stride - 2 * p + 2 * stride;
  a.epi = VRVQ_EPI_NONE;
  a.w3 = reinterpret_cast<const unsigned*>(w_x3);
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
