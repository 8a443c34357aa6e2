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

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

struct ConvArgs {
  const float* x;          // [B][cin][tin]
  const float* alpha;      // [cin] or null
  const float* inv_alpha;  // [cin]
  const float* w;          // [cin][KS][m_pad]
  const float* bias;       // [cout] or null
  const float* res;        // [B][cout][ylen] or null
  float* y;                // [B][cout][ylen]
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

template <int BM, int BN, int WM, int KS>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM;
  constexpr int TN = BN / WN;
  constexpr int RM = TM / 32;
  constexpr int RN = TN / 32;
  constexpr int CK = ChunkCfg<KS, BM>::CK;
  constexpr int KROWS = CK * KS;
  constexpr int WQ4 = KROWS * BM / 4;               // float4 of W per chunk
  constexpr int WQ = (WQ4 + 255) / 256;             // ... per thread
  constexpr int XROWS = CK / 4;                     // x rows per wave per chunk
  constexpr int XPR = WinCfg<KS, BN>::PER_ROW;
  static_assert(RM >= 1 && RN >= 1 && TM % 32 == 0 && TN % 32 == 0, "tile");
  static_assert(CK % 4 == 0, "chunk shape");

  // Two LDS stages: [W chunk | x window] x 2. The next chunk is prefetched into registers
  // while the current one feeds the MFMAs, then written (with Snake) to the other stage:
  // one barrier per K-chunk.
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

  float4 wreg[WQ];
  float xreg[XROWS][XPR];

  auto load_chunk = [&](int ci0) {
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int idx = tid + q * 256;
      const int rr = idx / (BM / 4);
      const int cc = (idx - rr * (BM / 4)) * 4;
      wreg[q] = (idx < WQ4 && ci0 + rr / KS < a.cin)
                    ? *reinterpret_cast<const float4*>(a.w + (size_t)(ci0 * KS + rr) * a.m_pad + m0 + cc)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int rw = 0; rw < XROWS; ++rw) {
      const int ci = ci0 + wave + 4 * rw;
      const float* xr = xb + (size_t)ci * a.tin;
#pragma unroll
      for (int u = 0; u < XPR; ++u) {
        const int p = lane + 64 * u;
        const int t = xbase + p;
        xreg[rw][u] = (ci < a.cin && p < XW && t >= 0 && t < a.tin) ? xr[t] : 0.0f;
      }
    }
  };
  auto store_chunk = [&](float* stg, int ci0) {
    float* ws = stg;
    float* xs = stg + KROWS * BM;
#pragma unroll
    for (int q = 0; q < WQ; ++q)
      if (tid + q * 256 < WQ4) reinterpret_cast<float4*>(ws)[tid + q * 256] = wreg[q];
#pragma unroll
    for (int rw = 0; rw < XROWS; ++rw) {
      const int cl = wave + 4 * rw;
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
#pragma unroll
    for (int k = 0; k < KS; ++k) {
#pragma unroll
      for (int cc = 0; cc < CK; cc += 2) {
        const int kr = cc + lh;
        float av[RM], bv[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) av[i] = ws[(kr * KS + k) * BM + wm * TM + i * 32 + lr];
        const int col = wn * TN + lr;
        const int xo = a.ssh ? kr * XWP + (k & (a.stride - 1)) * XP + col + (k >> a.ssh)
                             : kr * XWP + col + k * a.dil;
#pragma unroll
        for (int j = 0; j < RN; ++j) bv[j] = xs[xo + j * 32];
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store_chunk(smem + (cur ^ 1) * STG, ci0 + CK);
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue: bias, residual, activation, store ----
  // Per accumulator tile: every load (bias, residual) is issued before any store, so the
  // 16 round trips overlap instead of serialising behind possibly-aliasing stores.
  if (a.up == 0) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int mb = m0 + wm * TM + i * 32 + 4 * lh;
      float bv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + (r & 3) + 8 * (r >> 2);
        bv[r] = (a.bias && m < a.M) ? a.bias[m] : 0.0f;
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = n0 + wn * TN + j * 32 + lr;
        const size_t ob = ((size_t)b * a.cout + mb) * a.ylen + n;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[i][j][r] + bv[r];
        if (a.res) {
          float rv[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mo = (r & 3) + 8 * (r >> 2);
            rv[r] = (mb + mo < a.M && n < a.ng) ? a.res[ob + (size_t)mo * a.ylen] : 0.0f;
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = rv[r] + v[r];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mo = (r & 3) + 8 * (r >> 2);
          if (mb + mo < a.M && n < a.ng) a.y[ob + (size_t)mo * a.ylen] = apply_epi(v[r], a.epi);
        }
      }
    }
  } else {
    // transposed conv: GEMM row m = co*up + phase, output t = n*up + phase - up_pad
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int mb = m0 + wm * TM + i * 32 + 4 * lh;
      int cor[16], phr[16];
      float bv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + (r & 3) + 8 * (r >> 2);
        const int co = m / a.up;
        cor[r] = m < a.M ? co : -1;
        phr[r] = m - co * a.up - a.up_pad;
        bv[r] = (a.bias && m < a.M) ? a.bias[co] : 0.0f;
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = n0 + wn * TN + j * 32 + lr;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int t = n * a.up + phr[r];
          if (cor[r] >= 0 && n < a.ng && t >= 0 && t < a.ylen)
            a.y[((size_t)b * a.cout + cor[r]) * a.ylen + t] = acc[i][j][r] + bv[r];
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
        a.y[o] = apply_epi(v, a.epi);
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

template <int BM, int BN, int WM, int KS>
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
  const size_t lds = 2 * (size_t)(CK * KS * BM + CK * XWP) * sizeof(float);
  if (lds > 160 * 1024) return VRVQ_ERR_UNSUPPORTED;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_mfma_kernel<BM, BN, WM, KS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  const long long nblk = (long long)a.n_mt * a.n_nt * batch;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
  hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, KS>), dim3((unsigned)nblk), dim3(256), lds,
                     st, a);
  return vrvq_launch_status();
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
  if (a.M <= 32) return launch_cfg<32, 128, 1, KS>(a, batch, st);
  if (bn == 32) return launch_cfg<128, 32, 4, KS>(a, batch, st);
  if (bn == 96) return launch_cfg<128, 96, 4, KS>(a, batch, st);
  if (a.M <= 64) {
    if (bn == 64) return launch_cfg<64, 64, 2, KS>(a, batch, st);
    return launch_cfg<64, 128, 2, KS>(a, batch, st);
  }
  // 96- and 192-row tiles: no padded rows for the C = 96 / 192 decoder blocks
  if (a.M <= 96) return launch_cfg<96, 128, 1, KS>(a, batch, st);
  if (KS >= 3 && a.M % 128 != 0 && a.M % 192 == 0) return launch_cfg<192, 128, 2, KS>(a, batch, st);
  if (bn == 64) return launch_cfg<128, 64, 2, KS>(a, batch, st);
  return launch_cfg<128, 128, 2, KS>(a, batch, st);
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
                           vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && w_packed && y);
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
                                     const float* bias, float* y, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && w_packed && y);
  VRVQ_CHECK_ARG(batch > 0 && cin > 0 && tin > 0 && cout > 0 && stride > 0);
  VRVQ_CHECK_ARG(cout_pad >= cout * stride && cout_pad % 128 == 0);
  VRVQ_CHECK_ARG(alpha == nullptr || inv_alpha != nullptr);
  const int p = (stride + 1) / 2;  // math.ceil(stride / 2), models/layers.py:102
  ConvArgs a{};
  a.x = x; a.alpha = alpha; a.inv_alpha = inv_alpha; a.w = w_packed; a.bias = bias;
  a.res = nullptr; a.y = y;
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
