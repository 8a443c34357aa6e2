// Backward kernels of the VRVQ generator (the training step, SURVEY.md §8f row 1;
// scripts/train.py:262-335): weight gradients of the Snake-fused convolutions, Snake /
// activation / bias / weight-norm backward, and the adjoint-conv weight packing that lets the
// input gradient reuse the forward MFMA conv kernels (conv.hip):
//   Conv1d (stride 1, dilation d):   dXs = conv1d(dY, W^flip, pad' = d (K-1) - pad)
//   Conv1d (k = 2s, stride s):       dXs = conv_transpose1d(dY, W) (the polyphase kernel)
//   ConvTranspose1d (k = 2s):        dXs = conv1d(dY, W, stride s, pad)
// Every reduction is deterministic (fixed order; split-K partials summed in split order).
#include "common.h"
#include "conv_x3.h"  // split3x2 / mfma_bf16: the x3 (split bf16) products of the forward convs

namespace {

// ------------------------------------------------------------------------------------------
// Weight gradient as a split-K GEMM on v_mfma_f32_32x32x2_f32:
//   out[m][c][k] = sum_b sum_{t < TA} A[b][m][t] * Xs[b][c][t*s - p + k*d]
//   Xs = snake(X) when alpha != NULL (the layer's input activation), 0 outside [0, TX)
//   As = snake(A) when alpha_a != NULL
// Conv1d:          A = dY (m = Cout), X = the layer input (c = Cin)   -> dW[Cout][Cin][K]
// ConvTranspose1d: A = the layer input (m = Cin, snake on A), X = dY  -> dW[Cin][Cout][K]
//                  (y[co][t s - p + k] += W[ci][co][k] xs[ci][t])
// Workgroup = (64 m x 64 c tile, tap k, split); 4 waves of 32 x 32; K_red chunks of 32
// (b, t) values staged in LDS; partial[split][m][c][k] reduced in split order afterwards.
constexpr int WG_BM = 64, WG_BN = 64;
constexpr int WG_WMAX = 192;           // X-window samples per staged row

struct WgradArgs {
  const float* A; int M, TA;
  const float* X; int C, TX;
  const float* alpha_a; const float* inv_alpha_a;
  const float* alpha; const float* inv_alpha;
  int B, K, s, p, d;
  int n_split, chunks;   // (clip, time chunk) units, split evenly over n_split
  int kt_sh, W, WP, n_kg;  // log2 time chunk, window, padded row stride (odd), tap groups
  float* part;           // [n_split][M][C][K]
};

// Workgroup = (64 m x 64 c tile, group of KG taps, split). Per (clip, KT-sample) chunk the
// A rows [64][KT] and the X window [64 channels][(KT-1) s + (KG-1) d + 1] are staged once in
// LDS (snake applied while staging) and every tap of the group reads its shifted view of the
// window: 4 waves of 32 x 32 on v_mfma_f32_32x32x2_f32, KG accumulators each. Row strides are
// odd (conflict-free reads).
template <int KG>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradArgs a) {
  extern __shared__ float wsm[];
  const int KT = 1 << a.kt_sh;
  float* A_s = wsm;                    // [64][KT + 1]
  float* X_s = wsm + 64 * (KT + 1);    // [64][WP]
  const int n_mt = (a.M + WG_BM - 1) / WG_BM, n_ct = (a.C + WG_BN - 1) / WG_BN;
  int bid = blockIdx.x;
  const int mt = bid % n_mt; bid /= n_mt;
  const int ct = bid % n_ct; bid /= n_ct;
  const int kg = bid % a.n_kg;
  const int sp = bid / a.n_kg;
  const int m0 = mt * WG_BM, c0 = ct * WG_BN, k0 = kg * KG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int nct = (a.TA + KT - 1) >> a.kt_sh;
  const int q0 = (int)((long long)sp * a.chunks / a.n_split);
  const int q1 = (int)((long long)(sp + 1) * a.chunks / a.n_split);
  // staging: wave w fills A rows and X-window rows w, w+4, ... (16 each), in two halves of 8
  // rows: every load of a half is issued before its first LDS store (no per-row load -> store
  // round trips; the half bounds the registers), lanes walk the rows (coalesced), snake applied
  // between the loads and the stores.
  constexpr int NA = 8 * 64 / 64;       // A values per lane per half (KT <= 64)
  constexpr int NU = WG_WMAX / 64;      // X-window segments of 64 per row
  auto stage = [&](int q) {
    const int b = q / nct, t0 = (q - b * nct) << a.kt_sh;
    const int xb = t0 * a.s - a.p + k0 * a.d;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      float av[NA], xv[8][NU];
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = lane + 64 * i;
        const int r = wave + 4 * (8 * h + (e >> a.kt_sh)), j = e & (KT - 1);
        const int m = m0 + r, t = t0 + j;
        av[i] = (e < 8 * KT && m < a.M && t < a.TA) ? a.A[((size_t)b * a.M + m) * a.TA + t]
                                                    : 0.0f;
      }
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int c = c0 + wave + 4 * (8 * h + rr);
        const float* xr = a.X + ((size_t)b * a.C + (c < a.C ? c : 0)) * a.TX;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int pp = lane + 64 * u, tx = xb + pp;
          xv[rr][u] = (pp < a.W && c < a.C && tx >= 0 && tx < a.TX) ? xr[tx] : 0.0f;
        }
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int e = lane + 64 * i;
        if (e < 8 * KT) {
          const int r = wave + 4 * (8 * h + (e >> a.kt_sh)), j = e & (KT - 1);
          float v = av[i];
          if (a.alpha_a && m0 + r < a.M)
            v = snake_act(v, a.alpha_a[m0 + r], a.inv_alpha_a[m0 + r]);
          A_s[r * (KT + 1) + j] = v;
        }
      }
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int r = wave + 4 * (8 * h + rr), c = c0 + r;
        const bool sn = a.alpha && c < a.C;
        const float cl = sn ? a.alpha[c] : 0.0f, icl = sn ? a.inv_alpha[c] : 0.0f;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int pp = lane + 64 * u;
          if (pp < a.W) X_s[r * a.WP + pp] = sn ? snake_act(xv[rr][u], cl, icl) : xv[rr][u];
        }
      }
    }
  };
  f32x16 acc[KG];
#pragma unroll
  for (int kk = 0; kk < KG; ++kk)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[kk][r] = 0.0f;
  const float* arow = A_s + (wm * 32 + (lane & 31)) * (KT + 1) + (lane >> 5);
  const float* xrow = X_s + (wn * 32 + (lane & 31)) * a.WP + (lane >> 5) * a.s;
  for (int q = q0; q < q1; ++q) {
    stage(q);
    __syncthreads();
    // 32x32x2: A lane l -> A[m = l & 31][kr = l >> 5]; B lane l -> B[kr = l >> 5][n = l & 31]
    for (int tp = 0; tp < KT; tp += 2) {
      const float av = arow[tp];
      const float* xr = xrow + tp * a.s;
#pragma unroll
      for (int kk = 0; kk < KG; ++kk)
        acc[kk] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, xr[kk * a.d], acc[kk], 0, 0, 0);
    }
    __syncthreads();
  }
  // D: lane l, reg r -> row (r & 3) + 8 (r >> 2) + 4 (l >> 5), col l & 31
#pragma unroll
  for (int kk = 0; kk < KG; ++kk)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int c = c0 + wn * 32 + (lane & 31);
      if (m < a.M && c < a.C && k0 + kk < a.K)
        a.part[(((size_t)sp * a.M + m) * a.C + c) * a.K + k0 + kk] = acc[kk][r];
    }
}

// Weight gradient of the stride-1 convs on the split bf16 MFMA (the forward convs' "x3"
// products, conv_x3.h): both operands split exactly into three bf16 terms, six
// v_mfma_f32_32x32x16_bf16 per 16 time samples (m m, h l, l h, h m, m h, then h h), fp32
// accumulation -- fp32-accurate (dropped terms <= 2^-23 |ab|) at 2.7x the fp32 MFMA ceiling.
// Same workgroup geometry and split-K order as wgrad_kernel: (64 m x 64 c tile, KG taps, split),
// 64-sample time chunks. Both operands are staged pre-split, once per chunk: A rows as
// [3 planes][64][72] bf16 (16-byte rows), the X window as [3 planes][64][XPW] bf16 (odd dword
// stride). A tap's B operand is 8 consecutive samples from an offset of any parity: 4 dwords per
// plane when the tap shift k d is even, else 5 dwords re-aligned by 16 bits (v_alignbit) -- the
// same bf16 planes the per-tap split in registers produced, for a fraction of the VALU.
constexpr int WX_KT = 64;
constexpr int WX_ALD = WX_KT + 8;  // bf16 per A-plane row (144 B)

__host__ __device__ inline int wx_xpw(int w) {  // bf16 per X-plane row: >= w + 2, odd dwords
  const int dw = (w + 3) / 2;
  return 2 * (dw | 1);
}

template <int KG>
__global__ __launch_bounds__(256, 2) void wgrad_x3_kernel(WgradArgs a) {
  using namespace vrvq_conv;
  extern __shared__ float wsm[];
  unsigned* A3 = reinterpret_cast<unsigned*>(wsm);       // [3][64][WX_ALD / 2] bf16 pairs
  unsigned* X3 = A3 + 3 * 64 * WX_ALD / 2;               // [3][64][XPW / 2] bf16 pairs
  const int XD = wx_xpw(a.W) / 2;                         // dwords per X-plane row
  const int n_mt = (a.M + WG_BM - 1) / WG_BM, n_ct = (a.C + WG_BN - 1) / WG_BN;
  int bid = blockIdx.x;
  const int mt = bid % n_mt; bid /= n_mt;
  const int ct = bid % n_ct; bid /= n_ct;
  const int kg = bid % a.n_kg;
  const int sp = bid / a.n_kg;
  const int m0 = mt * WG_BM, c0 = ct * WG_BN, k0 = kg * KG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int nct = (a.TA + WX_KT - 1) / WX_KT;
  const int q0 = (int)((long long)sp * a.chunks / a.n_split);
  const int q1 = (int)((long long)(sp + 1) * a.chunks / a.n_split);
  constexpr int NU2 = (WG_WMAX + 127) / 128;  // sample pairs per lane and X row
  // staging in two halves (32 A rows, 32 X-window rows, both as sample pairs), every load of a
  // half before its stores, snake and the bf16 split between them
  auto stage = [&](int q) {
    const int b = q / nct, t0 = (q - b * nct) * WX_KT;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      float av[4][2], xv[8][NU2][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = tid + 256 * i, r = 32 * h + (e >> 5), j = (e & 31) * 2;
        const int m = m0 + r;
        const float* ap = a.A + ((size_t)b * a.M + min(m, a.M - 1)) * a.TA;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int t = t0 + j + u;
          av[i][u] = (m < a.M && t < a.TA) ? ap[min(t, a.TA - 1)] : 0.0f;
        }
      }
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int c = c0 + wave + 4 * (8 * h + rr);
        const float* xr = a.X + ((size_t)b * a.C + (c < a.C ? c : 0)) * a.TX;
#pragma unroll
        for (int u = 0; u < NU2; ++u)
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const int pp = 2 * (lane + 64 * u) + v, tx = t0 - a.p + k0 * a.d + pp;
            xv[rr][u][v] = (pp < a.W && c < a.C && tx >= 0 && tx < a.TX) ? xr[tx] : 0.0f;
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = tid + 256 * i, r = 32 * h + (e >> 5), j = (e & 31) * 2;
        float v0 = av[i][0], v1 = av[i][1];
        if (a.alpha_a && m0 + r < a.M) {
          v0 = snake_act(v0, a.alpha_a[m0 + r], a.inv_alpha_a[m0 + r]);
          v1 = snake_act(v1, a.alpha_a[m0 + r], a.inv_alpha_a[m0 + r]);
        }
        unsigned hh, mm, ll;
        split3x2(v0, v1, hh, mm, ll);
        const int o = r * (WX_ALD / 2) + j / 2;
        A3[o] = hh;
        A3[64 * (WX_ALD / 2) + o] = mm;
        A3[2 * 64 * (WX_ALD / 2) + o] = ll;
      }
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int r = wave + 4 * (8 * h + rr), c = c0 + r;
        const bool sn = a.alpha && c < a.C;
        const float cl = sn ? a.alpha[c] : 0.0f, icl = sn ? a.inv_alpha[c] : 0.0f;
#pragma unroll
        for (int u = 0; u < NU2; ++u) {
          const int pw = lane + 64 * u;  // pair index
          if (2 * pw < a.W) {
            float v0 = xv[rr][u][0], v1 = xv[rr][u][1];
            if (sn) {
              v0 = snake_act(v0, cl, icl);
              v1 = snake_act(v1, cl, icl);
            }
            unsigned hh, mm, ll;
            split3x2(v0, v1, hh, mm, ll);
            X3[r * XD + pw] = hh;
            X3[(64 + r) * XD + pw] = mm;
            X3[(128 + r) * XD + pw] = ll;
          }
        }
      }
    }
  };
  f32x16 acc[KG];
#pragma unroll
  for (int kk = 0; kk < KG; ++kk)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[kk][r] = 0.0f;
  const u32x4* arow = reinterpret_cast<const u32x4*>(A3 + (wm * 32 + lr) * (WX_ALD / 2)) + lh;
  const unsigned* xrow = X3 + (wn * 32 + lr) * XD + 4 * lh;  // sample 8 lh of row wn 32 + lr
  for (int q = q0; q < q1; ++q) {
    stage(q);
    __syncthreads();
    // 32x32x16 bf16: lane l holds A[m = l & 31][k = 8 (l >> 5) .. +7] and B[k][c = l & 31]
#pragma unroll 1
    for (int tp = 0; tp < WX_KT; tp += 16) {
      const u32x4 ah = arow[tp / 8], am = arow[64 * (WX_ALD / 8) + tp / 8],
                  al = arow[2 * 64 * (WX_ALD / 8) + tp / 8];
#pragma unroll
      for (int kk = 0; kk < KG; ++kk) {
        const int sh = kk * a.d;                       // tap shift (wave-uniform)
        const unsigned* xp = xrow + (tp + sh) / 2;
        u32x4 bp[3];
        if ((sh & 1) == 0) {
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const unsigned* r = xp + p * 64 * XD;
            bp[p] = u32x4{r[0], r[1], r[2], r[3]};
          }
        } else {
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const unsigned* r = xp + p * 64 * XD;
            const unsigned d0 = r[0], d1 = r[1], d2 = r[2], d3 = r[3], d4 = r[4];
            bp[p] = u32x4{__builtin_amdgcn_alignbit(d1, d0, 16), __builtin_amdgcn_alignbit(d2, d1, 16),
                          __builtin_amdgcn_alignbit(d3, d2, 16), __builtin_amdgcn_alignbit(d4, d3, 16)};
          }
        }
        f32x16 t = acc[kk];
        t = mfma_bf16(am, bp[1], t);  // m m
        t = mfma_bf16(ah, bp[2], t);  // h l
        t = mfma_bf16(al, bp[0], t);  // l h
        t = mfma_bf16(ah, bp[1], t);  // h m
        t = mfma_bf16(am, bp[0], t);  // m h
        acc[kk] = mfma_bf16(ah, bp[0], t);  // h h
      }
    }
    __syncthreads();
  }
  // D: lane l, reg r -> row (r & 3) + 8 (r >> 2) + 4 (l >> 5), col l & 31
#pragma unroll
  for (int kk = 0; kk < KG; ++kk)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int c = c0 + wn * 32 + lr;
      if (m < a.M && c < a.C && k0 + kk < a.K)
        a.part[(((size_t)sp * a.M + m) * a.C + c) * a.K + k0 + kk] = acc[kk][r];
    }
}

// The 1x1 form (KG = 1): X staged fp32 and each 8-sample B operand split in registers -- with
// one tap per staged window, splitting while staging buys nothing and costs a third LDS plane.
template <int KG>
__global__ __launch_bounds__(256, 2) void wgrad_x3_reg_kernel(WgradArgs a) {
  using namespace vrvq_conv;
  extern __shared__ float wsm[];
  unsigned* A3 = reinterpret_cast<unsigned*>(wsm);       // [3][64][WX_ALD / 2] bf16 pairs
  float* X_s = wsm + 3 * 64 * WX_ALD / 2;                // [64][WP]
  const int n_mt = (a.M + WG_BM - 1) / WG_BM, n_ct = (a.C + WG_BN - 1) / WG_BN;
  int bid = blockIdx.x;
  const int mt = bid % n_mt; bid /= n_mt;
  const int ct = bid % n_ct; bid /= n_ct;
  const int kg = bid % a.n_kg;
  const int sp = bid / a.n_kg;
  const int m0 = mt * WG_BM, c0 = ct * WG_BN, k0 = kg * KG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int nct = (a.TA + WX_KT - 1) / WX_KT;
  const int q0 = (int)((long long)sp * a.chunks / a.n_split);
  const int q1 = (int)((long long)(sp + 1) * a.chunks / a.n_split);
  constexpr int NU = WG_WMAX / 64;
  // staging in two halves (32 A rows as pairs, 32 X-window rows), every load of a half before
  // its stores, snake and the bf16 split between them
  auto stage = [&](int q) {
    const int b = q / nct, t0 = (q - b * nct) * WX_KT;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      float av[4][2], xv[8][NU];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = tid + 256 * i, r = 32 * h + (e >> 5), j = (e & 31) * 2;
        const int m = m0 + r;
        const float* ap = a.A + ((size_t)b * a.M + min(m, a.M - 1)) * a.TA;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int t = t0 + j + u;
          av[i][u] = (m < a.M && t < a.TA) ? ap[min(t, a.TA - 1)] : 0.0f;
        }
      }
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int c = c0 + wave + 4 * (8 * h + rr);
        const float* xr = a.X + ((size_t)b * a.C + (c < a.C ? c : 0)) * a.TX;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int pp = lane + 64 * u, tx = t0 - a.p + k0 * a.d + pp;
          xv[rr][u] = (pp < a.W && c < a.C && tx >= 0 && tx < a.TX) ? xr[tx] : 0.0f;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = tid + 256 * i, r = 32 * h + (e >> 5), j = (e & 31) * 2;
        float v0 = av[i][0], v1 = av[i][1];
        if (a.alpha_a && m0 + r < a.M) {
          v0 = snake_act(v0, a.alpha_a[m0 + r], a.inv_alpha_a[m0 + r]);
          v1 = snake_act(v1, a.alpha_a[m0 + r], a.inv_alpha_a[m0 + r]);
        }
        unsigned hh, mm, ll;
        split3x2(v0, v1, hh, mm, ll);
        const int o = r * (WX_ALD / 2) + j / 2;
        A3[o] = hh;
        A3[64 * (WX_ALD / 2) + o] = mm;
        A3[2 * 64 * (WX_ALD / 2) + o] = ll;
      }
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int r = wave + 4 * (8 * h + rr), c = c0 + r;
        const bool sn = a.alpha && c < a.C;
        const float cl = sn ? a.alpha[c] : 0.0f, icl = sn ? a.inv_alpha[c] : 0.0f;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int pp = lane + 64 * u;
          if (pp < a.W) X_s[r * a.WP + pp] = sn ? snake_act(xv[rr][u], cl, icl) : xv[rr][u];
        }
      }
    }
  };
  f32x16 acc[KG];
#pragma unroll
  for (int kk = 0; kk < KG; ++kk)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[kk][r] = 0.0f;
  const u32x4* arow = reinterpret_cast<const u32x4*>(A3 + (wm * 32 + lr) * (WX_ALD / 2)) + lh;
  const float* xrow = X_s + (wn * 32 + lr) * a.WP + 8 * lh;
  for (int q = q0; q < q1; ++q) {
    stage(q);
    __syncthreads();
    // 32x32x16 bf16: lane l holds A[m = l & 31][k = 8 (l >> 5) .. +7] and B[k][c = l & 31]
#pragma unroll 1
    for (int tp = 0; tp < WX_KT; tp += 16) {
      const u32x4 ah = arow[tp / 8], am = arow[64 * (WX_ALD / 8) + tp / 8],
                  al = arow[2 * 64 * (WX_ALD / 8) + tp / 8];
#pragma unroll
      for (int kk = 0; kk < KG; ++kk) {
        const float* xp = xrow + tp + kk * a.d;
        unsigned bh[4], bm[4], bl[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) split3x2(xp[2 * u], xp[2 * u + 1], bh[u], bm[u], bl[u]);
        const u32x4 h = {bh[0], bh[1], bh[2], bh[3]}, m = {bm[0], bm[1], bm[2], bm[3]},
                    l = {bl[0], bl[1], bl[2], bl[3]};
        f32x16 t = acc[kk];
        t = mfma_bf16(am, m, t);  // m m
        t = mfma_bf16(ah, l, t);  // h l
        t = mfma_bf16(al, h, t);  // l h
        t = mfma_bf16(ah, m, t);  // h m
        t = mfma_bf16(am, h, t);  // m h
        acc[kk] = mfma_bf16(ah, h, t);  // h h
      }
    }
    __syncthreads();
  }
  // D: lane l, reg r -> row (r & 3) + 8 (r >> 2) + 4 (l >> 5), col l & 31
#pragma unroll
  for (int kk = 0; kk < KG; ++kk)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int c = c0 + wn * 32 + lr;
      if (m < a.M && c < a.C && k0 + kk < a.K)
        a.part[(((size_t)sp * a.M + m) * a.C + c) * a.K + k0 + kk] = acc[kk][r];
    }
}

// out[e] = sum_{s < n} part[s][e], split order
__global__ void split_reduce_kernel(const float* __restrict__ part, size_t n_elem, int n_split,
                                    float* __restrict__ out) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_elem;
       e += (size_t)gridDim.x * blockDim.x) {
    float acc = part[e];
    for (int s = 1; s < n_split; ++s) acc = acc + part[(size_t)s * n_elem + e];
    out[e] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// Snake backward (models/layers.py:26-32 under torch autograd):
//   y = x + inv * sin(a x)^2,  inv = 1 / (a + 1e-9)
//   dx = g * (1 + inv * (2 sin(a x) cos(a x)) * a)
//   da = sum_{b,t} g * (-inv^2 * sin(a x)^2 + inv * (2 sin(a x) cos(a x)) * x)
// Workgroup = (channel c, split q = (clip b, time chunk of RCH)): coalesced row segments, no
// per-element index division; dalpha partials [n_split][C] reduced in split order.
constexpr int RCH = 4096;  // time samples per split

__global__ __launch_bounds__(256) void snake_backward_kernel(
    const float* __restrict__ x, const float* __restrict__ alpha,
    const float* __restrict__ inv_alpha, const float* __restrict__ g, int B, int C, int T,
    int n_split, float* __restrict__ dx, float* __restrict__ da_part) {
  __shared__ float red[256];
  const int c = blockIdx.x % C, q = blockIdx.x / C;
  const int ntc = (T + RCH - 1) / RCH;
  const int b = q / ntc, t0 = (q - b * ntc) * RCH, t1 = min(T, t0 + RCH);
  const float a = alpha[c], inv = inv_alpha[c];
  const size_t row = ((size_t)b * C + c) * T;
  float acc = 0.0f;
  for (int t = t0 + threadIdx.x; t < t1; t += 256) {
    const float xv = x[row + t], gv = g[row + t];
    float sn, cs;
    sincos_reduced(a * xv, &sn, &cs);
    const float s2 = (2.0f * sn) * cs;
    if (dx) dx[row + t] = gv * (1.0f + (inv * s2) * a);
    acc += gv * (-(inv * inv) * (sn * sn) + (inv * s2) * xv);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int h = 128; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0 && da_part) da_part[(size_t)q * C + c] = red[0];
}

// db partials: workgroup (channel, split) as above, sum of g over the chunk
__global__ __launch_bounds__(256) void bias_grad_kernel(const float* __restrict__ g, int B, int C,
                                                        int T, float* __restrict__ part) {
  __shared__ float red[256];
  const int c = blockIdx.x % C, q = blockIdx.x / C;
  const int ntc = (T + RCH - 1) / RCH;
  const int b = q / ntc, t0 = (q - b * ntc) * RCH, t1 = min(T, t0 + RCH);
  const float* gr = g + ((size_t)b * C + c) * T;
  float acc = 0.0f;
  for (int t = t0 + threadIdx.x; t < t1; t += 256) acc += gr[t];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int h = 128; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)q * C + c] = red[0];
}

// tanh / sigmoid backward from the stored output y (models/dac_vrvq.py:74,
// models/importance_subnet.py:44)
__global__ void act_backward_kernel(const float* __restrict__ y, const float* __restrict__ g,
                                    size_t n, int epi, float* __restrict__ out) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
       e += (size_t)gridDim.x * blockDim.x) {
    const float yv = y[e], gv = g[e];
    out[e] = epi == VRVQ_EPI_TANH ? gv * (1.0f - yv * yv) : gv * (yv * (1.0f - yv));
  }
}

// torch.nn.utils.weight_norm backward, per row r (norm over the other dims):
//   n = ||v_r||, dg_r = (dw_r . v_r) / n, dv_r = (g_r / n) (dw_r - v_r (dw_r . v_r) / n^2)
__global__ __launch_bounds__(256) void weight_norm_backward_kernel(
    const float* __restrict__ g, const float* __restrict__ v, const float* __restrict__ dw,
    int cols, float* __restrict__ dg, float* __restrict__ dv) {
  __shared__ float r1[256], r2[256];
  const size_t row = blockIdx.x;
  const float* vr = v + row * cols;
  const float* dr = dw + row * cols;
  float ss = 0.0f, dot = 0.0f;
  for (int c = threadIdx.x; c < cols; c += 256) {
    ss = fmaf(vr[c], vr[c], ss);
    dot = fmaf(dr[c], vr[c], dot);
  }
  r1[threadIdx.x] = ss;
  r2[threadIdx.x] = dot;
  __syncthreads();
  for (int h = 128; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) {
      r1[threadIdx.x] += r1[threadIdx.x + h];
      r2[threadIdx.x] += r2[threadIdx.x + h];
    }
    __syncthreads();
  }
  const float n = sqrtf(r1[0]), dvv = r2[0];
  const float gr = g[row];
  if (threadIdx.x == 0) dg[row] = dvv / n;
  const float sc = gr / n, corr = dvv / (n * n);
  for (int c = threadIdx.x; c < cols; c += 256) dv[row * cols + c] = sc * (dr[c] - vr[c] * corr);
}

// Adjoint-conv packing: the input gradient of a stride-1 Conv1d is a Conv1d of dY with
//   W'[ci][co][k] = W[co][ci][K-1-k], packed as vrvq_pack_conv1d_weight would pack W':
//   wp[co][k][ci_pad] (Cin' = Cout rows of K taps, Cout' = Cin padded to cout_pad)
__global__ void pack_conv1d_flip_kernel(const float* __restrict__ w, int cout, int cin, int K,
                                        int cin_pad, float* __restrict__ wp) {
  const size_t total = (size_t)cout * K * cin_pad;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cin_pad);
    const size_t rk = i / cin_pad;
    const int k = (int)(rk % K);
    const int co = (int)(rk / K);
    wp[i] = ci < cin ? w[((size_t)co * cin + ci) * K + (K - 1 - k)] : 0.0f;
  }
}

unsigned grid_n(size_t total, unsigned block) {
  size_t g = (total + block - 1) / block;
  return (unsigned)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

}  // namespace

static int wgrad_kg(int k) {  // taps per workgroup: all of them up to 8 (k = 16: two groups)
  if (k == 1 || k == 2 || k == 3 || k == 4 || k == 7 || k == 8) return k;
  if (k % 8 == 0) return 8;
  if (k % 4 == 0) return 4;
  return 1;
}

extern "C" int vrvq_wgrad_plan(int batch, int m, int ta, int c, int k, int* n_split,
                               long long* workspace_bytes) {
  VRVQ_CHECK_ARG(n_split && workspace_bytes && batch > 0 && m > 0 && ta > 0 && c > 0 && k > 0);
  const long long tiles = (long long)((m + WG_BM - 1) / WG_BM) * ((c + WG_BN - 1) / WG_BN) *
                          (k / wgrad_kg(k));
  const long long chunks = (long long)batch * ((ta + 7) / 8);  // upper bound (KT >= 8)
  long long s = (1024 + tiles - 1) / tiles;  // >= 4 workgroups per CU in total
  if (s > chunks) s = chunks;
  if (s > 256) s = 256;
  if (s < 1) s = 1;
  *n_split = (int)s;
  *workspace_bytes = s * m * (long long)c * k * (long long)sizeof(float);
  return 0;
}

template <int KG>
int launch_wgrad(WgradArgs w, hipStream_t st, bool x3) {
  const long long nblk = (long long)((w.M + WG_BM - 1) / WG_BM) * ((w.C + WG_BN - 1) / WG_BN) *
                         w.n_kg * w.n_split;
  if (nblk >= 0x7fffffffLL) return VRVQ_ERR_ARG;
  if (x3) {
    if constexpr (KG == 1) {
      const size_t lds = (size_t)(3 * 64 * WX_ALD / 2 + 64 * w.WP) * sizeof(float);
      hipLaunchKernelGGL(wgrad_x3_reg_kernel<KG>, dim3((unsigned)nblk), dim3(256), lds, st, w);
    } else {
      const size_t lds = (size_t)(3 * 64 * WX_ALD / 2 + 3 * 64 * wx_xpw(w.W) / 2) * sizeof(float);
      hipLaunchKernelGGL(wgrad_x3_kernel<KG>, dim3((unsigned)nblk), dim3(256), lds, st, w);
    }
    return vrvq_launch_status();
  }
  const size_t lds = (size_t)(64 * ((1 << w.kt_sh) + 1) + 64 * w.WP) * sizeof(float);
  hipLaunchKernelGGL(wgrad_kernel<KG>, dim3((unsigned)nblk), dim3(256), lds, st, w);
  return vrvq_launch_status();
}

// Stride-1 weight gradients on the split bf16 MFMA (wgrad_x3_kernel) unless VRVQ_WGRAD_X3=0
// (A/B and tests: the fp32-input MFMA kernel for every shape).
static bool wgrad_x3_enabled() {
  static const bool on = [] {
    const char* e = getenv("VRVQ_WGRAD_X3");
    return !(e && e[0] == '0');
  }();
  return on;
}

extern "C" int vrvq_conv1d_wgrad(const float* a, int batch, int m, int ta,
                                 const float* alpha_a, const float* inv_alpha_a, const float* x,
                                 int c, int tx, const float* alpha, const float* inv_alpha, int k,
                                 int stride, int pad, int dil, int n_split, float* workspace,
                                 long long workspace_bytes, float* out, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(a && x && out && workspace && batch > 0 && m > 0 && ta > 0 && c > 0 && tx > 0);
  VRVQ_CHECK_ARG(k > 0 && stride > 0 && pad >= 0 && dil > 0 && n_split > 0);
  VRVQ_CHECK_ARG(alpha == nullptr || inv_alpha != nullptr);
  VRVQ_CHECK_ARG(alpha_a == nullptr || inv_alpha_a != nullptr);
  VRVQ_CHECK_ARG(workspace_bytes >= (long long)n_split * m * (long long)c * k * 4);
  const int kg = wgrad_kg(k);
  WgradArgs w{a, m, ta, x, c, tx, alpha_a, inv_alpha_a, alpha, inv_alpha, batch, k, stride, pad,
              dil, n_split, 0, 5, 0, 0, k / kg, workspace};
  // time chunk: 64 samples unless the window then exceeds the staged row length
  for (w.kt_sh = 6; w.kt_sh >= 3; --w.kt_sh) {
    w.W = ((1 << w.kt_sh) - 1) * stride + (kg - 1) * dil + 1;
    if (w.W <= WG_WMAX) break;
  }
  if (w.W > WG_WMAX) return VRVQ_ERR_UNSUPPORTED;
  // the x3 kernel: stride 1, 64-sample chunks (window <= 64 + 7 * 9 samples)
  const bool x3 = wgrad_x3_enabled() && stride == 1 && w.kt_sh == 6;
  w.WP = w.W | 1;
  w.chunks = batch * ((ta + (1 << w.kt_sh) - 1) >> w.kt_sh);
  if (w.n_split > w.chunks) w.n_split = w.chunks;
  hipStream_t st = as_stream(stream);
  int rc;
  switch (kg) {
    case 1: rc = launch_wgrad<1>(w, st, x3); break;
    case 2: rc = launch_wgrad<2>(w, st, x3); break;
    case 3: rc = launch_wgrad<3>(w, st, x3); break;
    case 4: rc = launch_wgrad<4>(w, st, x3); break;
    case 7: rc = launch_wgrad<7>(w, st, x3); break;
    default: rc = launch_wgrad<8>(w, st, x3); break;
  }
  if (rc) return rc;
  const size_t n_elem = (size_t)m * c * k;
  hipLaunchKernelGGL(split_reduce_kernel, dim3(grid_n(n_elem, 256)), dim3(256), 0, st, workspace,
                     n_elem, w.n_split, out);
  return vrvq_launch_status();
}

static long long chunk_splits(int batch, int frames) {  // (clip, RCH-sample chunk) splits
  return (long long)batch * ((frames + RCH - 1) / RCH);
}

extern "C" int vrvq_snake_backward_workspace(int batch, int channels, int frames,
                                             long long* bytes) {
  VRVQ_CHECK_ARG(bytes && batch > 0 && channels > 0 && frames > 0);
  *bytes = chunk_splits(batch, frames) * channels * (long long)sizeof(float);
  return 0;
}

extern "C" int vrvq_snake_backward(const float* x, const float* alpha, const float* inv_alpha,
                                   const float* grad, int batch, int channels, int frames,
                                   float* dx, float* dalpha, float* workspace,
                                   long long workspace_bytes, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && alpha && inv_alpha && grad && (dx || dalpha) && batch > 0 &&
                 channels > 0 && frames > 0);
  const long long n_split = chunk_splits(batch, frames);
  VRVQ_CHECK_ARG(n_split * channels < 0x7fffffffLL);
  if (dalpha) VRVQ_CHECK_ARG(workspace && workspace_bytes >= n_split * channels * 4);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(snake_backward_kernel, dim3((unsigned)(channels * n_split)), dim3(256), 0, st,
                     x, alpha, inv_alpha, grad, batch, channels, frames, (int)n_split, dx,
                     dalpha ? workspace : nullptr);
  if (dalpha)
    hipLaunchKernelGGL(split_reduce_kernel, dim3(grid_n(channels, 256)), dim3(256), 0, st,
                       workspace, (size_t)channels, (int)n_split, dalpha);
  return vrvq_launch_status();
}

extern "C" int vrvq_bias_grad_workspace(int batch, int channels, int frames, long long* bytes) {
  VRVQ_CHECK_ARG(bytes && batch > 0 && channels > 0 && frames > 0);
  *bytes = chunk_splits(batch, frames) * channels * (long long)sizeof(float);
  return 0;
}

extern "C" int vrvq_bias_grad(const float* grad, int batch, int channels, int frames, float* db,
                              float* workspace, long long workspace_bytes, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(grad && db && workspace && batch > 0 && channels > 0 && frames > 0);
  const long long n_split = chunk_splits(batch, frames);
  VRVQ_CHECK_ARG(n_split * channels < 0x7fffffffLL);
  VRVQ_CHECK_ARG(workspace_bytes >= n_split * channels * 4);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(bias_grad_kernel, dim3((unsigned)(channels * n_split)), dim3(256), 0, st,
                     grad, batch, channels, frames, workspace);
  hipLaunchKernelGGL(split_reduce_kernel, dim3(grid_n(channels, 256)), dim3(256), 0, st,
                     workspace, (size_t)channels, (int)n_split, db);
  return vrvq_launch_status();
}

extern "C" int vrvq_act_backward(const float* y, const float* grad, long long n, int epilogue,
                                 float* out, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(y && grad && out && n > 0);
  VRVQ_CHECK_ARG(epilogue == VRVQ_EPI_TANH || epilogue == VRVQ_EPI_SIGMOID);
  hipLaunchKernelGGL(act_backward_kernel, dim3(grid_n((size_t)n, 256)), dim3(256), 0,
                     as_stream(stream), y, grad, (size_t)n, epilogue, out);
  return vrvq_launch_status();
}

extern "C" int vrvq_weight_norm_backward(const float* g, const float* v, const float* dw, int rows,
                                         int cols, float* dg, float* dv, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(g && v && dw && dg && dv && rows > 0 && cols > 0);
  hipLaunchKernelGGL(weight_norm_backward_kernel, dim3(rows), dim3(256), 0, as_stream(stream), g,
                     v, dw, cols, dg, dv);
  return vrvq_launch_status();
}

extern "C" int vrvq_pack_conv1d_flip(const float* w, int cout, int cin, int k, int cin_pad,
                                     float* w_packed, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(w && w_packed && cout > 0 && cin > 0 && k > 0 && cin_pad >= cin);
  const size_t total = (size_t)cout * k * cin_pad;
  hipLaunchKernelGGL(pack_conv1d_flip_kernel, dim3(grid_n(total, 256)), dim3(256), 0,
                     as_stream(stream), w, cout, cin, k, cin_pad, w_packed);
  return vrvq_launch_status();
}
