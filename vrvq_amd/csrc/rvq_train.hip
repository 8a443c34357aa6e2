// Training-mode residual vector quantisation on gfx950: the importance-mask STE and the
// backward pass of VBRResidualVectorQuantize.forward (models/quantize.py:328-443 in training,
// VectorQuantize.forward :42-79, generate_mask_ste / logcosh models/utils.py:11-53).
//
// Backward, for upstream dZ = dL/dz_q [B][D][T], gc = dL/dcommitment, gcb = dL/dcodebook and
// the stored forward state (z, zst, z_e = latents, codes, mask m), per frame in the 8-dim space:
//   Q_i    = W_out(i)^T dZ,  bdz_i = b_out(i) . dZ              (projection kernel on dZ)
//   dm_i   = Q_i . zst_i + bdz_i                                 (= dZ . z_q_i, the mask grad)
//   dzst_i = m_i Q_i - sum_{j>i} M_ji^T dze_j,   M_ji = W_in(j) W_out(i)
//   dze_i  = dzst_i + gc m_i / (B T) * 2 (z_e_i - cb[code_i]) / 8     (straight-through + commit)
//   dz     = sum_i W_in(i)^T dze_i                               (expansion kernel, bias 0)
// Weight gradients without the 1024-dim residuals r_i = z - sum_{j<i} (W_out(j) zst_j + b_out(j)):
//   S      = sum_{b,t} dze (x) [zst ; 1]          (8nq x (8nq + 1), split-K MFMA GEMM)
//   dW_in  = sum dze (x) z - sum_{j<i} S_ij W_out(j)^T - (sum dze_i) (x) sum_{j<i} b_out(j)
//   dW_out = sum dZ (x) m_i zst_i - sum_{j>i} W_in(j)^T S_ji
//   db_out = sum m_i dZ - sum_{j>i} W_in(j)^T sum dze_j,  db_in = sum dze_i
//   dcb[i][n] = sum_{frames with code n} gcb m_i / (B T) * 2 (cb[n] - z_e_i) / 8  (frame order)
// All sums deterministic.
#include "common.h"

namespace {

constexpr int RD = 1024;
constexpr int RCD = 8;
constexpr int BW_FR = 32;   // frames per backward-chain workgroup (8 lanes each)
constexpr int BW_NQMAX = 32;

// ------------------------------------------------------------------------------------------
// Mask STE forward (models/quantize.py:377-414 in training):
//   rows b < n_imps:  x = (imp * level_b) * nq, p = x - i,
//                     mask = smooth(p) + ((p >= 0) - smooth(p))   (generate_mask_ste)
//   dropout rows b = n_imps + j, j < n_drop: (dropout[j] - i >= 0) (generate_mask_hard of
//                     the first n_drop draws, quantize.py:412-413)
//   remaining rows (full codebook): 1
// smooth = logcosh(alpha, p), the two-branch form of models/utils.py:11-32 (EPS = 1e-10).
__device__ __forceinline__ float logcosh_smooth(float p, float alpha, float ea) {
  const float EPS = 1e-10f;
  if (p >= 0.0f) {
    const float numer = ea + expf((-2.0f * p) * alpha);
    const float denom = expf(alpha * ((-2.0f * p) + 1.0f)) + 1.0f;
    return (logf(numer + EPS) - logf(denom + EPS)) / (2.0f * alpha) + 0.5f;
  }
  const float numer = expf(alpha * ((2.0f * p) + 1.0f)) + 1.0f;
  const float denom = ea + expf((alpha * 2.0f) * p);
  return (logf(numer + EPS) - logf(denom + EPS)) / (2.0f * alpha) + 0.5f;
}

// d smooth / dp (what autograd differentiates through the same expressions)
__device__ __forceinline__ float logcosh_grad(float p, float alpha, float ea) {
  const float EPS = 1e-10f;
  if (p >= 0.0f) {
    const float e1 = expf((-2.0f * p) * alpha);
    const float e2 = expf(alpha * ((-2.0f * p) + 1.0f));
    return -e1 / ((ea + e1) + EPS) + e2 / ((e2 + 1.0f) + EPS);
  }
  const float e3 = expf(alpha * ((2.0f * p) + 1.0f));
  const float e4 = expf((alpha * 2.0f) * p);
  return e3 / ((e3 + 1.0f) + EPS) - e4 / ((ea + e4) + EPS);
}

__global__ void mask_ste_kernel(const float* __restrict__ imp, const float* __restrict__ levels,
                                const int64_t* __restrict__ dropout, int B, int T, int nq,
                                float alpha, float ea, int n_imps, int n_drop,
                                float* __restrict__ mask) {
  const size_t total = (size_t)B * nq * T;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
       e += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(e % T);
    const size_t bi = e / T;
    const int i = (int)(bi % nq), b = (int)(bi / nq);
    float m;
    if (b < n_imps) {
      // levels == null: imp already holds the scaled map x (public generate_mask_ste)
      const float x = levels ? (imp[(size_t)b * T + t] * levels[b]) * (float)nq
                             : imp[(size_t)b * T + t];
      const float p = x - (float)i;
      const float sm = logcosh_smooth(p, alpha, ea);
      const float q = p >= 0.0f ? 1.0f : 0.0f;
      m = sm + (q - sm);
    } else if (b < n_imps + n_drop) {
      m = ((float)dropout[b - n_imps] - (float)i >= 0.0f) ? 1.0f : 0.0f;  // dropout[:n_drop]
    } else {
      m = 1.0f;
    }
    mask[e] = m;
  }
}

// dimp[b][t] = ((sum_i dmask[b][i][t] smooth'(p_i)) * nq) * level_b for b < n_imps, else 0
// (levels == null: d/dx of the prescaled map, sum_i dmask smooth'(p_i))
// (the dropout / full-codebook rows are overwritten in the reference: no gradient).
__global__ void mask_ste_backward_kernel(const float* __restrict__ imp,
                                         const float* __restrict__ levels,
                                         const float* __restrict__ dmask, int B, int T, int nq,
                                         float alpha, float ea, int n_imps,
                                         float* __restrict__ dimp) {
  const size_t total = (size_t)B * T;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
       e += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(e % T), b = (int)(e / T);
    float g = 0.0f;
    if (b < n_imps) {
      const float x = levels ? (imp[e] * levels[b]) * (float)nq : imp[e];
      for (int i = 0; i < nq; ++i)
        g += dmask[((size_t)b * nq + i) * T + t] * logcosh_grad(x - (float)i, alpha, ea);
      if (levels) g = (g * (float)nq) * levels[b];
    }
    dimp[e] = g;
  }
}

// ------------------------------------------------------------------------------------------
// Projection weights for dZ: blocks 0..nq-1 = W_out (Q_i), blocks nq.. = b_out rows packed 8 per
// block (bdz_i = block nq + i/8, row i%8).
__global__ void build_wext_kernel(const float* __restrict__ w_out, const float* __restrict__ b_out,
                                  int nq, int nqb, float* __restrict__ wext) {
  const size_t total = (size_t)(nq + nqb) * RD * RCD;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
       e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % RCD);
    const size_t r = e / RCD;
    const int c = (int)(r % RD), blk = (int)(r / RD);
    float v;
    if (blk < nq) {
      v = w_out[e];
    } else {
      const int i = (blk - nq) * RCD + k;
      v = i < nq ? b_out[(size_t)i * RD + c] : 0.0f;
    }
    wext[e] = v;
  }
}

struct BwdArgs {
  const float* part;     // [8][NF][R]  R = 8 (nq + nqb)
  int B, T, nq, nqb, N, NF;
  const float* zst;      // [B][nq][T][8]
  const float* lat;      // [B][8nq][T]
  const int64_t* codes;  // [B][nq][T]
  const float* mask;     // [B][nq][T]
  const float* cb;       // [nq][N][8]
  const float* mcol;     // [nq][nq][8][8]
  const float* gc;       // device scalar: dL/d commitment_loss
  const float* gcb;      // device scalar: dL/d codebook_loss
  float* dze_t;          // [B][8nq][T]
  float* dze_z;          // [B][nq][T][8]
  float* zx1;            // [B][8nq + 1][T]   zst ; 1
  float* zx2;            // [B][9nq][T]       m zst ; m
  float* dm;             // [B][nq][T]
  float* dcb_f;          // [B][nq][T][8]
};

// Reverse chain: lane (frame f, component m), stages nq-1 .. 0.
__global__ __launch_bounds__(256) void rvq_bwd_chain_kernel(BwdArgs a) {
  __shared__ float dze_s[BW_FR][BW_NQMAX][RCD];
  const int tid = threadIdx.x, f = tid >> 3, m = tid & 7;
  const int n = blockIdx.x * BW_FR + f;
  const bool valid = n < a.NF;
  const int b = valid ? n / a.T : 0, t = valid ? n - b * a.T : 0;
  const int R = RCD * (a.nq + a.nqb);
  const float inv_bt = 1.0f / (float)((long long)a.B * a.T);
  const float gc = *a.gc, gcb = *a.gcb;
  const size_t NF = (size_t)a.NF;
  if (valid && m == 0) a.zx1[((size_t)b * (RCD * a.nq + 1) + RCD * a.nq) * a.T + t] = 1.0f;
  for (int i = a.nq - 1; i >= 0; --i) {
    if (valid) {
      float q = 0.0f, bdz = 0.0f;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const float* ps = a.part + ((size_t)s * NF + n) * R;
        q = q + ps[RCD * i + m];
        bdz = bdz + ps[RCD * a.nq + i];
      }
      const size_t fi = ((size_t)b * a.nq + i) * a.T + t;
      const float zs = a.zst[fi * RCD + m];
      const float ze = a.lat[((size_t)b * RCD * a.nq + RCD * i + m) * a.T + t];
      const int64_t code = a.codes[fi];
      const float zq = a.cb[((size_t)i * a.N + code) * RCD + m];
      const float mi = a.mask[fi];
      float acc = 0.0f;
      for (int j = i + 1; j < a.nq; ++j) {
        const float* mc = a.mcol + (((size_t)i * a.nq + j) * RCD) * RCD + m;
#pragma unroll
        for (int k = 0; k < RCD; ++k) acc = fmaf(mc[k * RCD], dze_s[f][j][k], acc);
      }
      const float dzst = mi * q - acc;
      const float dze = dzst + ((gc * inv_bt) * mi) * (0.25f * (ze - zq));
      dze_s[f][i][m] = dze;
      a.dze_t[((size_t)b * RCD * a.nq + RCD * i + m) * a.T + t] = dze;
      a.dze_z[fi * RCD + m] = dze;
      a.zx1[((size_t)b * (RCD * a.nq + 1) + RCD * i + m) * a.T + t] = zs;
      a.zx2[((size_t)b * 9 * a.nq + RCD * i + m) * a.T + t] = mi * zs;
      a.dcb_f[fi * RCD + m] = ((gcb * inv_bt) * mi) * (0.25f * (zq - ze));
      float p = q * zs;
      p += __shfl_xor(p, 1, 8);
      p += __shfl_xor(p, 2, 8);
      p += __shfl_xor(p, 4, 8);
      if (m == 0) {
        a.dm[fi] = p + bdz;
        a.zx2[((size_t)b * 9 * a.nq + RCD * a.nq + i) * a.T + t] = mi;
      }
    }
    __syncthreads();
  }
}

// Weight-gradient fix-ups (see the header): thread = channel c, blockIdx.y = stage i.
struct FixArgs {
  const float* P;      // [8nq][D]        sum dze (x) z
  const float* S;      // [8nq][8nq + 1]  sum dze (x) [zst ; 1]
  const float* G;      // [D][9nq]        sum dZ (x) [m zst ; m]
  const float* w_in_t; // [nq][D][8]
  const float* w_out;  // [nq][D][8]
  const float* b_out;  // [nq][D]
  int nq;
  float* dw_in;        // [nq][8][D]
  float* db_in;        // [nq][8]
  float* dw_out;       // [nq][D][8]
  float* db_out;       // [nq][D]
};

__global__ __launch_bounds__(256) void rvq_wfix_kernel(FixArgs a) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int i = blockIdx.y;
  if (c >= RD) return;
  const int nq = a.nq, SC = RCD * nq + 1;
  // dW_in rows 8i..8i+7
  float win[RCD];
#pragma unroll
  for (int k = 0; k < RCD; ++k) win[k] = a.P[(size_t)(RCD * i + k) * RD + c];
  float cumb = 0.0f;
  for (int j = 0; j < i; ++j) {
    const float* wo = a.w_out + ((size_t)j * RD + c) * RCD;
    float wv[RCD];
#pragma unroll
    for (int mm = 0; mm < RCD; ++mm) wv[mm] = wo[mm];
#pragma unroll
    for (int k = 0; k < RCD; ++k) {
      const float* srow = a.S + (size_t)(RCD * i + k) * SC + RCD * j;
      float acc = 0.0f;
#pragma unroll
      for (int mm = 0; mm < RCD; ++mm) acc = fmaf(srow[mm], wv[mm], acc);
      win[k] -= acc;
    }
    cumb = cumb + a.b_out[(size_t)j * RD + c];
  }
#pragma unroll
  for (int k = 0; k < RCD; ++k) {
    const float sdz = a.S[(size_t)(RCD * i + k) * SC + RCD * nq];
    a.dw_in[((size_t)i * RCD + k) * RD + c] = win[k] - sdz * cumb;
    if (c == 0) a.db_in[i * RCD + k] = sdz;
  }
  // dW_out(i)[c][:], db_out(i)[c]
  float wout[RCD];
#pragma unroll
  for (int mm = 0; mm < RCD; ++mm) wout[mm] = a.G[(size_t)c * 9 * nq + RCD * i + mm];
  float bo = a.G[(size_t)c * 9 * nq + RCD * nq + i];
  for (int j = i + 1; j < nq; ++j) {
    const float* wi = a.w_in_t + ((size_t)j * RD + c) * RCD;
    float wv[RCD];
#pragma unroll
    for (int k = 0; k < RCD; ++k) wv[k] = wi[k];
#pragma unroll
    for (int mm = 0; mm < RCD; ++mm) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < RCD; ++k) acc = fmaf(wv[k], a.S[(size_t)(RCD * j + k) * SC + RCD * i + mm], acc);
      wout[mm] -= acc;
    }
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < RCD; ++k) acc = fmaf(wv[k], a.S[(size_t)(RCD * j + k) * SC + RCD * nq], acc);
    bo -= acc;
  }
#pragma unroll
  for (int mm = 0; mm < RCD; ++mm) a.dw_out[((size_t)i * RD + c) * RCD + mm] = wout[mm];
  a.db_out[(size_t)i * RD + c] = bo;
}

// dcb[i][n][:] = sum over frames (in frame order) with codes[b][i][t] == n of dcb_f[b][i][t][:]
__global__ __launch_bounds__(256) void rvq_codebook_grad_kernel(const int64_t* __restrict__ codes,
                                                                const float* __restrict__ dcb_f,
                                                                int B, int T, int nq, int N,
                                                                float* __restrict__ dcb) {
  const int i = blockIdx.y;
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float acc[RCD];
#pragma unroll
  for (int k = 0; k < RCD; ++k) acc[k] = 0.0f;
  for (int b = 0; b < B; ++b) {
    const int64_t* cr = codes + ((size_t)b * nq + i) * T;
    for (int t = 0; t < T; ++t) {
      if (cr[t] == n) {
        const float* g = dcb_f + (((size_t)b * nq + i) * T + t) * RCD;
#pragma unroll
        for (int k = 0; k < RCD; ++k) acc[k] = acc[k] + g[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < RCD; ++k) dcb[((size_t)i * N + n) * RCD + k] = acc[k];
}

unsigned grid_cap(size_t total) {
  const size_t g = (total + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

// Workspace carve (floats), shared by the size query and the launcher.
struct BwdWs {
  size_t wext, part, dze_t, dze_z, zx1, zx2, dcb_f, S, G, P, zb, gemm, total;
  int split_s, split_g, split_p;
  BwdWs(int B, int T, int nq) {
    const size_t nf = (size_t)B * T;
    const int nqb = (nq + 7) / 8;
    auto al = [](size_t x) { return (x + 63) & ~(size_t)63; };
    size_t o = 0;
    wext = o; o += al((size_t)(nq + nqb) * RD * RCD);
    part = o; o += al((size_t)8 * nf * RCD * (nq + nqb));
    dze_t = o; o += al(nf * RCD * nq);
    dze_z = o; o += al(nf * RCD * nq);
    zx1 = o; o += al(nf * (RCD * nq + 1));
    zx2 = o; o += al(nf * 9 * nq);
    dcb_f = o; o += al(nf * RCD * nq);
    S = o; o += al((size_t)RCD * nq * (RCD * nq + 1));
    G = o; o += al((size_t)RD * 9 * nq);
    P = o; o += al((size_t)RCD * nq * RD);
    zb = o; o += al((size_t)nq * RD);
    long long bs = 0, bg = 0, bp = 0;
    vrvq_wgrad_plan(B, RCD * nq, T, RCD * nq + 1, 1, &split_s, &bs);
    vrvq_wgrad_plan(B, RD, T, 9 * nq, 1, &split_g, &bg);
    vrvq_wgrad_plan(B, RCD * nq, T, RD, 1, &split_p, &bp);
    long long mx = bs > bg ? bs : bg;
    mx = mx > bp ? mx : bp;
    gemm = o; o += al((size_t)(mx / 4));
    total = o;
  }
};

}  // namespace

extern "C" int vrvq_mask_ste(const float* imp, const float* levels, const int64_t* dropout,
                             int batch, int frames, int nq, float alpha, int n_imps, int n_drop,
                             float* mask, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(imp && mask && batch > 0 && frames > 0 && nq > 0 && alpha > 0.0f);
  VRVQ_CHECK_ARG(n_imps >= 0 && n_drop >= 0 && n_imps + n_drop <= batch);
  VRVQ_CHECK_ARG(n_drop == 0 || dropout != nullptr);
  const float ea = (float)exp((double)alpha);  // math.exp(alpha), rounded to the tensor dtype
  hipLaunchKernelGGL(mask_ste_kernel, dim3(grid_cap((size_t)batch * nq * frames)), dim3(256), 0,
                     as_stream(stream), imp, levels, dropout, batch, frames, nq, alpha, ea,
                     n_imps, n_drop, mask);
  return vrvq_launch_status();
}

extern "C" int vrvq_mask_ste_backward(const float* imp, const float* levels, const float* dmask,
                                      int batch, int frames, int nq, float alpha, int n_imps,
                                      float* dimp, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(imp && dmask && dimp && batch > 0 && frames > 0 && nq > 0);
  VRVQ_CHECK_ARG(alpha > 0.0f && n_imps >= 0 && n_imps <= batch);
  const float ea = (float)exp((double)alpha);
  hipLaunchKernelGGL(mask_ste_backward_kernel, dim3(grid_cap((size_t)batch * frames)), dim3(256),
                     0, as_stream(stream), imp, levels, dmask, batch, frames, nq, alpha, ea,
                     n_imps, dimp);
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_backward_workspace(int batch, int frames, int nq, long long* bytes) {
  VRVQ_CHECK_ARG(bytes && batch > 0 && frames > 0 && nq > 0 && nq <= BW_NQMAX);
  *bytes = (long long)BwdWs(batch, frames, nq).total * (long long)sizeof(float);
  return 0;
}

extern "C" int vrvq_rvq_backward(const float* dz_q, const float* g_commit, const float* g_codebook,
                                 const float* z, const float* zst, const float* latents,
                                 const int64_t* codes, const float* mask, int batch, int dim,
                                 int frames, int nq, int ncode, int cdim, const float* w_in_t,
                                 const float* w_out, const float* b_out, const float* mcol,
                                 const float* cb, float* dz, float* dmask, float* dw_in,
                                 float* db_in, float* dw_out, float* db_out, float* dcb,
                                 void* workspace, long long workspace_bytes,
                                 vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(dz_q && g_commit && g_codebook && z && zst && latents && codes && mask);
  VRVQ_CHECK_ARG(w_in_t && w_out && b_out && mcol && cb && dz && dmask && dw_in && db_in &&
                 dw_out && db_out && dcb && workspace);
  VRVQ_CHECK_ARG(batch > 0 && frames > 0 && nq > 0 && ncode > 0);
  if (dim != RD || cdim != RCD || nq > BW_NQMAX) return VRVQ_ERR_UNSUPPORTED;
  const BwdWs L(batch, frames, nq);
  VRVQ_CHECK_ARG(workspace_bytes >= (long long)L.total * 4);
  VRVQ_CHECK_ARG(((uintptr_t)workspace & 15) == 0);
  float* ws = static_cast<float*>(workspace);
  hipStream_t st = as_stream(stream);
  const int nqb = (nq + 7) / 8;
  const long long nf = (long long)batch * frames;
  VRVQ_CHECK_ARG(nf * 9 * nq < 0x7fffffffLL);
  hipLaunchKernelGGL(build_wext_kernel, dim3(grid_cap((size_t)(nq + nqb) * RD * RCD)), dim3(256), 0,
                     st, w_out, b_out, nq, nqb, ws + L.wext);
  int rc = vrvq_rvq_project(dz_q, batch, RD, frames, nq + nqb, RCD, ws + L.wext, ws + L.part,
                            stream);
  if (rc) return rc;
  BwdArgs a{ws + L.part, batch, frames, nq, nqb, ncode, (int)nf, zst, latents, codes, mask, cb,
            mcol, g_commit, g_codebook, ws + L.dze_t, ws + L.dze_z, ws + L.zx1, ws + L.zx2,
            dmask, ws + L.dcb_f};
  hipLaunchKernelGGL(rvq_bwd_chain_kernel, dim3((unsigned)((nf + BW_FR - 1) / BW_FR)), dim3(256),
                     0, st, a);
  rc = vrvq_launch_status();
  if (rc) return rc;
  const long long gb = (long long)(L.total - L.gemm) * 4;
  rc = vrvq_conv1d_wgrad(ws + L.dze_t, batch, RCD * nq, frames, nullptr, nullptr, ws + L.zx1,
                         RCD * nq + 1, frames, nullptr, nullptr, 1, 1, 0, 1, L.split_s,
                         ws + L.gemm, gb, ws + L.S, stream);
  if (rc) return rc;
  rc = vrvq_conv1d_wgrad(dz_q, batch, RD, frames, nullptr, nullptr, ws + L.zx2, 9 * nq, frames,
                         nullptr, nullptr, 1, 1, 0, 1, L.split_g, ws + L.gemm, gb, ws + L.G,
                         stream);
  if (rc) return rc;
  rc = vrvq_conv1d_wgrad(ws + L.dze_t, batch, RCD * nq, frames, nullptr, nullptr, z, RD, frames,
                         nullptr, nullptr, 1, 1, 0, 1, L.split_p, ws + L.gemm, gb, ws + L.P,
                         stream);
  if (rc) return rc;
  FixArgs fx{ws + L.P, ws + L.S, ws + L.G, w_in_t, w_out, b_out, nq, dw_in, db_in, dw_out, db_out};
  hipLaunchKernelGGL(rvq_wfix_kernel, dim3(RD / 256, nq), dim3(256), 0, st, fx);
  hipLaunchKernelGGL(rvq_codebook_grad_kernel, dim3((unsigned)((ncode + 255) / 256), nq),
                     dim3(256), 0, st, codes, ws + L.dcb_f, batch, frames, nq, ncode, dcb);
  rc = vrvq_launch_status();
  if (rc) return rc;
  // dz = sum_i W_in(i)^T dze_i: the expansion kernel with W_in^T as out_proj, zero bias, no mask
  if (hipMemsetAsync(ws + L.zb, 0, (size_t)nq * RD * sizeof(float), st) != hipSuccess)
    return vrvq_launch_status();
  return vrvq_rvq_expand(ws + L.dze_z, batch, RD, frames, nq, RCD, w_in_t, ws + L.zb, nullptr,
                         1.0f, nullptr, dz, nullptr, stream);
}
