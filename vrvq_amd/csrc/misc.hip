// Weight preparation, importance gating and small reductions for the VRVQ hot path.
#include "common.h"

namespace {

// One workgroup per row: w = v * (g / ||v||) (torch._weight_norm, dim = 0).
__global__ __launch_bounds__(256) void weight_norm_kernel(const float* __restrict__ g,
                                                          const float* __restrict__ v, int cols,
                                                          float* __restrict__ w) {
  __shared__ float part[256];
  const size_t row = blockIdx.x;
  const float* vr = v + row * cols;
  float ss = 0.0f;
  for (int c = threadIdx.x; c < cols; c += 256) ss = fmaf(vr[c], vr[c], ss);
  part[threadIdx.x] = ss;
  __syncthreads();
  for (int h = 128; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
    __syncthreads();
  }
  const float scale = g[row] / sqrtf(part[0]);
  for (int c = threadIdx.x; c < cols; c += 256) w[row * cols + c] = vr[c] * scale;
}

__global__ void inv_alpha_kernel(const float* __restrict__ alpha, int n, float* __restrict__ inv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) inv[i] = 1.0f / (alpha[i] + 1e-9f);
}

__global__ void codebook_prep_kernel(const float* __restrict__ cb, int rows, int dim,
                                     float* __restrict__ cbn, float* __restrict__ c2) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* x = cb + (size_t)r * dim;
  float ss = 0.0f;
  for (int k = 0; k < dim; ++k) ss = fmaf(x[k], x[k], ss);
  const float den = fmaxf(sqrtf(ss), 1e-12f);  // F.normalize: x / clamp_min(||x||, eps)
  float s2 = 0.0f;
  for (int k = 0; k < dim; ++k) {
    const float y = x[k] / den;
    cbn[(size_t)r * dim + k] = y;
    s2 = fmaf(y, y, s2);
  }
  c2[r] = s2;
}

// out[0] = sum_{b,t} (sum_i loss[b,i,t] * mask[b,i,t]) / (B*T); single workgroup, fixed order.
__global__ __launch_bounds__(1024) void masked_loss_kernel(const float* __restrict__ loss,
                                                           const float* __restrict__ mask, int B,
                                                           int nq, int T, float* __restrict__ out) {
  __shared__ float part[1024];
  float acc = 0.0f;
  const int NF = B * T;
  for (int n = threadIdx.x; n < NF; n += 1024) {
    const int b = n / T, t = n - b * T;
    float s = 0.0f;
    for (int i = 0; i < nq; ++i) {
      const size_t o = ((size_t)b * nq + i) * T + t;
      s = s + loss[o] * (mask ? mask[o] : 1.0f);
    }
    acc += s;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int h = 512; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = part[0] / (float)NF;
}

__global__ void mask_hard_kernel(const float* __restrict__ s, int B, int T, int nq,
                                 float* __restrict__ mask) {
  const size_t total = (size_t)B * nq * T;
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total;
       o += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(o % T);
    const size_t bi = o / T;
    const int i = (int)(bi % nq);
    const int b = (int)(bi / nq);
    mask[o] = (s[(size_t)b * T + t] - (float)i >= 0.0f) ? 1.0f : 0.0f;
  }
}

__global__ void scale_imp_kernel(const float* __restrict__ imp, int n, float a, float c,
                                 float* __restrict__ s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) s[i] = (imp[i] * a) * c;
}

// z_q[b, e] = sum_i mask[b,i,t(e)] * z_q_is[b,i,e] over the (D*T) slab, float4 per thread.
__global__ void masked_sum_kernel(const float* __restrict__ zqis, const float* __restrict__ mask,
                                  int B, int nq, int D, int T, float* __restrict__ zq) {
  const size_t slab4 = (size_t)D * T / 4;
  const size_t total = (size_t)B * slab4;
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < total;
       q += (size_t)gridDim.x * blockDim.x) {
    const size_t b = q / slab4;
    const size_t e4 = q - b * slab4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int tt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tt[k] = (int)((e4 * 4 + k) % T);
    for (int i = 0; i < nq; ++i) {
      const float4 v = reinterpret_cast<const float4*>(zqis + ((b * nq + i) * D) * (size_t)T)[e4];
      const float* mr = mask + (b * nq + i) * (size_t)T;
      acc[0] = acc[0] + v.x * mr[tt[0]];
      acc[1] = acc[1] + v.y * mr[tt[1]];
      acc[2] = acc[2] + v.z * mr[tt[2]];
      acc[3] = acc[3] + v.w * mr[tt[3]];
    }
    reinterpret_cast<float4*>(zq + b * (size_t)D * T)[e4] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

__global__ __launch_bounds__(1024) void bpf_kernel(const float* __restrict__ mask,
                                                   const float* __restrict__ bits, int B, int nq,
                                                   int T, float* __restrict__ out) {
  __shared__ float part[1024];
  const size_t total = (size_t)B * nq * T;
  float acc = 0.0f;
  for (size_t o = threadIdx.x; o < total; o += 1024) {
    const int i = (int)((o / T) % nq);
    acc += mask[o] * bits[i];
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int h = 512; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = part[0] / (float)((size_t)B * T);
}

unsigned grid_for(size_t total, unsigned block) {
  size_t g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g == 0) g = 1;
  return (unsigned)g;
}

// decode_code of models/quantize.py:81-85 for every stage at once (the gather half of
// ResidualVectorQuantize.from_codes, :217-249): z_p[b, i*d + k, t] = cb[i][codes[b,i,t]][k]
// (raw, un-normalised rows) in the reference's latents layout, plus the same rows as
// zst[b][i][t][d], the input layout of vrvq_rvq_expand (out_proj + masked sum). One thread per
// (b, i, t) (grid-stride: any B*nq*T); consecutive t -> consecutive lanes, so the z_p row
// stores coalesce.
__global__ __launch_bounds__(256) void rvq_gather_kernel(const int64_t* __restrict__ codes,
                                                         const float* __restrict__ cb, int batch,
                                                         int nq, int frames, int ncode, int cdim,
                                                         float* __restrict__ zst,
                                                         float* __restrict__ z_p,
                                                         int* __restrict__ err) {
  const size_t total = (size_t)batch * nq * frames;
  for (size_t n = (size_t)blockIdx.x * blockDim.x + threadIdx.x; n < total;
       n += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(n % frames);
    const size_t bi = n / frames;            // b * nq + i
    const int i = (int)(bi % nq);
    long long c = codes[n];
    if (c < 0 || c >= ncode) {               // F.embedding raises IndexError; report, read row 0
      if (err) *err = 1;
      c = 0;
    }
    const float* row = cb + ((size_t)i * ncode + (size_t)c) * cdim;
    float* zs = zst ? zst + n * cdim : nullptr;
    float* zp = z_p ? z_p + bi * cdim * frames + t : nullptr;
    for (int k = 0; k < cdim; ++k) {
      const float v = row[k];
      if (zs) zs[k] = v;
      if (zp) zp[(size_t)k * frames] = v;
    }
  }
}

// Nearest normalised codeword of each stage's own latent (ResidualVectorQuantize.from_latents,
// models/quantize.py:251-285 via decode_latents :87-103): no residual chain, so every
// (clip, stage, frame) is independent. Workgroup = (stage, 256 frames) with the stage's
// normalised codebook and squared norms in LDS (read as broadcasts); the distance is the chain
// kernel's expression: e = z / max(||z||, 1e-12) with pairwise sums, dot in k order,
// fma(dot, -2, sum e^2) + c2, lowest index on ties.
__global__ __launch_bounds__(256) void rvq_nearest_kernel(const float* __restrict__ latents,
                                                          int batch, int nlat, int frames,
                                                          const float* __restrict__ cbn,
                                                          const float* __restrict__ c2, int ncode,
                                                          int64_t* __restrict__ codes, int nq) {
  extern __shared__ float nsm[];  // [ncode][8] codebook, [ncode] c2
  const int i = blockIdx.y;
  float* cb_s = nsm;
  float* c2_s = nsm + ncode * 8;
  for (int e = threadIdx.x; e < ncode * 8; e += 256) cb_s[e] = cbn[(size_t)i * ncode * 8 + e];
  for (int e = threadIdx.x; e < ncode; e += 256) c2_s[e] = c2[(size_t)i * ncode + e];
  __syncthreads();
  const long long n = (long long)blockIdx.x * 256 + threadIdx.x;
  if (n >= (long long)batch * frames) return;
  const int b = (int)(n / frames), t = (int)(n - (long long)b * frames);
  float z[8], q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    z[k] = latents[((size_t)b * nlat + (size_t)i * 8 + k) * frames + t];
    q[k] = z[k] * z[k];
  }
  const float n2 = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  const float nrm = fmaxf(sqrtf(n2), 1e-12f);
  float e[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    e[k] = z[k] / nrm;
    q[k] = e[k] * e[k];
  }
  const float e2 = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  float best = INFINITY;
  int bi = 0;
  for (int c = 0; c < ncode; ++c) {
    const float* r = cb_s + c * 8;
    float d = r[0] * e[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) d = fmaf(r[k], e[k], d);
    const float dist = fmaf(d, -2.0f, e2) + c2_s[c];
    if (dist < best) {  // increasing code index: strict < keeps the first
      best = dist;
      bi = c;
    }
  }
  codes[((size_t)b * nq + i) * frames + t] = bi;
}

}  // namespace

extern "C" int vrvq_rvq_nearest(const float* latents, int batch, int nlat, int frames, int nq,
                                const float* cbn, const float* c2, int ncode, int cdim,
                                int64_t* codes, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(latents && cbn && c2 && codes && batch > 0 && frames > 0 && nq > 0);
  VRVQ_CHECK_ARG(ncode > 0 && nlat >= nq * 8);
  if (cdim != 8 || ncode > 4096) return VRVQ_ERR_UNSUPPORTED;
  const long long nf = (long long)batch * frames;
  VRVQ_CHECK_ARG((nf + 255) / 256 < 0x7fffffffLL);
  const size_t lds = (size_t)ncode * 9 * sizeof(float);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)rvq_nearest_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(rvq_nearest_kernel, dim3((unsigned)((nf + 255) / 256), nq), dim3(256), lds,
                     as_stream(stream), latents, batch, nlat, frames, cbn, c2, ncode, codes, nq);
  return vrvq_launch_status();
}

extern "C" const char* vrvq_status_string(int status) {
  switch (status) {
    case VRVQ_OK: return "ok";
    case VRVQ_ERR_ARG: return "vrvq: invalid argument (null pointer, size or shape mismatch)";
    case VRVQ_ERR_UNSUPPORTED: return "vrvq: shape outside the instantiated kernel set";
    default: return hipGetErrorString((hipError_t)status);
  }
}

extern "C" int vrvq_version(void) { return 100; }

extern "C" int vrvq_weight_norm(const float* g, const float* v, int rows, int cols, float* w,
                                vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(g && v && w && rows > 0 && cols > 0);
  hipLaunchKernelGGL(weight_norm_kernel, dim3(rows), dim3(256), 0, as_stream(stream), g, v, cols, w);
  return vrvq_launch_status();
}

// Snake1d forward over [rows = batch * channels][frames]: one workgroup per (row, 1024-sample
// segment), 4 samples per thread.
__global__ __launch_bounds__(256) void snake_rows_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ alpha,
                                                         const float* __restrict__ inv_alpha,
                                                         int channels, int frames, int nseg,
                                                         float* __restrict__ y) {
  const int row = blockIdx.x / nseg, seg = blockIdx.x - row * nseg;
  const int c = row % channels;
  const float al = alpha[c], ia = inv_alpha[c];
  const size_t base = (size_t)row * frames;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = seg * 1024 + u * 256 + (int)threadIdx.x;
    if (t < frames) y[base + t] = snake_act(x[base + t], al, ia);
  }
}

extern "C" int vrvq_snake(const float* x, int batch, int channels, int frames, const float* alpha,
                          const float* inv_alpha, float* y, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && alpha && inv_alpha && y && x != y && batch > 0 && channels > 0 && frames > 0);
  const int nseg = (frames + 1023) / 1024;
  const long long nblk = (long long)batch * channels * nseg;
  if (nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
  hipLaunchKernelGGL(snake_rows_kernel, dim3((unsigned)nblk), dim3(256), 0, as_stream(stream), x,
                     alpha, inv_alpha, channels, frames, nseg, y);
  return vrvq_launch_status();
}

// Phase-split view of a (Snake-activated) signal: y[b][c s + r][m] = snake_c(x[b][c][m s + r -
// pad]), 0 outside [0, frames). A stride-s product over taps j = q s + r (q = 0, 1) becomes a
// stride-1 2-tap one over the view (the forward x3 path addresses the same view while staging;
// the weight gradients of the strided encoder convs and of the ConvTranspose layers take it
// materialised, once per layer). Thread = one view element; the gathers read rows of x.
__global__ __launch_bounds__(256) void phase_split_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ alpha,
                                                          const float* __restrict__ inv_alpha,
                                                          int channels, int frames, int sh,
                                                          int pad, int out_frames,
                                                          float* __restrict__ y, long long n) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;  // no barrier in this kernel
  const int m = (int)(e % out_frames);
  const long long rowv = e / out_frames;                 // b * (channels << sh) + c s + r
  const int vr = (int)(rowv % ((long long)channels << sh));
  const long long b = rowv / ((long long)channels << sh);
  const int c = vr >> sh, r = vr & ((1 << sh) - 1);
  const int t = (m << sh) + r - pad;
  float v = 0.0f;
  if (t >= 0 && t < frames) {
    v = x[(b * channels + c) * (long long)frames + t];
    if (alpha) v = snake_act(v, alpha[c], inv_alpha[c]);
  }
  y[e] = v;
}

extern "C" int vrvq_phase_split(const float* x, int batch, int channels, int frames, int stride,
                                int pad, int out_frames, const float* alpha,
                                const float* inv_alpha, float* y, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(x && y && x != y && batch > 0 && channels > 0 && frames > 0 && out_frames > 0);
  VRVQ_CHECK_ARG(stride > 0 && (stride & (stride - 1)) == 0 && pad >= 0);
  VRVQ_CHECK_ARG(alpha == nullptr || inv_alpha != nullptr);
  int sh = 0;
  while ((1 << sh) < stride) ++sh;
  const long long n = (long long)batch * channels * stride * out_frames;
  const long long nblk = (n + 255) / 256;
  if (nblk > 0x7fffffffLL) return VRVQ_ERR_ARG;
  hipLaunchKernelGGL(phase_split_kernel, dim3((unsigned)nblk), dim3(256), 0, as_stream(stream), x,
                     alpha, inv_alpha, channels, frames, sh, pad, out_frames, y, n);
  return vrvq_launch_status();
}

extern "C" int vrvq_snake_inv_alpha(const float* alpha, int channels, float* inv,
                                    vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(alpha && inv && channels > 0);
  hipLaunchKernelGGL(inv_alpha_kernel, dim3((channels + 255) / 256), dim3(256), 0,
                     as_stream(stream), alpha, channels, inv);
  return vrvq_launch_status();
}

extern "C" int vrvq_codebook_prep(const float* cb, int rows, int dim, float* cbn, float* c2,
                                  vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(cb && cbn && c2 && rows > 0 && dim > 0);
  hipLaunchKernelGGL(codebook_prep_kernel, dim3((rows + 255) / 256), dim3(256), 0,
                     as_stream(stream), cb, rows, dim, cbn, c2);
  return vrvq_launch_status();
}

extern "C" int vrvq_masked_loss(const float* loss_pf, const float* mask, int batch, int nq,
                                int frames, float* out, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(loss_pf && out && batch > 0 && nq > 0 && frames > 0);
  hipLaunchKernelGGL(masked_loss_kernel, dim3(1), dim3(1024), 0, as_stream(stream), loss_pf,
                     mask, batch, nq, frames, out);
  return vrvq_launch_status();
}

extern "C" int vrvq_mask_hard(const float* s, int batch, int frames, int nq, float* mask,
                              vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(s && mask && batch > 0 && frames > 0 && nq > 0);
  hipLaunchKernelGGL(mask_hard_kernel, dim3(grid_for((size_t)batch * nq * frames, 256)), dim3(256),
                     0, as_stream(stream), s, batch, frames, nq, mask);
  return vrvq_launch_status();
}

extern "C" int vrvq_scale_imp(const float* imp, int n, float a, float c, float* s,
                              vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(imp && s && n > 0);
  hipLaunchKernelGGL(scale_imp_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     imp, n, a, c, s);
  return vrvq_launch_status();
}

extern "C" int vrvq_masked_sum(const float* z_q_is, const float* mask, int batch, int nq, int dim,
                               int frames, float* z_q, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(z_q_is && mask && z_q && batch > 0 && nq > 0 && dim > 0 && frames > 0);
  VRVQ_CHECK_ARG(((size_t)dim * frames) % 4 == 0);
  hipLaunchKernelGGL(masked_sum_kernel, dim3(grid_for((size_t)batch * dim * frames / 4, 256)),
                     dim3(256), 0, as_stream(stream), z_q_is, mask, batch, nq, dim, frames, z_q);
  return vrvq_launch_status();
}

extern "C" int vrvq_bpf(const float* mask, const float* bits, int batch, int nq, int frames,
                        float* out, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(mask && bits && out && batch > 0 && nq > 0 && frames > 0);
  hipLaunchKernelGGL(bpf_kernel, dim3(1), dim3(1024), 0, as_stream(stream), mask, bits, batch, nq,
                     frames, out);
  return vrvq_launch_status();
}

extern "C" int vrvq_rvq_gather(const int64_t* codes, int batch, int nq, int frames,
                               const float* cb, int ncode, int cdim, float* zst, float* z_p,
                               int* err, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(codes && cb && (zst || z_p) && batch > 0 && nq > 0 && frames > 0);
  VRVQ_CHECK_ARG(ncode > 0 && cdim > 0);
  const size_t total = (size_t)batch * nq * frames;
  hipLaunchKernelGGL(rvq_gather_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     as_stream(stream), codes, cb, batch, nq, frames, ncode, cdim, zst, z_p, err);
  return vrvq_launch_status();
}
