// Variable-length code packing from importance masks: the VBR encoder
// emits codes [B][nq][T] (int64) with a prefix-shaped mask [B][nq][T] (mask[i] = s - i >= 0,
// models/utils.py:55-61), so frame (b, t) carries count[b,t] = sum_i mask[b,i,t] meaningful
// codes. Packed stream: clip-major, frame-major, stage-minor uint16 —
//   packed[clip_off[b] + frame_off[b,t] + i] = codes[b,i,t],  i < count[b,t]
// with counts[b*T+t] stored alongside (the bitstream's side information).
// Three launches: per-clip counts + totals (prefix check), one-workgroup scan over clips,
// per-clip frame scan + scatter. Unpacking runs the same count scan over the stored counts.
// Byte work: HBM-bound, coalesced along t (lane = frame).
#include "common.h"

namespace {

constexpr int PK_NT = 256;

// Exclusive scan of one value per thread across the workgroup (PK_NT threads); returns the
// thread's exclusive prefix and writes the block total to *total.
__device__ int block_exclusive_scan(int v, int* s_buf, int* total) {
  const int tid = threadIdx.x;
  s_buf[tid] = v;
  __syncthreads();
  for (int off = 1; off < PK_NT; off <<= 1) {
    const int add = tid >= off ? s_buf[tid - off] : 0;
    __syncthreads();
    s_buf[tid] += add;
    __syncthreads();
  }
  const int incl = s_buf[tid];
  *total = s_buf[PK_NT - 1];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(PK_NT) void pack_count_kernel(const float* __restrict__ mask,
                                                           int nq, int T,
                                                           int* __restrict__ counts,
                                                           long long* __restrict__ clip_total,
                                                           int* __restrict__ err) {
  __shared__ int s_buf[PK_NT];
  const int b = blockIdx.x;
  long long acc = 0;
  for (int t0 = 0; t0 < T; t0 += PK_NT) {
    const int t = t0 + threadIdx.x;
    int c = 0;
    if (t < T) {
      bool seen_zero = false;
      for (int i = 0; i < nq; ++i) {
        const bool on = mask[((size_t)b * nq + i) * T + t] != 0.0f;
        if (on) {
          if (seen_zero && err) *err = 1;   // not prefix-shaped
          ++c;
        } else {
          seen_zero = true;
        }
      }
      counts[(size_t)b * T + t] = c;
    }
    int tot;
    block_exclusive_scan(c, s_buf, &tot);
    acc += tot;
  }
  if (threadIdx.x == 0) clip_total[b] = acc;
}

// Exclusive scan over clips (one workgroup, chunks of PK_NT with a running carry).
__global__ __launch_bounds__(PK_NT) void pack_clip_scan_kernel(const long long* __restrict__ tot,
                                                               int B,
                                                               long long* __restrict__ clip_off) {
  __shared__ long long s[PK_NT];
  long long carry = 0;
  for (int b0 = 0; b0 < B; b0 += PK_NT) {
    const int b = b0 + threadIdx.x;
    const long long v = b < B ? tot[b] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < PK_NT; off <<= 1) {
      const long long add = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
      __syncthreads();
      s[threadIdx.x] += add;
      __syncthreads();
    }
    if (b < B) clip_off[b] = carry + s[threadIdx.x] - v;
    const long long chunk = s[PK_NT - 1];
    __syncthreads();
    carry += chunk;
  }
  if (threadIdx.x == 0) clip_off[B] = carry;
}

// Per-clip total of stored counts (unpack side).
__global__ __launch_bounds__(PK_NT) void pack_sum_kernel(const int* __restrict__ counts, int T,
                                                         long long* __restrict__ clip_total) {
  __shared__ int s_buf[PK_NT];
  const int b = blockIdx.x;
  long long acc = 0;
  for (int t0 = 0; t0 < T; t0 += PK_NT) {
    const int t = t0 + threadIdx.x;
    int tot;
    block_exclusive_scan(t < T ? counts[(size_t)b * T + t] : 0, s_buf, &tot);
    acc += tot;
  }
  if (threadIdx.x == 0) clip_total[b] = acc;
}

// dir = 0: pack codes -> packed; dir = 1: unpack packed -> codes (+ mask).
__global__ __launch_bounds__(PK_NT) void pack_move_kernel(int dir, int nq, int T,
                                                          const int* __restrict__ counts,
                                                          const long long* __restrict__ clip_off,
                                                          int64_t* __restrict__ codes,
                                                          uint16_t* __restrict__ packed,
                                                          float* __restrict__ mask,
                                                          int ncode, int* __restrict__ err) {
  __shared__ int s_buf[PK_NT];
  const int b = blockIdx.x;
  long long base = clip_off[b];
  for (int t0 = 0; t0 < T; t0 += PK_NT) {
    const int t = t0 + threadIdx.x;
    const int c = t < T ? counts[(size_t)b * T + t] : 0;
    int tot;
    const int off = block_exclusive_scan(c, s_buf, &tot);
    if (t < T) {
      uint16_t* p = packed + base + off;
      for (int i = 0; i < nq; ++i) {
        const size_t ci = ((size_t)b * nq + i) * T + t;
        if (dir == 0) {
          if (i < c) {
            const long long v = codes[ci];
            if ((v < 0 || v >= ncode) && err) *err = 2;
            p[i] = (uint16_t)v;
          }
        } else {
          codes[ci] = i < c ? (int64_t)p[i] : 0;
          if (mask) mask[ci] = i < c ? 1.0f : 0.0f;
        }
      }
    }
    base += tot;
  }
}

}  // namespace

extern "C" int vrvq_pack_counts(const float* mask, int batch, int nq, int frames, int* counts,
                                long long* clip_total, long long* clip_off, int* err,
                                vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(mask && counts && clip_total && clip_off && batch > 0 && nq > 0 && frames > 0);
  VRVQ_CHECK_ARG(nq <= 255);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(pack_count_kernel, dim3(batch), dim3(PK_NT), 0, st, mask, nq, frames,
                     counts, clip_total, err);
  hipLaunchKernelGGL(pack_clip_scan_kernel, dim3(1), dim3(PK_NT), 0, st, clip_total, batch,
                     clip_off);
  return vrvq_launch_status();
}

extern "C" int vrvq_pack_codes(const int64_t* codes, const int* counts, const long long* clip_off,
                               int batch, int nq, int frames, int ncode, uint16_t* packed,
                               int* err, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(codes && counts && clip_off && packed && batch > 0 && nq > 0 && frames > 0);
  VRVQ_CHECK_ARG(ncode > 0 && ncode <= 65536);
  hipLaunchKernelGGL(pack_move_kernel, dim3(batch), dim3(PK_NT), 0, as_stream(stream), 0, nq,
                     frames, counts, clip_off, const_cast<int64_t*>(codes), packed, nullptr,
                     ncode, err);
  return vrvq_launch_status();
}

extern "C" int vrvq_unpack_offsets(const int* counts, int batch, int frames,
                                   long long* clip_total, long long* clip_off,
                                   vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(counts && clip_total && clip_off && batch > 0 && frames > 0);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(pack_sum_kernel, dim3(batch), dim3(PK_NT), 0, st, counts, frames,
                     clip_total);
  hipLaunchKernelGGL(pack_clip_scan_kernel, dim3(1), dim3(PK_NT), 0, st, clip_total, batch,
                     clip_off);
  return vrvq_launch_status();
}

extern "C" int vrvq_unpack_codes(const uint16_t* packed, const int* counts,
                                 const long long* clip_off, int batch, int nq, int frames,
                                 int64_t* codes, float* mask, vrvq_stream_t stream) {
  VRVQ_CHECK_ARG(packed && counts && clip_off && codes && batch > 0 && nq > 0 && frames > 0);
  hipLaunchKernelGGL(pack_move_kernel, dim3(batch), dim3(PK_NT), 0, as_stream(stream), 1, nq,
                     frames, counts, clip_off, codes, const_cast<uint16_t*>(packed), mask, 65536,
                     nullptr);
  return vrvq_launch_status();
}
