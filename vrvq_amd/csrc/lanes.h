// Cross-lane exchange helpers for wave64 reductions on gfx950, without the LDS crossbar
// (ds_bpermute): DPP row/quad permutes for distances 1..8, v_permlane16/32_swap for 16, 32.
#pragma once
#include <hip/hip_runtime.h>

namespace vrvq {

// DPP controls (gfx9 encoding).
constexpr int DPP_QUAD_XOR1 = 0xB1;       // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;       // quad_perm [2,3,0,1]
constexpr int DPP_ROW_HALF_MIRROR = 0x141;  // lane i <-> 7-i inside each 8-lane half-row
constexpr int DPP_ROW_ROR8 = 0x128;       // lane i <-> i^8 inside each 16-lane row

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL,
                                                    0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
  return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false);
}

// Partner value across 16-lane rows (lane l <-> l^16).
__device__ __forceinline__ unsigned partner16_u(unsigned x, int lane) {
  auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return (lane & 16) ? r[0] : r[1];
}
// Partner value across wave halves (lane l <-> l^32).
__device__ __forceinline__ unsigned partner32_u(unsigned x, int lane) {
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (lane & 32) ? r[0] : r[1];
}

// Exchange with the partner at "distance" H. For H = 4 the partner is the half-row mirror
// (7-i), which is a valid partner for butterfly all-reductions once lanes within each quad
// already agree (i.e. when H = 1 and 2 have been applied first) and for the reduce-scatter
// below (applied after H >= 8, before H = 2, 1).
template <int H>
__device__ __forceinline__ float xchg(float x, int lane) {
  if constexpr (H == 1) return dpp<DPP_QUAD_XOR1>(x);
  else if constexpr (H == 2) return dpp<DPP_QUAD_XOR2>(x);
  else if constexpr (H == 4) return dpp<DPP_ROW_HALF_MIRROR>(x);
  else if constexpr (H == 8) return dpp<DPP_ROW_ROR8>(x);
  else if constexpr (H == 16) return __uint_as_float(partner16_u(__float_as_uint(x), lane));
  else return __uint_as_float(partner32_u(__float_as_uint(x), lane));
}
template <int H>
__device__ __forceinline__ int xchg(int x, int lane) {
  if constexpr (H == 1) return dpp<DPP_QUAD_XOR1>(x);
  else if constexpr (H == 2) return dpp<DPP_QUAD_XOR2>(x);
  else if constexpr (H == 4) return dpp<DPP_ROW_HALF_MIRROR>(x);
  else if constexpr (H == 8) return dpp<DPP_ROW_ROR8>(x);
  else if constexpr (H == 16) return (int)partner16_u((unsigned)x, lane);
  else return (int)partner32_u((unsigned)x, lane);
}

// Sum over groups of 8 lanes (lanes 8g..8g+7), result in all 8 lanes.
__device__ __forceinline__ float sum8(float x, int lane) {
  x = x + xchg<1>(x, lane);
  x = x + xchg<2>(x, lane);
  x = x + xchg<4>(x, lane);
  return x;
}

// Reduce-scatter step with partner "distance" H over N = 2H values: lanes whose partner bit
// is clear keep v[0..H) and receive their partner's v[0..H); the others keep v[H..2H).
// Afterwards v[0..H) hold pairwise sums. `up` = this lane is the upper partner.
template <int H>
__device__ __forceinline__ void rs_step(float* v, int lane, bool up) {
  const unsigned m = up ? 0xffffffffu : 0u;
#pragma unroll
  for (int q = 0; q < H; ++q) {
    const unsigned lo = __float_as_uint(v[q]), hi = __float_as_uint(v[q + H]);
    const float keep = __uint_as_float((lo & ~m) | (hi & m));
    const float send = __uint_as_float((hi & ~m) | (lo & m));
    v[q] = keep + xchg<H>(send, lane);
  }
}

// Reduce-scatter steps for the two widest distances: one v_permlane{32,16}_swap exchanges a
// pair of registers between partner lanes, after which (X' + Y') is the partner-pair sum of
// v[q] in the lanes whose partner bit is clear and of v[q+H] in the others -- no selects.
__device__ __forceinline__ void rs_step32_swap(float* v) {
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[q]), __float_as_uint(v[q + 32]),
                                              false, false);
    v[q] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}
__device__ __forceinline__ void rs_step16_swap(float* v) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[q]), __float_as_uint(v[q + 16]),
                                              false, false);
    v[q] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}

// Sum-reduce-scatter of 64 per-lane values: afterwards lane l holds sum over the wave of v[l].
__device__ __forceinline__ float reduce_scatter64(float (&v)[64], int lane) {
  rs_step32_swap(v);
  rs_step16_swap(v);
  rs_step<8>(v, lane, (lane & 8) != 0);
  rs_step<4>(v, lane, (lane & 4) != 0);
  rs_step<2>(v, lane, (lane & 2) != 0);
  rs_step<1>(v, lane, (lane & 1) != 0);
  return v[0];
}

// Value select through bit masks (a ternary on array elements can be folded into a
// dynamically indexed load, which sends the array to scratch memory).
__device__ __forceinline__ float bsel(unsigned m, float a_if_set, float b) {
  return __uint_as_float((__float_as_uint(b) & ~m) | (__float_as_uint(a_if_set) & m));
}
__device__ __forceinline__ int bsel(unsigned m, int a_if_set, int b) {
  return (int)(((unsigned)b & ~m) | ((unsigned)a_if_set & m));
}

// (dist, index) argmin combine: smaller distance wins, lower index on ties.
__device__ __forceinline__ void amin(float& d, int& i, float od, int oi) {
  const bool take = (od < d) | ((od == d) & (oi < i));  // bitwise: no short-circuit branches
  d = take ? od : d;
  i = take ? oi : i;
}

// Argmin-reduce-scatter of F = 8 (dist, index) pairs over the wave: afterwards every lane of
// the 8-lane group g = (lane >> 3) holds the wave-wide argmin of frame g.
__device__ __forceinline__ void argmin_scatter8(float (&d)[8], int (&ix)[8], int lane) {
  {  // H = 32: frames 0-3 stay in lower lanes, 4-7 in upper
    const unsigned up = (lane & 32) ? 0xffffffffu : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float kd = bsel(up, d[q + 4], d[q]), sd = bsel(up, d[q], d[q + 4]);
      const int ki = bsel(up, ix[q + 4], ix[q]), si = bsel(up, ix[q], ix[q + 4]);
      d[q] = kd; ix[q] = ki;
      amin(d[q], ix[q], xchg<32>(sd, lane), xchg<32>(si, lane));
    }
  }
  {  // H = 16
    const unsigned up = (lane & 16) ? 0xffffffffu : 0u;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float kd = bsel(up, d[q + 2], d[q]), sd = bsel(up, d[q], d[q + 2]);
      const int ki = bsel(up, ix[q + 2], ix[q]), si = bsel(up, ix[q], ix[q + 2]);
      d[q] = kd; ix[q] = ki;
      amin(d[q], ix[q], xchg<16>(sd, lane), xchg<16>(si, lane));
    }
  }
  {  // H = 8
    const unsigned up = (lane & 8) ? 0xffffffffu : 0u;
    const float kd = bsel(up, d[1], d[0]), sd = bsel(up, d[0], d[1]);
    const int ki = bsel(up, ix[1], ix[0]), si = bsel(up, ix[0], ix[1]);
    d[0] = kd; ix[0] = ki;
    amin(d[0], ix[0], xchg<8>(sd, lane), xchg<8>(si, lane));
  }
  // all-reduce inside each 8-lane group
  amin(d[0], ix[0], xchg<1>(d[0], lane), xchg<1>(ix[0], lane));
  amin(d[0], ix[0], xchg<2>(d[0], lane), xchg<2>(ix[0], lane));
  amin(d[0], ix[0], xchg<4>(d[0], lane), xchg<4>(ix[0], lane));
}

// Sum-reduce-scatter of 32 per-lane values: afterwards lanes l and l^32 both hold the
// wave-wide sum of v[l & 31].
__device__ __forceinline__ float reduce_scatter32(float (&v)[32], int lane) {
  rs_step16_swap(v);
  rs_step<8>(v, lane, (lane & 8) != 0);
  rs_step<4>(v, lane, (lane & 4) != 0);
  rs_step<2>(v, lane, (lane & 2) != 0);
  rs_step<1>(v, lane, (lane & 1) != 0);
  return v[0] + xchg<32>(v[0], lane);
}

// Argmin-reduce-scatter of 4 (dist, index) pairs over the wave: afterwards every lane of the
// 16-lane group g = (lane >> 4) holds the wave-wide argmin of frame g.
__device__ __forceinline__ void argmin_scatter4(float (&d)[4], int (&ix)[4], int lane) {
  {  // H = 32: frames 0-1 stay in lower lanes, 2-3 in upper
    const unsigned up = (lane & 32) ? 0xffffffffu : 0u;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float kd = bsel(up, d[q + 2], d[q]), sd = bsel(up, d[q], d[q + 2]);
      const int ki = bsel(up, ix[q + 2], ix[q]), si = bsel(up, ix[q], ix[q + 2]);
      d[q] = kd; ix[q] = ki;
      amin(d[q], ix[q], xchg<32>(sd, lane), xchg<32>(si, lane));
    }
  }
  {  // H = 16
    const unsigned up = (lane & 16) ? 0xffffffffu : 0u;
    const float kd = bsel(up, d[1], d[0]), sd = bsel(up, d[0], d[1]);
    const int ki = bsel(up, ix[1], ix[0]), si = bsel(up, ix[0], ix[1]);
    d[0] = kd; ix[0] = ki;
    amin(d[0], ix[0], xchg<16>(sd, lane), xchg<16>(si, lane));
  }
  // all-reduce inside each 16-lane row (quads first, then the mirror, then ror 8)
  amin(d[0], ix[0], xchg<1>(d[0], lane), xchg<1>(ix[0], lane));
  amin(d[0], ix[0], xchg<2>(d[0], lane), xchg<2>(ix[0], lane));
  amin(d[0], ix[0], xchg<4>(d[0], lane), xchg<4>(ix[0], lane));
  amin(d[0], ix[0], xchg<8>(d[0], lane), xchg<8>(ix[0], lane));
}

// Argmin-reduce-scatter of 16 (dist, index) pairs over the wave: afterwards the 4 lanes
// 4f .. 4f+3 hold the wave-wide argmin of frame f (smaller distance, lower index on ties).
// Every level's exchanges are independent (ILP 8, 4, 2, 1, then two 1-wide all-reduce steps).
__device__ __forceinline__ void argmin_scatter16(float (&d)[16], int (&ix)[16], int lane) {
  {  // H = 32: frames 0-7 stay in the lower half, 8-15 in the upper
    const unsigned up = (lane & 32) ? 0xffffffffu : 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float kd = bsel(up, d[q + 8], d[q]), sd = bsel(up, d[q], d[q + 8]);
      const int ki = bsel(up, ix[q + 8], ix[q]), si = bsel(up, ix[q], ix[q + 8]);
      d[q] = kd; ix[q] = ki;
      amin(d[q], ix[q], xchg<32>(sd, lane), xchg<32>(si, lane));
    }
  }
  {  // H = 16
    const unsigned up = (lane & 16) ? 0xffffffffu : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float kd = bsel(up, d[q + 4], d[q]), sd = bsel(up, d[q], d[q + 4]);
      const int ki = bsel(up, ix[q + 4], ix[q]), si = bsel(up, ix[q], ix[q + 4]);
      d[q] = kd; ix[q] = ki;
      amin(d[q], ix[q], xchg<16>(sd, lane), xchg<16>(si, lane));
    }
  }
  {  // H = 8
    const unsigned up = (lane & 8) ? 0xffffffffu : 0u;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float kd = bsel(up, d[q + 2], d[q]), sd = bsel(up, d[q], d[q + 2]);
      const int ki = bsel(up, ix[q + 2], ix[q]), si = bsel(up, ix[q], ix[q + 2]);
      d[q] = kd; ix[q] = ki;
      amin(d[q], ix[q], xchg<8>(sd, lane), xchg<8>(si, lane));
    }
  }
  {  // H = 4 (half-row mirror partner: lane i <-> 7-i, the upper lanes have bit 2 set)
    const unsigned up = (lane & 4) ? 0xffffffffu : 0u;
    const float kd = bsel(up, d[1], d[0]), sd = bsel(up, d[0], d[1]);
    const int ki = bsel(up, ix[1], ix[0]), si = bsel(up, ix[0], ix[1]);
    d[0] = kd; ix[0] = ki;
    amin(d[0], ix[0], xchg<4>(sd, lane), xchg<4>(si, lane));
  }
  // all-reduce inside each quad
  amin(d[0], ix[0], xchg<1>(d[0], lane), xchg<1>(ix[0], lane));
  amin(d[0], ix[0], xchg<2>(d[0], lane), xchg<2>(ix[0], lane));
}

}  // namespace vrvq
