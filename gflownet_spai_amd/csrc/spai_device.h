// Device helpers shared by the gfx950 kernels: Philox4x32-10, the deterministic fp32
// log used by the Gumbel keys, order-preserving float bits and wave64 reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spai {

constexpr int kWave = 64;  // CDNA wavefront

// Random123 Philox4x32-10 (KAT-checked in tests against oracle/spai_oracle.py).
__device__ __forceinline__ uint4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product (lo and hi together) instead of mul_lo + mul_hi
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    c1 = (uint32_t)p1;
    c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ uint32_t pick_word(const uint4& r, int s) {
  return s == 0 ? r.x : (s == 1 ? r.y : (s == 2 ? r.z : r.w));
}

// Deterministic ln(x) for positive normal fp32 x: bit-exact with oracle.det_logf.
// Only separately rounded fp32 multiplies/adds (contraction disabled), so the
// result does not depend on the compiler's FMA choices.
__device__ __forceinline__ float det_logf(float x) {
#pragma clang fp contract(off)
  uint32_t bits = __float_as_uint(x);
  int e = (int)(bits >> 23) - 127;
  uint32_t mb = (bits & 0x7FFFFFu) | 0x3F800000u;
  if (mb > 0x3FB504F3u) {
    mb -= 0x00800000u;
    e += 1;
  }
  const float t = __uint_as_float(mb) - 1.0f;
  float p = __uint_as_float(0x3db31375u);
  p = p * t + __uint_as_float(0xbe13394fu);
  p = p * t + __uint_as_float(0x3e191428u);
  p = p * t + __uint_as_float(0xbe2994dfu);
  p = p * t + __uint_as_float(0x3e4c5c05u);
  p = p * t + __uint_as_float(0xbe8002d3u);
  p = p * t + __uint_as_float(0x3eaaabc8u);
  p = p * t + __uint_as_float(0xbefffffcu);
  p = p * t + __uint_as_float(0x3f800000u);
  p = p * t;
  return (float)e * __uint_as_float(0x3f317218u) + p;
}

// key = l - ln(-ln u), u = (2*(word >> 9) + 1) * 2^-24 (exact), canonical +0.
__device__ __forceinline__ float gumbel_key(float logit, uint32_t word) {
#pragma clang fp contract(off)
  const uint32_t k = word >> 9;
  const float u = (2.0f * (float)k + 1.0f) * 5.9604644775390625e-08f;
  const float q = -det_logf(u);
  const float key = logit - det_logf(q);
  return key + 0.0f;
}

// Monotone map float -> uint32 (larger float => larger uint).
__device__ __forceinline__ uint32_t orderable(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64); result valid in every thread.
template <int NT, typename T>
__device__ __forceinline__ T block_sum(T v, T* lds /* NT/64 */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) lds[w] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += lds[i];
  return s;
}

}  // namespace spai
