// Issue-rate probe (dev tool): wave64 v_mad_u64_u32 vs v_xad / v_add on independent chains.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int K>
__global__ __launch_bounds__(256) void k_mad(uint32_t* out, int iters) {
  uint32_t a[8], c[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 7 + i; c[i] = blockIdx.x + i; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (K == 0) {  // 64-bit product of 32-bit operands (Philox's multiply)
        const uint64_t p = (uint64_t)0xD2511F53u * a[i];
        a[i] = (uint32_t)(p >> 32) ^ c[i];
        c[i] = (uint32_t)p;
      } else if constexpr (K == 1) {  // 32-bit low product
        a[i] = a[i] * 0xD2511F53u + c[i];
      } else {  // add / xor / rotate (ARX)
        a[i] = (a[i] + c[i]);
        c[i] = __builtin_amdgcn_alignbit(c[i], c[i], 13) ^ a[i];
      }
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i] ^ c[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  uint32_t* d;
  const int blocks = 256 * 8, iters = 4096;
  hipMalloc(&d, blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"mad_u64_u32 (+xor)", "mul_lo+add (mad_u32)", "add+alignbit+xor"};
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (k == 0) k_mad<0><<<blocks, 256>>>(d, iters);
      if (k == 1) k_mad<1><<<blocks, 256>>>(d, iters);
      if (k == 2) k_mad<2><<<blocks, 256>>>(d, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double waves = blocks * 4.0, chains = 8.0 * iters;
      // wave-instruction slots per SIMD per cycle estimate at 2.4 GHz, 1024 SIMDs
      const double per_wave_op_ns = ms * 1e6 / (waves * chains / 1024.0);
      if (rep) printf("%-24s %.3f ms  %.2f ns per wave-op per SIMD (%.1f cycles @2.4GHz)\n", names[k], ms, per_wave_op_ns, per_wave_op_ns * 2.4);
    }
  }
  hipFree(d);
  return 0;
}
