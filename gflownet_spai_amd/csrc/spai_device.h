// Device helpers shared by the gfx950 kernels: Philox4x32-10, the deterministic fp32
// log used by the Gumbel keys, order-preserving float bits and wave64 reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spai {

constexpr int kWave = 64;  // CDNA wavefront

// Streaming output stores (M of the fill, the trajectory log of k_sort2): `nt` stores, which do
// not keep the written lines in the caches — nothing in the step reads these outputs back, and
// these interleaved read/write streams run faster without allocating them (fill: 73 -> 64 us
// at C4).  Not for a pure write stream: k_pad's padding took 2x longer with them.
typedef unsigned int nt_u4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ void nt_store(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

constexpr int kNtAux = 2;              // buffer-store cache policy: nt (streaming output, gfx950)
constexpr int kBufWord3 = 0x00020000;  // buffer resource dword 3 (raw byte addressing)
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

// One sample's M block of a line block (ne = nvl * wrt values, contiguous at dst) from its LDS
// staging copy sm (NT * W values), with a FIXED number of buffer stores per thread: 16-byte
// stores over the whole 16-byte chunks, then one element store for the tail.  Stores past the
// block — all of them when dst is null (no M requested) — fall outside the buffer's bound and are
// dropped.  No branch skips a store, so the compiler's wait for the next sample's bitmap words
// (loaded before these stores; vmcnt counts in order) is vmcnt(stores), not vmcnt(0): a drain of
// the M stores per sample is an HBM write latency per sample.
// NT = 64 with t = the lane: one wave stores its own 64 lines (no block barrier before it: a
// wave's LDS operations complete in order).
template <int NT, int W, typename TM>
__device__ __forceinline__ void store_m_block(TM* dst, const TM* sm, int ne, int t = (int)threadIdx.x) {
  constexpr int kV = 16 / (int)sizeof(TM), kChunks = NT * W / kV;
  constexpr int kSt = (kChunks + NT - 1) / NT;
  static_assert(NT * W % kV == 0, "whole 16-byte chunks in the staging buffer");
  const int nfull = ne / kV;
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(dst, 0, dst ? nfull * 16 : 0, kBufWord3);
  const __amdgpu_buffer_rsrc_t re =
      __builtin_amdgcn_make_buffer_rsrc(dst, 0, dst ? ne * (int)sizeof(TM) : 0, kBufWord3);
#pragma unroll
  for (int i = 0; i < kSt; ++i) {
    const int c = i * NT + t;
    const u4v v = reinterpret_cast<const u4v*>(sm)[min(c, kChunks - 1)];
    __builtin_amdgcn_raw_buffer_store_b128(v, rv, c * 16, 0, kNtAux);
  }
  const int e = nfull * kV + min(t, kV - 1);  // the tail (< kV values): threads 0 .. kV - 1
  const int off = t < kV ? e * (int)sizeof(TM) : 0x7ffffff0;
  const TM x = sm[min(e, NT * W - 1)];
  if constexpr (sizeof(TM) == 4)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), re, off, 0, kNtAux);
  else {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    __builtin_amdgcn_raw_buffer_store_b64((u2v){(uint32_t)u, (uint32_t)(u >> 32)}, re, off, 0, kNtAux);
  }
}

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
// Horner in single-rounded fp32 FMAs (IEEE fmaf; the oracle emulates it exactly) and no
// other contraction, so the result never depends on the compiler's choices.
constexpr uint32_t kLogC[9] = {0x3f800000u, 0xbefffffcu, 0x3eaaabc8u, 0xbe8002d3u, 0x3e4c5c05u,
                               0xbe2994dfu, 0x3e191428u, 0xbe13394fu, 0x3db31375u};
__device__ __forceinline__ void log_reduce(float x, float& t, float& ef) {
  const uint32_t bits = __float_as_uint(x);
  int e = (int)(bits >> 23) - 127;
  uint32_t mb = (bits & 0x7FFFFFu) | 0x3F800000u;
  if (mb > 0x3FB504F3u) {
    mb -= 0x00800000u;
    e += 1;
  }
  t = __uint_as_float(mb) - 1.0f;  // exact
  ef = (float)e;
}
__device__ __forceinline__ float det_logf(float x) {
#pragma clang fp contract(off)
  float t, ef;
  log_reduce(x, t, ef);
  float p = __uint_as_float(kLogC[8]);
#pragma unroll
  for (int i = 7; i >= 0; --i) p = __builtin_fmaf(p, t, __uint_as_float(kLogC[i]));
  p = p * t;
  return __builtin_fmaf(ef, __uint_as_float(0x3f317218u), p);
}

// Two logs at once: the polynomial runs on packed fp32 (v_pk_fma_f32 / v_pk_mul_f32),
// bit-identical to two det_logf calls.
typedef float spai_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ spai_f2 det_logf2(spai_f2 x) {
#pragma clang fp contract(off)
  float t0, t1, e0, e1;
  log_reduce(x.x, t0, e0);
  log_reduce(x.y, t1, e1);
  const spai_f2 t = (spai_f2){t0, t1}, ef = (spai_f2){e0, e1};
  spai_f2 p = (spai_f2){__uint_as_float(kLogC[8]), __uint_as_float(kLogC[8])};
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    const float c = __uint_as_float(kLogC[i]);
    p = __builtin_elementwise_fma(p, t, (spai_f2){c, c});
  }
  p = p * t;
  const float l2 = __uint_as_float(0x3f317218u);
  return __builtin_elementwise_fma(ef, (spai_f2){l2, l2}, p);
}

// key = l - ln(-ln u), u = (2*(word >> 9) + 1) * 2^-24 (exact), canonical +0.
__device__ __forceinline__ float gumbel_u(uint32_t word) {
#pragma clang fp contract(off)
  const uint32_t k = word >> 9;
  return (2.0f * (float)k + 1.0f) * 5.9604644775390625e-08f;
}
__device__ __forceinline__ float gumbel_key(float logit, uint32_t word) {
#pragma clang fp contract(off)
  const float q = -det_logf(gumbel_u(word));
  const float key = logit - det_logf(q);
  return key + 0.0f;
}
// keys of two actions (words w0, w1) with the packed log
__device__ __forceinline__ spai_f2 gumbel_key2(spai_f2 logit, uint32_t w0, uint32_t w1) {
#pragma clang fp contract(off)
  const spai_f2 q = -det_logf2((spai_f2){gumbel_u(w0), gumbel_u(w1)});
  const spai_f2 key = logit - det_logf2(q);
  return key + (spai_f2){0.0f, 0.0f};
}

// Deterministic e^x in fp32, bit-exact with oracle.det_expf: k = rint(x * log2 e) (fp32),
// Cody-Waite r = x - k ln2 in two single-rounded FMAs, degree-7 Taylor Horner in fp32 FMAs,
// 2^k by ldexp (exact: results stay normal).  x > 88.72 -> +inf, x < -87.33 -> 0.
constexpr uint32_t kExpC[8] = {0x3f800000u, 0x3f800000u, 0x3f000000u, 0x3e2aaaabu,
                               0x3d2aaaabu, 0x3c088889u, 0x3ab60b61u, 0x39500d01u};
__device__ __forceinline__ float det_expf(float x) {
#pragma clang fp contract(off)
  if (x > 88.72f) return __uint_as_float(0x7f800000u);
  if (x < -87.33f) return 0.0f;
  const float k = __builtin_rintf(x * __uint_as_float(0x3fb8aa3bu));  // log2(e)
  float r = __builtin_fmaf(-k, __uint_as_float(0x3f317200u), x);      // ln2 head (exact k * head)
  r = __builtin_fmaf(-k, __uint_as_float(0x35bfbe8eu), r);            // ln2 tail
  float p = __uint_as_float(kExpC[7]);
#pragma unroll
  for (int i = 6; i >= 0; --i) p = __builtin_fmaf(p, r, __uint_as_float(kExpC[i]));
  return __builtin_ldexpf(p, (int)k);
}

// Exponential race (throughput sampler): action a arrives at t_a = q_a * r_a with
// q_a = -ln u_a ~ Exp(1) and r_a = e^(l_E - l_a) (the inverse rate relative to the terminal
// E, whose r is exactly 1), so t_a < t_E <=> key_a > key_E of the Gumbel keys l - ln q and
// the arrival order is the Plackett-Luce (sequential sampling) order.
__device__ __forceinline__ float arrival_q(uint32_t word) { return -det_logf(gumbel_u(word)); }
__device__ __forceinline__ spai_f2 arrival_q2(uint32_t w0, uint32_t w1) {
  return -det_logf2((spai_f2){gumbel_u(w0), gumbel_u(w1)});
}
// Trajectory-order key of an arrival time t >= 0: larger = earlier (ties: action ascending).
__device__ __forceinline__ uint32_t arrival_ord(float t) { return ~__float_as_uint(t); }

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

// Wave scans on DPP row shifts + row broadcasts (no LDS-permute traffic, no per-lane address
// registers): row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast 15 (rows 1, 3) and
// row_bcast 31 (rows 2, 3).  Lanes without a source add the identity (`old`).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int dpp_i(int ident, int v) {
  return __builtin_amdgcn_update_dpp(ident, v, kCtrl, kRowMask, 0xf, false);
}
// Inclusive wave scan (int).
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += dpp_i<0x111, 0xf>(0, v);
  v += dpp_i<0x112, 0xf>(0, v);
  v += dpp_i<0x114, 0xf>(0, v);
  v += dpp_i<0x118, 0xf>(0, v);
  v += dpp_i<0x142, 0xa>(0, v);
  v += dpp_i<0x143, 0xc>(0, v);
  return v;
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = __double_as_longlong(v);
  const int lo = dpp_i<kCtrl, kRowMask>(0, (int)(uint32_t)u), hi = dpp_i<kCtrl, kRowMask>(0, (int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));  // 0 bits = +0.0
}
// Inclusive wave scan (double, fixed association => deterministic).
__device__ __forceinline__ double wave_incl_scan_d(double v) {
  v += dpp_d<0x111, 0xf>(v);
  v += dpp_d<0x112, 0xf>(v);
  v += dpp_d<0x114, 0xf>(v);
  v += dpp_d<0x118, 0xf>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  return v;
}
// Wave-wide sum of doubles in a fixed association (deterministic), valid in every lane.
__device__ __forceinline__ double wave_sum_dpp(double v) {
  const uint64_t u = __double_as_longlong(wave_incl_scan_d(v));
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)u, 63), hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
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

// ---- exact, partition-invariant sums of fp64 partials (SPAI_RES2_LIMBS in spai_hip.h)
// A partial x is truncated (toward zero) to a multiple of 2^-96 and held as six signed 32-bit
// limbs in int64 slots, value = sum_i L_i 2^(32 i - 96), |x| < 2^94; slot 6 counts the partials
// that are not representable (NaN: bit 32 up, inf / |x| >= 2^94: bit 0 up).  Integer sums are
// associative, so summing the slots in any order, over any partition of the partials (the line
// shards of a multi-GPU job: one all_reduce of the slots), gives the same bits.
constexpr int kLimbSlots = 8;  // 6 limbs + flags + 1 pad (64 bytes per sample)
__device__ __forceinline__ void fixed_add(double x, int64_t (&L)[kLimbSlots]) {
  // branch-free (selects only): keeps L in registers
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  const int ex = (int)((u >> 52) & 0x7ff);
  const uint64_t frac = u & ((1ull << 52) - 1);
  const bool nan = ex == 0x7ff && frac != 0;
  const bool over = !nan && ex >= 1023 + 94;  // inf or |x| >= 2^94
  const uint64_t m = (nan || over) ? 0ull : (frac | (ex ? (1ull << 52) : 0ull));
  const int shift = (ex ? ex : 1) - 1075 + 96;  // x = m * 2^(shift - 96)
  const bool neg = (u >> 63) != 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int k = 32 * i - shift;  // limb i holds bits [k, k + 32) of m
    const uint64_t hi = (m >> min(max(k, 0), 63)) & 0xffffffffull;
    const uint64_t lo = (m << min(max(-k, 0), 63)) & 0xffffffffull;
    const uint64_t c = k >= 0 ? (k < 64 ? hi : 0ull) : (-k < 32 ? lo : 0ull);
    L[i] += neg ? -(int64_t)c : (int64_t)c;
  }
  L[6] += nan ? (1ll << 32) : (over ? 1ll : 0ll);
}
template <typename LA>
__device__ __forceinline__ double fixed_value(const LA& L) {
  const int64_t fl = L[6];
  if (fl >> 32) return __longlong_as_double(0x7ff8000000000000ll);  // NaN
  if (fl) return __longlong_as_double(0x7ff0000000000000ll);        // +inf
  int64_t c[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) c[i] = L[i];
#pragma unroll
  for (int i = 0; i < 5; ++i) {  // carry-normalise: c[0..4] in [0, 2^32), c[5] signed
    const int64_t carry = c[i] >> 32;
    c[i] -= carry * 4294967296ll;
    c[i + 1] += carry;
  }
  double v = (double)c[5];
#pragma unroll
  for (int i = 4; i >= 0; --i) v = fma(v, 4294967296.0, (double)c[i]);
  return v * 0x1p-96;
}
// Reward of preconditioner.py:55-66 + 137-165 with the reference's torch type promotion
// reproduced op for op: alpha is fp32, the residual ratio fp64, the flop ratio a python float,
// (1 - alpha) * (1 - flop_ratio) an fp32 product and the sum fp64.  Contraction is disabled so
// every op rounds as torch's separate kernels do.
struct RewardArgs {
  const int32_t* counts;  // removed per sample (nnz(M) = nnz0 - counts[b])
  int64_t nnz0;
  int32_t n;
  double r0, f0;
  const float* alpha;     // device fp32 scalar
  double* residual;       // [B] sqrt(res2)
  double* reward;         // [B] fp64
  float* reward32;        // [B] fp32 copy (Log.rewards' dtype, gflownet.py:193) or null
};
__device__ __forceinline__ void write_reward(int b, double res2, const RewardArgs& ra) {
#pragma clang fp contract(off)
  const double r = sqrt(res2);
  ra.residual[b] = r;
  const double rr = ra.r0 != 0.0 ? r / ra.r0 : INFINITY;
  const double flops = (double)(ra.nnz0 - ra.counts[b]) * 2.0 * (double)ra.n;
  const double cr = ra.f0 != 0.0 ? flops / ra.f0 : INFINITY;
  const float a = *ra.alpha;
  const double t1 = (double)a * (1.0 - rr);
  const float t2 = (1.0f - a) * (float)(1.0 - cr);
  const double rw = (t1 + (double)t2) * 1000.0;
  ra.reward[b] = rw;
  if (ra.reward32) ra.reward32[b] = (float)rw;
}

// Wave-wide int64 sum by DPP (row shifts + row broadcasts, as wave_incl_scan; no LDS permutes),
// valid in every lane.  Integer: any association gives the same bits.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int64_t dpp_add_i64(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const int lo = dpp_i<kCtrl, kRowMask>(0, (int)(uint32_t)u), hi = dpp_i<kCtrl, kRowMask>(0, (int)(uint32_t)(u >> 32));
  return v + (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
  v = dpp_add_i64<0x111, 0xf>(v);
  v = dpp_add_i64<0x112, 0xf>(v);
  v = dpp_add_i64<0x114, 0xf>(v);
  v = dpp_add_i64<0x118, 0xf>(v);
  v = dpp_add_i64<0x142, 0xa>(v);
  v = dpp_add_i64<0x143, 0xc>(v);
  const uint64_t u = (uint64_t)v;
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)u, 63), hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// res2_out[b] and/or limbs_out[b][kLimbSlots] from per-block fp64 partials [B][nparts], one block
// per sample (the fill kernels' second half).  Every load of a round is issued before the
// conversions (a dependent load per partial made this a 16 us latency chain at C4); DPP wave
// sums of the limbs.  The conversions are the VALU chain: 1024 threads x 4 partials (C4's 4096
// in one round); 256 threads x 16 took 13 us against 10.
template <int NT>
__global__ __launch_bounds__(NT) void k_fixed_reduce(const double* __restrict__ partials, int32_t nparts,
                                                     double* __restrict__ res2_out, int64_t* __restrict__ limbs_out,
                                                     RewardArgs ra) {
  constexpr int kPer = 4;
  __shared__ int64_t sred[NT / 64][kLimbSlots];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double* p = partials + (int64_t)b * nparts;
  int64_t L[kLimbSlots] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 1
  for (int i0 = 0; i0 < nparts; i0 += kPer * NT) {
    double v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = i0 + j * NT + (int)threadIdx.x;
      v[j] = i < nparts ? p[i] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) fixed_add(v[j], L);
  }
#pragma unroll
  for (int q = 0; q < 7; ++q) L[q] = wave_sum_i64(L[q]);
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < 7; ++q) sred[wave][q] = L[q];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t T[kLimbSlots] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int w = 0; w < NT / 64; ++w)
#pragma unroll
      for (int q = 0; q < 7; ++q) T[q] += sred[w][q];
    if (limbs_out) {
#pragma unroll
      for (int q = 0; q < kLimbSlots; ++q) limbs_out[(int64_t)b * kLimbSlots + q] = T[q];
    }
    const double r2 = fixed_value(T);
    if (res2_out) res2_out[b] = r2;
    if (ra.reward) write_reward(b, r2, ra);  // fused reward (one GPU: the sums are complete here)
  }
}

}  // namespace spai
