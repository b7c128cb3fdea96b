// Rollout kernels for gfx950: logits statistics, the reference-parity sampling step and the
// actions -> removal-bitmap conversion (the one-pass sampler lives in trajectory.hip).
//
// Replaces the T-step Python loop of GFlowNet.sample_states (gflownet/gflownet.py:135-179)
// and Log.log (gflownet/log.py:24-89).  Layout in HBM (per rollout of B samples, E edges):
//   logits      fp32 [B or 1][E+1]        (policy output, state-independent per rollout)
//   removed     u32  [B][ceil(E/32)]      bit a = edge a removed (keep-bitmap complement)
//   actions     i64  [B][t_cap]           trajectory per sample (Log.actions is its transpose)
//   fwd_probs   f32  [B][t_cap]
// Every kernel is HBM/L2-bound integer + transcendental work: coalesced 4-wide action
// runs per lane, wave64 ballots/shuffles for the bitmap words and the block-local
// compaction, no MFMA (there is no matrix product on this path).
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kNT = 256;         // threads per block
constexpr int kStatChunk = 8192;
constexpr int kParChunk = 4096;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// ------------------------------------------------------------------ logits statistics
__global__ __launch_bounds__(kNT) void k_stats_partial(const float* __restrict__ logits, int64_t bstride,
                                                       int32_t E1, int32_t nchunk, float* __restrict__ pm,
                                                       double* __restrict__ ps) {
  const int b = blockIdx.y;
  const float* lg = logits + (int64_t)b * bstride;
  const int64_t beg = (int64_t)blockIdx.x * kStatChunk;
  const int64_t end = min(beg + (int64_t)kStatChunk, (int64_t)E1);
  __shared__ float sm[kNT / 64];
  __shared__ double sd[kNT / 64];
  float m = -INFINITY;
  for (int64_t i = beg + threadIdx.x; i < end; i += kNT) m = fmaxf(m, lg[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
  __syncthreads();
  m = sm[0];
#pragma unroll
  for (int i = 1; i < kNT / 64; ++i) m = fmaxf(m, sm[i]);
  double s = 0.0;
  for (int64_t i = beg + threadIdx.x; i < end; i += kNT) s += exp((double)lg[i] - (double)m);
  s = block_sum<kNT>(s, sd);
  if (threadIdx.x == 0) {
    pm[b * nchunk + blockIdx.x] = m;
    ps[b * nchunk + blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(64) void k_stats_final(const float* __restrict__ pm, const double* __restrict__ ps,
                                                    int32_t nchunk, int32_t B, int32_t shared,
                                                    float* __restrict__ lmax, double* __restrict__ z) {
  const int b = blockIdx.x;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < nchunk; i += 64) m = fmaxf(m, pm[b * nchunk + i]);
  m = wave_max(m);
  double s = 0.0;
  for (int i = threadIdx.x; i < nchunk; i += 64)
    s += ps[b * nchunk + i] * exp((double)pm[b * nchunk + i] - (double)m);
  s = wave_sum(s);
  if (threadIdx.x == 0) {
    if (shared) {
      for (int k = 0; k < B; ++k) {
        lmax[k] = m;
        z[k] = s;
      }
    } else {
      lmax[b] = m;
      z[b] = s;
    }
  }
}

// ------------------------------------------------------------------ reference-parity step
__device__ __forceinline__ void argmax_merge(float& s, int& a, float os, int oa) {
  if (os > s || (os == s && oa < a)) {
    s = os;
    a = oa;
  }
}

__global__ __launch_bounds__(kNT) void k_parity_partial(const float* __restrict__ logits, int64_t bstride,
                                                        int32_t E1, const float* __restrict__ noise,
                                                        const float* __restrict__ lmax,
                                                        const uint32_t* __restrict__ chosen, int32_t words1,
                                                        int32_t nchunk, float* __restrict__ pscore,
                                                        int32_t* __restrict__ pact) {
  const int b = blockIdx.y;
  const float* lg = logits + (int64_t)b * bstride;
  const float* nz = noise + (int64_t)b * E1;
  const uint32_t* ch = chosen + (int64_t)b * words1;
  const float lm = lmax[b];
  const int beg = blockIdx.x * kParChunk;
  const int end = min(beg + kParChunk, E1);
  float best = -1.0f;
  int besta = 0x7FFFFFFF;
  for (int a = beg + threadIdx.x; a < end; a += kNT) {
    const bool taken = (ch[a >> 5] >> (a & 31)) & 1u;
    const float s = taken ? 0.0f : expf(lg[a] - lm) / nz[a];
    argmax_merge(best, besta, s, a);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float os = __shfl_xor(best, o, kWave);
    const int oa = __shfl_xor(besta, o, kWave);
    argmax_merge(best, besta, os, oa);
  }
  __shared__ float ss[kNT / 64];
  __shared__ int sa[kNT / 64];
  if ((threadIdx.x & 63) == 0) {
    ss[threadIdx.x >> 6] = best;
    sa[threadIdx.x >> 6] = besta;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    best = ss[0];
    besta = sa[0];
    for (int w = 1; w < kNT / 64; ++w) argmax_merge(best, besta, ss[w], sa[w]);
    pscore[b * nchunk + blockIdx.x] = best;
    pact[b * nchunk + blockIdx.x] = besta;
  }
}

__global__ __launch_bounds__(64) void k_parity_commit(const float* __restrict__ logits, int64_t bstride,
                                                      int32_t E1, const float* __restrict__ lmax,
                                                      const float* __restrict__ pscore,
                                                      const int32_t* __restrict__ pact, int32_t nchunk,
                                                      uint32_t* __restrict__ chosen, int32_t words1,
                                                      uint8_t* __restrict__ active, double* __restrict__ zrem,
                                                      int64_t* __restrict__ out_action,
                                                      float* __restrict__ out_prob) {
  const int b = blockIdx.x;
  float best = -1.0f;
  int besta = 0x7FFFFFFF;
  for (int i = threadIdx.x; i < nchunk; i += 64) argmax_merge(best, besta, pscore[b * nchunk + i], pact[b * nchunk + i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float os = __shfl_xor(best, o, kWave);
    const int oa = __shfl_xor(besta, o, kWave);
    argmax_merge(best, besta, os, oa);
  }
  if (threadIdx.x == 0) {
    if (active[b]) {
      const int a = besta;
      chosen[(int64_t)b * words1 + (a >> 5)] |= 1u << (a & 31);
      const double w = exp((double)logits[(int64_t)b * bstride + a] - (double)lmax[b]);
      const double zr = zrem[b];
      out_action[b] = a;
      out_prob[b] = (float)(w / zr);
      zrem[b] = zr - w;
      if (a == E1 - 1) active[b] = 0;
    } else {
      out_action[b] = -1;
      out_prob[b] = 1.0f;
    }
  }
}

// ------------------------------------------------------------------ actions -> removal sets
__global__ __launch_bounds__(kNT) void k_actions_to_bits(const int64_t* __restrict__ actions, int64_t sb,
                                                         int64_t st, int32_t T, int32_t E,
                                                         uint32_t* __restrict__ removed, int32_t words) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * kNT + threadIdx.x;
  if (t >= T) return;
  const int64_t a = actions[(int64_t)b * sb + (int64_t)t * st];
  if (a >= 0 && a < E) atomicOr(&removed[(int64_t)b * words + (a >> 5)], 1u << (a & 31));
}

__global__ __launch_bounds__(kNT) void k_popcount(const uint32_t* __restrict__ removed, int32_t words,
                                                  int32_t* __restrict__ counts) {
  const int b = blockIdx.y;
  __shared__ int si[kNT / 64];
  int c = 0;
  for (int i = blockIdx.x * kNT + threadIdx.x; i < words; i += gridDim.x * kNT)
    c += __popc(removed[(int64_t)b * words + i]);
  c = block_sum<kNT>(c, si);
  if (threadIdx.x == 0 && c) atomicAdd(&counts[b], c);
}

}  // namespace
}  // namespace spai

using namespace spai;

// ================================================================== C ABI
extern "C" size_t spai_logits_stats_workspace_bytes(int32_t E1, int32_t B) {
  const int64_t nchunk = (E1 + kStatChunk - 1) / kStatChunk;
  Carve c(nullptr);
  c.take<float>(nchunk * B);
  c.take<double>(nchunk * B);
  return c.off;
}

extern "C" int spai_logits_stats(const float* logits, int64_t bstride, int32_t E1, int32_t B, float* lmax, double* z,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(logits && lmax && z && E1 > 0 && B > 0 && bstride >= 0, "spai_logits_stats: bad arguments");
  SPAI_CHECK_ARG(workspace_bytes >= spai_logits_stats_workspace_bytes(E1, B), "spai_logits_stats: workspace too small");
  const int nchunk = (E1 + kStatChunk - 1) / kStatChunk;
  const int Bl = bstride == 0 ? 1 : B;
  Carve c(workspace);
  float* pm = c.take<float>((size_t)nchunk * B);
  double* ps = c.take<double>((size_t)nchunk * B);
  hipStream_t s = (hipStream_t)stream;
  k_stats_partial<<<dim3(nchunk, Bl), kNT, 0, s>>>(logits, bstride, E1, nchunk, pm, ps);
  SPAI_CHECK_LAUNCH();
  k_stats_final<<<Bl, 64, 0, s>>>(pm, ps, nchunk, B, bstride == 0, lmax, z);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" size_t spai_parity_step_workspace_bytes(int32_t E1, int32_t B) {
  const int64_t nchunk = (E1 + kParChunk - 1) / kParChunk;
  Carve c(nullptr);
  c.take<float>(nchunk * B);
  c.take<int32_t>(nchunk * B);
  return c.off;
}

extern "C" int spai_parity_step(const float* logits, int64_t bstride, int32_t E1, int32_t B, const float* noise,
                                const float* lmax, uint32_t* chosen, int32_t words1, uint8_t* active, double* zrem,
                                int64_t* out_action, float* out_prob, void* workspace, size_t workspace_bytes,
                                void* stream) {
  SPAI_CHECK_ARG(logits && noise && lmax && chosen && active && zrem && out_action && out_prob,
                 "spai_parity_step: null pointer");
  SPAI_CHECK_ARG(E1 > 0 && B > 0 && bstride >= 0 && words1 == (E1 + 31) / 32, "spai_parity_step: bad shape");
  SPAI_CHECK_ARG(workspace_bytes >= spai_parity_step_workspace_bytes(E1, B), "spai_parity_step: workspace too small");
  const int nchunk = (E1 + kParChunk - 1) / kParChunk;
  Carve c(workspace);
  float* ps = c.take<float>((size_t)nchunk * B);
  int32_t* pa = c.take<int32_t>((size_t)nchunk * B);
  hipStream_t s = (hipStream_t)stream;
  k_parity_partial<<<dim3(nchunk, B), kNT, 0, s>>>(logits, bstride, E1, noise, lmax, chosen, words1, nchunk, ps, pa);
  SPAI_CHECK_LAUNCH();
  k_parity_commit<<<B, 64, 0, s>>>(logits, bstride, E1, lmax, ps, pa, nchunk, chosen, words1, active, zrem,
                                   out_action, out_prob);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_actions_to_removed(const int64_t* actions, int64_t stride_b, int64_t stride_t, int32_t B,
                                       int32_t T, int32_t E, uint32_t* removed, int32_t words, int32_t* counts,
                                       void* stream) {
  SPAI_CHECK_ARG(removed && counts && B > 0 && T >= 0 && E > 0, "spai_actions_to_removed: bad arguments");
  SPAI_CHECK_ARG(words == (E + 31) / 32, "spai_actions_to_removed: words must be ceil(E/32)");
  SPAI_CHECK_ARG(T == 0 || actions, "spai_actions_to_removed: null actions");
  hipStream_t s = (hipStream_t)stream;
  SPAI_CHECK_HIP(hipMemsetAsync(removed, 0, sizeof(uint32_t) * (size_t)B * words, s));
  SPAI_CHECK_HIP(hipMemsetAsync(counts, 0, sizeof(int32_t) * B, s));
  if (T > 0) {
    k_actions_to_bits<<<dim3((T + kNT - 1) / kNT, B), kNT, 0, s>>>(actions, stride_b, stride_t, T, E, removed, words);
    SPAI_CHECK_LAUNCH();
  }
  const int gx = std::min(64, (words + kNT - 1) / kNT);
  k_popcount<<<dim3(gx, B), kNT, 0, s>>>(removed, words, counts);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
