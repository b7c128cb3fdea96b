// Rollout kernels for gfx950: logits statistics, the reference-parity sampling step and
// the one-pass Gumbel-top-k trajectory sampler with its ordered trajectory log.
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
#include <hipcub/hipcub.hpp>

#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kNT = 256;         // threads per block
constexpr int kPer = 4;          // actions per thread (one Philox call)
constexpr int kBlk = kNT * kPer; // actions per block
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

// ------------------------------------------------------------------ throughput rollout
struct RolloutWs {
  int32_t nblk;
  int32_t* block_counts;  // [B][nblk]
  int32_t* block_offsets; // [B][nblk]
  int32_t* seg_start;     // [B]
  double* stot;           // [B]
  uint64_t* loc_keys;     // [B][nblk*kBlk]  (reused as scan output after compaction)
  int32_t* loc_acts;      // [B][nblk*kBlk]
  uint64_t* keys_in;      // [B*E]           (reused as fp64 weights after the sort)
  int32_t* acts_in;       // [B*E]           (reused as segment ids after the sort)
  uint64_t* keys_out;     // [B*E]
  int32_t* acts_out;      // [B*E]
  void* temp;
  size_t temp_bytes;
  size_t total_bytes;
};

static hipError_t cub_temp_bytes(int64_t n, size_t* out) {
  size_t sort_b = 0, scan_b = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                    (const int32_t*)nullptr, (int32_t*)nullptr, (int64_t)n, 0, 64,
                                                    (hipStream_t)0);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSumByKey(nullptr, scan_b, (const int32_t*)nullptr, (const double*)nullptr,
                                            (double*)nullptr, (int64_t)n, hipcub::Equality(), (hipStream_t)0);
  if (e != hipSuccess) return e;
  *out = std::max(sort_b, scan_b);
  return hipSuccess;
}

static hipError_t rollout_ws(void* base, int32_t E, int32_t B, RolloutWs* w) {
  Carve c(base);
  w->nblk = (E + kBlk - 1) / kBlk;
  const int64_t nb = (int64_t)B * w->nblk;
  const int64_t cap = (int64_t)B * E;
  w->block_counts = c.take<int32_t>(nb);
  w->block_offsets = c.take<int32_t>(nb);
  w->seg_start = c.take<int32_t>(B);
  w->stot = c.take<double>(B);
  w->loc_keys = c.take<uint64_t>(nb * kBlk);
  w->loc_acts = c.take<int32_t>(nb * kBlk);
  w->keys_in = c.take<uint64_t>(cap);
  w->acts_in = c.take<int32_t>(cap);
  w->keys_out = c.take<uint64_t>(cap);
  w->acts_out = c.take<int32_t>(cap);
  hipError_t e = cub_temp_bytes(cap > 0 ? cap : 1, &w->temp_bytes);
  if (e != hipSuccess) return e;
  w->temp = c.take<char>(w->temp_bytes);
  w->total_bytes = c.off;
  return hipSuccess;
}

__global__ __launch_bounds__(kNT) void k_select(const float* __restrict__ logits, int64_t bstride, int32_t E,
                                                int32_t nblk, uint32_t seed0, uint32_t seed1, uint32_t st0,
                                                uint32_t st1, int32_t sample_base, uint32_t* __restrict__ removed,
                                                int32_t words, int32_t* __restrict__ counts,
                                                int32_t* __restrict__ block_counts,
                                                uint64_t* __restrict__ loc_keys, int32_t* __restrict__ loc_acts) {
  const int b = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const float* lg = logits + (int64_t)b * bstride;
  const uint32_t bg = (uint32_t)(sample_base + b);
  __shared__ float s_tk;
  __shared__ int s_wc[kNT / 64];
  if (tid == 0) {
    const uint4 r = philox4x32_10((uint32_t)E >> 2, bg, st0, st1, seed0, seed1);
    s_tk = gumbel_key(lg[E], pick_word(r, E & 3));
  }
  __syncthreads();
  const float tk = s_tk;
  const int a0 = blk * kBlk + tid * kPer;
  uint32_t nib = 0;
  float key[kPer];
  if (a0 < E) {
    const uint4 r = philox4x32_10((uint32_t)a0 >> 2, bg, st0, st1, seed0, seed1);
#pragma unroll
    for (int s = 0; s < kPer; ++s) {
      key[s] = 0.0f;
      if (a0 + s < E) {
        key[s] = gumbel_key(lg[a0 + s], pick_word(r, s));
        if (key[s] > tk) nib |= 1u << s;
      }
    }
  }
  // removal bitmap: 8 lanes x 4 bits = one 32-bit word
  uint32_t x = nib << ((tid & 7) * kPer);
  x |= __shfl_xor(x, 1, kWave);
  x |= __shfl_xor(x, 2, kWave);
  x |= __shfl_xor(x, 4, kWave);
  if ((tid & 7) == 0) {
    const int wi = (blk * kBlk + (tid & ~7) * kPer) >> 5;
    if (wi < words) removed[(int64_t)b * words + wi] = x;
  }
  // block-local ordered compaction of the winners (key, action)
  const int c = __popc(nib);
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, kWave);
    if ((tid & 63) >= o) incl += y;
  }
  if ((tid & 63) == 63) s_wc[tid >> 6] = incl;
  __syncthreads();
  int wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kNT / 64; ++w) {
    if (w < (tid >> 6)) wbase += s_wc[w];
    tot += s_wc[w];
  }
  int pos = wbase + incl - c;
  const int64_t lbase = ((int64_t)b * nblk + blk) * kBlk;
#pragma unroll
  for (int s = 0; s < kPer; ++s) {
    if ((nib >> s) & 1u) {
      loc_keys[lbase + pos] = ((uint64_t)b << 32) | (uint64_t)(uint32_t)(~orderable(key[s]));
      loc_acts[lbase + pos] = a0 + s;
      ++pos;
    }
  }
  if (tid == 0) {
    block_counts[b * nblk + blk] = tot;
    if (tot) atomicAdd(&counts[b], tot);
  }
}

// Exclusive scan of the per-block winner counts of one sample (one 1024-thread block per sample).
__global__ __launch_bounds__(1024) void k_scan_blocks(const int32_t* __restrict__ block_counts, int32_t nblk,
                                                      int32_t* __restrict__ block_offsets) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int per = (nblk + 1023) / 1024;
  const int beg = min(tid * per, nblk), end = min(beg + per, nblk);
  const int32_t* bc = block_counts + (int64_t)b * nblk;
  int32_t* bo = block_offsets + (int64_t)b * nblk;
  int loc = 0;
  for (int i = beg; i < end; ++i) loc += bc[i];
  int incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, kWave);
    if ((tid & 63) >= o) incl += y;
  }
  __shared__ int s_wc[16];
  if ((tid & 63) == 63) s_wc[tid >> 6] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < (tid >> 6); ++w) base += s_wc[w];
  int run = base + incl - loc;
  for (int i = beg; i < end; ++i) {
    bo[i] = run;
    run += bc[i];
  }
}

__global__ void k_seg_start(const int32_t* __restrict__ counts, int32_t B, int32_t* __restrict__ seg_start,
                            double* __restrict__ stot) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int run = 0;
    for (int b = 0; b < B; ++b) {
      seg_start[b] = run;
      run += counts[b];
      stot[b] = 0.0;
    }
  }
}

__global__ __launch_bounds__(kNT) void k_compact(int32_t nblk, const int32_t* __restrict__ block_counts,
                                                 const int32_t* __restrict__ block_offsets,
                                                 const int32_t* __restrict__ seg_start,
                                                 const uint64_t* __restrict__ loc_keys,
                                                 const int32_t* __restrict__ loc_acts, uint64_t* __restrict__ keys,
                                                 int32_t* __restrict__ acts) {
  const int b = blockIdx.y, blk = blockIdx.x;
  const int n = block_counts[b * nblk + blk];
  const int64_t dst = (int64_t)seg_start[b] + block_offsets[b * nblk + blk];
  const int64_t src = ((int64_t)b * nblk + blk) * kBlk;
  for (int i = threadIdx.x; i < n; i += kNT) {
    keys[dst + i] = loc_keys[src + i];
    acts[dst + i] = loc_acts[src + i];
  }
}

__global__ __launch_bounds__(kNT) void k_weights(int64_t total, const uint64_t* __restrict__ keys,
                                                 const int32_t* __restrict__ acts, const float* __restrict__ logits,
                                                 int64_t bstride, const float* __restrict__ lmax,
                                                 int32_t* __restrict__ segid, double* __restrict__ wv) {
  const int64_t t = (int64_t)blockIdx.x * kNT + threadIdx.x;
  if (t >= total) return;
  const int b = (int)(keys[t] >> 32);
  const int a = acts[t];
  wv[t] = exp((double)logits[(int64_t)b * bstride + a] - (double)lmax[b]);
  segid[t] = b;
}

__global__ __launch_bounds__(kNT) void k_log_write(int64_t total, const int32_t* __restrict__ segid,
                                                   const int32_t* __restrict__ acts, const double* __restrict__ wv,
                                                   const double* __restrict__ S, const double* __restrict__ z,
                                                   const int32_t* __restrict__ seg_start,
                                                   const int32_t* __restrict__ counts, int64_t t_cap,
                                                   int64_t* __restrict__ actions, float* __restrict__ fwd,
                                                   double* __restrict__ stot) {
  const int64_t t = (int64_t)blockIdx.x * kNT + threadIdx.x;
  if (t >= total) return;
  const int b = segid[t];
  const int64_t tl = t - seg_start[b];
  const double w = wv[t], s = S[t];
  actions[(int64_t)b * t_cap + tl] = acts[t];
  fwd[(int64_t)b * t_cap + tl] = (float)(w / (z[b] - s));
  if (tl == counts[b] - 1) stot[b] = s + w;
}

__global__ __launch_bounds__(kNT) void k_log_pad(int32_t T, int32_t E, const int32_t* __restrict__ counts,
                                                 const double* __restrict__ stot, const double* __restrict__ z,
                                                 const float* __restrict__ logits, int64_t bstride,
                                                 const float* __restrict__ lmax, int64_t t_cap,
                                                 int64_t* __restrict__ actions, float* __restrict__ fwd) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * kNT + threadIdx.x;
  const int k = counts[b];
  if (t >= T || t < k) return;
  if (t == k) {
    const double wE = exp((double)logits[(int64_t)b * bstride + E] - (double)lmax[b]);
    actions[(int64_t)b * t_cap + t] = E;
    fwd[(int64_t)b * t_cap + t] = (float)(wE / (z[b] - stot[b]));
  } else {
    actions[(int64_t)b * t_cap + t] = -1;
    fwd[(int64_t)b * t_cap + t] = 1.0f;
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

extern "C" size_t spai_rollout_workspace_bytes(int32_t E, int32_t B) {
  if (E <= 0 || B <= 0) return 0;
  RolloutWs w;
  if (rollout_ws(nullptr, E, B, &w) != hipSuccess) return 0;
  return w.total_bytes;
}

extern "C" int spai_rollout_select(const float* logits, int64_t bstride, int32_t E, int32_t B, uint64_t seed,
                                   uint64_t stream_id, int32_t sample_base, uint32_t* removed, int32_t words,
                                   int32_t* counts, void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(logits && removed && counts && workspace, "spai_rollout_select: null pointer");
  SPAI_CHECK_ARG(E > 0 && B > 0 && bstride >= 0 && sample_base >= 0, "spai_rollout_select: bad shape");
  SPAI_CHECK_ARG(words == (E + 31) / 32, "spai_rollout_select: words must be ceil(E/32)");
  RolloutWs w;
  SPAI_CHECK_HIP(rollout_ws(workspace, E, B, &w));
  SPAI_CHECK_ARG(workspace_bytes >= w.total_bytes, "spai_rollout_select: workspace too small (%zu < %zu)",
                 workspace_bytes, w.total_bytes);
  hipStream_t s = (hipStream_t)stream;
  SPAI_CHECK_HIP(hipMemsetAsync(counts, 0, sizeof(int32_t) * B, s));
  k_select<<<dim3(w.nblk, B), kNT, 0, s>>>(logits, bstride, E, w.nblk, (uint32_t)seed, (uint32_t)(seed >> 32),
                                           (uint32_t)stream_id, (uint32_t)(stream_id >> 32), sample_base, removed,
                                           words, counts, w.block_counts, w.loc_keys, w.loc_acts);
  SPAI_CHECK_LAUNCH();
  k_scan_blocks<<<B, 1024, 0, s>>>(w.block_counts, w.nblk, w.block_offsets);
  SPAI_CHECK_LAUNCH();
  k_seg_start<<<1, 64, 0, s>>>(counts, B, w.seg_start, w.stot);
  SPAI_CHECK_LAUNCH();
  k_compact<<<dim3(w.nblk, B), kNT, 0, s>>>(w.nblk, w.block_counts, w.block_offsets, w.seg_start, w.loc_keys,
                                            w.loc_acts, w.keys_in, w.acts_in);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_rollout_order(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                  const double* z, const int32_t* counts, int64_t total, int32_t T, int64_t t_cap,
                                  int64_t* actions, float* fwd_probs, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  SPAI_CHECK_ARG(logits && lmax && z && counts && actions && fwd_probs && workspace,
                 "spai_rollout_order: null pointer");
  SPAI_CHECK_ARG(E > 0 && B > 0 && total >= 0 && total <= (int64_t)B * E && T >= 1 && t_cap >= T && T <= E + 1,
                 "spai_rollout_order: bad shape (E=%d B=%d total=%lld T=%d t_cap=%lld)", E, B, (long long)total, T,
                 (long long)t_cap);
  RolloutWs w;
  SPAI_CHECK_HIP(rollout_ws(workspace, E, B, &w));
  SPAI_CHECK_ARG(workspace_bytes >= w.total_bytes, "spai_rollout_order: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  if (total > 0) {
    int bbits = 0;
    while ((1 << bbits) < B) ++bbits;
    size_t tb = w.temp_bytes;
    SPAI_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.keys_in, w.keys_out, w.acts_in, w.acts_out,
                                                      total, 0, 32 + bbits, s));
    int32_t* segid = w.acts_in;                                   // reuse
    double* wv = reinterpret_cast<double*>(w.keys_in);            // reuse
    double* S = reinterpret_cast<double*>(w.loc_keys);            // reuse
    const int nb = (int)((total + kNT - 1) / kNT);
    k_weights<<<nb, kNT, 0, s>>>(total, w.keys_out, w.acts_out, logits, bstride, lmax, segid, wv);
    SPAI_CHECK_LAUNCH();
    tb = w.temp_bytes;
    SPAI_CHECK_HIP(hipcub::DeviceScan::ExclusiveSumByKey(w.temp, tb, segid, wv, S, total, hipcub::Equality(), s));
    k_log_write<<<nb, kNT, 0, s>>>(total, segid, w.acts_out, wv, S, z, w.seg_start, counts, t_cap, actions,
                                   fwd_probs, w.stot);
    SPAI_CHECK_LAUNCH();
  }
  k_log_pad<<<dim3((T + kNT - 1) / kNT, B), kNT, 0, s>>>(T, E, counts, w.stot, z, logits, bstride, lmax, t_cap,
                                                          actions, fwd_probs);
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
