// One-pass trajectory sampler for gfx950 (throughput mode) — replaces the T-step loop of
// GFlowNet.sample_states (gflownet/gflownet.py:135-179) and Log.log (gflownet/log.py:24-89).
//
// Sampling without replacement until the terminal id E is drawn == an exponential race:
// action a arrives at t_a = q_a * r_a (q_a = -ln u_a ~ Exp(1), r_a = e^(l_E - l_a), r_E = 1);
// the removed set is {a < E : t_a < t_E} and the trajectory lists it by t ascending (ties:
// action ascending), then E.  (Equivalently the Gumbel keys l - ln q, ordered descending.)
//
// Ordering ~1e6 winners per sample is a SAMPLE SORT whose only global data movement is
// one coalesced staging write and one gather of contiguous runs:
//   k_presample  arrival times of a pseudo-random stratified subset of <= 65536 actions per
//                sample (1.2 % of the Philox work at C4); winners kept in subset order, each
//                block's key range, the terminal's arrival time; with the policy's fc block
//                maxima (spai_rollout_select_pm) one extra block reduces them to lmax.
//   k_splitters  per sample: value-linear histogram quantiles of the sampled winner keys
//                -> nb ~ est/4096 bucket splitters and a 4096-bin bucket lookup table.  Its
//                extra blocks precompute the per-action inverse rates r and weights
//                w = e^(l - lmax) once per logits row (shared by every sample of the row).
//   k_tile       one kTile (8192)-action tile of one sample per 512-thread block, two blocks
//                per CU (the samples of a tile share an XCD and its L2): Philox4x32-10 +
//                deterministic fp32 arrival times (in registers), removal bitmap words, the
//                fp64 mass of the untouched actions, bucket histogram with in-bucket ranks
//                and fixed-point per-bucket weight sums, and the tile's winners written
//                grouped by bucket through an LDS window as 12-byte records {action, key,
//                weight}; per-(bucket, tile) runs in a bucket-major table (one contiguous
//                row per bucket).
//   k_bsum       per (sample, bucket): winner count and weight sum over the tiles (the
//                exchange array of a split rollout).
//   k_bscan      per sample: bucket starts, winner count, untouched mass, later-bucket
//                suffix sums, T.
//   k_sort2      persistent, software-pipelined: the next bucket's runs (one per tile) are
//                gathered into registers while the current bucket is ranked in value-linear
//                LDS sub-buckets; fp64 in-bucket suffix sums and
//                fwd_probs = w / (W_rest + later buckets + in-bucket suffix).  Outputs stored
//                during the next bucket.  Buckets above the LDS capacity: an exact radix in
//                global memory by the block that meets them (big_bucket; rare).
//   k_pad        terminal step, -1 / 1.0 padding up to T = max_b k_b + 1.
// The step probability is formed from the mass still available at step t (untouched
// actions + trajectory suffix), so no "Z - prefix" cancellation occurs.  Every sum is taken
// in a fixed order: results are bit-reproducible run to run.
#include "spai_device.h"
#include "spai_status.h"
#include "spai_timer.h"

namespace spai {
namespace {

#ifndef KTILE
#define KTILE 8192
#endif
constexpr int kTile = KTILE;               // actions per tile (k_tile block; a run per bucket)
static_assert(kTile <= 65535, "run offsets and counts are packed in 16 bits (k_tile, k_sort2)");
#ifndef KGRPNT
#define KGRPNT 512
#endif
constexpr int kGrpNT = KGRPNT;             // threads of a k_tile block (16 actions each)
constexpr int kWin = 2048;                 // records per LDS output window of k_tile's slot path
constexpr int kList = 4000;                // compacted winners per k_tile block (<= 49 % of the tile; denser: slot path)
#ifndef KSAMPM
#define KSAMPM 65536
#endif
constexpr int kSampM = KSAMPM;             // subset size (power of two, capped by E)
constexpr int kSampNT = 256;
constexpr int kSampCap = 32768;            // sampled winners behind the splitters
constexpr int kMaxNsb = kSampM / kSampNT;  // presample blocks per sample (256)
#ifndef KTARGET
#define KTARGET 4096
#endif
constexpr int kTarget = KTARGET;            // winners per bucket (target)
constexpr int kMaxB = 2048;                // buckets per sample (11 bits in the LDS record)
constexpr int kCap2 = 8192;               // LDS capacity of k_sort2 (records per bucket)
constexpr int kMaxSub = 4096;              // value sub-buckets per bucket in k_sort2
constexpr int kBigWords = 256;             // k_sort2: buckets per block tracked for the oversized pass (x32)
constexpr int kSortNT = 1024;
constexpr int kRwChunk = 4 * kSortNT;      // actions per rate/weight block of k_splitters
constexpr int kMaxTiles = 2048;            // E <= kMaxTiles * kTile actions
constexpr int kFinNT = 256;
constexpr int kMaxSamples = 1024;          // B per rollout call
typedef unsigned int spai_u2 __attribute__((ext_vector_type(2)));
typedef unsigned int spai_u3 __attribute__((ext_vector_type(3)));
typedef unsigned int spai_u4 __attribute__((ext_vector_type(4)));
// (kBufWord3, kNtAux: spai_device.h)
constexpr int kBins = 4096;                // splitter histogram / bucket lookup table bins

struct TrajWs {
  int32_t ntiles, M;
  int32_t* ctl;           // zeroed per rollout: bigcnt | tdev | lastbig | pad
  int32_t* bigcnt;        // number of oversized buckets k_sort2 met (k_pad moves it to lastbig, then 0)
  int32_t* tdev;
  int32_t* lastbig;       // bigcnt of the last sort (kept for tests / diagnostics)
  double* xch;            // exchange array: [B][2][kMaxB] bucket weight sums | winner counts, then
                          // [B][8] caller slots (the residual limbs); a part fills its own buckets
  int32_t* samp_cnt;      // [B][M / kSampNT] winners per presample block
  uint32_t* samp_mm;      // [B][M / kSampNT][2] min / max winner key per presample block
  uint32_t* samp;         // [B][M] winner keys (orderable), block-compacted
  int32_t* nb;            // [B] buckets
  uint32_t* spl;          // [B][kMaxB] ascending orderable splitters
  uint16_t* lut;          // [B][kBins] bucket lookup table
  uint32_t* lut_base;     // [B][2] (min key, shift) of the table
  uint32_t* staging;      // [B][ntiles][kTile][3] records {action, ~ord, bits of w}, grouped by bucket per tile
  int64_t wstride;        // row stride of rr / ww: E + 1 rounded up to 4 (16-byte aligned rows)
  float* rr;              // [B][wstride] inverse rates r_a = e^(l_E - l_a) (row 0 only: shared logits)
  float* ww;              // [B][wstride] weights w_a = e^(l_a - lmax)
  uint64_t* wfix;         // [B][nwb][2] fixed-point weight total of each kRwChunk-action chunk (row 0 only: shared)
  uint32_t* runs;         // [B][kMaxB][ntiles] run of bucket k in tile t: offset << 16 | count (k_tile)
  double* tbw;            // [B][kMaxB][ntiles] weight sum of that run
  double* tile_wrest;     // [B][ntiles]
  int32_t* bstart;        // [B][kMaxB + 1]
  double* wrest;          // [B]
  double* bwsuf;          // [B][kMaxB]
  uint64_t* scratch;      // [B][E] oversized-bucket radix scratch
  float* tE;              // [B] the terminal's arrival time (k_presample; k_tile reads it)
  size_t total_bytes;
};

static size_t xch_doubles(int32_t B) { return (size_t)B * 2 * kMaxB + (size_t)B * 8; }

static void traj_ws(void* base, int32_t E, int32_t B, TrajWs* w) {
  Carve c(base);
  w->ntiles = (E + kTile - 1) / kTile;
  int M = 1;
  while (M * 2 <= E && M * 2 <= kSampM) M *= 2;
  w->M = M;
  const int nsb = (M + kSampNT - 1) / kSampNT;
  w->ctl = c.take<int32_t>(4);
  w->bigcnt = w->ctl;
  w->tdev = w->ctl + 1;
  w->lastbig = w->ctl + 2;
  w->xch = c.take<double>(xch_doubles(B));
  w->samp_cnt = c.take<int32_t>((size_t)B * nsb);
  w->samp_mm = c.take<uint32_t>((size_t)B * nsb * 2);
  w->samp = c.take<uint32_t>((size_t)B * M);
  w->nb = c.take<int32_t>(B);
  w->spl = c.take<uint32_t>((size_t)B * kMaxB);
  w->lut = c.take<uint16_t>((size_t)B * kBins);
  w->lut_base = c.take<uint32_t>((size_t)B * 2);
  w->staging = c.take<uint32_t>((size_t)B * w->ntiles * kTile * 3);
  w->wstride = ((int64_t)E + 1 + 3) & ~(int64_t)3;
  w->rr = c.take<float>((size_t)B * w->wstride);
  w->ww = c.take<float>((size_t)B * w->wstride);
  w->wfix = c.take<uint64_t>((size_t)B * 2 * ((w->wstride + kRwChunk - 1) / kRwChunk));
  w->runs = c.take<uint32_t>((size_t)B * kMaxB * w->ntiles);
  w->tbw = c.take<double>((size_t)B * kMaxB * w->ntiles);
  w->tile_wrest = c.take<double>((size_t)B * w->ntiles);
  w->bstart = c.take<int32_t>((size_t)B * (kMaxB + 1));
  w->wrest = c.take<double>(B);
  w->bwsuf = c.take<double>((size_t)B * kMaxB);
  w->scratch = c.take<uint64_t>((size_t)B * E);
  w->tE = c.take<float>(B);
  w->total_bytes = c.off;
}

// Wave-wide min / max of uint32 (uniform result): an inclusive scan, lane 63 read out.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = min(v, (uint32_t)dpp_i<0x111, 0xf>(-1, (int)v));
  v = min(v, (uint32_t)dpp_i<0x112, 0xf>(-1, (int)v));
  v = min(v, (uint32_t)dpp_i<0x114, 0xf>(-1, (int)v));
  v = min(v, (uint32_t)dpp_i<0x118, 0xf>(-1, (int)v));
  v = min(v, (uint32_t)dpp_i<0x142, 0xa>(-1, (int)v));
  v = min(v, (uint32_t)dpp_i<0x143, 0xc>(-1, (int)v));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)dpp_i<0x111, 0xf>(0, (int)v));
  v = max(v, (uint32_t)dpp_i<0x112, 0xf>(0, (int)v));
  v = max(v, (uint32_t)dpp_i<0x114, 0xf>(0, (int)v));
  v = max(v, (uint32_t)dpp_i<0x118, 0xf>(0, (int)v));
  v = max(v, (uint32_t)dpp_i<0x142, 0xa>(0, (int)v));
  v = max(v, (uint32_t)dpp_i<0x143, 0xc>(0, (int)v));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads (which __syncthreads would drain), so prefetches stay in flight.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool kLdsOnly>
__device__ __forceinline__ void scan_barrier() {
  if constexpr (kLdsOnly) lds_barrier();
  else __syncthreads();
}

// Block-wide exclusive scan of one int per thread (NT <= 1024); *total = block total.
// kLdsOnly: LDS-only barriers (outstanding global loads of the caller stay in flight).
template <int NT, bool kLdsOnly = false>
__device__ __forceinline__ int block_excl_scan(int v, int* lds /* NT/64 */, int* total) {
  const int incl = wave_incl_scan(v);
  scan_barrier<kLdsOnly>();
  if ((threadIdx.x & 63) == 63) lds[threadIdx.x >> 6] = incl;
  scan_barrier<kLdsOnly>();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const int x = lds[w];
    base += (w < (int)(threadIdx.x >> 6)) ? x : 0;
    tot += x;
  }
  *total = tot;
  return base + incl - v;
}

// Same for doubles (fixed summation order => deterministic).
template <int NT, bool kLdsOnly = false>
__device__ __forceinline__ double block_excl_scan_d(double v, double* lds, double* total) {
  const double incl = wave_incl_scan_d(v);
  scan_barrier<kLdsOnly>();
  if ((threadIdx.x & 63) == 63) lds[threadIdx.x >> 6] = incl;
  scan_barrier<kLdsOnly>();
  double base = 0.0, tot = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const double x = lds[w];
    if (w < (int)(threadIdx.x >> 6)) base += x;
    tot += x;
  }
  *total = tot;
  return base + (incl - v);
}

__device__ __forceinline__ uint32_t wave_and_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v &= (uint32_t)__shfl_xor((int)v, o, kWave);
  return v;
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, kWave);
  return v;
}

// Arrival time of the terminal: t_E = q_E (its inverse rate is exactly 1).
__device__ __forceinline__ float terminal_t(int32_t E, uint32_t bg, uint32_t st0, uint32_t st1, uint32_t seed0,
                                            uint32_t seed1) {
  const uint4 r = philox4x32_10((uint32_t)E >> 2, bg, st0, st1, seed0, seed1);
  return arrival_q(pick_word(r, E & 3));
}

// w = e^(l - lmax) in fp32 to within ~1 ulp: l - lmax is exact in fp64, split into a float
// head and a tiny tail, e^(hi + lo) = e^hi (1 + lo).
__device__ __forceinline__ float action_weight(float l, float lm) {
  const double d = (double)l - (double)lm;
  const float hi = (float)d, lo = (float)(d - (double)hi);
  const float e = det_expf(hi);
  return fmaf(e, lo, e);
}

// Stratified pseudo-random subset: subset index i -> stratum (i * odd) mod M -> one action
// of that stratum chosen by an integer hash; independent of the noise and of the logits.
__device__ __forceinline__ int32_t subset_action(int i, int M, int32_t E) {
  const uint32_t s = ((uint32_t)i * 0x9E3779B1u) & (uint32_t)(M - 1);
  const int64_t lo = (int64_t)s * E / M, hi = (int64_t)(s + 1) * E / M;
  uint32_t h = (uint32_t)i * 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (int32_t)(lo + (int64_t)(h % (uint32_t)(hi - lo)));
}

// First bucket of part p of np (buckets in trajectory order; part p orders [lo(p), lo(p+1))).
__host__ __device__ __forceinline__ int part_lo(int nb, int p, int np) { return (int)(((int64_t)nb * p) / np); }

// Block-wide exclusive scan of one uint64 per thread (packed 16-bit fields never overflow).
template <int NT>
__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t c, uint64_t* lds /* NT/64 */, uint64_t* total) {
  uint64_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(incl, o, kWave);
    if ((threadIdx.x & 63) >= o) incl += y;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 63) lds[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint64_t base = 0, t = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint64_t x = lds[w];
    base += (w < (int)(threadIdx.x >> 6)) ? x : 0ull;
    t += x;
  }
  *total = t;
  return base + incl - c;
}

#ifdef SPAI_PROF  // phase timing (variant builds only: make EXTRA=-DSPAI_PROF); slots 16*kernel + phase
__device__ unsigned long long g_prof[64];
__device__ __forceinline__ uint64_t prof_stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define PROF_INIT uint64_t pf_t = prof_stamp(), pf_acc[16] = {};
#define PROF(i)                          \
  if (threadIdx.x == 0) {                \
    const uint64_t pf_n = prof_stamp();   \
    pf_acc[i] += pf_n - pf_t;            \
    pf_t = pf_n;                         \
  }
#define PROF_END(base)     \
  if (threadIdx.x == 0)    \
    for (int q = 0; q < 16; ++q) atomicAdd(&g_prof[(base) + q], (unsigned long long)pf_acc[q]);
extern "C" int spai_debug_prof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof)) != hipSuccess) return 2;
  if (reset) {
    static const unsigned long long z[64] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#else
#define PROF_INIT
#define PROF(i)
#define PROF_END(base)
#endif

// ------------------------------------------------------------------ k_presample
// Philox stream id of this rollout: the kernel argument, or the device counter when the caller
// keeps one (graph replays draw fresh rollouts; k_bsum advances it at the end of the select phase).
__device__ __forceinline__ void stream_words(const uint64_t* sctr, uint32_t& st0, uint32_t& st1) {
  if (sctr) {
    const uint64_t v = *sctr;
    st0 = (uint32_t)v;
    st1 = (uint32_t)(v >> 32);
  }
}

// w (fp32 in [0, 1]) as the fixed-point integer of k_tile's per-bucket sums: w * 2^47 for
// w >= 2^-20, else w * 2^69, truncated — from the float's bits (mantissa shifted by its
// exponent), identical to (uint64)(w * 2^s) in fp64 at a fraction of its instructions.
__device__ __forceinline__ uint64_t weight_fixed(float w) {
  const uint32_t bits = __float_as_uint(w);
  const int ex = (int)(bits >> 23);  // w >= 0: no sign bit
  if (ex == 0) return 0ull;          // zero or denormal (< 2^-126): below both units
  const uint64_t man = (uint64_t)((bits & 0x7FFFFFu) | 0x800000u);  // w = man * 2^(ex - 150)
  const int sh = ex - 150 + (ex >= 107 ? 47 : 69);                  // 2^-20 <=> ex >= 107
  return sh >= 0 ? man << sh : man >> min(-sh, 63);
}

// Inverse rates r = e^(l_E - l) and weights w = e^(l - lmax) of one chunk (NT * 4 actions) of
// one logits row, for k_tile; the row padding past E gets r = inf (never a winner), w = 0.  Also
// the chunk's total weight over its actions < E as exact fixed point (weight_fixed: hi units for
// w >= 2^-20, lo units below), wfix[row][chunk][2]: k_tile forms a tile's untouched mass as that
// total minus its winners' (integers, so the result is independent of any summation order).
// Run by the extra blocks of k_splitters, so this HBM stream overlaps the B splitter blocks.
template <int NT>
__device__ __forceinline__ void rates_weights_chunk(int q, const float* __restrict__ logits, int64_t bstride,
                                                    int32_t E, const float* __restrict__ lmax,
                                                    float* __restrict__ rr, float* __restrict__ ww, int64_t wstride,
                                                    uint64_t* __restrict__ wfix) {
  constexpr int kPer = 4, kChunkA = NT * kPer;
  const int tid = threadIdx.x;
  const int nwb = (int)((wstride + kChunkA - 1) / kChunkA);
  const int row = q / nwb;
  const float* lg = logits + (int64_t)row * bstride;
  const int64_t beg = (int64_t)(q % nwb) * kChunkA + tid;
  const float lE = lg[E], lm = lmax[row];
  float* r = rr + (int64_t)row * wstride;
  float* w = ww + (int64_t)row * wstride;
  float l[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {  // every load in flight before the math
    const int64_t i = beg + j * NT;
    l[j] = i <= E ? lg[i] : 0.0f;
  }
  uint64_t fh = 0, fl = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = beg + j * NT;
    if (i <= E) {
      r[i] = det_expf(lE - l[j]);
      const float wv = action_weight(l[j], lm);
      w[i] = wv;
      if (i < E) {
        const uint64_t f = weight_fixed(wv);
        if (wv >= 9.5367431640625e-07f) fh += f;
        else fl += f;
      }
    } else if (i < wstride) {
      r[i] = __uint_as_float(0x7f800000u);
      w[i] = 0.0f;
    }
  }
  __shared__ uint64_t s_fx[NT / 64][2];
  fh = (uint64_t)wave_sum_i64((int64_t)fh);
  fl = (uint64_t)wave_sum_i64((int64_t)fl);
  if ((tid & 63) == 0) {
    s_fx[tid >> 6][0] = fh;
    s_fx[tid >> 6][1] = fl;
  }
  __syncthreads();
  if (tid < 2) {
    uint64_t t = 0;
#pragma unroll
    for (int v = 0; v < NT / 64; ++v) t += s_fx[v][tid];
    wfix[(int64_t)q * 2 + tid] = t;
  }
}

__global__ __launch_bounds__(kSampNT) void k_presample(const float* __restrict__ logits, int64_t bstride, int32_t E,
                                                       int32_t M, int32_t nsb, uint32_t seed0, uint32_t seed1,
                                                       uint32_t st0, uint32_t st1, const uint64_t* __restrict__ sctr,
                                                       int32_t sample_base,
                                                       uint32_t* __restrict__ samp, int32_t* __restrict__ samp_cnt,
                                                       uint32_t* __restrict__ samp_mm,
                                                       int32_t* __restrict__ ctl, int32_t nctl, float* __restrict__ tE_out,
                                                       const float* __restrict__ lmax_parts, int32_t n_lmax_parts,
                                                       float* __restrict__ lmax_out, int32_t B) {
  const int tid = threadIdx.x;
  if (lmax_parts != nullptr && blockIdx.x == gridDim.x - 1) {
    // the deferred logits maximum (spai_policy_logits with B = 0 left its fc block maxima): one block
    // reduces them here, so the policy needs no reduction launch; its first reader is k_splitters
    constexpr int kRound = 8;
    float v = -INFINITY;
#pragma unroll 1
    for (int k0 = 0; k0 < n_lmax_parts; k0 += kRound * kSampNT) {
      float x[kRound];
#pragma unroll
      for (int j = 0; j < kRound; ++j) {
        const int k = k0 + j * kSampNT + tid;
        x[j] = k < n_lmax_parts ? lmax_parts[k] : -INFINITY;
      }
#pragma unroll
      for (int j = 0; j < kRound; ++j) v = fmaxf(v, x[j]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    __shared__ float s_mx[kSampNT / 64];
    if ((tid & 63) == 0) s_mx[tid >> 6] = v;
    __syncthreads();
    float r = s_mx[0];
#pragma unroll
    for (int k = 1; k < kSampNT / 64; ++k) r = fmaxf(r, s_mx[k]);
    for (int bb = tid; bb < B; bb += kSampNT) lmax_out[bb] = r;
    return;
  }
  stream_words(sctr, st0, st1);
  {  // the rollout's control block (bucket totals, oversized-bucket list count, tdev) starts at 0;
     // its first users (k_tile, k_sort2, k_bscan) run after this launch on the same stream
    const int nthr = gridDim.x * kSampNT;
    for (int q = blockIdx.x * kSampNT + tid; q < nctl; q += nthr) ctl[q] = 0;
  }
  const int b = blockIdx.x / nsb, blk = blockIdx.x % nsb;
  const float* lg = logits + (int64_t)b * bstride;
  const uint32_t bg = (uint32_t)(sample_base + b);
  __shared__ float s_tk;
  __shared__ int s_wc[kSampNT / 64];
  if (tid == 0) {
    s_tk = terminal_t(E, bg, st0, st1, seed0, seed1);
    if (blk == 0) tE_out[b] = s_tk;  // for k_tile: one Philox call per sample instead of per thread
  }
  __syncthreads();
  const int i = blk * kSampNT + tid;
  int win = 0;
  uint32_t o = 0;
  if (i < M) {
    const int32_t a = subset_action(i, M, E);
    const uint4 r = philox4x32_10((uint32_t)a >> 2, bg, st0, st1, seed0, seed1);
    const float t = arrival_q(pick_word(r, a & 3)) * det_expf(lg[E] - lg[a]);
    if (t < s_tk) {
      win = 1;
      o = arrival_ord(t);
    }
  }
  // the block's winner key range (for k_splitters' histogram range: no staging pass there)
  __shared__ uint32_t s_kmn[kSampNT / 64], s_kmx[kSampNT / 64];
  {
    const uint32_t wmn = wave_min_u32(win ? o : 0xFFFFFFFFu), wmx = wave_max_u32(win ? o : 0u);
    if ((tid & 63) == 0) {
      s_kmn[tid >> 6] = wmn;
      s_kmx[tid >> 6] = wmx;
    }
  }
  int tot;
  const int pos = block_excl_scan<kSampNT>(win, s_wc, &tot);  // (its barriers publish s_kmn / s_kmx)
  if (win) samp[(int64_t)b * M + blk * kSampNT + pos] = o;
  if (tid == 0) {
    samp_cnt[b * nsb + blk] = tot;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
#pragma unroll
    for (int w = 0; w < kSampNT / 64; ++w) {
      mn = min(mn, s_kmn[w]);
      mx = max(mx, s_kmx[w]);
    }
    samp_mm[(b * nsb + blk) * 2] = mn;
    samp_mm[(b * nsb + blk) * 2 + 1] = mx;
  }
}

// ------------------------------------------------------------------ k_splitters
// Splitters at equal-count quantiles of the sampled winner keys (up to kSampCap, in subset
// order) from a 4096-bin value-linear histogram over [min, max] of the sample (orderable
// space), interpolating inside a bin: monotone in j, no sort, four block barriers.
__global__ __launch_bounds__(kSortNT) void k_splitters(int32_t E, int32_t M, int32_t nsb,
                                                       const uint32_t* __restrict__ samp,
                                                       const int32_t* __restrict__ samp_cnt,
                                                       const uint32_t* __restrict__ samp_mm,
                                                       int32_t* __restrict__ nb_out, uint32_t* __restrict__ spl,
                                                       uint16_t* __restrict__ lut, uint32_t* __restrict__ lut_base,
                                                       int32_t B, const float* __restrict__ logits, int64_t bstride,
                                                       const float* __restrict__ lmax, float* __restrict__ rr,
                                                       float* __restrict__ ww, int64_t wstride,
                                                       uint64_t* __restrict__ wfix) {
  if ((int)blockIdx.x >= B) {  // blocks [B, ...): rates and weights of the logits rows
    rates_weights_chunk<kSortNT>(blockIdx.x - B, logits, bstride, E, lmax, rr, ww, wstride, wfix);
    return;
  }
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  PROF_INIT
  // (no key staging in LDS: the histogram is built from the keys' registers; ~21 KB of LDS)
  __shared__ int hist[kBins + 1];
  __shared__ int sblk[kMaxNsb + 1];
  __shared__ int s_wc[kSortNT / 64];
  __shared__ uint32_t s_mn[kSortNT / 64], s_mx[kSortNT / 64];
  const int c = tid < nsb ? samp_cnt[b * nsb + tid] : 0;
  // the winner key range from k_presample's per-block ranges (one load round with the counts)
  uint32_t mn = tid < nsb ? samp_mm[(b * nsb + tid) * 2] : 0xFFFFFFFFu;
  uint32_t mx = tid < nsb ? samp_mm[(b * nsb + tid) * 2 + 1] : 0u;
  mn = wave_min_u32(mn);
  mx = wave_max_u32(mx);
  if (lane == 0) {
    s_mn[wave] = mn;
    s_mx[wave] = mx;
  }
  int total;
  const int ex = block_excl_scan<kSortNT>(c, s_wc, &total);
  if (tid < nsb) sblk[tid] = ex;
  if (tid == 0) sblk[nsb] = total;
  for (int i = tid; i <= kBins; i += kSortNT) hist[i] = 0;
  __syncthreads();
  PROF(0)
  const int ns = min(total, kSampCap);
  mn = 0xFFFFFFFFu;
  mx = 0u;
#pragma unroll
  for (int w = 0; w < kSortNT / 64; ++w) {
    mn = min(mn, s_mn[w]);
    mx = max(mx, s_mx[w]);
  }
  const uint32_t range = ns > 0 ? mx - mn : 0u;
  const int shift = range >= (uint32_t)kBins ? 32 - __clz((int)(range >> 12)) : 0;  // (range >> shift) < kBins
  const uint32_t* sb = samp + (int64_t)b * M;
  // histogram of the first ns sampled winners, read in two halves with every load of a half in
  // flight at once: wave w reads presample blocks w*kBPW .. w*kBPW + kBPW - 1 (kSampNT keys
  // each, kLPB per lane)
  constexpr int kBPW = kMaxNsb / (kSortNT / 64), kLPB = kSampNT / 64, kHalf = kBPW / 2;
  static_assert(kMaxNsb % (kSortNT / 64) == 0 && kSampNT % 64 == 0 && kBPW % 2 == 0 && kHalf * kLPB <= 32,
                "k_splitters key rounds (the 32-bit validity mask of a half)");
#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    uint32_t v[kHalf * kLPB];
    uint32_t ok = 0;
#pragma unroll
    for (int j = 0; j < kHalf; ++j) {
      const int k = wave * kBPW + h * kHalf + j;
      const int beg = k < nsb ? sblk[k] : ns, cnt = k < nsb ? min(sblk[k + 1], ns) - beg : 0;
#pragma unroll
      for (int q = 0; q < kLPB; ++q) {
        const int i = lane + 64 * q;
        const bool in = i < cnt;
        v[j * kLPB + q] = in ? sb[k * kSampNT + i] : 0u;
        ok |= (uint32_t)in << (j * kLPB + q);
      }
    }
#pragma unroll
    for (int j = 0; j < kHalf; ++j)
#pragma unroll
      for (int q = 0; q < kLPB; ++q)
        if ((ok >> (j * kLPB + q)) & 1u) atomicAdd(&hist[(v[j * kLPB + q] - mn) >> shift], 1);
  }
  __syncthreads();
  PROF(2)
  // exclusive scan of the bins (4 per thread), in place
  {
    int cv[4], loc = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cv[q] = hist[tid * 4 + q];
      loc += cv[q];
    }
    int t2;
    int run = block_excl_scan<kSortNT>(loc, s_wc, &t2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      hist[tid * 4 + q] = run;
      run += cv[q];
    }
    if (tid == 0) hist[kBins] = t2;
  }
  __syncthreads();
  PROF(3)
  // bucket count from the winner estimate: >= 16 sampled winners per bucket
  const double est = (double)total * (double)E / (double)M;
  int nb = (int)ceil(est / (double)kTarget);
  nb = max(1, min(nb, min(kMaxB, max(1, ns / 16))));
  __shared__ uint32_t s_spl[kMaxB];
  for (int j = tid + 1; j < nb; j += kSortNT) {
    const int64_t rj = (int64_t)j * ns / nb;  // target rank
    int lo = 0, hi = kBins - 1;               // last bin with start <= rj
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (hist[mid] <= rj) lo = mid;
      else hi = mid - 1;
    }
    const int cnt = hist[lo + 1] - hist[lo];
    const double frac = cnt > 0 ? (double)(rj - hist[lo]) / (double)cnt : 0.0;
    const uint64_t v = (uint64_t)mn + ((uint64_t)lo << shift) + (uint64_t)(frac * (double)(1ull << shift));
    const uint32_t sv = (uint32_t)min(v, (uint64_t)mx);
    spl[(int64_t)b * kMaxB + j - 1] = sv;
    s_spl[j - 1] = sv;
  }
  __syncthreads();
  PROF(4)
  // lookup table over the same bins: lut[bin] = #(splitters < start of bin); a key's bucket
  // count is then lut[bin] plus the few splitters inside its bin (bucket_lut)
  for (int bin = tid; bin < kBins; bin += kSortNT) {
    const uint64_t start = (uint64_t)mn + ((uint64_t)bin << shift);
    int lo = 0, hi = nb - 1;  // lower_bound over s_spl[0 .. nb-2]
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((uint64_t)s_spl[mid] < start) lo = mid + 1;
      else hi = mid;
    }
    lut[(int64_t)b * kBins + bin] = (uint16_t)lo;
  }
  if (tid == 0) {
    nb_out[b] = nb;
    lut_base[2 * b] = mn;
    lut_base[2 * b + 1] = (uint32_t)shift;
  }
  PROF(5)
  PROF_END(16)
}


// ------------------------------------------------------------------ k_tile
// Selection and grouping fused, one 8192-action tile of one sample per block: arrival times
// of the tile (16 actions per thread; times and weights kept in registers), the removed
// bitmap, the rest mass of the tile's non-winners, then the grouping steps on the
// register-resident winners: bucket histogram, per-(bucket, tile) runs, and the winners
// re-written grouped by bucket through LDS windows (whole cache lines out).  The splitter
// tables load while the times are computed, so the only exposed global trip is the read of
// the tile's inverse rates and weights.  Block -> (tile, sample): the samples of one tile are
// consecutive blocks of one XCD (bijective XCD remap), so the rate/weight rows are read from
// HBM once per tile and served to the other samples by that XCD's L2.
constexpr int kTileG = kTile / (kGrpNT * 4);  // Philox groups (of 4 actions) per thread: 4
constexpr int kXcd = 8;
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int x = orig % kXcd, q = nwg / kXcd, r = nwg % kXcd;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / kXcd;
}
__global__ __launch_bounds__(kGrpNT) __attribute__((amdgpu_waves_per_eu(2 * kGrpNT / 256)))  // two blocks per CU
void k_tile(const float* __restrict__ rr, const float* __restrict__ ww, int64_t wstride, int64_t rowsel,
            int32_t E, int32_t B, int32_t ntiles, uint32_t seed0, uint32_t seed1, uint32_t st0, uint32_t st1,
            const uint64_t* __restrict__ sctr, int32_t sample_base, int32_t part, int32_t nparts,
            uint32_t* __restrict__ removed, int32_t words, const int32_t* __restrict__ nb_,
            const uint32_t* __restrict__ spl_, const uint16_t* __restrict__ lut_,
            const uint32_t* __restrict__ lut_base, uint32_t* __restrict__ staging,
            uint32_t* __restrict__ runs, double* __restrict__ tbw, double* __restrict__ tile_wrest,
            const float* __restrict__ tE_in, const uint64_t* __restrict__ wfix, int32_t nwb) {
  // LDS regions (two blocks per CU: <= 80 KB per block):
  //   s_r0: the slot path's record window
  //   s_r1: the compacted winner list: keys, weights, tile-local ids; once the list is read into
  //         registers, the fixed-point bucket sums (slot path: those sums, then the window's weights)
  // one array: the compact path's output staging (3 words per winner) spans both regions
  __shared__ __attribute__((aligned(16))) uint32_t s_r01[2 * kWin + 2 * kList + kList / 2];
  static_assert(2 * kWin + 2 * kList + kList / 2 >= 3 * kList, "compact staging fits the two regions");
  uint64_t* s_r0 = reinterpret_cast<uint64_t*>(s_r01);
  uint32_t* s_r1 = s_r01 + 2 * kWin;
  static_assert(kWin <= 2 * kList + kList / 2 && kList % 2 == 0, "LDS region sizes");
  uint64_t* w_rec = s_r0;  // one window of the slot path's grouped output
  float* w_log = reinterpret_cast<float*>(s_r1);
  uint32_t* l_ord = s_r1;
  float* l_w = reinterpret_cast<float*>(s_r1 + kList);  // the weight travels with the winner: no reload
  uint16_t* l_id = reinterpret_cast<uint16_t*>(s_r1 + 2 * kList);
  __shared__ __attribute__((aligned(16))) uint32_t s_spl[kMaxB];
  __shared__ int s_off[kMaxB + 1];  // histogram, then tile-local bucket offsets
  __shared__ __attribute__((aligned(16))) uint16_t s_lut[kBins];
  __shared__ int s_wc[kGrpNT / 64];
  __shared__ uint64_t s_fxo[2];              // fixed-point weight of the winners of OTHER parts' buckets
  __shared__ uint64_t s_fxw[kGrpNT / 64][2];  // per wave: the tile's winner weight (hi, lo units)
#ifdef KTILE_NOREMAP
  const int wg = (blockIdx.x % (gridDim.x / B)) * B + blockIdx.x / (gridDim.x / B);  // sample-major order
#else
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
#endif
  const int b = wg % B, tile = wg / B, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  PROF_INIT
  stream_words(sctr, st0, st1);
  const float* rrow = rr + (int64_t)b * rowsel * wstride;  // rowsel 0: one shared row
  const float* wrow = ww + (int64_t)b * rowsel * wstride;
  const uint32_t bg = (uint32_t)(sample_base + b);
  const int nb = nb_[b];
  // buckets [k0, k1) are ordered by this part (the others only counted: the removal bitmap,
  // the bucket totals and the untouched mass cover every action in every part)
  const int k0 = part_lo(nb, part, nparts), k1 = part_lo(nb, part + 1, nparts);
  // splitter tables (consumed only after the times; their latency hides behind the Philox work)
  static_assert(kBins * 2 == 512 * 16 && kMaxB * 4 <= 512 * 16 && kGrpNT == 512, "prologue vector widths");
  // direct global -> LDS loads (no VGPR destination, nothing waits on them until the barrier
  // after the times): 16 bytes per lane into a wave-contiguous 1 KB of the table
  for (int i0 = 0; i0 < 1024; i0 += kGrpNT) {
    const int i = i0 + tid, wb = i0 + (tid & ~63);  // wave base (uniform within the wave)
    if (wb < 512)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(lut_ + (int64_t)b * kBins) + i,
                                       reinterpret_cast<uint4*>(s_lut) + wb, 16, 0, 0);
    else if ((i - 512) * 4 < nb - 1)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(spl_ + (int64_t)b * kMaxB) + (i - 512),
                                       reinterpret_cast<uint4*>(s_spl) + (wb - 512), 16, 0, 0);
  }
  for (int k = tid; k < nb; k += kGrpNT) s_off[k] = 0;
  // per-bucket weight sums of the tile's winners as exact fixed point (integer LDS atomics: the
  // result is independent of their order): w >= 2^-20 in units of 2^-47, smaller w in units of
  // 2^-69 (a tile adds <= 2^14 terms, so neither overflows 64 bits; every w >= 2^-45 is exact).
  // The two [kMaxB] u64 arrays live in the list region once the list has been read (zeroed then).
  static_assert((2 * kList + kList / 2) * 4 >= 2 * kMaxB * 8, "fixed-point accumulators alias the list");
  uint64_t* s_fx = reinterpret_cast<uint64_t*>(s_r1);
  if (tid < 2) s_fxo[tid] = 0ull;
  // the tile's total weight (k_splitters' chunk sums, fixed point): the untouched mass is that
  // minus the winners' weight, exact in integers (no fp64 sum per slot)
  static_assert(kTile % kRwChunk == 0, "whole rate/weight chunks per tile");
  uint64_t tot_h = 0, tot_l = 0;
  {
    const uint64_t* wf = wfix + ((int64_t)(rowsel ? b : 0) * nwb + (int64_t)tile * (kTile / kRwChunk)) * 2;
#pragma unroll
    for (int c = 0; c < kTile / kRwChunk; ++c)
      if (tile * (kTile / kRwChunk) + c < nwb) {
        tot_h += wf[2 * c];
        tot_l += wf[2 * c + 1];
      }
  }
  const uint32_t lmn = lut_base[2 * b];
  const int lsh = (int)lut_base[2 * b + 1];
  const int a_t = tile * kTile;  // first action of the tile
  // all rates and weights of the thread in flight at once (group g: actions a_t + g * (4 *
  // kGrpNT) + 4 * tid + 0..3, coalesced float4 from the 16-byte aligned rows; the padding
  // past E reads r = inf, w = 0); no barrier before the times
  float lvk[4 * kTileG];  // the weights stay in registers for the grouped weight stream
  float rvk[4 * kTileG];
#pragma unroll
  for (int g = 0; g < kTileG; ++g) {
    const int a0 = a_t + g * 4 * kGrpNT + 4 * tid;
    if (a0 < wstride) {
      const float4 r4 = *reinterpret_cast<const float4*>(rrow + a0);
      const float4 w4 = *reinterpret_cast<const float4*>(wrow + a0);
      rvk[4 * g] = r4.x, rvk[4 * g + 1] = r4.y, rvk[4 * g + 2] = r4.z, rvk[4 * g + 3] = r4.w;
      lvk[4 * g] = w4.x, lvk[4 * g + 1] = w4.y, lvk[4 * g + 2] = w4.z, lvk[4 * g + 3] = w4.w;
    } else {  // past the row: never a winner (r = inf, as the row's own padding)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        rvk[4 * g + s] = __uint_as_float(0x7f800000u);
        lvk[4 * g + s] = 0.0f;
      }
    }
  }
  // the terminal's arrival time, computed once per sample by k_presample (a scalar load issued
  // with the block's other scalar loads, instead of a Philox call per thread on the critical path)
  const float tE = tE_in[b];
  PROF(0)
  uint32_t ord[4 * kTileG];  // trajectory-order keys (read for the winners only)
  uint32_t win = 0;  // bit 4g + s: action a_t + g * 4 * kGrpNT + 4 * tid + s is a winner
#pragma unroll
  for (int g = 0; g < kTileG; ++g) {
    const int a0 = a_t + g * 4 * kGrpNT + 4 * tid;
    const uint4 ph = philox4x32_10((uint32_t)a0 >> 2, bg, st0, st1, seed0, seed1);
    const spai_f2 t01 = arrival_q2(ph.x, ph.y) * (spai_f2){rvk[4 * g], rvk[4 * g + 1]};
    const spai_f2 t23 = arrival_q2(ph.z, ph.w) * (spai_f2){rvk[4 * g + 2], rvk[4 * g + 3]};
    const float ts[4] = {t01.x, t01.y, t23.x, t23.y};
    uint32_t nib = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // branch-free; a slot past E has r = inf (never a winner) and the
                                   // terminal's own slot t = t_E (not below it)
      nib |= (uint32_t)(ts[s] < tE) << s;
      ord[4 * g + s] = arrival_ord(ts[s]);
    }
    win |= nib << (4 * g);
    // removed bitmap: 8 adjacent threads make one 32-bit word (OR over the 8 lanes by DPP:
    // quad_perm [1,0,3,2], [2,3,0,1], then row_half_mirror joins the two quads)
    uint32_t x = nib << ((tid & 7) * 4);
    x |= (uint32_t)dpp_i<0xB1, 0xf>(0, (int)x);
    x |= (uint32_t)dpp_i<0x4E, 0xf>(0, (int)x);
    x |= (uint32_t)dpp_i<0x141, 0xf>(0, (int)x);
    const int wi = a0 >> 5;
    if ((tid & 7) == 0 && a0 < E && wi < words) removed[(int64_t)b * words + wi] = x;
  }
  __syncthreads();  // splitter tables, zeroed histogram
  PROF(1)
  const int nbl = nb - 1;
  // bucket histogram of the part's winners (buckets [k0, k1); the winners of other parts only add
  // their weight to s_fxo, for the untouched mass); each winner keeps its bucket and its rank inside
  // the bucket (the histogram atomic's return; any order: the level-2 sort orders buckets fully)
  static_assert(kMaxB <= (1 << 11) && kTile <= (1 << 21), "bucket | rank << 11 packing");
  // Compacted path (the usual case: the part's winners fit the list, i.e. <= ~49 % of the tile):
  // the winners are first packed into an LDS list, so the bucket lookup, the rank and weight
  // atomics and the placement run once per WINNER over all lanes, instead of once per slot
  // (16 per thread, mostly losers) as on the slot path below.
  int totw;
  const int wbase = block_excl_scan<kGrpNT>(__popc(win), s_wc, &totw);
  const bool compact = totw <= kList;  // block-uniform
  constexpr int kPerT = (kList + kGrpNT - 1) / kGrpNT;
  uint32_t ebr[kPerT];  // bucket | rank << 11 of the thread's list entries (kept across the scan)
  uint32_t eo[kPerT], eid[kPerT];  // key, tile-local id, weight of the thread's list entries
  float ew[kPerT];
  int bc[4 * kTileG];
  uint32_t br[4 * kTileG];
  if (compact) {
#pragma unroll
    for (int q = 0; q < 4 * kTileG; ++q)
      if ((win >> q) & 1u) {
        const int k = wbase + __popc(win & ((1u << q) - 1u));
        l_ord[k] = ord[q];
        l_w[k] = lvk[q];
        l_id[k] = (uint16_t)((q >> 2) * 4 * kGrpNT + 4 * tid + (q & 3));
      }
    __syncthreads();
    PROF(6)
    // list rounds in use (block-uniform, usually 3-4 of kPerT): the unrolled per-entry loops
    // branch over the empty rounds instead of evaluating them under a false predicate
    const int nI = (totw + kGrpNT - 1) / kGrpNT;
#pragma unroll
    for (int i = 0; i < kPerT; ++i) {
      eo[i] = 0u;
      eid[i] = 0u;
      ew[i] = 0.0f;
      if (i < nI) {
        const int e = tid + i * kGrpNT;
        const bool v = e < totw;
        eo[i] = v ? l_ord[e] : 0u;
        eid[i] = v ? (uint32_t)l_id[e] : 0u;
        ew[i] = v ? l_w[e] : 0.0f;
      }
    }
    lds_barrier();  // the list is in registers: its region takes the bucket sums
    for (int k = tid; k < 2 * kMaxB; k += kGrpNT) s_fx[k] = 0ull;
    int ebc[kPerT];
#pragma unroll
    for (int i = 0; i < kPerT; ++i) {
      ebc[i] = 0;
      if (i < nI) {
        const uint32_t o = eo[i];
        const uint32_t bin = o < lmn ? 0u : min((uint32_t)(kBins - 1), (o - lmn) >> lsh);
        ebc[i] = s_lut[bin];
      }
    }
    bool more;
    do {
      more = false;
#pragma unroll
      for (int i = 0; i < kPerT; ++i) {
        if (i < nI) {
          const uint32_t sv = s_spl[max(0, min(ebc[i], nbl - 1))];
          const bool step = tid + i * kGrpNT < totw && ebc[i] < nbl && sv <= eo[i];
          ebc[i] += step;
          more |= step;
        }
      }
    } while (__any(more));
    PROF(7)
    lds_barrier();  // the sums are zero
#pragma unroll
    for (int i = 0; i < kPerT; ++i) {
      ebr[i] = 0xFFFFFFFFu;  // (not stored: beyond the list or another part's bucket)
      if (tid + i * kGrpNT < totw) {
        const int bk = nbl - ebc[i];
        const bool hi = ew[i] >= 9.5367431640625e-07f;
        const unsigned long long f = (unsigned long long)weight_fixed(ew[i]);
        if (bk >= k0 && bk < k1) {
          ebr[i] = (uint32_t)bk | ((uint32_t)atomicAdd(&s_off[bk], 1) << 11);
          atomicAdd((unsigned long long*)&s_fx[bk + (hi ? 0 : kMaxB)], f);
        } else {
          atomicAdd((unsigned long long*)&s_fxo[hi ? 0 : 1], f);
        }
      }
    }
  } else {
  for (int k = tid; k < 2 * kMaxB; k += kGrpNT) s_fx[k] = 0ull;
  // slot path (dense tiles): bucket of a winner's orderable key (buckets numbered in
  // trajectory order, descending key): value-linear lookup table, then the splitters, for all
  // the thread's slots at once: the table guesses of every slot are read together, then
  // wave-uniform correction rounds over the splitters (usually one step and one check), so the
  // LDS reads of the slots overlap instead of forming one dependent chain each
#pragma unroll
  for (int q = 0; q < 4 * kTileG; ++q) {
    const uint32_t o = ord[q];
    const uint32_t bin = o < lmn ? 0u : min((uint32_t)(kBins - 1), (o - lmn) >> lsh);
    bc[q] = s_lut[bin];
  }
  bool more;
  do {
    more = false;
#pragma unroll
    for (int q = 0; q < 4 * kTileG; ++q) {
      const uint32_t sv = s_spl[max(0, min(bc[q], nbl - 1))];
      const bool step = ((win >> q) & 1u) && bc[q] < nbl && sv <= ord[q];
      bc[q] += step;
      more |= step;
    }
  } while (__any(more));
  lds_barrier();  // the sums are zero
  uint32_t mine = 0;  // the winners of this part's buckets
#pragma unroll
  for (int q = 0; q < 4 * kTileG; ++q) {
    br[q] = 0u;
    if ((win >> q) & 1u) {
      const int bk = nbl - bc[q];
      const bool hi = lvk[q] >= 9.5367431640625e-07f;
      const unsigned long long f = (unsigned long long)weight_fixed(lvk[q]);
      if (bk >= k0 && bk < k1) {
        mine |= 1u << q;
        br[q] = (uint32_t)bk | ((uint32_t)atomicAdd(&s_off[bk], 1) << 11);
        atomicAdd((unsigned long long*)&s_fx[bk + (hi ? 0 : kMaxB)], f);
      } else {
        atomicAdd((unsigned long long*)&s_fxo[hi ? 0 : 1], f);
      }
    }
  }
  win = mine;
  }
  __syncthreads();
  PROF(2)
  // bucket offsets inside the tile (exclusive scan, kMaxB / kGrpNT buckets per thread; buckets
  // of other parts count 0)
  constexpr int kQ = kMaxB / kGrpNT;
  int hv[kQ], loc = 0;
  uint64_t wh = tid == 0 ? s_fxo[0] : 0ull, wl = tid == 0 ? s_fxo[1] : 0ull;  // the tile's winner weight
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const int k = tid * kQ + q;
    hv[q] = k < nb ? s_off[k] : 0;
    loc += hv[q];
    wh += s_fx[k];  // (0 past nb and outside [k0, k1))
    wl += s_fx[kMaxB + k];
  }
  wh = (uint64_t)wave_sum_i64((int64_t)wh);
  wl = (uint64_t)wave_sum_i64((int64_t)wl);
  if (lane == 0) {
    s_fxw[wave][0] = wh;
    s_fxw[wave][1] = wl;
  }
  int tot;
  int run = block_excl_scan<kGrpNT>(loc, s_wc, &tot);  // (its barriers publish s_fxw)
  if (tid == 0) {  // the untouched mass of the tile: its total weight minus its winners', exact
#pragma unroll
    for (int w = 0; w < kGrpNT / 64; ++w) {
      tot_h -= s_fxw[w][0];
      tot_l -= s_fxw[w][1];
    }
    tile_wrest[(int64_t)b * ntiles + tile] = (double)tot_h * 7.105427357601002e-15 + (double)tot_l * 1.6940658945086007e-21;
  }
  // bucket-major run table [b][bucket][tile] written directly (k_sort2 reads one bucket's runs
  // as a contiguous row): neighbouring tiles fill neighbouring words of a row, so the scattered
  // 4-byte stores merge in L2; this replaced a separate transpose kernel (k_runs, 26 us at C4)
  uint32_t* rcol = runs + (int64_t)b * kMaxB * ntiles + tile;
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const int k = tid * kQ + q;
    if (k >= k0 && k < k1) {
      s_off[k] = run;
      rcol[(int64_t)k * ntiles] = ((uint32_t)run << 16) | (uint32_t)hv[q];
    }
    run += hv[q];
    if (k >= k0 && k < k1)  // the run's weight sum (k_bsum adds them over the tiles)
      tbw[((int64_t)b * kMaxB + k) * ntiles + tile] =
          (double)s_fx[k] * 7.105427357601002e-15 + (double)s_fx[kMaxB + k] * 1.6940658945086007e-21;
  }
  __syncthreads();
  PROF(3)
  uint3* st = reinterpret_cast<uint3*>(staging) + ((int64_t)b * ntiles + tile) * kTile;
  if (compact) {
    // placed at their tile-local positions in LDS, then written out in order as 16-byte vectors
    // (whole cache lines instead of one scattered 12-byte store per winner)
#pragma unroll
    for (int i = 0; i < kPerT; ++i) {
      if (ebr[i] != 0xFFFFFFFFu) {
        const int p = s_off[ebr[i] & 0x7FFu] + (int)(ebr[i] >> 11);
        s_r01[3 * p] = (uint32_t)a_t + eid[i];
        s_r01[3 * p + 1] = ~eo[i];
        s_r01[3 * p + 2] = __float_as_uint(ew[i]);
      }
    }
    __syncthreads();
    {
      const int nw = 3 * tot, nv = nw >> 2;
      uint4* sv = reinterpret_cast<uint4*>(st);
      const uint4* lv = reinterpret_cast<const uint4*>(s_r01);
      for (int v = tid; v < nv; v += kGrpNT) sv[v] = lv[v];
      uint32_t* sw = reinterpret_cast<uint32_t*>(st);
      if (tid < nw - 4 * nv) sw[4 * nv + tid] = s_r01[4 * nv + tid];
    }
    PROF(4)
    PROF(5)
    PROF_END(32)
    return;
  }
  // final tile-local position of every winner, two per VGPR
  uint32_t pp[2 * kTileG];
#pragma unroll
  for (int q = 0; q < 4 * kTileG; ++q) {
    const uint32_t pos = (win >> q) & 1u ? min((uint32_t)s_off[br[q] & 0x7FFu] + (br[q] >> 11), 0xFFFFu) : 0xFFFFu;
    if (q & 1) pp[q >> 1] |= pos << 16;
    else pp[q >> 1] = pos;
  }
  // positional windows of kWin records staged in LDS, written out as whole cache lines
#pragma unroll 1
  for (int w0 = 0; w0 < tot; w0 += kWin) {
    int tv = tid;
    asm volatile("" : "+v"(tv));  // opaque per window: keeps per-slot addresses out of registers
#pragma unroll
    for (int q = 0; q < 4 * kTileG; ++q) {
      const int p = (int)((pp[q >> 1] >> (16 * (q & 1))) & 0xFFFFu) - w0;
      if ((unsigned)p < (unsigned)kWin) {  // (non-winners carry 0xFFFF, beyond every window)
        const int a = a_t + (q >> 2) * 4 * kGrpNT + 4 * tv + (q & 3);
        w_rec[p] = ((uint64_t)(~ord[q]) << 32) | (uint32_t)a;
        w_log[p] = lvk[q];
      }
    }
    __syncthreads();
    PROF(4)
    const int cnt = min(kWin, tot - w0);
    for (int e = tid; e < cnt; e += kGrpNT) {  // one 12-byte record per lane
      const uint64_t r = w_rec[e];
      st[w0 + e] = make_uint3((uint32_t)r, (uint32_t)(r >> 32), __float_as_uint(w_log[e]));
    }
    __syncthreads();
    PROF(5)
  }
  PROF_END(32)
}

// ------------------------------------------------------------------ k_bsum
// Per (sample, bucket) of this part, one block: the winner count and the weight sum over the
// tiles (thread t adds tiles t, t + kBsumNT, ... in order, then a fixed butterfly per wave and
// the waves in order) of the per-(bucket, tile) runs and run sums k_tile left, into the exchange
// array xch[b][0][k] (weights) / xch[b][1][k] (counts); the other buckets are zeroed, so the
// sum of the parts' arrays is the one-part array.  Also advances the device stream counter:
// every k_presample / k_tile block has read it.
constexpr int kBsumNT = 256;
__global__ __launch_bounds__(kBsumNT) void k_bsum(int32_t ntiles, const int32_t* __restrict__ nb_,
                                                  const uint32_t* __restrict__ runs, const double* __restrict__ tbw,
                                                  double* __restrict__ xch, uint64_t* __restrict__ sctr,
                                                  int32_t part, int32_t nparts) {
  const int b = blockIdx.y, k = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (sctr && b == 0 && k == 0 && tid == 0) *sctr += 1;
  const int nb = nb_[b];
  double* xw = xch + (int64_t)b * 2 * kMaxB;
  if (k >= nb) {  // beyond this sample's buckets: zero the rest of its rows (one block does it)
    if (k == nb)
      for (int j = nb + tid; j < kMaxB; j += kBsumNT) xw[j] = xw[kMaxB + j] = 0.0;
    return;
  }
  if (k < part_lo(nb, part, nparts) || k >= part_lo(nb, part + 1, nparts)) {
    if (tid == 0) xw[k] = xw[kMaxB + k] = 0.0;
    return;
  }
  __shared__ double s_d[kBsumNT / 64];
  __shared__ int s_c[kBsumNT / 64];
  const int64_t row = ((int64_t)b * kMaxB + k) * ntiles;
  double s = 0.0;
  int c = 0;
  for (int t = tid; t < ntiles; t += kBsumNT) {  // coalesced over the tiles, in order per thread
    s += tbw[row + t];
    c += (int)(runs[row + t] & 0xFFFFu);
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if (lane == 0) {
    s_d[wave] = s;
    s_c[wave] = c;
  }
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    int ct = 0;
#pragma unroll
    for (int w = 0; w < kBsumNT / 64; ++w) {
      t += s_d[w];
      ct += s_c[w];
    }
    xw[k] = t;
    xw[kMaxB + k] = (double)ct;
  }
}

// ------------------------------------------------------------------ k_bscan
// Per sample, once the exchange array holds every part's buckets: bucket starts (trajectory
// positions), winner count, T, the untouched mass W_rest (terminal included) and the mass of
// all later buckets per bucket (fixed-order suffix).
__global__ __launch_bounds__(1024) void k_bscan(int32_t E, int32_t ntiles, const float* __restrict__ ww,
                                                int64_t wrow_stride, const int32_t* __restrict__ nb_,
                                                const double* __restrict__ xch, const double* __restrict__ tile_wrest,
                                                int32_t* __restrict__ bstart, int32_t* __restrict__ counts,
                                                double* __restrict__ wrest, int32_t* __restrict__ tdev,
                                                double* __restrict__ bwsuf) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ int s_wc[16];
  __shared__ double s_wr[16], s_wd[16];
  const int nb = nb_[b];
  double wr = 0.0;
  for (int t = tid; t < ntiles; t += 1024) wr += tile_wrest[(int64_t)b * ntiles + t];
  wr = wave_sum(wr);
  if (lane == 0) s_wr[wave] = wr;
  const double* xw = xch + (int64_t)b * 2 * kMaxB;
  const double* xc = xw + kMaxB;
  const int k0 = 2 * tid, k1 = 2 * tid + 1;
  const int h0 = k0 < nb ? (int)xc[k0] : 0, h1 = k1 < nb ? (int)xc[k1] : 0;
  int tot;
  const int ex = block_excl_scan<1024>(h0 + h1, s_wc, &tot);
  int32_t* bs = bstart + (int64_t)b * (kMaxB + 1);
  if (k0 < nb) bs[k0] = ex;
  if (k1 < nb) bs[k1] = ex + h0;
  if (tid == 0) {
    bs[nb] = tot;
    double t = (double)ww[(int64_t)b * wrow_stride + E];  // the terminal stays available
#pragma unroll
    for (int w = 0; w < 16; ++w) t += s_wr[w];
    wrest[b] = t;
    counts[b] = tot;
    atomicMax(tdev, tot + 1);
  }
  // bwsuf[k] = sum of the weights of all buckets after k: thread t owns the t-th chunk counted
  // from the end (contiguous, fixed order)
  const int per = (nb + 1023) / 1024;
  const int hi_ = nb - min(tid * per, nb), lo_ = max(hi_ - per, 0);
  double loc = 0.0;
  for (int k = hi_ - 1; k >= lo_; --k) loc += xw[k];
  double total;
  double run = block_excl_scan_d<1024>(loc, s_wd, &total);
  double* wp = bwsuf + (int64_t)b * kMaxB;
  for (int k = hi_ - 1; k >= lo_; --k) {
    wp[k] = run;
    run += xw[k];
  }
}

// In-block exact sort of an oversized bucket (n > kCap2) in global memory: 1-bit LSD radix
// over the varying bits of the 64-bit records, ping-ponging between the bucket's slots of
// the actions output (src0) and of out_suf (src1); ends with the sorted records in src0.
__device__ void big_bucket_sort(uint64_t* __restrict__ s0, uint64_t* __restrict__ s1, int n, int* s_wc,
                                uint32_t* s_red) {
  const int tid = threadIdx.x;
  uint64_t an = ~0ull, orr = 0ull;
  for (int i = tid; i < n; i += kSortNT) {
    an &= s0[i];
    orr |= s0[i];
  }
  uint32_t alo = wave_and_u32((uint32_t)an), ahi = wave_and_u32((uint32_t)(an >> 32));
  uint32_t olo = wave_or_u32((uint32_t)orr), ohi = wave_or_u32((uint32_t)(orr >> 32));
  __syncthreads();
  if ((tid & 63) == 0) {
    s_red[(tid >> 6) * 4 + 0] = alo;
    s_red[(tid >> 6) * 4 + 1] = ahi;
    s_red[(tid >> 6) * 4 + 2] = olo;
    s_red[(tid >> 6) * 4 + 3] = ohi;
  }
  __syncthreads();
  alo = ahi = 0xFFFFFFFFu;
  olo = ohi = 0u;
  for (int w = 0; w < kSortNT / 64; ++w) {
    alo &= s_red[w * 4 + 0];
    ahi &= s_red[w * 4 + 1];
    olo |= s_red[w * 4 + 2];
    ohi |= s_red[w * 4 + 3];
  }
  const uint64_t vary = ((((uint64_t)ahi) << 32) | alo) ^ ((((uint64_t)ohi) << 32) | olo);
  uint64_t* src = s0;
  uint64_t* dst = s1;
#pragma unroll 1
  for (int bit = 0; bit < 64; ++bit) {
    if (!((vary >> bit) & 1ull)) continue;
    // zeros of the whole bucket
    int z = 0;
    for (int i = tid; i < n; i += kSortNT) z += ((src[i] >> bit) & 1ull) ? 0 : 1;
    int ztot;
    (void)block_excl_scan<kSortNT>(z, s_wc, &ztot);
    int zc = 0, oc = ztot;  // running bases (uniform)
#pragma unroll 1
    for (int i0 = 0; i0 < n; i0 += kSortNT) {
      const int i = i0 + tid;
      const uint64_t v = i < n ? src[i] : 0ull;
      const int one = (i < n) ? (int)((v >> bit) & 1ull) : 0;
      const int zero = (i < n) ? 1 - one : 0;
      int zt;
      const int zex = block_excl_scan<kSortNT>(zero, s_wc, &zt);
      const int chunk = min(kSortNT, n - i0);
      if (i < n) dst[one ? oc + (tid - zex) : zc + zex] = v;
      zc += zt;
      oc += chunk - zt;
    }
    __syncthreads();
    uint64_t* t = src;
    src = dst;
    dst = t;
  }
  if (src != s0) {
    for (int i = tid; i < n; i += kSortNT) s0[i] = src[i];
    __syncthreads();
  }
}


// ------------------------------------------------------------------ k_sort2

// Oversized bucket (the sampled splitters missed; rare): gather into scratch, exact
// in-block radix in global memory, then the same outputs as the LDS path.
__device__ __forceinline__ void big_bucket(const int n, const int ntiles, const int* s_pre, const int* s_loc,
                                           const uint32_t* stb, const float* wrow, int64_t* act_out,
                                           float* fwd_out, uint64_t* s0, uint64_t* s1, const double later,
                                           int* s_wc, double* s_wd, uint32_t* s_red) {
  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += kSortNT) {
    int lo = 0, hi = ntiles - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t* r = stb + 3 * ((int64_t)lo * kTile + s_loc[lo] + (i - s_pre[lo]));
    s0[i] = ((uint64_t)r[1] << 32) | r[0];
  }
  __syncthreads();
  big_bucket_sort(s0, s1, n, s_wc, s_red);
  double carry = 0.0;  // suffix sums chunk by chunk from the end
  for (int c1e = n; c1e > 0; c1e -= kSortNT) {
    const int i = c1e - 1 - tid;
    const uint32_t a = i >= 0 ? (uint32_t)s0[i] : 0u;
    const double w = i >= 0 ? (double)wrow[a] : 0.0;
    double t;
    const double exs = block_excl_scan_d<kSortNT>(w, s_wd, &t);
    if (i >= 0) {
      act_out[i] = (int64_t)a;
      const double den = later + (carry + exs + w);  // (as k_sort2)
      fwd_out[i] = den >= 1e-30 ? (float)w * __builtin_amdgcn_rcpf((float)den) : (float)(w / den);
    }
    carry += t;
  }
}

// Level-2 sort, persistent: one resident block per CU walks the FLATTENED (sample, bucket)
// list, so the samples' very different winner counts (the terminal's own Gumbel key sets
// them) do not pile work on the blocks of one sample.  Per bucket (<= kCap2 records):
// the runs (one per select tile) are mapped into an LDS gather table and every record is
// loaded into registers in one round trip; records are ranked inside value-linear
// sub-buckets of ~0.5 record (almost always a direct placement) and re-laid in trajectory
// order in LDS together with their weights; then fp64 in-bucket suffix sums, the step
// probabilities fwd = w / (W_rest + later buckets + in-bucket suffix) and coalesced stores.
// The next bucket's run
// table is prefetched while the current one is processed (LDS-only barriers keep it in
// flight).  Oversized buckets are sorted in global memory by the block that meets them.
__global__ __launch_bounds__(kSortNT) void k_sort2(int32_t E, int32_t B, int32_t ntiles,
                                                   const int32_t* __restrict__ nb_,
                                                   const int32_t* __restrict__ bstart,
                                                   const uint32_t* __restrict__ runs,
                                                   const uint32_t* __restrict__ staging,
                                                   const uint32_t* __restrict__ spl,
                                                   int64_t t_cap, int64_t* __restrict__ actions,
                                                   float* __restrict__ fwd, const double* __restrict__ wrest,
                                                   const double* __restrict__ bwsuf, int32_t* __restrict__ bigcnt,
                                                   const float* __restrict__ ww, int64_t wrow_stride,
                                                   uint64_t* __restrict__ scratch, int32_t part, int32_t nparts) {
  // the bucket's records (ranked in place; once placed, {weight bits, action} in trajectory order);
  // high half: actions awaiting store
  __shared__ __attribute__((aligned(16))) uint64_t A[kCap2];
  __shared__ __attribute__((aligned(16))) float S[kCap2];  // step probabilities awaiting store
  __shared__ __attribute__((aligned(16))) int s_sub[kMaxSub + 4];
  __shared__ int s_nbp[kMaxSamples + 1];
  __shared__ int s_wc[kSortNT / 64];
  __shared__ double s_wd[kSortNT / 64];
  __shared__ uint32_t s_red[4 * (kSortNT / 64)];
  __shared__ uint32_t s_bigm[kBigWords];  // bit j: this block's j-th bucket is oversized (sorted after the loop)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ int s_anybig;
  for (int i = tid; i < kBigWords; i += kSortNT) s_bigm[i] = 0u;
  if (tid == 0) s_anybig = 0;
  {  // prefix of the part's bucket counts over the samples (parallel loads)
    const int nbb = tid < B ? nb_[tid] : 0;
    const int v = part_lo(nbb, part + 1, nparts) - part_lo(nbb, part, nparts);
    int tot;
    const int ex = block_excl_scan<kSortNT>(v, s_wc, &tot);
    if (tid < B) s_nbp[tid] = ex;
    if (tid == 0) s_nbp[B] = tot;
  }
  for (int i = tid; i < kMaxSub + 4; i += kSortNT) s_sub[i] = 0;  // zero again after each bucket's ranking
  __syncthreads();
  const int total = s_nbp[B];
  const int t0 = 2 * tid, t1 = 2 * tid + 1;
  PROF_INIT
  // bucket f: sample, bucket index, start/size, and the count and tile-local offset of its
  // runs in tiles t0, t1
  // and, for an interior bucket, its key range from the splitters: bucket kk holds the keys o with
  // spl[j - 1] <= o < spl[j], j = nb - 1 - kk (records carry ~o), so no min / max reduction is
  // needed to lay out its sub-buckets (the two end buckets have an open side: reduced)
  auto fetch = [&](int f, int& bb, int& kk, int& s0, int& s1, uint32_t& r0, uint32_t& r1, double& lt, uint32_t& bmn,
                   uint32_t& bmx, bool& bnd) {
    r0 = r1 = 0u;
    bb = kk = s0 = s1 = 0;
    lt = 0.0;
    uint32_t lo = 0u, hi = 0u;
    int nbl = 0;
    if (f < total) {
      while (s_nbp[bb + 1] <= f) ++bb;
      kk = f - s_nbp[bb] + part_lo(nb_[bb], part, nparts);
      const int32_t* bs = bstart + (int64_t)bb * (kMaxB + 1);
      s0 = bs[kk];
      s1 = bs[kk + 1];
      lt = wrest[bb] + bwsuf[(int64_t)bb * kMaxB + kk];  // mass of the untouched actions + later buckets
      const uint32_t* rr = runs + ((int64_t)bb * kMaxB + kk) * ntiles;  // [b][bucket][tile]
      if (t0 < ntiles) r0 = rr[t0];
      if (t1 < ntiles) r1 = rr[t1];
      nbl = nb_[bb] - 1;
      const int j = nbl - kk;
      if (j >= 1 && j <= nbl - 1) {
        lo = spl[(int64_t)bb * kMaxB + j - 1];
        hi = spl[(int64_t)bb * kMaxB + j];
      }
    }
    {
      const int j = __builtin_amdgcn_readfirstlane(nbl - kk);
      bnd = f < total && j >= 1 && j <= __builtin_amdgcn_readfirstlane(nbl) - 1;
      bmn = ~(uint32_t)__builtin_amdgcn_readfirstlane((int)hi) + 1u;  // ~o of the largest o < hi
      bmx = ~(uint32_t)__builtin_amdgcn_readfirstlane((int)lo);
    }
    // block-uniform: scalar registers (scalar-base addressing of the gather and the stores)
    bb = __builtin_amdgcn_readfirstlane(bb);
    kk = __builtin_amdgcn_readfirstlane(kk);
    s0 = __builtin_amdgcn_readfirstlane(s0);
    s1 = __builtin_amdgcn_readfirstlane(s1);
  };
  int nxb, nxk, nxs0, nxs1;
  bool nxbnd;
  uint32_t nxmn, nxmx;
  double nxl;
  uint32_t r0, r1;  // packed runs (offset << 16 | count) of the next bucket in tiles t0, t1
  // gather map of the bucket being staged (in S: free from the flush until the suffix phase)
  int* dlt = reinterpret_cast<int*>(S);
  uint32_t* a_out = reinterpret_cast<uint32_t*>(A) + kCap2;
  // Outputs of a bucket are stored during the NEXT bucket, after its records have landed.
  int pv_n = 0;
  int64_t* pv_act = nullptr;
  float* pv_fwd = nullptr;
  auto flush = [&]() {  // 16-byte buffer stores with scalar bases (2 actions / 4 step probabilities per lane)
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(pv_act, 0, pv_n * 8, kBufWord3);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(pv_fwd, 0, pv_n * 4, kBufWord3);
    int tv = tid;
    asm volatile("" : "+v"(tv));  // opaque: the lane offsets are recomputed here, not held across the loop
#pragma unroll
    for (int j = 0; j < kCap2 / (2 * kSortNT); ++j) {
      const int e = 2 * (j * kSortNT + tv);
      if (2 * j * kSortNT < pv_n) {
        const uint2 a = reinterpret_cast<const uint2*>(a_out)[e >> 1];
        if (e + 1 < pv_n) __builtin_amdgcn_raw_buffer_store_b128((spai_u4){a.x, 0u, a.y, 0u}, ra, e * 8, 0, kNtAux);
        else if (e < pv_n) __builtin_amdgcn_raw_buffer_store_b64((spai_u2){a.x, 0u}, ra, e * 8, 0, kNtAux);
      }
    }
#pragma unroll
    for (int j = 0; j < kCap2 / (4 * kSortNT); ++j) {
      const int e = 4 * (j * kSortNT + tv);
      if (4 * j * kSortNT < pv_n) {
        const uint4 v = reinterpret_cast<const uint4*>(S)[e >> 2];
        if (e + 3 < pv_n) {
          __builtin_amdgcn_raw_buffer_store_b128((spai_u4){v.x, v.y, v.z, v.w}, rf, e * 4, 0, kNtAux);
        } else if (e < pv_n) {  // the bucket's last 1-3 step probabilities
          __builtin_amdgcn_raw_buffer_store_b32(v.x, rf, e * 4, 0, kNtAux);
          if (e + 1 < pv_n) __builtin_amdgcn_raw_buffer_store_b32(v.y, rf, e * 4 + 4, 0, kNtAux);
          if (e + 2 < pv_n) __builtin_amdgcn_raw_buffer_store_b32(v.z, rf, e * 4 + 8, 0, kNtAux);
        }
      }
    }
    pv_n = 0;
  };
  // gather map of a bucket: record i sits at staging offset dlt[i] + i; each thread writes
  // the entries of its two runs (after the scan's barriers: the flush has read S)
  auto build_map = [&]() {
    const int c0 = (int)(r0 & 0xFFFFu), l0 = (int)(r0 >> 16), c1 = (int)(r1 & 0xFFFFu), l1 = (int)(r1 >> 16);
    int tot;
    const int ex = block_excl_scan<kSortNT, true>(c0 + c1, s_wc, &tot);
    if (tot <= kCap2) {
      const int d0 = t0 * kTile + l0 - ex, d1 = t1 * kTile + l1 - ex - c0;
#pragma unroll 1
      for (int i = 0; i < c0; ++i) dlt[ex + i] = d0;
#pragma unroll 1
      for (int i = 0; i < c1; ++i) dlt[ex + c0 + i] = d1;
    }
  };
  // Software pipeline: the records of bucket f + G (G = gridDim.x) are gathered into gm/gw
  // while bucket f goes through its LDS phases (LDS-only barriers keep them in flight), and
  // the run table of bucket f + 2G is in flight with them.
  constexpr int kPer = kCap2 / kSortNT;
  int cb = 0, ck = 0, cs = 0, cn = 0;
  bool cbnd = false;
  uint32_t cmn = 0u, cmx = 0u;
  double cl = 0.0;
  uint64_t gm[kPer];
  float gw[kPer];
  auto stage = [&](int fnext) {  // the bucket whose runs are in r0/r1 becomes the staged one
    cb = nxb;
    ck = nxk;
    cs = nxs0;
    cn = nxs1 - nxs0;
    cl = nxl;
    cbnd = nxbnd;
    cmn = nxmn;
    cmx = nxmx;
    build_map();
    PROF(2)
    fetch(fnext, nxb, nxk, nxs0, nxs1, r0, r1, nxl, nxmn, nxmx, nxbnd);
    lds_barrier();
    PROF(3)
  };
  // the staged bucket's gather, records [j0, j0 + 2) of every thread: one 12-byte buffer load per
  // record (scalar base, 32-bit offsets; positions past the bucket read out of range: 0, never
  // used).  Issued two at a time between the current bucket's LDS phases, so the waves do not
  // stall on one burst of memory instructions; the map stays in S until the suffix phase.
  auto issue = [&](const int j0) {
    const bool ok = cn > 0 && cn <= kCap2;  // empty / oversized buckets are not gathered
    const uint32_t nrec = (uint32_t)ntiles * kTile;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(staging + (int64_t)cb * nrec * 3), 0, nrec * 12, kBufWord3);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = j0 + jj;
      const int i = j * kSortNT + tid;
      const bool in = ok && i < cn;
      const uint32_t d = in ? (uint32_t)(dlt[i] + i) : 0x08000000u;  // >= nrec: out of range
      const spai_u3 r = __builtin_amdgcn_raw_buffer_load_b96(rs, d * 12, 0, 0);
      gm[j] = ((uint64_t)r.y << 32) | r.x;
      gw[j] = __uint_as_float(r.z);
    }
  };
  static_assert(kPer == 8, "four gather issues of two records");
  // XCD-aware bucket order: in each round the blocks of one XCD take consecutive buckets, so
  // the cache lines two neighbouring runs share in a tile's staging region (bucket k's run ends
  // where bucket k + 1's begins) are fetched once into that XCD's L2
  const int slot = xcd_remap(blockIdx.x, gridDim.x);
  fetch(slot, nxb, nxk, nxs0, nxs1, r0, r1, nxl, nxmn, nxmx, nxbnd);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  stage(slot + gridDim.x);
  issue(0);
  issue(2);
  issue(4);
  issue(6);
  int it = -1;  // this block's iteration (bit of s_bigm)
#pragma unroll 1
  for (int f = slot; f < total; f += gridDim.x) {
    ++it;
    // this bucket's records and the next bucket's run table have landed (and the previous
    // bucket's stores drained)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    const int b = cb, s = cs, n = cn;
    const bool bbnd = cbnd;
    uint32_t mn = cmn, mx = cmx;
    const double later = cl;
    uint64_t mine[kPer];
    float lw[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      mine[j] = gm[j];
      lw[j] = gw[j];
    }
    PROF(0)
    flush();  // the previous bucket's outputs (drain during this bucket's LDS phases)
    PROF(1)
    stage(f + 2 * gridDim.x);  // map of the next bucket; its gather is issued in four parts below
    issue(0);
    PROF(4)
    if (n == 0 || n > kCap2) {
      issue(2);
      issue(4);
      issue(6);
      if (n > kCap2 && tid == 0) {  // oversized (the sampled splitters missed; rare): sorted after the loop
        s_bigm[it >> 5] |= 1u << (it & 31);
        s_anybig = 1;
        atomicAdd(bigcnt, 1);  // diagnostic count (spai_rollout_ws_offset field 0)
      }
      continue;
    }
    if (!bbnd) {  // an end bucket: the key range by a block reduction (s_sub is already zero)
      mn = 0xFFFFFFFFu;
      mx = 0u;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int i = j * kSortNT + tid;
        if (i < n) {
          mn = min(mn, (uint32_t)(mine[j] >> 32));
          mx = max(mx, (uint32_t)(mine[j] >> 32));
        }
      }
      mn = wave_min_u32(mn);
      mx = wave_max_u32(mx);
      if (lane == 0) {
        s_red[wave * 2] = mn;
        s_red[wave * 2 + 1] = mx;
      }
      lds_barrier();
      mn = 0xFFFFFFFFu;
      mx = 0u;
#pragma unroll
      for (int w = 0; w < kSortNT / 64; ++w) {
        mn = min(mn, s_red[2 * w]);
        mx = max(mx, s_red[2 * w + 1]);
      }
    }
    const int nsub = max(1, min(kMaxSub, 2 * n));
    PROF(5)
    issue(2);
    // sub-bucket = floor((key - mn) * nsub / span) in fp32, clamped: monotone in the key (all
    // that the ranking needs), no 64-bit division per record
    const float scale = (float)nsub / ((float)(mx - mn) + 1.0f);
    int sb[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      sb[j] = 0;
      if (j * kSortNT + tid < n) {
        sb[j] = min(nsub - 1, (int)((float)((uint32_t)(mine[j] >> 32) - mn) * scale));
        atomicAdd(&s_sub[sb[j]], 1);
      }
    }
    lds_barrier();
    PROF(6)
    {  // exclusive scan of the sub-bucket counts: 4 per thread, one 16-byte LDS access each way
       // (conflict-free; entries at or past nsub are zero and their scanned values unused)
      static_assert(kMaxSub == 4 * kSortNT, "one int4 of sub-buckets per thread");
      int4 cv = reinterpret_cast<const int4*>(s_sub)[tid];
      int t2;
      int run = block_excl_scan<kSortNT, true>(cv.x + cv.y + cv.z + cv.w, s_wc, &t2);
      int4 ex;
      ex.x = run;
      ex.y = ex.x + cv.x;
      ex.z = ex.y + cv.y;
      ex.w = ex.z + cv.z;
      reinterpret_cast<int4*>(s_sub)[tid] = ex;
    }
    lds_barrier();
    PROF(7)
    issue(4);
    // scatter by sub-bucket (the cursor is the start; afterwards s_sub[i] = END of i)
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (j * kSortNT + tid < n) A[atomicAdd(&s_sub[sb[j]], 1)] = mine[j];
    lds_barrier();
    PROF(8)
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (j * kSortNT + tid < n) {
        const int lo = sb[j] ? s_sub[sb[j] - 1] : 0, hi = s_sub[sb[j]];
        int r = lo;
#pragma unroll 1
        for (int q = lo; q < hi; ++q) r += A[q] < mine[j];
        sb[j] = r;  // rank
      }
    }
    lds_barrier();
    PROF(9)
    // the sub-bucket counts are dead until the next bucket's histogram (several barriers away)
    for (int i = tid; i < kMaxSub; i += kSortNT) s_sub[i] = 0;  // all of it: the scan reads whole int4s
    issue(6);
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (j * kSortNT + tid < n)  // the key has done its work: the weight's bits take its place
        A[sb[j]] = ((uint64_t)__float_as_uint(lw[j]) << 32) | (uint32_t)mine[j];
    lds_barrier();
    PROF(10)
    // fp64 in-bucket inclusive suffix sums: thread t owns the kPer-record chunk
    // c = kSortNT - 1 - t (chunks counted from the end of the bucket, so the exclusive scan over
    // lower threads is the mass of every later record), read and written as aligned 16-byte
    // vectors (conflict-free); fixed order -> deterministic
    static_assert(kPer == 8 && kPer * kSortNT == kCap2, "four 16-byte record pairs per chunk");
    const int cb = (kSortNT - 1 - tid) * kPer;  // first record of this thread's chunk
    float lv[kPer];
#pragma unroll
    for (int k = 0; k < kPer / 2; ++k) {  // 16-byte LDS reads of the chunk's placed records
      const ulonglong2 r2 = reinterpret_cast<const ulonglong2*>(A)[cb / 2 + k];
      lv[2 * k] = __uint_as_float((uint32_t)(r2.x >> 32));
      lv[2 * k + 1] = __uint_as_float((uint32_t)(r2.y >> 32));
    }
    double loc = 0.0;
#pragma unroll
    for (int j = kPer - 1; j >= 0; --j) loc += cb + j < n ? (double)lv[j] : 0.0;
    uint32_t av[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = j * kSortNT + tid;
      av[j] = i < n ? (uint32_t)A[i] : 0u;
    }
    double wsum;
    double run = block_excl_scan_d<kSortNT, true>(loc, s_wd, &wsum);  // mass of all later records
    PROF(11)
    // (every read of A above is behind the scan's barriers)
    float fv[kPer];
#pragma unroll
    for (int j = kPer - 1; j >= 0; --j) {
      fv[j] = 0.0f;
      if (cb + j < n) {
        run += (double)lv[j];
        // w / (mass still available): the fp64 mass rounded to fp32, then the hardware reciprocal
        // (1 ulp) and one product: <= ~2.5 ulp of the exact quotient (the log's fp32 tolerance);
        // masses below 1e-30 (fp32 denormals for the reciprocal) divide in fp64
        const double den = later + run;
        fv[j] = den >= 1e-30 ? lv[j] * __builtin_amdgcn_rcpf((float)den) : (float)((double)lv[j] / den);
      }
    }
    reinterpret_cast<float4*>(S)[cb / 4] = make_float4(fv[0], fv[1], fv[2], fv[3]);
    reinterpret_cast<float4*>(S)[cb / 4 + 1] = make_float4(fv[4], fv[5], fv[6], fv[7]);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = j * kSortNT + tid;
      if (i < n) a_out[i] = av[j];
    }
    pv_n = n;
    pv_act = actions + (int64_t)b * t_cap + s;
    pv_fwd = fwd + (int64_t)b * t_cap + s;
    lds_barrier();  // LDS reuse by the next bucket
    PROF(12)
  }
  flush();
  PROF_END(0)
  // the oversized buckets this block met: exact radix in global memory (rare; the loop's
  // registers are dead here, so this path costs the main loop nothing)
  __syncthreads();
  if (!s_anybig) return;  // the usual case: no oversized bucket met
#pragma unroll 1
  for (int wd = 0; wd <= (it >> 5); ++wd) {
    uint32_t m = s_bigm[wd];
#pragma unroll 1
    while (m) {
      const int j = wd * 32 + __ffs((int)m) - 1;
      m &= m - 1u;
      const int f = slot + j * gridDim.x;
      int bb = 0;
      while (s_nbp[bb + 1] <= f) ++bb;
      const int kk = f - s_nbp[bb] + part_lo(nb_[bb], part, nparts);
      const int32_t* bs = bstart + (int64_t)bb * (kMaxB + 1);
      const int s0 = bs[kk], n = bs[kk + 1] - s0;
      const double later = wrest[bb] + bwsuf[(int64_t)bb * kMaxB + kk];
      int* s_pre = reinterpret_cast<int*>(S);  // (S is free after the loop's last flush)
      int* s_loc = s_pre + (kMaxTiles + 1);
      const uint32_t* rr = runs + ((int64_t)bb * kMaxB + kk) * ntiles;  // [b][bucket][tile]
      const uint32_t q0 = t0 < ntiles ? rr[t0] : 0u, q1 = t1 < ntiles ? rr[t1] : 0u;
      const int c0 = (int)(q0 & 0xFFFFu);
      int tot;
      const int ex = block_excl_scan<kSortNT>(c0 + (int)(q1 & 0xFFFFu), s_wc, &tot);
      if (t0 < ntiles) {
        s_pre[t0] = ex;
        s_loc[t0] = (int)(q0 >> 16);
      }
      if (t1 < ntiles) {
        s_pre[t1] = ex + c0;
        s_loc[t1] = (int)(q1 >> 16);
      }
      if (tid == 0) s_pre[ntiles] = tot;
      __syncthreads();
      int64_t* act_out = actions + (int64_t)bb * t_cap + s0;
      big_bucket(n, ntiles, s_pre, s_loc, staging + (int64_t)bb * ntiles * kTile * 3, ww + (int64_t)bb * wrow_stride,
                 act_out, fwd + (int64_t)bb * t_cap + s0, scratch + (int64_t)bb * E + s0,
                 reinterpret_cast<uint64_t*>(act_out), later, s_wc, s_wd, s_red);
      __syncthreads();
    }
  }
}

// Terminal step and the -1 / 1.0 padding up to T (grid-stride: the padding of a sample
// with few removals can be millions of steps).
__global__ __launch_bounds__(kFinNT) void k_pad(int32_t E, int32_t B, const int32_t* __restrict__ counts,
                                                const int32_t* __restrict__ tdev, const double* __restrict__ wrest,
                                                const float* __restrict__ ww, int64_t wrow_stride, int64_t t_cap,
                                                int64_t* __restrict__ actions, float* __restrict__ fwd,
                                                int32_t* __restrict__ t_out, int32_t* __restrict__ bigcnt,
                                                int32_t* __restrict__ lastbig, int32_t do_pad) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (t_out) *t_out = *tdev;
    // retire the oversized-bucket count of this sort (k_sort2, its only writer, ran before this
    // launch on the same stream): a second sort on the same select starts from 0
    *lastbig = *bigcnt;
    *bigcnt = 0;
  }
  if (!do_pad) return;  // the terminal step and the padding belong to the last part
  // every block takes the same share of every sample's padding (samples differ by up to ~1e6
  // slots: a per-sample grid left most blocks idle behind the longest pad), in 16-byte vectors
  // on 16-byte aligned addresses; block 0 also stores the terminal steps and the unaligned ends
  const int T = *tdev, G = gridDim.x, g = blockIdx.x;
#pragma unroll 1
  for (int b = 0; b < B; ++b) {
    const int k = counts[b];
    int64_t* ab = actions + (int64_t)b * t_cap;
    float* fb = fwd + (int64_t)b * t_cap;
    if (g == 0 && threadIdx.x == 0 && k < T) {  // the terminal step
      const double wE = (double)ww[(int64_t)b * wrow_stride + E];
      ab[k] = E;
      fb[k] = (float)(wE / wrest[b]);
    }
    const int lo = k + 1, hi = T;
    if (lo >= hi) continue;
    {  // actions: pairs of int64 (-1)
      const int a0 = min(hi, lo + (int)((((uintptr_t)(ab + lo)) >> 3) & 1));
      const int nv = (hi - a0) >> 1, a1 = a0 + 2 * nv;
      const int v0 = (int)((int64_t)nv * g / G), v1 = (int)((int64_t)nv * (g + 1) / G);
      longlong2* av = reinterpret_cast<longlong2*>(ab + a0);
      for (int v = v0 + threadIdx.x; v < v1; v += kFinNT) av[v] = make_longlong2(-1, -1);
      if (g == 0 && threadIdx.x == 0) {
        for (int t = lo; t < a0; ++t) ab[t] = -1;
        for (int t = a1; t < hi; ++t) ab[t] = -1;
      }
    }
    {  // step probabilities: float4 of 1.0
      const int a0 = min(hi, lo + (int)((4 - ((((uintptr_t)(fb + lo)) >> 2) & 3)) & 3));
      const int nv = (hi - a0) >> 2, a1 = a0 + 4 * nv;
      const int v0 = (int)((int64_t)nv * g / G), v1 = (int)((int64_t)nv * (g + 1) / G);
      float4* fv = reinterpret_cast<float4*>(fb + a0);
      for (int v = v0 + threadIdx.x; v < v1; v += kFinNT) fv[v] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
      if (g == 0 && threadIdx.x == 0) {
        for (int t = lo; t < a0; ++t) fb[t] = 1.0f;
        for (int t = a1; t < hi; ++t) fb[t] = 1.0f;
      }
    }
  }
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

static int max_buckets(int32_t E) { return std::min(kMaxB, E / kTarget + 2); }

// persistent grid of k_sort2 (0: one block per CU); spai_set_sort_blocks
static int g_sort_blocks = 0;

}  // namespace
}  // namespace spai

// k_sort2 takes a whole CU per block (153 KB of LDS, the register file at 4 waves per SIMD), so
// nothing runs beside it on its CUs: fewer persistent blocks leave CUs to a concurrent kernel
// (the fill on the second stream, GFlowNet overlap).  Process-wide; 0 = one block per CU.
extern "C" int spai_set_sort_blocks(int32_t blocks) {
  SPAI_CHECK_ARG(blocks >= 0, "spai_set_sort_blocks: blocks %d < 0", blocks);
  spai::g_sort_blocks = blocks;
  return SPAI_OK;
}

using namespace spai;

extern "C" size_t spai_rollout_workspace_bytes(int32_t E, int32_t B) {
  if (E <= 0 || B <= 0) return 0;
  if ((int64_t)E > (int64_t)kMaxTiles * kTile) {
    set_error("spai_rollout_workspace_bytes: E=%d above the %lld actions the sampler is compiled for", E,
              (long long)kMaxTiles * kTile);
    return 0;
  }
  TrajWs w;
  traj_ws(nullptr, E, B, &w);
  return w.total_bytes;
}

// Byte offset of a diagnostic / exchange array inside the rollout workspace (tests and the
// multi-part exchange address it in the caller-owned buffer instead of hard-coding the carve):
//   0 = int32 oversized buckets of the last sort (sorted in global memory by k_sort2)
//   1 = int32 T of the last rollout
//   2 = fp64 exchange array: [B][2][kMaxB] bucket weight sums | bucket winner counts (a part
//       fills its own buckets, the rest are 0 — so the int64 bit patterns of the parts' arrays
//       sum exactly too), then [B][8] slots for the caller's exact residual limbs
//   3 = kMaxB (the row length of field 2), as a value, not an offset
//   4 = int32 [B][kMaxB + 1] trajectory position of each bucket's first winner (bucket nb: count)
//   5 = int32 [B] buckets of each sample
//   6 = the number of fp64 values of field 2, as a value
// -1 for a bad field or shape.
extern "C" int64_t spai_rollout_ws_offset(int32_t E, int32_t B, int32_t field) {
  if (E <= 0 || B <= 0) return -1;
  TrajWs w;
  char* base = reinterpret_cast<char*>((uintptr_t)1 << 20);  // any aligned non-null base: offsets only
  traj_ws(base, E, B, &w);
  switch (field) {
    case 0: return reinterpret_cast<char*>(w.lastbig) - base;
    case 1: return reinterpret_cast<char*>(w.tdev) - base;
    case 2: return reinterpret_cast<char*>(w.xch) - base;
    case 3: return kMaxB;
    case 4: return reinterpret_cast<char*>(w.bstart) - base;
    case 5: return reinterpret_cast<char*>(w.nb) - base;
    case 6: return (int64_t)xch_doubles(B);
    default: return -1;
  }
}

static int select_args(const float* logits, const float* lmax, int32_t E, int32_t B, int64_t bstride,
                       int32_t sample_base, int32_t part, int32_t nparts, const void* workspace,
                       size_t workspace_bytes, TrajWs* w, const char* who) {
  SPAI_CHECK_ARG(logits && lmax && workspace, "%s: null pointer", who);
  SPAI_CHECK_ARG(E > 0 && B > 0 && bstride >= 0 && sample_base >= 0, "%s: bad shape", who);
  SPAI_CHECK_ARG((int64_t)E <= (int64_t)kMaxTiles * kTile, "%s: E=%d too large", who, E);
  SPAI_CHECK_ARG(B <= kMaxSamples, "%s: B=%d above %d", who, B, kMaxSamples);
  SPAI_CHECK_ARG(nparts >= 1 && part >= 0 && part < nparts, "%s: part %d of %d", who, part, nparts);
  traj_ws(const_cast<void*>(workspace), E, B, w);
  SPAI_CHECK_ARG(workspace_bytes >= w->total_bytes, "%s: workspace too small (%zu < %zu)", who, workspace_bytes,
                 w->total_bytes);
  return SPAI_OK;
}

static void launch_merge(const TrajWs& w, int32_t E, int32_t B, int64_t bstride, int32_t* counts, hipStream_t s) {
  k_bscan<<<B, 1024, 0, s>>>(E, w.ntiles, w.ww, bstride ? w.wstride : 0, w.nb, w.xch, w.tile_wrest, w.bstart,
                             counts, w.wrest, w.tdev, w.bwsuf);
}

static int rollout_select(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                          const float* lmax_parts, int32_t n_lmax_parts, uint64_t seed, uint64_t stream_id,
                          uint64_t* stream_ctr, int32_t sample_base, int32_t part, int32_t nparts, uint32_t* removed,
                          int32_t words, int32_t* counts, void* workspace, size_t workspace_bytes, void* stream) {
  TrajWs w;
  const int st = select_args(logits, lmax, E, B, bstride, sample_base, part, nparts, workspace, workspace_bytes, &w,
                             "spai_rollout_select");
  if (st != SPAI_OK) return st;
  SPAI_CHECK_ARG(!lmax_parts || (n_lmax_parts > 0 && bstride == 0),
                 "spai_rollout_select_pm: block maxima need n > 0 and one shared logits row");
  SPAI_CHECK_ARG(removed && counts, "spai_rollout_select: null pointer");
  SPAI_CHECK_ARG(words == (E + 31) / 32, "spai_rollout_select: words must be ceil(E/32)");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t s0 = (uint32_t)seed, s1 = (uint32_t)(seed >> 32);
  const uint32_t t0 = (uint32_t)stream_id, t1 = (uint32_t)(stream_id >> 32);
  const int nsb = (w.M + kSampNT - 1) / kSampNT;
  const int nwb = (int)((w.wstride + kRwChunk - 1) / kRwChunk);  // rate/weight blocks per logits row
  const int64_t rowsel = bstride ? 1 : 0;
  // (+1 block: the deferred logits maximum, when given)
  k_presample<<<nsb * B + (lmax_parts ? 1 : 0), kSampNT, 0, s>>>(logits, bstride, E, w.M, nsb, s0, s1, t0, t1,
                                                                 stream_ctr, sample_base, w.samp, w.samp_cnt, w.samp_mm,
                                                                 w.ctl, 4,
                                                                 w.tE, lmax_parts, n_lmax_parts,
                                                                 const_cast<float*>(lmax), B);
  SPAI_CHECK_LAUNCH();
  k_splitters<<<B + nwb * (bstride ? B : 1), kSortNT, 0, s>>>(E, w.M, nsb, w.samp, w.samp_cnt, w.samp_mm, w.nb, w.spl,
                                                             w.lut,
                                                             w.lut_base, B, logits, bstride, lmax, w.rr, w.ww,
                                                             w.wstride, w.wfix);
  SPAI_CHECK_LAUNCH();
  {
    KernelTimer kt(SPAI_TIMER_TILE, s);
    k_tile<<<w.ntiles * B, kGrpNT, 0, s>>>(w.rr, w.ww, w.wstride, rowsel, E, B, w.ntiles, s0, s1, t0, t1, stream_ctr,
                                           sample_base, part, nparts, removed, words, w.nb, w.spl, w.lut, w.lut_base,
                                           w.staging, w.runs, w.tbw, w.tile_wrest, w.tE, w.wfix, nwb);
  }
  SPAI_CHECK_LAUNCH();
  k_bsum<<<dim3(max_buckets(E) + 1, B), kBsumNT, 0, s>>>(w.ntiles, w.nb, w.runs, w.tbw, w.xch, stream_ctr, part,
                                                         nparts);
  SPAI_CHECK_LAUNCH();
  if (nparts == 1) {
    launch_merge(w, E, B, bstride, counts, s);
    SPAI_CHECK_LAUNCH();
  }
  return SPAI_OK;
}

extern "C" int spai_rollout_select(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                   uint64_t seed, uint64_t stream_id, uint64_t* stream_ctr, int32_t sample_base,
                                   int32_t part, int32_t nparts, uint32_t* removed, int32_t words, int32_t* counts,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  return rollout_select(logits, bstride, E, B, lmax, nullptr, 0, seed, stream_id, stream_ctr, sample_base, part,
                        nparts, removed, words, counts, workspace, workspace_bytes, stream);
}

extern "C" int spai_rollout_select_pm(const float* logits, int64_t bstride, int32_t E, int32_t B, float* lmax,
                                      const float* lmax_parts, int32_t n_lmax_parts, uint64_t seed,
                                      uint64_t stream_id, uint64_t* stream_ctr, int32_t sample_base, int32_t part,
                                      int32_t nparts, uint32_t* removed, int32_t words, int32_t* counts,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(lmax_parts != nullptr, "spai_rollout_select_pm: null lmax_parts");
  return rollout_select(logits, bstride, E, B, lmax, lmax_parts, n_lmax_parts, seed, stream_id, stream_ctr,
                        sample_base, part, nparts, removed, words, counts, workspace, workspace_bytes, stream);
}

extern "C" int spai_rollout_merge(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                  int32_t part, int32_t nparts, int32_t* counts, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  TrajWs w;
  const int st = select_args(logits, lmax, E, B, bstride, 0, part, nparts, workspace, workspace_bytes, &w,
                             "spai_rollout_merge");
  if (st != SPAI_OK) return st;
  SPAI_CHECK_ARG(counts, "spai_rollout_merge: null pointer");
  launch_merge(w, E, B, bstride, counts, (hipStream_t)stream);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

static int order_args(const float* logits, const float* lmax, const void* actions, const void* fwd,
                      const void* workspace, int32_t E, int32_t B, int64_t t_cap, int32_t part, int32_t nparts,
                      size_t workspace_bytes, TrajWs* w, const char* who) {
  SPAI_CHECK_ARG(logits && lmax && actions && fwd && workspace, "%s: null pointer", who);
  SPAI_CHECK_ARG(E > 0 && B > 0 && t_cap >= (int64_t)E + 1, "%s: bad shape (E=%d B=%d t_cap=%lld)", who, E, B,
                 (long long)t_cap);
  SPAI_CHECK_ARG((int64_t)E <= (int64_t)kMaxTiles * kTile, "%s: E=%d too large", who, E);
  SPAI_CHECK_ARG(B <= kMaxSamples, "%s: B=%d above %d", who, B, kMaxSamples);
  SPAI_CHECK_ARG(nparts >= 1 && part >= 0 && part < nparts, "%s: part %d of %d", who, part, nparts);
  traj_ws(const_cast<void*>(workspace), E, B, w);
  SPAI_CHECK_ARG(workspace_bytes >= w->total_bytes, "%s: workspace too small", who);
  return SPAI_OK;
}

extern "C" int spai_rollout_sort(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                 int32_t part, int32_t nparts, int64_t t_cap, int64_t* actions, float* fwd_probs,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  TrajWs w;
  const int st = order_args(logits, lmax, actions, fwd_probs, workspace, E, B, t_cap, part, nparts, workspace_bytes,
                            &w, "spai_rollout_sort");
  if (st != SPAI_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  const int nbm = max_buckets(E);
  const int nbt = (nbm + nparts - 1) / nparts * B;  // buckets of the part over the samples (upper bound)
  // persistent blocks, enough that none walks more than the 32 * kBigWords its oversized mask tracks
  const int cus = g_sort_blocks > 0 ? std::min(g_sort_blocks, num_cus()) : num_cus();
  const int g2 = std::max(std::max(1, std::min(nbt, cus)), (nbt + 32 * kBigWords - 1) / (32 * kBigWords));
  const int64_t wrs = bstride ? w.wstride : 0;
  {
    KernelTimer kt(SPAI_TIMER_SORT, s);
    k_sort2<<<g2, kSortNT, 0, s>>>(E, B, w.ntiles, w.nb, w.bstart, w.runs, w.staging, w.spl, t_cap, actions,
                                   fwd_probs, w.wrest, w.bwsuf, w.bigcnt, w.ww, wrs, w.scratch, part, nparts);
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_rollout_finish(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                   const int32_t* counts, int32_t part, int32_t nparts, int64_t t_cap,
                                   int64_t* actions, float* fwd_probs, int32_t* t_out, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  TrajWs w;
  const int st = order_args(logits, lmax, actions, fwd_probs, workspace, E, B, t_cap, part, nparts, workspace_bytes,
                            &w, "spai_rollout_finish");
  if (st != SPAI_OK) return st;
  SPAI_CHECK_ARG(counts, "spai_rollout_finish: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int last = part == nparts - 1;
  k_pad<<<last ? 4 * num_cus() : 1, kFinNT, 0, s>>>(E, B, counts, w.tdev, w.wrest, w.ww,
                                                                     bstride ? w.wstride : 0, t_cap, actions,
                                                                     fwd_probs, t_out, w.bigcnt, w.lastbig, last);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_rollout_order(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                  const int32_t* counts, int64_t t_cap, int64_t* actions, float* fwd_probs,
                                  int32_t* t_out, void* workspace, size_t workspace_bytes, void* stream) {
  const int st = spai_rollout_sort(logits, bstride, E, B, lmax, 0, 1, t_cap, actions, fwd_probs, workspace,
                                   workspace_bytes, stream);
  if (st != SPAI_OK) return st;
  return spai_rollout_finish(logits, bstride, E, B, lmax, counts, 0, 1, t_cap, actions, fwd_probs, t_out, workspace,
                             workspace_bytes, stream);
}
