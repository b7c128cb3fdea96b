// One-pass trajectory sampler for gfx950 (throughput mode) — replaces the T-step loop of
// GFlowNet.sample_states (gflownet/gflownet.py:135-179) and Log.log (gflownet/log.py:24-89).
//
// Sampling without replacement until the terminal id E is drawn == the Plackett-Luce order
// of the Gumbel keys key_a = l_a - ln(-ln u_a); the removed set is {a < E : key_a > key_E}
// and the trajectory lists it by key descending (ties: action ascending), then E.
//
// Pipeline (all stream-ordered, no host synchronisation; B samples per launch):
//   k_select        Philox4x32-10 + deterministic fp32 keys for 4 actions per lane; removal
//                   bitmap words via wave shuffles; block-local ordered staging of the
//                   winners (orderable key, action); per-block count/min/max and the mass
//                   of the untouched actions.
//   k_sample_stats  per-sample count, key range and bucket count (no global atomics).
//   k_part<0>       MSD bucketing: per (sample, part) LDS histogram, buckets linear in the
//                   key value over [min, max] of the sample's winners.
//   k_bucket_count  per-bucket part offsets and totals; k_bucket_scan: bucket starts.
//   k_part<1>       scatter winners into their buckets (LDS cursors).
//   k_sort_small    one wave per bucket of <= 256 winners: rank by counting in LDS by
//                   (key desc, action asc); fp64 weights w = exp(l - lmax) and in-bucket
//                   inclusive SUFFIX sums.  k_sort_large: bitonic in LDS for larger buckets.
//   k_wscan         per-sample suffix scan of the bucket weight sums (fixed order).
//   k_final         fwd_probs = w_t / (W_rest + sum_{s>=t} w_s), actions, [B][t_cap] layout.
// The step probability is formed from the mass still available at step t (the untouched
// actions W_rest, summed directly in k_select, plus the suffix of the trajectory), so no
// "Z - prefix" cancellation occurs however much of the mass the removed edges carry.
//   k_pad           terminal step and -1 / 1.0 padding up to T = max_b k_b + 1.
// Buckets hold ~160 winners on average (k_sample_stats picks the count), far below the
// 2048-element LDS capacity; an over-full bucket (pathologically clustered keys) falls
// back to an exact rank-counting sort in global memory inside the same kernel.
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kNT = 256;
constexpr int kPer = 4;
constexpr int kBlk = kNT * kPer;   // actions per select block
constexpr int kParts = 64;         // histogram/scatter parts per sample
constexpr int kPT = 1024;          // threads of the part kernels (2 blocks per CU with a 64 KiB LDS histogram)
constexpr int kMaxBuckets = 16384; // per sample
constexpr int kPerBucket = 96;     // target mean bucket occupancy
constexpr int kCap = 2048;         // LDS bitonic capacity per bucket
constexpr int kSortNT = 256;
constexpr int kSortGrid = 512;     // bucket-sort blocks per sample (grid-stride over buckets)
constexpr int kWaveMax = 256;      // buckets up to this size: one wave ranks them by counting (4 per lane)
constexpr int kSmallNT = 256;      // 4 waves per block in the small-bucket kernels
constexpr int kSmallGrid = 2048;   // small-bucket blocks per sample (grid-stride, 4 waves each)

struct TrajWs {
  int32_t nblk;
  int32_t *block_counts;
  uint32_t *block_min, *block_max;
  double* block_wrest;
  double* wrest;
  double *klo, *kscale;
  int32_t *nbk, *seg, *tdev;
  uint32_t* st_ord;
  int32_t* st_act;
  int32_t* part_hist;
  int32_t* bucket_start;
  int32_t* bucket_tot;
  double *bucket_wsum, *bucket_wsuf;
  uint64_t* bk_key;  // (~orderable(key) << 32) | action: ascending == trajectory order
  int32_t* out_act;
  double *out_w, *out_suf;
  size_t total_bytes;
};

static void traj_ws(void* base, int32_t E, int32_t B, TrajWs* w) {
  Carve c(base);
  w->nblk = (E + kBlk - 1) / kBlk;
  const size_t nb = (size_t)B * w->nblk, stage = nb * kBlk, cap = (size_t)B * E;
  w->block_counts = c.take<int32_t>(nb);
  w->block_min = c.take<uint32_t>(nb);
  w->block_max = c.take<uint32_t>(nb);
  w->block_wrest = c.take<double>(nb);
  w->wrest = c.take<double>(B);
  w->klo = c.take<double>(B);
  w->kscale = c.take<double>(B);
  w->nbk = c.take<int32_t>(B);
  w->seg = c.take<int32_t>(B);
  w->tdev = c.take<int32_t>(1);
  w->st_ord = c.take<uint32_t>(stage);
  w->st_act = c.take<int32_t>(stage);
  w->part_hist = c.take<int32_t>((size_t)B * kParts * kMaxBuckets);
  w->bucket_start = c.take<int32_t>((size_t)B * (kMaxBuckets + 1));
  w->bucket_tot = c.take<int32_t>((size_t)B * kMaxBuckets);
  w->bucket_wsum = c.take<double>((size_t)B * kMaxBuckets);
  w->bucket_wsuf = c.take<double>((size_t)B * kMaxBuckets);
  w->bk_key = c.take<uint64_t>(cap);
  w->out_act = c.take<int32_t>(cap);
  w->out_w = c.take<double>(cap);
  w->out_suf = c.take<double>(cap);
  w->total_bytes = c.off;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, kWave));
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, kWave));
  return v;
}

// Inclusive wave scan (int).
__device__ __forceinline__ int wave_incl_scan(int v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, kWave);
    if ((threadIdx.x & 63) >= o) v += y;
  }
  return v;
}

// Block-wide exclusive scan of one int per thread (NT <= 1024); returns the exclusive
// prefix, *total receives the block total.  Uses lds[NT/64].
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* lds, int* total) {
  const int incl = wave_incl_scan(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 63) lds[threadIdx.x >> 6] = incl;
  __syncthreads();
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
template <int NT>
__device__ __forceinline__ double block_excl_scan_d(double v, double* lds, double* total) {
  double incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(incl, o, kWave);
    if ((threadIdx.x & 63) >= o) incl += y;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 63) lds[threadIdx.x >> 6] = incl;
  __syncthreads();
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

__device__ __forceinline__ float from_orderable(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// Bucket of a key: linear in the key VALUE over [kmin, kmax] (the orderable bits are
// log-like per exponent and badly skewed when the range crosses zero); bucket 0 holds
// the LARGEST keys.  Monotone in the key, which is all the ordering needs.
__device__ __forceinline__ int bucket_of(uint32_t o, double klo, double scale, int nbk) {
  int k = (int)(((double)from_orderable(o) - klo) * scale);
  k = max(0, min(k, nbk - 1));
  return nbk - 1 - k;
}

// ------------------------------------------------------------------ k_select
__global__ __launch_bounds__(kNT) void k_select(const float* __restrict__ logits, int64_t bstride, int32_t E,
                                                int32_t nblk, uint32_t seed0, uint32_t seed1, uint32_t st0,
                                                uint32_t st1, int32_t sample_base, uint32_t* __restrict__ removed,
                                                int32_t words, const float* __restrict__ lmax,
                                                int32_t* __restrict__ block_counts,
                                                uint32_t* __restrict__ block_min, uint32_t* __restrict__ block_max,
                                                double* __restrict__ block_wrest, uint32_t* __restrict__ st_ord,
                                                int32_t* __restrict__ st_act) {
  const int b = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const float* lg = logits + (int64_t)b * bstride;
  const uint32_t bg = (uint32_t)(sample_base + b);
  const double lm = (double)lmax[b];
  __shared__ float s_tk;
  __shared__ int s_wc[kNT / 64];
  __shared__ uint32_t s_mn[kNT / 64], s_mx[kNT / 64];
  __shared__ double s_wr[kNT / 64];
  if (tid == 0) {
    const uint4 r = philox4x32_10((uint32_t)E >> 2, bg, st0, st1, seed0, seed1);
    s_tk = gumbel_key(lg[E], pick_word(r, E & 3));
  }
  __syncthreads();
  const float tk = s_tk;
  const int a0 = blk * kBlk + tid * kPer;
  uint32_t nib = 0, ord[kPer];
  float lv[kPer];
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
  double wr = 0.0;  // mass of the actions this lane leaves untouched
  if (a0 < E) {
    const uint4 r = philox4x32_10((uint32_t)a0 >> 2, bg, st0, st1, seed0, seed1);
#pragma unroll
    for (int s = 0; s < kPer; ++s) {
      ord[s] = 0;
      lv[s] = 0.0f;
      if (a0 + s < E) {
        lv[s] = lg[a0 + s];
        const float key = gumbel_key(lv[s], pick_word(r, s));
        if (key > tk) {
          nib |= 1u << s;
          ord[s] = orderable(key);
          mn = min(mn, ord[s]);
          mx = max(mx, ord[s]);
        } else {
          wr += (double)__expf(lv[s] - (float)lm);
        }
      }
    }
  }
  uint32_t x = nib << ((tid & 7) * kPer);
  x |= __shfl_xor(x, 1, kWave);
  x |= __shfl_xor(x, 2, kWave);
  x |= __shfl_xor(x, 4, kWave);
  if ((tid & 7) == 0) {
    const int wi = (blk * kBlk + (tid & ~7) * kPer) >> 5;
    if (wi < words) removed[(int64_t)b * words + wi] = x;
  }
  const int c = __popc(nib);
  const int incl = wave_incl_scan(c);
  mn = wave_min_u32(mn);
  mx = wave_max_u32(mx);
  wr = wave_sum(wr);
  if ((tid & 63) == 63) s_wc[tid >> 6] = incl;
  if ((tid & 63) == 0) {
    s_mn[tid >> 6] = mn;
    s_mx[tid >> 6] = mx;
    s_wr[tid >> 6] = wr;
  }
  __syncthreads();
  int pos = incl - c, tot = 0;
#pragma unroll
  for (int w = 0; w < kNT / 64; ++w) {
    pos += (w < (tid >> 6)) ? s_wc[w] : 0;
    tot += s_wc[w];
  }
  const int64_t lbase = ((int64_t)b * nblk + blk) * kBlk;
#pragma unroll
  for (int s = 0; s < kPer; ++s) {
    if ((nib >> s) & 1u) {
      st_ord[lbase + pos] = ord[s];
      st_act[lbase + pos] = a0 + s;
      ++pos;
    }
  }
  if (tid == 0) {
    uint32_t bmn = s_mn[0], bmx = s_mx[0];
    double bwr = s_wr[0];
#pragma unroll
    for (int w = 1; w < kNT / 64; ++w) {
      bmn = min(bmn, s_mn[w]);
      bmx = max(bmx, s_mx[w]);
      bwr += s_wr[w];
    }
    block_counts[b * nblk + blk] = tot;
    block_min[b * nblk + blk] = bmn;
    block_max[b * nblk + blk] = bmx;
    block_wrest[b * nblk + blk] = bwr;
  }
}

// ------------------------------------------------------------------ k_sample_stats
__global__ __launch_bounds__(1024) void k_sample_stats(int32_t nblk, int32_t E, const float* __restrict__ logits,
                                                       int64_t bstride, const float* __restrict__ lmax,
                                                       const int32_t* __restrict__ block_counts,
                                                       const uint32_t* __restrict__ block_min,
                                                       const uint32_t* __restrict__ block_max,
                                                       const double* __restrict__ block_wrest,
                                                       int32_t* __restrict__ counts, double* __restrict__ klo,
                                                       double* __restrict__ kscale, int32_t* __restrict__ nbk,
                                                       double* __restrict__ wrest) {
  const int b = blockIdx.x;
  __shared__ int si[16];
  __shared__ uint32_t smn[16], smx[16];
  __shared__ double sw[16];
  int c = 0;
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
  double wr = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 1024) {
    c += block_counts[b * nblk + i];
    mn = min(mn, block_min[b * nblk + i]);
    mx = max(mx, block_max[b * nblk + i]);
    wr += block_wrest[b * nblk + i];
  }
  c = wave_sum(c);
  mn = wave_min_u32(mn);
  mx = wave_max_u32(mx);
  wr = wave_sum(wr);
  if ((threadIdx.x & 63) == 0) {
    si[threadIdx.x >> 6] = c;
    smn[threadIdx.x >> 6] = mn;
    smx[threadIdx.x >> 6] = mx;
    sw[threadIdx.x >> 6] = wr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    wr = exp((double)logits[(int64_t)b * bstride + E] - (double)lmax[b]);  // the terminal id stays available
    for (int w = 0; w < 16; ++w) {
      tot += si[w];
      mn = min(mn, smn[w]);
      mx = max(mx, smx[w]);
      wr += sw[w];
    }
    wrest[b] = wr;
    int k = 1;
    while (k < kMaxBuckets && (int64_t)k * kPerBucket < tot) k <<= 1;
    counts[b] = tot;
    const double vlo = tot ? (double)from_orderable(mn) : 0.0, vhi = tot ? (double)from_orderable(mx) : 0.0;
    klo[b] = vlo;
    kscale[b] = vhi > vlo ? (double)k / (vhi - vlo) : 0.0;
    nbk[b] = k;
  }
}

// Shared body of the MSD histogram (SCATTER = false) and scatter (SCATTER = true) passes.
// Part p of sample b owns a contiguous range of select blocks; each wave walks whole select
// blocks (their winners are contiguous in the staging area) 4 elements per lane at a time,
// so loads are coalesced and independent.  Histograms/cursors live in LDS; the scatter
// writes one 8-byte sort key per winner.
template <bool SCATTER>
__global__ __launch_bounds__(kPT) void k_part(int32_t nblk, const int32_t* __restrict__ block_counts,
                                              const double* __restrict__ klo_, const double* __restrict__ kscale_,
                                              const int32_t* __restrict__ nbk_, const int32_t* __restrict__ seg_,
                                              const int32_t* __restrict__ bucket_start,
                                              const uint32_t* __restrict__ st_ord, const int32_t* __restrict__ st_act,
                                              int32_t* __restrict__ part_hist, uint64_t* __restrict__ bk_key) {
  const int p = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  __shared__ int cnt[kMaxBuckets];
  const int nbk = nbk_[b];
  const double klo = klo_[b], scale = kscale_[b];
  int32_t* ph = part_hist + ((int64_t)b * kParts + p) * kMaxBuckets;
  const int32_t* bs = bucket_start + (int64_t)b * (kMaxBuckets + 1);
  for (int k = tid; k < nbk; k += kPT) cnt[k] = SCATTER ? ph[k] + bs[k] : 0;
  __syncthreads();
  const int bb = (int)((int64_t)p * nblk / kParts), be = (int)((int64_t)(p + 1) * nblk / kParts);
  const int64_t seg = SCATTER ? (int64_t)seg_[b] : 0;
  for (int blk = bb + wave; blk < be; blk += kPT / 64) {
    const int n = block_counts[b * nblk + blk];
    const int64_t src0 = ((int64_t)b * nblk + blk) * kBlk;
    for (int i0 = 0; i0 < n; i0 += 256) {
      uint32_t o[4];
      int a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 64 + lane;
        o[u] = i < n ? st_ord[src0 + i] : 0u;
        if constexpr (SCATTER) a[u] = i < n ? st_act[src0 + i] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (i0 + u * 64 + lane < n) {
          const int slot = atomicAdd(&cnt[bucket_of(o[u], klo, scale, nbk)], 1);
          if constexpr (SCATTER) bk_key[seg + slot] = ((uint64_t)(~o[u]) << 32) | (uint32_t)a[u];
        }
      }
    }
  }
  if constexpr (!SCATTER) {
    __syncthreads();
    for (int k = tid; k < nbk; k += kPT) ph[k] = cnt[k];
  }
}

// Per bucket k (one thread each): exclusive prefix of the part counts (in place) and the
// bucket total.  Coalesced across k.
__global__ __launch_bounds__(256) void k_bucket_count(const int32_t* __restrict__ nbk_, int32_t* __restrict__ part_hist,
                                                      int32_t* __restrict__ bucket_tot) {
  const int b = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
  if (k >= nbk_[b]) return;
  int32_t* ph = part_hist + (int64_t)b * kParts * kMaxBuckets + k;
  int run = 0;
#pragma unroll 8
  for (int p = 0; p < kParts; ++p) {
    const int c = ph[(int64_t)p * kMaxBuckets];
    ph[(int64_t)p * kMaxBuckets] = run;
    run += c;
  }
  bucket_tot[(int64_t)b * kMaxBuckets + k] = run;
}

// Per sample: exclusive scan of the bucket totals -> bucket starts; segment offsets and T.
__global__ __launch_bounds__(1024) void k_bucket_scan(int32_t B, const int32_t* __restrict__ counts,
                                                      const int32_t* __restrict__ nbk_,
                                                      const int32_t* __restrict__ bucket_tot,
                                                      int32_t* __restrict__ bucket_start, int32_t* __restrict__ seg,
                                                      int32_t* __restrict__ tdev, int32_t* __restrict__ t_out) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int sw[16];
  const int nbk = nbk_[b];
  const int per = (nbk + 1023) / 1024;  // <= 16
  const int kb = min(tid * per, nbk), ke = min(kb + per, nbk);
  const int32_t* bt = bucket_tot + (int64_t)b * kMaxBuckets;
  int loc = 0;
  for (int k = kb; k < ke; ++k) loc += bt[k];
  int total;
  int base = block_excl_scan<1024>(loc, sw, &total);
  int32_t* bs = bucket_start + (int64_t)b * (kMaxBuckets + 1);
  for (int k = kb; k < ke; ++k) {
    bs[k] = base;
    base += bt[k];
  }
  if (tid == 0) {
    bs[nbk] = total;
    int s = 0, t = 0;
    for (int i = 0; i < B; ++i) {
      if (i < b) s += counts[i];
      t = max(t, counts[i]);
    }
    seg[b] = s;
    if (b == 0) {
      *tdev = t + 1;
      if (t_out) *t_out = t + 1;
    }
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Exclusive scan over the 64 lanes in lane order (fixed order -> deterministic).
__device__ __forceinline__ double wave_excl_scan_d(double v, double* total) {
  double incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(incl, o, kWave);
    if ((threadIdx.x & 63) >= o) incl += y;
  }
  *total = __shfl(incl, 63, kWave);
  const double ex = __shfl_up(incl, 1, kWave);
  return (threadIdx.x & 63) ? ex : 0.0;
}

// Buckets of <= kWaveMax winners (the common case): one wave per bucket, no block barriers.
// Rank by counting against the bucket's keys in the wave's LDS slice (broadcast reads), then
// gather the logits, fp64 weights and suffix sums over contiguous per-lane chunks.
__global__ __launch_bounds__(kSmallNT) void k_sort_small(const int32_t* __restrict__ nbk_,
                                                         const int32_t* __restrict__ seg_,
                                                         const int32_t* __restrict__ bucket_start,
                                                         const uint64_t* __restrict__ bk_key,
                                                         const float* __restrict__ logits, int64_t bstride,
                                                         const float* __restrict__ lmax_,
                                                         int32_t* __restrict__ out_act, double* __restrict__ out_w,
                                                         double* __restrict__ out_suf,
                                                         double* __restrict__ bucket_wsum) {
  const int b = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ uint64_t kin[kSmallNT / 64][kWaveMax];
  __shared__ uint64_t kso[kSmallNT / 64][kWaveMax];
  uint64_t* ki = kin[wave];
  uint64_t* ks = kso[wave];
  const int nbk = nbk_[b];
  const int64_t seg = seg_[b];
  const double lmax = (double)lmax_[b];
  const float* lg = logits + (int64_t)b * bstride;
  const int32_t* bs = bucket_start + (int64_t)b * (kMaxBuckets + 1);
  const int wstride = gridDim.x * (kSmallNT / 64);
  for (int k = blockIdx.x * (kSmallNT / 64) + wave; k < nbk; k += wstride) {
    const int s = bs[k], n = bs[k + 1] - s;
    if (n > kWaveMax) continue;  // k_sort_large
    double wsum = 0.0;
    if (n > 0) {
      const int64_t base = seg + s;
      uint64_t mine[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = u * 64 + lane;
        mine[u] = e < n ? bk_key[base + e] : ~0ull;
        ki[e] = mine[u];
      }
      wave_sync();
      int rank[4] = {0, 0, 0, 0};
      for (int j = 0; j < n; ++j) {
        const uint64_t kj = ki[j];
#pragma unroll
        for (int u = 0; u < 4; ++u) rank[u] += kj < mine[u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u * 64 + lane < n) ks[rank[u]] = mine[u];
      wave_sync();
      const int c = (n + 63) >> 6;                               // chunk length (<= 4)
      const int hi = n - min(lane * c, n), lo = max(hi - c, 0);  // lane 0 owns the tail
      double wv[4];
      double loc = 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = hi - 1 - u;
        wv[u] = (i >= lo) ? exp((double)lg[(uint32_t)ks[i]] - lmax) : 0.0;
        loc += wv[u];
      }
      double run = wave_excl_scan_d(loc, &wsum);  // mass of all later elements
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = hi - 1 - u;
        if (i >= lo) {
          run += wv[u];
          out_act[base + i] = (int32_t)(uint32_t)ks[i];
          out_w[base + i] = wv[u];
          out_suf[base + i] = run;
        }
      }
      wave_sync();  // LDS slices are reused by the next bucket
    }
    if (lane == 0) bucket_wsum[(int64_t)b * kMaxBuckets + k] = wsum;
  }
}

// Buckets of more than kWaveMax winners: up to kCap keys are split in LDS into value
// sub-buckets of ~32 and ranked inside them; beyond kCap an exact tiled rank count; then
// sorted actions, fp64 weights w = exp(l - lmax) (logit gathered by action) and in-bucket
// inclusive suffix sums.
__global__ __launch_bounds__(kSortNT) void k_sort_large(const int32_t* __restrict__ nbk_,
                                                          const int32_t* __restrict__ seg_,
                                                          const int32_t* __restrict__ bucket_start,
                                                          const uint64_t* __restrict__ bk_key,
                                                          const float* __restrict__ logits, int64_t bstride,
                                                          const float* __restrict__ lmax_, int32_t* __restrict__ out_act,
                                                          double* __restrict__ out_w, double* __restrict__ out_suf,
                                                          double* __restrict__ bucket_wsum) {
  constexpr int kMaxSub = 64;
  const int b = blockIdx.y, tid = threadIdx.x;
  __shared__ uint64_t key[kCap];
  __shared__ uint64_t kmid[kCap];
  __shared__ int scnt[kMaxSub], sst[kMaxSub], scur[kMaxSub];
  __shared__ float sfl[8];
  __shared__ double sd[kSortNT / 64];
  const int nbk = nbk_[b];
  const int64_t seg = seg_[b];
  const double lmax = (double)lmax_[b];
  const float* lg = logits + (int64_t)b * bstride;
  const int32_t* bs = bucket_start + (int64_t)b * (kMaxBuckets + 1);
  for (int k = blockIdx.x; k < nbk; k += gridDim.x) {
    const int s = bs[k], n = bs[k + 1] - s;
    const int64_t base = seg + s;
    double wsum = 0.0;
    if (n <= kWaveMax) continue;  // k_sort_small (block-uniform branch)
    if (n <= kCap) {
      // sub-bucket by value inside the bucket (linear over its own [min, max]), then rank
      // each key against its sub-bucket only: ~6 barriers instead of a bitonic network
      constexpr int kPerT = kCap / kSortNT;  // keys per thread (8)
      uint64_t mine[kPerT];
      float v[kPerT];
      float vmn = INFINITY, vmx = -INFINITY;
#pragma unroll
      for (int u = 0; u < kPerT; ++u) {
        const int i = u * kSortNT + tid;
        mine[u] = i < n ? bk_key[base + i] : ~0ull;
        v[u] = i < n ? from_orderable(~(uint32_t)(mine[u] >> 32)) : 0.0f;
        if (i < n) {
          vmn = fminf(vmn, v[u]);
          vmx = fmaxf(vmx, v[u]);
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        vmn = fminf(vmn, __shfl_xor(vmn, o, kWave));
        vmx = fmaxf(vmx, __shfl_xor(vmx, o, kWave));
      }
      if ((tid & 63) == 0) {
        sfl[tid >> 6] = vmn;
        sfl[4 + (tid >> 6)] = vmx;
      }
      const int nsub = min(kMaxSub, (n + 31) / 32);
      for (int i = tid; i < nsub; i += kSortNT) scnt[i] = 0;
      __syncthreads();
      vmn = fminf(fminf(sfl[0], sfl[1]), fminf(sfl[2], sfl[3]));
      vmx = fmaxf(fmaxf(sfl[4], sfl[5]), fmaxf(sfl[6], sfl[7]));
      const double sc = vmx > vmn ? (double)nsub / ((double)vmx - (double)vmn) : 0.0;
      int sb[kPerT];
#pragma unroll
      for (int u = 0; u < kPerT; ++u) {
        sb[u] = 0;
        if (u * kSortNT + tid < n) {
          // reversed: sub-bucket 0 holds the largest values (trajectory order)
          sb[u] = nsub - 1 - min(nsub - 1, (int)(((double)v[u] - (double)vmn) * sc));
          atomicAdd(&scnt[sb[u]], 1);
        }
      }
      __syncthreads();
      if (tid < 64) {  // exclusive scan of <= 64 sub-bucket counts by one wave
        const int c = tid < nsub ? scnt[tid] : 0;
        const int inc = wave_incl_scan(c);
        if (tid < nsub) {
          sst[tid] = inc - c;
          scur[tid] = inc - c;
        }
      }
      __syncthreads();
      int pos[kPerT];
#pragma unroll
      for (int u = 0; u < kPerT; ++u) {
        if (u * kSortNT + tid < n) {
          pos[u] = atomicAdd(&scur[sb[u]], 1);
          kmid[pos[u]] = mine[u];
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kPerT; ++u) {
        if (u * kSortNT + tid < n) {
          const int a = sst[sb[u]], e = a + scnt[sb[u]];
          int r = a;
          for (int j = a; j < e; ++j) r += kmid[j] < mine[u];
          key[r] = mine[u];
        }
      }
      __syncthreads();
      // inclusive suffix sums: thread t owns the t-th chunk counted from the END of the
      // bucket (contiguous, fixed order -> deterministic, all terms positive)
      const int per = (n + kSortNT - 1) / kSortNT;
      const int hi_ = n - min(tid * per, n), lo_ = max(hi_ - per, 0);  // chunk = [lo_, hi_)
      double wv[kCap / kSortNT];
      double loc = 0.0;
      for (int i = hi_ - 1, u = 0; i >= lo_; --i, ++u) {
        wv[u] = exp((double)lg[(uint32_t)key[i]] - lmax);
        loc += wv[u];
      }
      double run = block_excl_scan_d<kSortNT>(loc, sd, &wsum);  // mass of all later elements
      for (int i = hi_ - 1, u = 0; i >= lo_; --i, ++u) {
        run += wv[u];
        out_act[base + i] = (int32_t)(uint32_t)key[i];
        out_w[base + i] = wv[u];
        out_suf[base + i] = run;
      }
      __syncthreads();
    } else if (n > kCap) {
      // exact fallback: rank by counting with the j-loop tiled through LDS; only reached by
      // pathologically clustered keys
      for (int i0 = 0; i0 < n; i0 += kSortNT) {
        const int i = i0 + tid;
        const uint64_t ki = i < n ? bk_key[base + i] : ~0ull;
        int rank = 0;
        for (int j0 = 0; j0 < n; j0 += kCap) {
          const int m = min(kCap, n - j0);
          __syncthreads();
          for (int j = tid; j < m; j += kSortNT) key[j] = bk_key[base + j0 + j];
          __syncthreads();
          if (i < n)
            for (int j = 0; j < m; ++j) rank += key[j] < ki;
        }
        if (i < n) {
          const int a = (int32_t)(uint32_t)ki;
          out_act[base + rank] = a;
          out_w[base + rank] = exp((double)lg[a] - lmax);
        }
      }
      __syncthreads();
      double carry = 0.0;  // suffix sums from the end, chunk by chunk
      for (int c1 = n; c1 > 0; c1 -= kSortNT) {
        const int i = c1 - 1 - tid;  // thread 0 takes the last element of the chunk
        const double w = i >= 0 ? out_w[base + i] : 0.0;
        double tot;
        const double ex = block_excl_scan_d<kSortNT>(w, sd, &tot);
        if (i >= 0) out_suf[base + i] = carry + ex + w;
        carry += tot;
      }
      wsum = carry;
      __syncthreads();
    }
    if (tid == 0) bucket_wsum[(int64_t)b * kMaxBuckets + k] = wsum;
  }
}

// bucket_wsuf[k] = sum of the weights of all buckets after k (exclusive suffix, fixed order).
__global__ __launch_bounds__(1024) void k_wscan(const int32_t* __restrict__ nbk_, const double* __restrict__ bucket_wsum,
                                                double* __restrict__ bucket_wsuf) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ double sd[16];
  const int nbk = nbk_[b];
  const int per = (nbk + 1023) / 1024;
  const int hi_ = nbk - min(tid * per, nbk), lo_ = max(hi_ - per, 0);
  const double* ws = bucket_wsum + (int64_t)b * kMaxBuckets;
  double* wp = bucket_wsuf + (int64_t)b * kMaxBuckets;
  double loc = 0.0;
  for (int k = hi_ - 1; k >= lo_; --k) loc += ws[k];
  double total;
  double run = block_excl_scan_d<1024>(loc, sd, &total);
  for (int k = hi_ - 1; k >= lo_; --k) {
    wp[k] = run;
    run += ws[k];
  }
}

// One wave per bucket: fwd_probs = w / (W_rest + later buckets + in-bucket suffix).
__global__ __launch_bounds__(kSmallNT) void k_final(const int32_t* __restrict__ nbk_, const int32_t* __restrict__ seg_,
                                                    const int32_t* __restrict__ bucket_start,
                                                    const double* __restrict__ bucket_wsuf,
                                                    const int32_t* __restrict__ out_act,
                                                    const double* __restrict__ out_w,
                                                    const double* __restrict__ out_suf,
                                                    const double* __restrict__ wrest, int64_t t_cap,
                                                    int64_t* __restrict__ actions, float* __restrict__ fwd) {
  const int b = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nbk = nbk_[b];
  const int64_t seg = seg_[b];
  const int32_t* bs = bucket_start + (int64_t)b * (kMaxBuckets + 1);
  const double* wp = bucket_wsuf + (int64_t)b * kMaxBuckets;
  const double rest = wrest[b];
  int64_t* act_b = actions + (int64_t)b * t_cap;
  float* fwd_b = fwd + (int64_t)b * t_cap;
  const int wstride = gridDim.x * (kSmallNT / 64);
  for (int k = blockIdx.x * (kSmallNT / 64) + wave; k < nbk; k += wstride) {
    const int s = bs[k], e = bs[k + 1];
    const double later = rest + wp[k];
    for (int t = s + lane; t < e; t += 64) {
      const int64_t i = seg + t;
      act_b[t] = out_act[i];
      fwd_b[t] = (float)(out_w[i] / (later + out_suf[i]));
    }
  }
}

__global__ __launch_bounds__(kNT) void k_pad(int32_t E, const int32_t* __restrict__ counts,
                                             const int32_t* __restrict__ tdev, const double* __restrict__ wrest,
                                             const float* __restrict__ logits,
                                             int64_t bstride, const float* __restrict__ lmax, int64_t t_cap,
                                             int64_t* __restrict__ actions, float* __restrict__ fwd) {
  const int b = blockIdx.y;
  const int k = counts[b], T = *tdev;
  for (int t = k + blockIdx.x * kNT + threadIdx.x; t < T; t += gridDim.x * kNT) {
    if (t == k) {
      const double wE = exp((double)logits[(int64_t)b * bstride + E] - (double)lmax[b]);
      actions[(int64_t)b * t_cap + t] = E;
      fwd[(int64_t)b * t_cap + t] = (float)(wE / wrest[b]);
    } else {
      actions[(int64_t)b * t_cap + t] = -1;
      fwd[(int64_t)b * t_cap + t] = 1.0f;
    }
  }
}

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" size_t spai_rollout_workspace_bytes(int32_t E, int32_t B) {
  if (E <= 0 || B <= 0) return 0;
  TrajWs w;
  traj_ws(nullptr, E, B, &w);
  return w.total_bytes;
}

extern "C" int spai_rollout_select(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                   uint64_t seed, uint64_t stream_id, int32_t sample_base, uint32_t* removed,
                                   int32_t words, int32_t* counts, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  SPAI_CHECK_ARG(logits && lmax && removed && counts && workspace, "spai_rollout_select: null pointer");
  SPAI_CHECK_ARG(E > 0 && B > 0 && bstride >= 0 && sample_base >= 0, "spai_rollout_select: bad shape");
  SPAI_CHECK_ARG(words == (E + 31) / 32, "spai_rollout_select: words must be ceil(E/32)");
  TrajWs w;
  traj_ws(workspace, E, B, &w);
  SPAI_CHECK_ARG(workspace_bytes >= w.total_bytes, "spai_rollout_select: workspace too small (%zu < %zu)",
                 workspace_bytes, w.total_bytes);
  hipStream_t s = (hipStream_t)stream;
  k_select<<<dim3(w.nblk, B), kNT, 0, s>>>(logits, bstride, E, w.nblk, (uint32_t)seed, (uint32_t)(seed >> 32),
                                           (uint32_t)stream_id, (uint32_t)(stream_id >> 32), sample_base, removed,
                                           words, lmax, w.block_counts, w.block_min, w.block_max, w.block_wrest,
                                           w.st_ord, w.st_act);
  SPAI_CHECK_LAUNCH();
  k_sample_stats<<<B, 1024, 0, s>>>(w.nblk, E, logits, bstride, lmax, w.block_counts, w.block_min, w.block_max,
                                    w.block_wrest, counts, w.klo, w.kscale, w.nbk, w.wrest);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_rollout_order(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                                  const int32_t* counts, int64_t t_cap, int64_t* actions, float* fwd_probs,
                                  int32_t* t_out, void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(logits && lmax && counts && actions && fwd_probs && workspace,
                 "spai_rollout_order: null pointer");
  SPAI_CHECK_ARG(E > 0 && B > 0 && t_cap >= (int64_t)E + 1, "spai_rollout_order: bad shape (E=%d B=%d t_cap=%lld)",
                 E, B, (long long)t_cap);
  TrajWs w;
  traj_ws(workspace, E, B, &w);
  SPAI_CHECK_ARG(workspace_bytes >= w.total_bytes, "spai_rollout_order: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  k_part<false><<<dim3(kParts, B), kPT, 0, s>>>(w.nblk, w.block_counts, w.klo, w.kscale, w.nbk, w.seg,
                                                w.bucket_start, w.st_ord, w.st_act, w.part_hist, nullptr);
  SPAI_CHECK_LAUNCH();
  k_bucket_count<<<dim3(kMaxBuckets / 256, B), 256, 0, s>>>(w.nbk, w.part_hist, w.bucket_tot);
  SPAI_CHECK_LAUNCH();
  k_bucket_scan<<<B, 1024, 0, s>>>(B, counts, w.nbk, w.bucket_tot, w.bucket_start, w.seg, w.tdev, t_out);
  SPAI_CHECK_LAUNCH();
  k_part<true><<<dim3(kParts, B), kPT, 0, s>>>(w.nblk, w.block_counts, w.klo, w.kscale, w.nbk, w.seg,
                                               w.bucket_start, w.st_ord, w.st_act, w.part_hist, w.bk_key);
  SPAI_CHECK_LAUNCH();
  k_sort_small<<<dim3(kSmallGrid, B), kSmallNT, 0, s>>>(w.nbk, w.seg, w.bucket_start, w.bk_key, logits, bstride,
                                                        lmax, w.out_act, w.out_w, w.out_suf, w.bucket_wsum);
  SPAI_CHECK_LAUNCH();
  k_sort_large<<<dim3(kSortGrid, B), kSortNT, 0, s>>>(w.nbk, w.seg, w.bucket_start, w.bk_key, logits, bstride,
                                                      lmax, w.out_act, w.out_w, w.out_suf, w.bucket_wsum);
  SPAI_CHECK_LAUNCH();
  k_wscan<<<B, 1024, 0, s>>>(w.nbk, w.bucket_wsum, w.bucket_wsuf);
  SPAI_CHECK_LAUNCH();
  k_final<<<dim3(kSmallGrid, B), kSmallNT, 0, s>>>(w.nbk, w.seg, w.bucket_start, w.bucket_wsuf, w.out_act, w.out_w,
                                             w.out_suf, w.wrest, t_cap, actions, fwd_probs);
  SPAI_CHECK_LAUNCH();
  k_pad<<<dim3(64, B), kNT, 0, s>>>(E, counts, w.tdev, w.wrest, logits, bstride, lmax, t_cap, actions, fwd_probs);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
