// Gram-cached fill + residual for gfx950 (the bench's roofline kernel).
//
// For one line l of M (slots p -> other index k_p) the fill and its residual only need
//     G_pq = <A_line(k_p), A_line(k_q)>   and   c_p = A_line(k_p)[l]
// (line residual^2 = m^T G m - 2 c^T m + 1, LSQ fill m = argmin = masked solve of G m = c).
// G and c depend on the pattern and on A only, never on the sample, and the candidate
// pattern is fixed for the lifetime of a PreconditionerEnv (preconditioner.py:23-25).  So
// they are built ONCE per env (k_gram_build, the same arithmetic the per-call kernel
// fill.hip:k_line used to redo on every launch) and stored structure-of-arrays in fp64:
//     gram[l / 64][q][l % 64], q < T = Wc(Wc+1)/2: G upper triangle (p <= q, row-major),
//     then Wc c_p (blocks of 64 lines: a wave's Gram data is one contiguous region, never
//     T + Wc power-of-two-strided streams on the same HBM channels).
// The per-rollout kernel (k_gram_fill) is then a stream: per line the Wc action ids, the
// T + Wc Gram values and, per
// sample, Wc mask bits and the Wc stored values of M, with a masked LDL^T in fp64 whose
// pivots use v_rcp_f64 + one Newton step instead of IEEE division.  The LSQ line residual
// is 1 - c^T m* = 1 - sum_k y_k^2 / D_k from the factorisation; it equals the residual of
// the stored (rounded) values up to d^T G d, d = rounding of m (<= 1e-14 relative for fp32 M).
#include "spai_device.h"
#include "spai_status.h"
#include "spai_timer.h"

namespace spai {
namespace {

constexpr int kNT = 256;
constexpr int kChunk = 8;  // samples per LDS residual chunk of the fill kernel
#ifndef FILL_WPE5
#define FILL_WPE5 4  // waves/SIMD of the 5-wide fill (7-wide: 2, no spills)
#endif

__host__ __device__ constexpr int tri(int w) { return w * (w + 1) / 2; }

// index of G_pq (p <= q) in the packed upper triangle of a W-wide line
template <int W>
__device__ __forceinline__ constexpr int gidx(int p, int q) {
  return p * W - p * (p - 1) / 2 + (q - p);
}

// 1/x to ~1 ulp: hardware reciprocal + one Newton step (the pivots are positive, normal).
__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  const double e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

template <int W, int WA, typename TA>
__global__ __launch_bounds__(kNT) void k_gram_build(int32_t n, int32_t wrt, int32_t wart,
                                                    const int32_t* __restrict__ pat_idx,
                                                    const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val,
                                                    double* __restrict__ gram) {
  const int j = blockIdx.x * kNT + threadIdx.x;
  if (j >= n) return;
  int idx[W];
#pragma unroll
  for (int p = 0; p < W; ++p) idx[p] = p < wrt ? pat_idx[(int64_t)j * wrt + p] : -1;
  int ai[W][WA];
  double av[W][WA];
#pragma unroll
  for (int p = 0; p < W; ++p) {
#pragma unroll
    for (int s = 0; s < WA; ++s) {
      ai[p][s] = -1;
      av[p][s] = 0.0;
      if (idx[p] >= 0 && s < wart) {
        const int64_t o = (int64_t)idx[p] * wart + s;
        ai[p][s] = a_idx[o];
        av[p][s] = (double)a_val[o];
      }
    }
  }
#pragma unroll
  for (int p = 0; p < W; ++p) {
    double cp = 0.0, gpp = 0.0;
#pragma unroll
    for (int s = 0; s < WA; ++s) {
      gpp += av[p][s] * av[p][s];
      cp += (ai[p][s] == j) ? av[p][s] : 0.0;
    }
    double* gj = gram + (int64_t)(j >> 6) * (tri(W) + W) * 64 + (j & 63);  // blocked layout
    gj[gidx<W>(p, p) * 64] = gpp;
    gj[(tri(W) + p) * 64] = cp;
#pragma unroll
    for (int q = p + 1; q < W; ++q) {
      double g = 0.0;
      // A lines are sorted by index: each entry of line p matches at most one of line q
#pragma unroll
      for (int s = 0; s < WA; ++s) {
        double m = 0.0;
#pragma unroll
        for (int t = 0; t < WA; ++t) m = (ai[p][s] >= 0 && ai[p][s] == ai[q][t]) ? av[q][t] : m;
        g += av[p][s] * m;
      }
      gj[gidx<W>(p, q) * 64] = g;
    }
  }
}

// One thread per line: the line's action ids and Gram values are loaded once (coalesced:
// consecutive lines are consecutive doubles), then the thread solves every sample; the
// squared line residuals of a chunk of kChunk samples go to LDS and are summed per sample
// by one wave each in a fixed order (two barriers per chunk, none per sample).
// kDict: gram is the cache's dictionary (spai_line_cache_dict: distinct entries of T + W values,
// contiguous) and line_entry[j] names line j's entry; else the full cache, 64 lines interleaved.
template <int W, typename TM, bool LSQ, typename GT, bool kDict>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(W <= 5 ? FILL_WPE5 : 2))) void k_gram_fill(int32_t n, int32_t line_begin, int32_t line_end, int32_t wrt,
                                                   const int32_t* __restrict__ pat_act,
                                                   const float* __restrict__ pat_val,
                                                   const GT* __restrict__ gram,
                                                   const int32_t* __restrict__ line_entry, int32_t B,
                                                   const uint32_t* __restrict__ removed, int32_t words,
                                                   int32_t word_base, TM* __restrict__ m_out,
                                                   double* __restrict__ partials) {
  constexpr int T = tri(W);
  __shared__ double s_r2[kChunk][kNT];
#ifdef FILL_BLOCK_M
  __shared__ __attribute__((aligned(16))) TM s_m[2][kNT * W];
#else
  __shared__ __attribute__((aligned(16))) TM s_m[1][kNT * W];  // per-wave regions
#endif
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lb = blockIdx.x;
  const int j = line_begin + lb * kNT + t;
  const bool valid = j < line_end;
  const int64_t nloc = line_end - line_begin;
  const int jj = valid ? j : line_begin;  // clamped: loads stay in bounds

  int act[W];
  float val[W];
  const int32_t* pa = pat_act + (int64_t)jj * wrt;
#pragma unroll
  for (int p = 0; p < W; ++p) {
    act[p] = (valid && p < wrt) ? pa[p] : -1;
    val[p] = (!LSQ && valid && p < wrt) ? pat_val[(int64_t)jj * wrt + p] : 0.0f;
  }
  double G[T], c[W];
  constexpr int kStride = kDict ? 1 : 64;  // blocked: one 64-line block contiguous
  const GT* gp = kDict ? gram + (int64_t)line_entry[jj] * (T + W) : gram + (int64_t)(jj >> 6) * (T + W) * 64 + (jj & 63);
#pragma unroll
  for (int q = 0; q < T; ++q) G[q] = (double)gp[q * kStride];  // fp32 storage only when exact (spai_gram_compact)
#pragma unroll
  for (int p = 0; p < W; ++p) c[p] = (double)gp[(T + p) * kStride];
  int wofs[W];  // bitmap word offsets / bit positions of the slots
#pragma unroll
  for (int p = 0; p < W; ++p) wofs[p] = act[p] >= 0 ? (act[p] >> 5) - word_base : 0;  // row-relative
  const int nvl = min(kNT, line_end - (line_begin + lb * kNT));  // valid lines of the block

  // the bitmap words of the next sample are loaded while the current one is solved
  uint32_t wd[W];
#pragma unroll
  for (int p = 0; p < W; ++p) wd[p] = removed[wofs[p]];
#pragma unroll 1
  for (int b0 = 0; b0 < B; b0 += kChunk) {
    const int nb = min(kChunk, B - b0);
#pragma unroll 1
    for (int s = 0; s < nb; ++s) {
      const int b = b0 + s;
      bool keep[W];
#pragma unroll
      for (int p = 0; p < W; ++p) keep[p] = act[p] >= 0 && !((wd[p] >> (act[p] & 31)) & 1u);
      if (b + 1 < B) {
        const uint32_t* rn = removed + (int64_t)(b + 1) * words;
#pragma unroll
        for (int p = 0; p < W; ++p) wd[p] = rn[wofs[p]];
      }

      double mr[W];
      double r2ls = 1.0;  // LSQ: 1 - c^T m* = 1 - sum_k y_k^2 / D_k (G m* = c on the kept slots)
      if constexpr (!LSQ) {
#pragma unroll
        for (int p = 0; p < W; ++p) mr[p] = keep[p] ? (double)val[p] : 0.0;
#ifdef FILL_NOCOMPUTE  // diagnostic variant: memory traffic without the solve
      } else if (true) {
#pragma unroll
        for (int p = 0; p < W; ++p) mr[p] = keep[p] ? c[p] * G[gidx<W>(p, p)] : 0.0;
        r2ls = mr[0] + mr[W - 1];
#endif
      } else {
        // masked LDL^T of the normal equations. A removed slot k only gets iD[k] = 0: every
        // L[.][k] = EL[.][k] * iD[k] is then exactly 0, so the kept unknowns see exactly the
        // factorisation of G restricted to the kept slots (the removed rows' own values are
        // finite and only ever multiplied by those zeros), and m[k] = 0 for the removed slots.
        // No per-entry masking of G or c.
        // (EL[i][q] = L[i][q] * D[q] is the unscaled elimination value: one FMA per term)
        double L[W][W], EL[W][W], iD[W], y[W];
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const double gkk = G[gidx<W>(k, k)];
          double dk = gkk;
#pragma unroll
          for (int q = 0; q < k; ++q) dk -= L[k][q] * EL[k][q];
          iD[k] = (keep[k] && dk > 1e-13 * gkk) ? fast_rcp(dk) : 0.0;
#pragma unroll
          for (int i = k + 1; i < W; ++i) {
            double v = G[gidx<W>(k, i)];
#pragma unroll
            for (int q = 0; q < k; ++q) v -= L[i][q] * EL[k][q];
            EL[i][k] = v;
            L[i][k] = v * iD[k];
          }
        }
#pragma unroll
        for (int k = 0; k < W; ++k) {
          double v = c[k];
#pragma unroll
          for (int q = 0; q < k; ++q) v -= L[k][q] * y[q];
          y[k] = v;
        }
#pragma unroll
        for (int k = 0; k < W; ++k) r2ls -= y[k] * y[k] * iD[k];
#pragma unroll
        for (int k = W - 1; k >= 0; --k) {
          double v = y[k] * iD[k];
#pragma unroll
          for (int q = k + 1; q < W; ++q) v -= L[q][k] * mr[q];
          mr[k] = v;
        }
      }
#ifdef FILL_BLOCK_M  // A/B: M staged per block (a block barrier per sample)
      if (m_out != nullptr) {
        // M through LDS (double-buffered per sample): the block's lines of one sample are one
        // contiguous run of nvl * wrt values, written with 16-byte stores
        TM* sm = s_m[b & 1];
        if (valid) {
#pragma unroll
          for (int p = 0; p < W; ++p)
            if (p < wrt) sm[t * wrt + p] = (TM)mr[p];
        }
        __syncthreads();
        TM* dst = m_out + ((int64_t)b * nloc + (int64_t)lb * kNT) * wrt;
        const int ne = nvl * wrt;
        constexpr int V = 16 / sizeof(TM);
        int e0 = 0;
        if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
          for (int e = t; e < ne / V; e += kNT)
            nt_store(reinterpret_cast<nt_u4*>(dst) + e, reinterpret_cast<const nt_u4*>(sm)[e]);
          e0 = ne / V * V;
        }
        for (int e = e0 + t; e < ne; e += kNT) nt_store(dst + e, sm[e]);
      }
#else
      {  // M staged per WAVE (its 64 lines are one contiguous run of M): no block barrier per sample
        const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: scalar offsets
      TM* sm = s_m[0] + wv * 64 * W;
        if (valid) {
#pragma unroll
          for (int p = 0; p < W; ++p)
            if (p < wrt) sm[lane * wrt + p] = (TM)mr[p];
        }
        __builtin_amdgcn_wave_barrier();
        const int nw = min(max(nvl - wv * 64, 0), 64);
        store_m_block<64, W, TM>(m_out ? m_out + ((int64_t)b * nloc + (int64_t)lb * kNT + wv * 64) * wrt : nullptr,
                                 sm, nw * wrt, lane);
        __builtin_amdgcn_wave_barrier();
      }
#endif
      double r2 = 0.0;
      if (valid) {
        if constexpr (LSQ) {
          r2 = r2ls;
        } else {
          r2 = 1.0;
#pragma unroll
          for (int p = 0; p < W; ++p) {
            double acc = mr[p] * G[gidx<W>(p, p)] - 2.0 * c[p];
#pragma unroll
            for (int q = p + 1; q < W; ++q) acc += 2.0 * mr[q] * G[gidx<W>(p, q)];
            r2 += mr[p] * acc;
          }
        }
      }
      s_r2[s][t] = r2;
    }
    __syncthreads();
    for (int s = wave; s < nb; s += kNT / 64) {  // fixed-order per-sample block sums
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kNT / 64; ++q) acc += s_r2[s][q * 64 + lane];
      acc = wave_sum(acc);
      if (lane == 0) partials[(int64_t)(b0 + s) * gridDim.x + lb] = acc;
    }
    __syncthreads();
  }
}

// The masked LDL^T solve of one wide line and sample, in place: a = G (packed upper triangle),
// y = c on entry; y = m on exit (0 on removed slots); returns the line residual^2 1 - c^T m.
template <int W>
__device__ __forceinline__ double wide_lsq_solve(double (&a)[tri(W)], double (&y)[W], uint32_t keep) {
  double r2 = 1.0;
  // left-looking LDL^T in place (column k of the packed upper triangle at step k), so the
  // pivot test reads the ORIGINAL G_kk: the per-pivot floor 1e-13 G_kk of k_gram_fill and
  // fill.hip's k_line, with no extra registers.  Column k first becomes u_jk = G_jk -
  // sum_{q<j} l_qj u_qk (j < k), then l_qk = u_qk / D_q; the diagonal slot ends as 1/D_k
  // (0 for a removed or singular pivot: l_k. = 0 and m_k = 0, as in k_gram_fill).
#pragma unroll
  for (int k = 0; k < W; ++k) {
#pragma unroll
    for (int j = 1; j < k; ++j) {
      double u = a[gidx<W>(j, k)];
#pragma unroll
      for (int q = 0; q < j; ++q) u -= a[gidx<W>(q, j)] * a[gidx<W>(q, k)];
      a[gidx<W>(j, k)] = u;
    }
    const double gkk = a[gidx<W>(k, k)];
    double d = gkk;
#pragma unroll
    for (int q = 0; q < k; ++q) {
      const double l = a[gidx<W>(q, k)] * a[gidx<W>(q, q)];  // u_qk / D_q
      d -= l * a[gidx<W>(q, k)];
      a[gidx<W>(q, k)] = l;
    }
    a[gidx<W>(k, k)] = (((keep >> k) & 1u) && d > 1e-13 * gkk) ? fast_rcp(d) : 0.0;
  }
#pragma unroll
  for (int k = 0; k < W; ++k) {  // forward substitution in place (y[q < k] are final)
    double v = y[k];
#pragma unroll
    for (int q = 0; q < k; ++q) v -= a[gidx<W>(q, k)] * y[q];
    y[k] = v;
  }
#pragma unroll
  for (int k = 0; k < W; ++k) r2 -= y[k] * y[k] * a[gidx<W>(k, k)];
#pragma unroll
  for (int k = W - 1; k >= 0; --k) {  // back substitution in place: y[q > k] already hold m_q
    double v = y[k] * a[gidx<W>(k, k)];
#pragma unroll
    for (int q = k + 1; q < W; ++q) v -= a[gidx<W>(k, q)] * y[q];
    y[k] = v;
  }
  return r2;
}

// Wide lines (8 <= W <= 13, e.g. the 13-point 3-D star of config C3): the same stream and
// outputs as k_gram_fill, but the factorisation runs in place on one packed working copy of G
// per sample (left-looking LDL^T, T = W(W+1)/2 doubles in registers), one wave per SIMD.
// Masking and the per-pivot floor are those of k_gram_fill: a removed slot k only gets
// 1/D_k := 0, so L[.][k] = 0 and m_k = 0.
// kDict: the dictionary form of the cache (as k_gram_fill).  Its few entries stay in the caches,
// so the line's Gram values are re-read for every sample instead of held in registers: one
// packed working copy (~250 VGPRs), two waves per SIMD.
template <int W, typename TM, bool LSQ, typename GT, bool kDict>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(kDict ? 2 : 1))) void k_gram_fill_wide(int32_t n, int32_t line_begin, int32_t line_end, int32_t wrt,
                                                        const int32_t* __restrict__ pat_act,
                                                        const float* __restrict__ pat_val,
                                                        const GT* __restrict__ gram,
                                                        const int32_t* __restrict__ line_entry, int32_t B,
                                                        const uint32_t* __restrict__ removed, int32_t words,
                                                        int32_t word_base, TM* __restrict__ m_out,
                                                        double* __restrict__ partials) {
  constexpr int T = tri(W);
  static_assert(W <= 32, "keep mask is one 32-bit word");
  // per-sample line residuals of a chunk of kChunk samples (summed after the chunk: one barrier
  // pair per chunk, not per sample) and M staged through two LDS buffers (sample b writes buffer
  // b & 1 while sample b - 1's stores may still read the other)
  // (kDict: ONE M buffer, a barrier before it is rewritten: <= 80 KB of LDS, two blocks per CU)
  __shared__ double s_r2[kChunk][kNT];
#ifdef FILL_BLOCK_M
  __shared__ __attribute__((aligned(16))) TM s_m[kDict ? 1 : 2][kNT * W];
#else
  __shared__ __attribute__((aligned(16))) TM s_m[1][kNT * W];  // per-wave regions
#endif
  __shared__ int32_t s_act[W][kNT];  // action ids of the slots (LDS, not registers: G needs them)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lb = blockIdx.x;
  const int j = line_begin + lb * kNT + t;
  const bool valid = j < line_end;
  const int64_t nloc = line_end - line_begin;
  const int jj = valid ? j : line_begin;
  {
    int av[W];  // every load issued before any is used (no branch per slot)
#pragma unroll
    for (int p = 0; p < W; ++p) av[p] = pat_act[(int64_t)jj * wrt + min(p, wrt - 1)];
#pragma unroll
    for (int p = 0; p < W; ++p) s_act[p][t] = (valid && p < wrt) ? av[p] : -1;
  }
  constexpr int kStride = kDict ? 1 : 64;
  const GT* gp = kDict ? gram + (int64_t)line_entry[jj] * (T + W) : gram + (int64_t)(jj >> 6) * (T + W) * 64 + (jj & 63);
  const int nvl = min(kNT, line_end - (line_begin + lb * kNT));
  // the slots' bitmap words of the next sample are loaded while the current one is solved (kDict:
  // loaded per sample, no registers held across the samples; the other wave of the SIMD hides them)
  constexpr int kWd = kDict ? 1 : W;
  uint32_t wd[kWd];
  if constexpr (!kDict) {
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const int ap = s_act[p][t];
      wd[p] = removed[ap >= 0 ? (ap >> 5) - word_base : 0];  // unconditional (masked at use): no branch per slot
    }
  }
#pragma unroll 1
  for (int b = 0; b < B; ++b) {
    uint32_t keep = 0;
    if constexpr (kDict) {
      const uint32_t* rb = removed + (int64_t)b * words;
      uint32_t wv[W];
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const int ap = s_act[p][t];
        wv[p] = rb[ap >= 0 ? (ap >> 5) - word_base : 0];
      }
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const int ap = s_act[p][t];
        keep |= (uint32_t)((ap >= 0) & !((wv[p] >> (ap & 31)) & 1u)) << p;
      }
    } else {
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const int ap = s_act[p][t];
        keep |= (uint32_t)((ap >= 0) & !((wd[p] >> (ap & 31)) & 1u)) << p;
      }
      if (b + 1 < B) {
        const uint32_t* rn = removed + (int64_t)(b + 1) * words;
#pragma unroll
        for (int p = 0; p < W; ++p) {
          const int ap = s_act[p][t];
          wd[kDict ? 0 : p] = rn[ap >= 0 ? (ap >> 5) - word_base : 0];
        }
      }
    }
    double a[T], y[W];
    // loop-invariant: the compiler keeps one copy of the line's Gram values in registers across
    // the samples and factors a second, working copy per sample (463 VGPRs, one wave per SIMD,
    // no spills).  Re-reading them per sample instead (an opaque address, 254 VGPRs, two waves
    // per SIMD) measured 286 vs 183 us at C3: the L2 re-reads cost more than the occupancy buys.
    const GT* gps = gp;  // fp32 storage only when exact (spai_gram_compact): the same values
    if constexpr (kDict) asm volatile("" : "+v"(gps));  // re-read per sample (cache hits), not held
#pragma unroll
    for (int q = 0; q < T; ++q) a[q] = (double)gps[q * kStride];
    double r2 = 1.0;
    if constexpr (LSQ) {
#pragma unroll
      for (int k = 0; k < W; ++k) y[k] = (double)gps[(T + k) * kStride];  // c, solved in place below
      r2 = wide_lsq_solve<W>(a, y, keep);
    } else {
#pragma unroll
      for (int p = 0; p < W; ++p)
        y[p] = ((keep >> p) & 1u) ? (double)pat_val[(int64_t)jj * wrt + (p < wrt ? p : 0)] : 0.0;
#pragma unroll
      for (int p = 0; p < W; ++p) {
        double acc = y[p] * a[gidx<W>(p, p)] - 2.0 * (double)gps[(T + p) * kStride];
#pragma unroll
        for (int q = p + 1; q < W; ++q) acc += 2.0 * y[q] * a[gidx<W>(p, q)];
        r2 += y[p] * acc;
      }
    }
    s_r2[b % kChunk][t] = valid ? r2 : 0.0;
#ifdef FILL_BLOCK_M
    {  // M (no branch on m_out: store_m_block drops every store when it is null)
      TM* sm = s_m[kDict ? 0 : (b & 1)];
      if constexpr (kDict) __syncthreads();  // the previous sample's stores have read the buffer
      if (valid) {
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p < wrt) sm[t * wrt + p] = (TM)y[p];
      }
      __syncthreads();
      store_m_block<kNT, W, TM>(m_out ? m_out + ((int64_t)b * nloc + (int64_t)lb * kNT) * wrt : nullptr, sm, nvl * wrt);
    }
#else
    {  // M staged per WAVE (its 64 lines are one contiguous run of M): no block barrier per sample
      const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: scalar offsets
      TM* sm = s_m[0] + wv * 64 * W;
      if (valid) {
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p < wrt) sm[lane * wrt + p] = (TM)y[p];
      }
      __builtin_amdgcn_wave_barrier();
      const int nw = min(max(nvl - wv * 64, 0), 64);
      store_m_block<64, W, TM>(m_out ? m_out + ((int64_t)b * nloc + (int64_t)lb * kNT + wv * 64) * wrt : nullptr,
                               sm, nw * wrt, lane);
      __builtin_amdgcn_wave_barrier();
    }
#endif
    if (b % kChunk == kChunk - 1 || b == B - 1) {  // the chunk's fixed-order block sums
      const int c0 = b - b % kChunk, nb = b - c0 + 1;
      __syncthreads();
      for (int u = wave; u < nb; u += kNT / 64) {
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < kNT / 64; ++q) acc += s_r2[u][q * 64 + lane];
        acc = wave_sum(acc);
        if (lane == 0) partials[(int64_t)(c0 + u) * gridDim.x + lb] = acc;
      }
      __syncthreads();
    }
  }
}

static int gram_width(int32_t W) { return W <= 5 ? 5 : (W <= 7 ? 7 : (W <= 13 ? 13 : 0)); }

template <int W, typename TM, bool LSQ, typename GT, bool kDict>
void launch_fill_t(int32_t n, int32_t lb, int32_t le, int32_t wrt, const int32_t* pa, const float* pv, const void* g,
                   const int32_t* ent, int32_t B, const uint32_t* rm, int32_t words, int32_t wb, void* mo,
                   double* partials, int32_t nparts, hipStream_t s) {
  KernelTimer kt(SPAI_TIMER_GRAM, s);
  if constexpr (W > 7)
    k_gram_fill_wide<W, TM, LSQ, GT, kDict><<<nparts, kNT, 0, s>>>(n, lb, le, wrt, pa, pv, static_cast<const GT*>(g),
                                                                    ent, B, rm, words, wb, static_cast<TM*>(mo),
                                                                    partials);
  else
    k_gram_fill<W, TM, LSQ, GT, kDict><<<nparts, kNT, 0, s>>>(n, lb, le, wrt, pa, pv, static_cast<const GT*>(g), ent,
                                                               B, rm, words, wb, static_cast<TM*>(mo), partials);
}
template <int W, typename TM, bool LSQ>
hipError_t launch_fill(int32_t n, int32_t lb, int32_t le, int32_t wrt, const int32_t* pa, const float* pv,
                       const void* g, bool g32, const int32_t* ent, int32_t B, const uint32_t* rm, int32_t words,
                       int32_t wb, void* mo, double* partials, int32_t nparts, hipStream_t s) {
  if (g32) {
    if (ent)
      launch_fill_t<W, TM, LSQ, float, true>(n, lb, le, wrt, pa, pv, g, ent, B, rm, words, wb, mo, partials, nparts, s);
    else
      launch_fill_t<W, TM, LSQ, float, false>(n, lb, le, wrt, pa, pv, g, ent, B, rm, words, wb, mo, partials, nparts, s);
  } else if (ent) {
    launch_fill_t<W, TM, LSQ, double, true>(n, lb, le, wrt, pa, pv, g, ent, B, rm, words, wb, mo, partials, nparts, s);
  } else {
    launch_fill_t<W, TM, LSQ, double, false>(n, lb, le, wrt, pa, pv, g, ent, B, rm, words, wb, mo, partials, nparts, s);
  }
  return hipGetLastError();
}

// fp32 copy of the Gram cache; *exact is cleared if any entry does not survive the round trip
__global__ __launch_bounds__(kNT) void k_gram_compact(int64_t count, const double* __restrict__ g,
                                                      float* __restrict__ g32, int32_t* __restrict__ exact) {
  const int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x;
  if (i >= count) return;
  const double v = g[i];
  const float f = (float)v;
  g32[i] = f;
  if ((double)f != v) *exact = 0;  // benign race: every writer stores 0
}

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" size_t spai_gram_bytes(int32_t n, int32_t W) {
  const int wc = gram_width(W);
  if (n <= 0 || wc == 0) return 0;
  return sizeof(double) * (size_t)(tri(wc) + wc) * (size_t)((n + 63) / 64 * 64);
}

extern "C" int spai_gram_build(int32_t n, int32_t W, const int32_t* pat_idx, int32_t WA, const int32_t* a_idx,
                               const void* a_val, int32_t a_dtype, double* gram, void* stream) {
  SPAI_CHECK_ARG(n >= 1 && W >= 1 && WA >= 1 && pat_idx && a_idx && a_val && gram, "spai_gram_build: bad arguments");
  SPAI_CHECK_ARG(a_dtype == SPAI_DTYPE_F32 || a_dtype == SPAI_DTYPE_F64, "spai_gram_build: bad a_dtype");
  const int wc = gram_width(W);
  if (wc == 0 || WA > 7) {
    set_error("spai_gram_build: widths W=%d (max 13) WA=%d (max 7) above the compiled kernels", W, WA);
    return SPAI_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int grid = (n + kNT - 1) / kNT;
  if (a_dtype == SPAI_DTYPE_F32) {
    if (wc == 5 && WA <= 5)
      k_gram_build<5, 5, float><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const float*)a_val, gram);
    else if (wc == 5)
      k_gram_build<5, 7, float><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const float*)a_val, gram);
    else if (wc == 7)
      k_gram_build<7, 7, float><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const float*)a_val, gram);
    else
      k_gram_build<13, 7, float><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const float*)a_val, gram);
  } else {
    if (wc == 5 && WA <= 5)
      k_gram_build<5, 5, double><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const double*)a_val, gram);
    else if (wc == 5)
      k_gram_build<5, 7, double><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const double*)a_val, gram);
    else if (wc == 7)
      k_gram_build<7, 7, double><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const double*)a_val, gram);
    else
      k_gram_build<13, 7, double><<<grid, kNT, 0, s>>>(n, W, WA, pat_idx, a_idx, (const double*)a_val, gram);
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_gram_compact(int32_t n, int32_t W, const double* gram, float* gram32, int32_t* exact,
                                 void* stream) {
  SPAI_CHECK_ARG(n >= 1 && gram && gram32 && exact, "spai_gram_compact: bad arguments");
  const int wc = gram_width(W);
  SPAI_CHECK_ARG(wc != 0, "spai_gram_compact: width %d above 13", W);
  const int64_t count = (int64_t)(tri(wc) + wc) * ((n + 63) / 64 * 64);
  hipStream_t s = (hipStream_t)stream;
  k_gram_compact<<<(int)((count + kNT - 1) / kNT), kNT, 0, s>>>(count, gram, gram32, exact);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

// Fill + per-block partial sums only (res2 partials stay in the workspace for spai_fill_reduce).
static int fill_lines_gram(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                           const int32_t* pat_act, const float* pat_val, const void* gram, int32_t gram_dtype,
                           const int32_t* line_entry, int32_t B, const uint32_t* removed, int32_t words,
                           int32_t word_base, void* m_out, int32_t m_dtype, void* workspace, size_t workspace_bytes,
                           void* stream) {
  SPAI_CHECK_ARG(fill_mode == SPAI_FILL_COPY || fill_mode == SPAI_FILL_LSQ,
                 "spai_fill_lines_gram(_dict): bad fill_mode %d", fill_mode);
  SPAI_CHECK_ARG(m_dtype == SPAI_DTYPE_F32 || m_dtype == SPAI_DTYPE_F64, "spai_fill_lines_gram(_dict): bad m_dtype");
  SPAI_CHECK_ARG(n >= 1 && line_begin >= 0 && line_end >= line_begin && line_end <= n && W >= 1 && B >= 1 &&
                     words >= 1 && word_base >= 0,
                 "spai_fill_lines_gram(_dict): bad shape");
  SPAI_CHECK_ARG(workspace != nullptr, "spai_fill_lines_gram(_dict): null workspace");
  SPAI_CHECK_ARG(fill_mode != SPAI_FILL_COPY || m_dtype == SPAI_DTYPE_F32,
                 "spai_fill_lines_gram(_dict): copy fill stores fp32 values (utils.py:350)");
  hipStream_t s = (hipStream_t)stream;
  const int32_t nl = line_end - line_begin;
  if (nl == 0) return SPAI_OK;
  SPAI_CHECK_ARG(pat_act && gram && removed && (fill_mode == SPAI_FILL_LSQ || pat_val),
                 "spai_fill_lines_gram(_dict): null input");
  const int wc = gram_width(W);
  if (wc == 0) {
    set_error("spai_fill_lines_gram(_dict): width W=%d above the compiled 13", W);
    return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_ARG(gram_dtype == SPAI_DTYPE_F64 || gram_dtype == SPAI_DTYPE_F32, "spai_fill_lines_gram(_dict): gram dtype %d",
                 gram_dtype);
  const bool g32 = gram_dtype == SPAI_DTYPE_F32;
  const int32_t nparts = (nl + kNT - 1) / kNT;
  SPAI_CHECK_ARG(workspace_bytes >= sizeof(double) * (size_t)nparts * B, "spai_fill_lines_gram(_dict): workspace too small");
  double* partials = static_cast<double*>(workspace);
  const uint32_t* rm = removed;
  const int32_t wb = word_base;
  hipError_t e;
  const bool lsq = fill_mode == SPAI_FILL_LSQ, f64 = m_dtype == SPAI_DTYPE_F64;
#define SPAI_FILL_ARGS n, line_begin, line_end, W, pat_act, pat_val, gram, g32, line_entry, B, rm, words, wb, m_out, partials, nparts, s
  if (wc == 5) {
    e = !lsq ? launch_fill<5, float, false>(SPAI_FILL_ARGS)
        : f64 ? launch_fill<5, double, true>(SPAI_FILL_ARGS)
              : launch_fill<5, float, true>(SPAI_FILL_ARGS);
  } else if (wc == 7) {
    e = !lsq ? launch_fill<7, float, false>(SPAI_FILL_ARGS)
        : f64 ? launch_fill<7, double, true>(SPAI_FILL_ARGS)
              : launch_fill<7, float, true>(SPAI_FILL_ARGS);
  } else {
    e = !lsq ? launch_fill<13, float, false>(SPAI_FILL_ARGS)
        : f64 ? launch_fill<13, double, true>(SPAI_FILL_ARGS)
              : launch_fill<13, float, true>(SPAI_FILL_ARGS);
  }
#undef SPAI_FILL_ARGS
  SPAI_CHECK_HIP(e);
  return SPAI_OK;
}
extern "C" int spai_fill_lines_gram(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                                    const int32_t* pat_act, const float* pat_val, const void* gram,
                                    int32_t gram_dtype, int32_t B, const uint32_t* removed, int32_t words,
                                    int32_t word_base, void* m_out, int32_t m_dtype, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  return fill_lines_gram(fill_mode, n, line_begin, line_end, W, pat_act, pat_val, gram, gram_dtype, nullptr, B,
                         removed, words, word_base, m_out, m_dtype, workspace, workspace_bytes, stream);
}
extern "C" int spai_fill_lines_gram_dict(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end,
                                         int32_t W, const int32_t* pat_act, const float* pat_val, const void* dict,
                                         int32_t gram_dtype, const int32_t* line_entry, int32_t B,
                                         const uint32_t* removed, int32_t words, int32_t word_base, void* m_out,
                                         int32_t m_dtype, void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(line_entry != nullptr, "spai_fill_lines_gram_dict: null line_entry");
  return fill_lines_gram(fill_mode, n, line_begin, line_end, W, pat_act, pat_val, dict, gram_dtype, line_entry, B,
                         removed, words, word_base, m_out, m_dtype, workspace, workspace_bytes, stream);
}

extern "C" int spai_fill_reduce(int32_t n_lines, int32_t B, const void* workspace, double* res2_out,
                                int64_t* limbs_out, void* stream) {
  SPAI_CHECK_ARG(n_lines >= 0 && B >= 1 && workspace && (res2_out || limbs_out), "spai_fill_reduce: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  if (n_lines == 0) {
    if (res2_out) SPAI_CHECK_HIP(hipMemsetAsync(res2_out, 0, sizeof(double) * B, s));
    if (limbs_out) SPAI_CHECK_HIP(hipMemsetAsync(limbs_out, 0, sizeof(int64_t) * kLimbSlots * B, s));
    return SPAI_OK;
  }
  k_fixed_reduce<1024><<<B, 1024, 0, s>>>(static_cast<const double*>(workspace), (n_lines + kNT - 1) / kNT, res2_out,
                                          limbs_out, RewardArgs{});
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

// One GPU: the fill's partial sums ARE the whole residuals, so the reward formula is applied in
// the same launch (replaces spai_fill_reduce + spai_rewards + the fp32 copy of the rewards).
extern "C" int spai_fill_reduce_rewards(int32_t n_lines, int32_t B, const void* workspace,
                                        const int32_t* removed_counts, int64_t nnz0, int32_t n, double r0, double f0,
                                        const float* alpha, double* residual, double* reward, float* reward32,
                                        void* stream) {
  SPAI_CHECK_ARG(n_lines >= 1 && B >= 1 && workspace && removed_counts && alpha && residual && reward && n >= 1 &&
                     nnz0 >= 0,
                 "spai_fill_reduce_rewards: bad arguments");
  const RewardArgs ra{removed_counts, nnz0, n, r0, f0, alpha, residual, reward, reward32};
  k_fixed_reduce<1024><<<B, 1024, 0, (hipStream_t)stream>>>(static_cast<const double*>(workspace),
                                                            (n_lines + kNT - 1) / kNT, nullptr, nullptr, ra);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_fill_residual_gram(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                                       const int32_t* pat_act, const float* pat_val, const void* gram,
                                       int32_t gram_dtype, int32_t B, const uint32_t* removed, int32_t words,
                                       int32_t word_base, void* m_out, int32_t m_dtype, double* res2_out,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(res2_out != nullptr, "spai_fill_residual_gram: null res2_out");
  const int st = spai_fill_lines_gram(fill_mode, n, line_begin, line_end, W, pat_act, pat_val, gram, gram_dtype, B,
                                      removed, words, word_base, m_out, m_dtype, workspace, workspace_bytes, stream);
  if (st != SPAI_OK) return st;
  return spai_fill_reduce(line_end - line_begin, B, workspace, res2_out, nullptr, stream);
}

namespace spai {
namespace {
__global__ void k_limbs_to_res2(int32_t B, const int64_t* __restrict__ limbs, double* __restrict__ res2) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) res2[b] = fixed_value(limbs + (int64_t)b * kLimbSlots);
}
}  // namespace
}  // namespace spai

extern "C" int spai_res2_from_limbs(int32_t B, const int64_t* limbs, double* res2_out, void* stream) {
  SPAI_CHECK_ARG(B >= 1 && limbs && res2_out, "spai_res2_from_limbs: bad arguments");
  k_limbs_to_res2<<<1, 256, 0, (hipStream_t)stream>>>(B, limbs, res2_out);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
