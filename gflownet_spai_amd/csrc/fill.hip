// Fill + residual kernel for gfx950: builds M from the pattern and the per-sample removal
// bitmaps (copy fill of gflownet/utils.py:331-353, or the north-star per-line least-squares
// fill) and accumulates ||M A - I||_F^2 (row lines, preconditioner.py:79-93) or
// ||A M - I||_F^2 (column lines) without materialising the product.
//
// Identity used (one line l of M with slots p -> other index k_p, values m_p):
//     || sum_p m_p A_line(k_p) - e_l ||^2 = m^T G m - 2 c^T m + 1
// with G_pq = <A_line(k_p), A_line(k_q)> and c_p = A_line(k_p)[l].  G and c depend only on
// the pattern, so one thread per line computes them ONCE from the W x WA entries it
// gathers and then loops over all B samples: per sample it reads W mask bits, solves the
// masked W x W normal equations in fp64 (LSQ) or copies (COPY), stores m in the target
// precision and evaluates the quadratic form on the STORED values.  HBM traffic per
// launch is the pattern + A lines once and B x (mask bits + M values); the B-fold
// re-reads of A that an SpGEMM per sample would make never happen.
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kNT = 256;

template <int W, int WA, typename TA, typename TM, bool LSQ>
__global__ __launch_bounds__(kNT) void k_line(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                              const int32_t* __restrict__ pat_idx,
                                              const int32_t* __restrict__ pat_act,
                                              const float* __restrict__ pat_val, const int32_t* __restrict__ a_idx,
                                              const TA* __restrict__ a_val, int32_t B,
                                              const uint32_t* __restrict__ removed, int32_t words,
                                              int32_t word_base, TM* __restrict__ m_out,
                                              double* __restrict__ partials) {
  __shared__ double sred[kNT / 64];
  const int j = line_begin + blockIdx.x * kNT + threadIdx.x;
  const bool valid = j < line_end;
  const int64_t nloc = line_end - line_begin;

  int idx[W], act[W];
  float val[W];
#pragma unroll
  for (int p = 0; p < W; ++p) {
    idx[p] = -1;
    act[p] = 0;
    val[p] = 0.0f;
    if (valid && p < wrt) {
      const int64_t o = (int64_t)j * wrt + p;
      idx[p] = pat_idx[o];
      act[p] = pat_act[o];
      val[p] = pat_val[o];
    }
  }

  double G[W][W];
  double c[W];
  {
    int ai[W][WA];
    TA av[W][WA];
#pragma unroll
    for (int p = 0; p < W; ++p) {
#pragma unroll
      for (int q = 0; q < WA; ++q) {
        ai[p][q] = -1;
        av[p][q] = (TA)0;
        if (idx[p] >= 0 && q < wart) {
          const int64_t o = (int64_t)idx[p] * wart + q;
          ai[p][q] = a_idx[o];
          av[p][q] = a_val[o];
        }
      }
    }
#pragma unroll
    for (int p = 0; p < W; ++p) {
      double cp = 0.0, gpp = 0.0;
#pragma unroll
      for (int s = 0; s < WA; ++s) {
        const double v = (double)av[p][s];
        gpp += v * v;
        cp += (ai[p][s] == j) ? v : 0.0;
      }
      c[p] = cp;
      G[p][p] = gpp;
#pragma unroll
      for (int q = p + 1; q < W; ++q) {
        double g = 0.0;
#pragma unroll
        for (int s = 0; s < WA; ++s) {
#pragma unroll
          for (int t = 0; t < WA; ++t) {
            g += (ai[p][s] >= 0 && ai[p][s] == ai[q][t]) ? (double)av[p][s] * (double)av[q][t] : 0.0;
          }
        }
        G[p][q] = g;
      }
    }
  }

  for (int b = 0; b < B; ++b) {
    const uint32_t* rb = removed + (int64_t)b * words;
    bool keep[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const int wo = idx[p] >= 0 ? (act[p] >> 5) - word_base : 0;  // row-relative word (window rows)
      keep[p] = idx[p] >= 0 && !((rb[wo] >> (act[p] & 31)) & 1u);
    }

    double mr[W];
    if constexpr (!LSQ) {
#pragma unroll
      for (int p = 0; p < W; ++p) mr[p] = keep[p] ? (double)val[p] : 0.0;
    } else {
      // masked LDL^T of the normal equations: removed slots become identity rows, rhs 0
      double L[W][W], D[W], iD[W], y[W];
#pragma unroll
      for (int k = 0; k < W; ++k) {
        double dk = keep[k] ? G[k][k] : 1.0;
        const double ref = dk;
#pragma unroll
        for (int s = 0; s < k; ++s) dk -= L[k][s] * L[k][s] * D[s];
        D[k] = dk;
        iD[k] = (dk > 1e-13 * ref) ? 1.0 / dk : 0.0;
#pragma unroll
        for (int i = k + 1; i < W; ++i) {
          double v = (keep[k] && keep[i]) ? G[k][i] : 0.0;
#pragma unroll
          for (int s = 0; s < k; ++s) v -= L[i][s] * L[k][s] * D[s];
          L[i][k] = v * iD[k];
        }
      }
#pragma unroll
      for (int k = 0; k < W; ++k) {
        double v = keep[k] ? c[k] : 0.0;
#pragma unroll
        for (int s = 0; s < k; ++s) v -= L[k][s] * y[s];
        y[k] = v;
      }
#pragma unroll
      for (int k = W - 1; k >= 0; --k) {
        double v = y[k] * iD[k];
#pragma unroll
        for (int s = k + 1; s < W; ++s) v -= L[s][k] * mr[s];
        mr[k] = v;
      }
#pragma unroll
      for (int p = 0; p < W; ++p) mr[p] = keep[p] ? (double)(TM)mr[p] : 0.0;  // stored precision
    }

    if (m_out != nullptr && valid) {
      TM* dst = m_out + ((int64_t)b * nloc + (j - line_begin)) * wrt;
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (p < wrt) dst[p] = (TM)mr[p];
    }

    double r2 = 0.0;
    if (valid) {
      r2 = 1.0;
#pragma unroll
      for (int p = 0; p < W; ++p) {
        double acc = mr[p] * G[p][p] - 2.0 * c[p];
#pragma unroll
        for (int q = p + 1; q < W; ++q) acc += 2.0 * mr[q] * G[p][q];
        r2 += mr[p] * acc;
      }
    }
    r2 = block_sum<kNT>(r2, sred);
    if (threadIdx.x == 0) partials[(int64_t)b * gridDim.x + blockIdx.x] = r2;
  }
}

// Generic COPY-fill residual for lines of any width (e.g. the reference drivers' spilu
// L@U candidate patterns, GFlowNet100.py:137-153): one workgroup per line accumulates the
// line of M*A (or A*M) of one sample in an LDS open-addressing table of fp64 sums keyed by
// the other index (the diagonal is seeded with -1), then sums the squares.  The table is sized
// per line: 2 x (1 + the products the line can make), capped by the launch's allocation; the A
// lines are walked up to their first -1 slot (left-packed ELL, as build_lines lays them out), so
// the work is the line's real products, not its padded width squared.  A probe that finds the table
// full (more distinct keys than the cap) flags the line: its partial is NaN, never a hang.
__device__ __forceinline__ bool hash_add(int* keys, double* vals, int tb, int key, double v) {
  unsigned h = ((unsigned)key * 2654435761u) % (unsigned)tb;
  for (int probe = 0; probe < tb; ++probe) {
    const int prev = atomicCAS(&keys[h], -1, key);
    if (prev == -1 || prev == key) {
      atomicAdd(&vals[h], v);
      return true;
    }
    h = (h + 1 == (unsigned)tb) ? 0u : h + 1;
  }
  return false;  // full
}

template <typename TA>
__global__ __launch_bounds__(kNT) void k_line_hash(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                   const int32_t* __restrict__ pat_idx,
                                                   const int32_t* __restrict__ pat_act,
                                                   const float* __restrict__ pat_val,
                                                   const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val,
                                                   int32_t B, const uint32_t* __restrict__ removed, int32_t words,
                                                   int32_t word_base, float* __restrict__ m_out,
                                                   double* __restrict__ partials, int32_t tb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* vals = reinterpret_cast<double*>(smem);
  int* keys = reinterpret_cast<int*>(smem + (size_t)tb * sizeof(double));
  __shared__ double sred[kNT / 64];
  __shared__ int s_cnt[kNT / 64];
  __shared__ int s_full;
  const int j = line_begin + blockIdx.x;
  const int64_t nloc = line_end - line_begin;
  const int64_t base = (int64_t)j * wrt;
  // this line's table size: 2 x (1 + its products over every slot), a multiple of 64, capped by tb
  int np = 0;
  for (int p = threadIdx.x; p < wrt; p += kNT) {
    const int k = pat_idx[base + p];
    if (k < 0) continue;
    int s = 0;
    while (s < wart && a_idx[(int64_t)k * wart + s] >= 0) ++s;
    np += s;
  }
  np = wave_sum(np);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = np;
  if (threadIdx.x == 0) s_full = 0;
  __syncthreads();
  int tot = 0;
#pragma unroll
  for (int w = 0; w < kNT / 64; ++w) tot += s_cnt[w];
  const int tbl = min(tb, max(64, (2 * (tot + 1) + 63) / 64 * 64));
  for (int b = 0; b < B; ++b) {
    const uint32_t* rb = removed + (int64_t)b * words;
    for (int t = threadIdx.x; t < tbl; t += kNT) {
      keys[t] = -1;
      vals[t] = 0.0;
    }
    __syncthreads();
    if (threadIdx.x == 0 && !hash_add(keys, vals, tbl, j, -1.0)) s_full = 1;
    if (m_out != nullptr) {
      for (int p = threadIdx.x; p < wrt; p += kNT) {
        const int k = pat_idx[base + p], a = pat_act[base + p];
        const bool keep = k >= 0 && !((rb[(a >> 5) - word_base] >> (a & 31)) & 1u);
        m_out[((int64_t)b * nloc + (j - line_begin)) * wrt + p] = keep ? pat_val[base + p] : 0.0f;
      }
    }
    for (int p = threadIdx.x; p < wrt; p += kNT) {
      const int k = pat_idx[base + p];
      if (k < 0) continue;
      const int a = pat_act[base + p];
      if ((rb[(a >> 5) - word_base] >> (a & 31)) & 1u) continue;
      const double mv = (double)pat_val[base + p];
      for (int s = 0; s < wart; ++s) {
        const int64_t o = (int64_t)k * wart + s;
        const int l = a_idx[o];
        if (l < 0) break;
        if (!hash_add(keys, vals, tbl, l, mv * (double)a_val[o])) s_full = 1;
      }
    }
    __syncthreads();
    double s2 = 0.0;
    for (int t = threadIdx.x; t < tbl; t += kNT)
      if (keys[t] >= 0) s2 += vals[t] * vals[t];
    s2 = block_sum<kNT>(s2, sred);
    if (threadIdx.x == 0) partials[(int64_t)b * gridDim.x + blockIdx.x] = s_full ? __builtin_nan("") : s2;
    __syncthreads();
  }
}

constexpr int kHashMaxEntries = 13000;  // 13000 x 12 B = 152 KiB of the 160 KiB LDS

template <typename TA>
hipError_t launch_hash(int32_t lb, int32_t le, int32_t wrt, int32_t wart, const int32_t* pi, const int32_t* pa,
                       const float* pv, const int32_t* ai, const void* av, int32_t B, const uint32_t* rm,
                       int32_t words, int32_t wb, void* mo, double* partials, int32_t tb, hipStream_t s) {
  const size_t lds = (size_t)tb * (sizeof(double) + sizeof(int));
  hipError_t e = hipFuncSetAttribute((const void*)k_line_hash<TA>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  k_line_hash<TA><<<le - lb, kNT, lds, s>>>(lb, le, wrt, wart, pi, pa, pv, ai, static_cast<const TA*>(av), B, rm,
                                             words, wb, static_cast<float*>(mo), partials, tb);
  return hipGetLastError();
}

__global__ void k_rewards(const double* __restrict__ res2, int32_t B, RewardArgs ra) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) write_reward(b, res2[b], ra);
}

template <int W, int WA, typename TA, typename TM, bool LSQ>
hipError_t launch_line(int32_t lb, int32_t le, int32_t wrt, int32_t wart, const int32_t* pi, const int32_t* pa,
                       const float* pv, const int32_t* ai, const void* av, int32_t B, const uint32_t* rm,
                       int32_t words, int32_t wb, void* mo, double* partials, int32_t nparts, hipStream_t s) {
  k_line<W, WA, TA, TM, LSQ><<<nparts, kNT, 0, s>>>(lb, le, wrt, wart, pi, pa, pv, ai, static_cast<const TA*>(av), B,
                                                     rm, words, wb, static_cast<TM*>(mo), partials);
  return hipGetLastError();
}

using LaunchFn = hipError_t (*)(int32_t, int32_t, int32_t, int32_t, const int32_t*, const int32_t*, const float*,
                                const int32_t*, const void*, int32_t, const uint32_t*, int32_t, int32_t, void*,
                                double*, int32_t, hipStream_t);

struct Variant {
  int W, WA, a_dtype, m_dtype, mode;
  LaunchFn fn;
};

// Compiled (width, A dtype, M dtype, fill) combinations; dispatch takes the first that fits.
static const Variant kVariants[] = {
    {5, 5, SPAI_DTYPE_F32, SPAI_DTYPE_F32, SPAI_FILL_COPY, launch_line<5, 5, float, float, false>},
    {7, 7, SPAI_DTYPE_F32, SPAI_DTYPE_F32, SPAI_FILL_COPY, launch_line<7, 7, float, float, false>},
    {5, 5, SPAI_DTYPE_F64, SPAI_DTYPE_F32, SPAI_FILL_COPY, launch_line<5, 5, double, float, false>},
    {7, 7, SPAI_DTYPE_F64, SPAI_DTYPE_F32, SPAI_FILL_COPY, launch_line<7, 7, double, float, false>},
    {5, 5, SPAI_DTYPE_F32, SPAI_DTYPE_F32, SPAI_FILL_LSQ, launch_line<5, 5, float, float, true>},
    {7, 7, SPAI_DTYPE_F32, SPAI_DTYPE_F32, SPAI_FILL_LSQ, launch_line<7, 7, float, float, true>},
    {5, 5, SPAI_DTYPE_F64, SPAI_DTYPE_F64, SPAI_FILL_LSQ, launch_line<5, 5, double, double, true>},
    {7, 7, SPAI_DTYPE_F64, SPAI_DTYPE_F64, SPAI_FILL_LSQ, launch_line<7, 7, double, double, true>},
};

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" size_t spai_fill_workspace_bytes(int32_t n_lines, int32_t B) {
  const int64_t nparts = std::max(n_lines, 1);  // one partial per line (hash variant) or per block
  Carve c(nullptr);
  c.take<double>((size_t)nparts * std::max(B, 1));
  return c.off;
}

extern "C" int spai_fill_residual(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                                  const int32_t* pat_idx, const int32_t* pat_act, const float* pat_val, int32_t WA,
                                  const int32_t* a_idx, const void* a_val, int32_t a_dtype, int32_t B,
                                  const uint32_t* removed, int32_t words, int32_t word_base, void* m_out,
                                  int32_t m_dtype, double* res2_out, int64_t* limbs_out, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(fill_mode == SPAI_FILL_COPY || fill_mode == SPAI_FILL_LSQ, "spai_fill_residual: bad fill_mode %d",
                 fill_mode);
  SPAI_CHECK_ARG(a_dtype == SPAI_DTYPE_F32 || a_dtype == SPAI_DTYPE_F64, "spai_fill_residual: bad a_dtype");
  SPAI_CHECK_ARG(m_dtype == SPAI_DTYPE_F32 || m_dtype == SPAI_DTYPE_F64, "spai_fill_residual: bad m_dtype");
  SPAI_CHECK_ARG(n >= 1 && line_begin >= 0 && line_end >= line_begin && line_end <= n && W >= 1 && WA >= 1 &&
                     B >= 1 && words >= 1 && word_base >= 0,
                 "spai_fill_residual: bad shape");
  SPAI_CHECK_ARG((res2_out || limbs_out) && workspace, "spai_fill_residual: null output/workspace");
  hipStream_t s = (hipStream_t)stream;
  const int32_t nl = line_end - line_begin;
  if (nl == 0) {
    if (res2_out) SPAI_CHECK_HIP(hipMemsetAsync(res2_out, 0, sizeof(double) * B, s));
    if (limbs_out) SPAI_CHECK_HIP(hipMemsetAsync(limbs_out, 0, sizeof(int64_t) * kLimbSlots * B, s));
    return SPAI_OK;
  }
  SPAI_CHECK_ARG(pat_idx && pat_act && pat_val && a_idx && a_val && removed, "spai_fill_residual: null input");
  SPAI_CHECK_ARG(workspace_bytes >= spai_fill_workspace_bytes(nl, B), "spai_fill_residual: workspace too small");
  const int32_t want_m = fill_mode == SPAI_FILL_COPY ? SPAI_DTYPE_F32 : m_dtype;
  SPAI_CHECK_ARG(fill_mode != SPAI_FILL_COPY || m_dtype == SPAI_DTYPE_F32,
                 "spai_fill_residual: copy fill stores fp32 values (utils.py:350)");
  const Variant* v = nullptr;
  for (const Variant& cand : kVariants) {
    if (cand.mode == fill_mode && cand.a_dtype == a_dtype && cand.m_dtype == want_m && cand.W >= W && cand.WA >= WA) {
      v = &cand;
      break;
    }
  }
  if (!v) {
    // any width: the hash kernel (copy fill); its table holds up to kHashMaxEntries keys per line
    // (a line with more distinct keys gets a NaN residual)
    const int64_t bound = std::min<int64_t>((int64_t)W * WA + 1, (int64_t)n);
    if (fill_mode == SPAI_FILL_COPY) {
      const int32_t tb = (int32_t)std::min<int64_t>(kHashMaxEntries, std::max<int64_t>(64, 2 * bound));
      double* partials = static_cast<double*>(workspace);
      hipError_t e = a_dtype == SPAI_DTYPE_F32
                         ? launch_hash<float>(line_begin, line_end, W, WA, pat_idx, pat_act, pat_val, a_idx, a_val, B,
                                              removed, words, word_base, m_out, partials, tb, s)
                         : launch_hash<double>(line_begin, line_end, W, WA, pat_idx, pat_act, pat_val, a_idx, a_val,
                                               B, removed, words, word_base, m_out, partials, tb, s);
      SPAI_CHECK_HIP(e);
      k_fixed_reduce<1024><<<B, 1024, 0, s>>>(partials, nl, res2_out, limbs_out, RewardArgs{});
      SPAI_CHECK_LAUNCH();
      return SPAI_OK;
    }
    set_error("spai_fill_residual: no compiled kernel for W=%d WA=%d a_dtype=%d m_dtype=%d mode=%d", W, WA, a_dtype,
              m_dtype, fill_mode);
    return SPAI_ERR_UNSUPPORTED;
  }
  const int32_t nparts = (nl + kNT - 1) / kNT;
  double* partials = static_cast<double*>(workspace);
  SPAI_CHECK_HIP(v->fn(line_begin, line_end, W, WA, pat_idx, pat_act, pat_val, a_idx, a_val, B, removed, words,
                       word_base, m_out, partials, nparts, s));
  k_fixed_reduce<1024><<<B, 1024, 0, s>>>(partials, nparts, res2_out, limbs_out, RewardArgs{});
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_rewards(const double* res2, const int32_t* removed_counts, int32_t B, int64_t nnz0, int32_t n,
                            double r0, double f0, const float* alpha, double* residual, double* reward, float* reward32,
                            void* stream) {
  SPAI_CHECK_ARG(res2 && removed_counts && alpha && residual && reward && B >= 1 && n >= 1 && nnz0 >= 0,
                 "spai_rewards: bad arguments");
  const RewardArgs ra{removed_counts, nnz0, n, r0, f0, alpha, residual, reward, reward32};
  k_rewards<<<1, 256, 0, (hipStream_t)stream>>>(res2, B, ra);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
