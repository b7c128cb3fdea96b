// Batched ||M_b A - I||_F^2 / ||A M_b - I||_F^2 of B ARBITRARY sparse M_b (gfx950) — the
// generic SpMM residual of PreconditionerEnv.calculate_residual (preconditioner.py:79-93),
// for any M, not only the masked copies / least-squares fills of one candidate pattern.
//
// Every matrix is a set of LINES (rows for M A, columns for A M) in ELL form, W slots per
// line of M (index k_p, value m_p; k_p < 0 = empty slot), WA per line of A.  One line l of
// M contributes
//     || sum_p m_p A_line(k_p) - e_l ||^2 = 1 - 2 sum_p m_p A_line(k_p)[l]
//                                         + sum_{p,q} m_p m_q <A_line(k_p), A_line(k_q)>
// (sparse dot products by index matching over the WA x WA entry pairs; fp64 accumulation of
// the products, as k_line).  One thread per (line, sample): it reads the W slots of its line
// of M_b and gathers the W lines of A they name.  A block covers 256 consecutive lines of one
// sample; the B blocks of one line range are consecutive blocks of ONE XCD (bijective XCD
// remap), so the A lines they gather (the same neighbourhood for every sample) are fetched
// from HBM once and served to the other samples by that XCD's L2.  Per-block partial sums,
// then a fixed-order reduction per sample: the result is bit-reproducible.
//
// Algorithmic bytes per sample: bytes(A) + bytes(M_b).
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kNT = 256;
constexpr int kXcd = 8;

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int x = orig % kXcd, q = nwg / kXcd, r = nwg % kXcd;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / kXcd;
}

template <int W, int WA, typename TA, typename TV>
__global__ __launch_bounds__(kNT) void k_resid(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                               int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                               int64_t idx_bstride, const TV* __restrict__ m_val,
                                               int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                               const TA* __restrict__ a_val, double* __restrict__ partials) {
  __shared__ double sred[kNT / 64];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % B, blk = wg / B;
  const int j = line_begin + blk * kNT + threadIdx.x;
  const bool valid = j < line_end;
  const int jj = valid ? j : line_begin;
  const int32_t* mi = m_idx + (int64_t)b * idx_bstride + (int64_t)jj * wrt;
  const TV* mv = m_val + (int64_t)b * val_bstride + (int64_t)jj * wrt;
  int k[W];
  double v[W];
#pragma unroll
  for (int p = 0; p < W; ++p) {
    k[p] = (valid && p < wrt) ? mi[p] : -1;
    v[p] = k[p] >= 0 ? (double)mv[p] : 0.0;  // empty slots contribute nothing (their value is not read)
  }
  int ai[W][WA];
  TA av[W][WA];
#pragma unroll
  for (int p = 0; p < W; ++p) {
#pragma unroll
    for (int s = 0; s < WA; ++s) {
      ai[p][s] = -1;
      av[p][s] = (TA)0;
      if (k[p] >= 0 && s < wart) {
        const int64_t o = (int64_t)k[p] * wart + s;
        ai[p][s] = a_idx[o];
        av[p][s] = a_val[o];
      }
    }
  }
  double r2 = 0.0;
  if (valid) {
    r2 = 1.0;
#pragma unroll
    for (int p = 0; p < W; ++p) {
      double cp = 0.0, gpp = 0.0;
#pragma unroll
      for (int s = 0; s < WA; ++s) {
        const double x = (double)av[p][s];
        gpp += x * x;  // padding entries carry 0
        cp += (ai[p][s] == j) ? x : 0.0;
      }
      double acc = v[p] * gpp - 2.0 * cp;
#pragma unroll
      for (int q = p + 1; q < W; ++q) {
        double g = 0.0;
#pragma unroll
        for (int s = 0; s < WA; ++s) {
#pragma unroll
          for (int t = 0; t < WA; ++t)
            g += (ai[p][s] >= 0 && ai[p][s] == ai[q][t]) ? (double)av[p][s] * (double)av[q][t] : 0.0;
        }
        acc += 2.0 * v[q] * g;
      }
      r2 += v[p] * acc;
    }
  }
  r2 = block_sum<kNT>(r2, sred);
  if (threadIdx.x == 0) partials[(int64_t)b * nblk + blk] = r2;
}

// Sort-based line residual: the W x WA products m_p * A_line(k_p)[s] of one line of M_b sit
// one per lane (IPL per lane) in a SEG-lane segment of a wave (64 / SEG lines per wave); a
// bitonic network over the segment orders them by (index, item) — unique keys, so the order
// and every sum below are deterministic — then a segmented inclusive scan gives each index's
// total T at the last product of its run, and
//     ||r - e_l||^2 = sum_runs T^2 - 2 T_l + 1
// (T_l = the total at index l, 0 when absent).  ~100 VALU per line where the pairwise index
// matching of k_resid needs W^2 WA^2 / 2 compare-and-adds.
template <int W, int WA, int SEG, int IPL, typename TA, typename TV>
__global__ __launch_bounds__(kNT) void k_resid_sort(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                    int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                    int64_t idx_bstride, const TV* __restrict__ m_val,
                                                    int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                    const TA* __restrict__ a_val, double* __restrict__ partials) {
  static_assert(W * WA <= SEG * IPL && (SEG == 32 || SEG == 64) && (IPL == 1 || IPL == 2), "segment shape");
  constexpr int N = SEG * IPL;         // items per line (power of two)
  constexpr int LPW = 64 / SEG;        // lines per wave and round
  constexpr int LPR = kNT / 64 * LPW;  // lines per block and round; a block covers kNT lines
  __shared__ double sred[kNT / 64];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wg % B, blk = wg / B;
  const int lane = threadIdx.x & 63, ls = lane & (SEG - 1), seg0 = lane & ~(SEG - 1);
  const int32_t* mib = m_idx + (int64_t)b * idx_bstride;
  const TV* mvb = m_val + (int64_t)b * val_bstride;
  double contrib = 0.0;
#pragma unroll 1
  for (int rd = 0; rd < kNT / LPR; ++rd) {
    const int j = line_begin + blk * kNT + rd * LPR + (threadIdx.x >> 6) * LPW + lane / SEG;
    const bool valid = j < line_end;
    const int jj = valid ? j : line_begin;
    uint32_t key[IPL];
    double val[IPL];
#pragma unroll
    for (int r = 0; r < IPL; ++r) {
      const int item = r * SEG + ls;  // product (p, s) = (item / WA, item % WA)
      const int p = item / WA, s = item - p * WA;
      key[r] = 0xFFFFFF80u | (uint32_t)item;  // empty: sorts after every index
      val[r] = 0.0;
      if (valid && item < W * WA && p < wrt && s < wart) {
        const int k = mib[(int64_t)jj * wrt + p];
        if (k >= 0) {
          const int64_t o = (int64_t)k * wart + s;
          const int ai = a_idx[o];
          if (ai >= 0) {
            key[r] = ((uint32_t)ai << 7) | (uint32_t)item;
            val[r] = (double)mvb[(int64_t)jj * wrt + p] * (double)a_val[o];
          }
        }
      }
    }
    // bitonic sort of the segment's N items (item i = r * SEG + ls), ascending keys
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
      for (int jx = k >> 1; jx >= 1; jx >>= 1) {
        if (jx >= SEG) {  // k == N == 2 SEG: the partner is the other register of this lane
          if (key[0] > key[IPL - 1]) {
            const uint32_t tk = key[0];
            key[0] = key[IPL - 1];
            key[IPL - 1] = tk;
            const double tv = val[0];
            val[0] = val[IPL - 1];
            val[IPL - 1] = tv;
          }
        } else {
#pragma unroll
          for (int r = 0; r < IPL; ++r) {
            const int i = r * SEG + ls;
            const uint32_t ok = (uint32_t)__shfl_xor((int)key[r], jx, 64);
            const double ov = __shfl_xor(val[r], jx, 64);
            const bool up = (i & k) == 0, lower = (i & jx) == 0;
            if ((lower == up) ? ok < key[r] : ok > key[r]) {
              key[r] = ok;
              val[r] = ov;
            }
          }
        }
      }
    }
    // segmented inclusive scan over equal indices, register by register; the run that crosses
    // from register 0 into register 1 (a prefix of register 1) gets register 0's carry
    double S[IPL];
    uint32_t ix[IPL];
#pragma unroll
    for (int r = 0; r < IPL; ++r) {
      ix[r] = key[r] >> 7;
      double v = val[r];
#pragma unroll
      for (int o = 1; o < SEG; o <<= 1) {
        const double y = __shfl_up(v, o, 64);
        const uint32_t ky = (uint32_t)__shfl_up((int)ix[r], o, 64);
        if (ls >= o && ky == ix[r]) v += y;
      }
      S[r] = v;
    }
    if constexpr (IPL == 2) {
      const double c0 = __shfl(S[0], seg0 + SEG - 1, 64);
      const uint32_t k0 = (uint32_t)__shfl((int)ix[0], seg0 + SEG - 1, 64);
      if (ix[1] == k0) S[1] += c0;
    }
    const uint32_t r1first = (uint32_t)__shfl((int)ix[IPL - 1], seg0, 64);
#pragma unroll
    for (int r = 0; r < IPL; ++r) {
      // last of its run: the next item (lane + 1, or register r + 1 at lane 0) has another index
      const uint32_t dn = (uint32_t)__shfl_down((int)ix[r], 1, 64);
      const uint32_t nk = ls < SEG - 1 ? dn : (r + 1 < IPL ? r1first : 0xFFFFFFFFu);
      if (valid && nk != ix[r] && ix[r] != 0x1FFFFFFu) contrib += S[r] * (ix[r] == (uint32_t)j ? S[r] - 2.0 : S[r]);
    }
    if (valid && ls == 0) contrib += 1.0;  // ||e_l||^2, once per line
  }
  const double r2 = block_sum<kNT>(contrib, sred);
  if (threadIdx.x == 0) partials[(int64_t)b * nblk + blk] = r2;
}

__global__ __launch_bounds__(kNT) void k_resid_reduce(const double* __restrict__ partials, int32_t nblk,
                                                      double* __restrict__ out) {
  __shared__ double sred[kNT / 64];
  const int b = blockIdx.x;
  double s = 0.0;
  for (int i = threadIdx.x; i < nblk; i += kNT) s += partials[(int64_t)b * nblk + i];
  s = block_sum<kNT>(s, sred);
  if (threadIdx.x == 0) out[b] = s;
}

using ResidFn = void (*)(int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, const int32_t*, int64_t,
                         const void*, int64_t, const int32_t*, const void*, double*, hipStream_t);

template <int W, int WA, typename TA, typename TV>
void launch_resid(int32_t lb, int32_t le, int32_t wrt, int32_t wart, int32_t B, int32_t nblk, const int32_t* mi,
                  int64_t ib, const void* mv, int64_t vb, const int32_t* ai, const void* av, double* partials,
                  hipStream_t s) {
#ifdef RESID_PAIRWISE  // the pairwise index-matching kernel (A/B builds)
  k_resid<W, WA, TA, TV><<<nblk * B, kNT, 0, s>>>(lb, le, wrt, wart, B, nblk, mi, ib, static_cast<const TV*>(mv), vb,
                                                   ai, static_cast<const TA*>(av), partials);
#else
  constexpr int SEG = W * WA <= 32 ? 32 : 64, IPL = W * WA <= 64 ? 1 : 2;
  k_resid_sort<W, WA, SEG, IPL, TA, TV><<<nblk * B, kNT, 0, s>>>(lb, le, wrt, wart, B, nblk, mi, ib,
                                                                  static_cast<const TV*>(mv), vb, ai,
                                                                  static_cast<const TA*>(av), partials);
#endif
}

struct ResidVariant {
  int W, WA, a_dtype, m_dtype;
  ResidFn fn;
};

static const ResidVariant kResid[] = {
    {5, 5, SPAI_DTYPE_F32, SPAI_DTYPE_F32, launch_resid<5, 5, float, float>},
    {7, 7, SPAI_DTYPE_F32, SPAI_DTYPE_F32, launch_resid<7, 7, float, float>},
    {5, 5, SPAI_DTYPE_F64, SPAI_DTYPE_F64, launch_resid<5, 5, double, double>},
    {7, 7, SPAI_DTYPE_F64, SPAI_DTYPE_F64, launch_resid<7, 7, double, double>},
    {13, 7, SPAI_DTYPE_F64, SPAI_DTYPE_F64, launch_resid<13, 7, double, double>},
    {5, 5, SPAI_DTYPE_F64, SPAI_DTYPE_F32, launch_resid<5, 5, double, float>},
    {7, 7, SPAI_DTYPE_F64, SPAI_DTYPE_F32, launch_resid<7, 7, double, float>},
    {13, 7, SPAI_DTYPE_F64, SPAI_DTYPE_F32, launch_resid<13, 7, double, float>},
    {13, 7, SPAI_DTYPE_F32, SPAI_DTYPE_F32, launch_resid<13, 7, float, float>},
    {5, 5, SPAI_DTYPE_F32, SPAI_DTYPE_F64, launch_resid<5, 5, float, double>},
    {7, 7, SPAI_DTYPE_F32, SPAI_DTYPE_F64, launch_resid<7, 7, float, double>},
    {13, 7, SPAI_DTYPE_F32, SPAI_DTYPE_F64, launch_resid<13, 7, float, double>},
};

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" size_t spai_residual_workspace_bytes(int32_t n_lines, int32_t B) {
  if (n_lines < 0 || B < 1) return 0;
  Carve c(nullptr);
  c.take<double>((size_t)std::max(1, (n_lines + kNT - 1) / kNT) * B);
  return c.off;
}

extern "C" int spai_residual_lines(int32_t n, int32_t line_begin, int32_t line_end, int32_t W, const int32_t* m_idx,
                                   int64_t idx_bstride, const void* m_val, int32_t m_dtype, int64_t val_bstride,
                                   int32_t WA, const int32_t* a_idx, const void* a_val, int32_t a_dtype, int32_t B,
                                   double* res2_out, void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(n >= 1 && line_begin >= 0 && line_end >= line_begin && line_end <= n && W >= 1 && WA >= 1 &&
                     B >= 1 && idx_bstride >= 0 && val_bstride >= 0,
                 "spai_residual_lines: bad shape");
  SPAI_CHECK_ARG(m_idx && m_val && a_idx && a_val && res2_out && workspace, "spai_residual_lines: null pointer");
  SPAI_CHECK_ARG(a_dtype == SPAI_DTYPE_F32 || a_dtype == SPAI_DTYPE_F64, "spai_residual_lines: bad a_dtype");
  SPAI_CHECK_ARG(m_dtype == SPAI_DTYPE_F32 || m_dtype == SPAI_DTYPE_F64, "spai_residual_lines: bad m_dtype");
  const int32_t nl = line_end - line_begin;
  hipStream_t s = (hipStream_t)stream;
  if (nl == 0) {
    SPAI_CHECK_HIP(hipMemsetAsync(res2_out, 0, sizeof(double) * B, s));
    return SPAI_OK;
  }
  SPAI_CHECK_ARG(workspace_bytes >= spai_residual_workspace_bytes(nl, B), "spai_residual_lines: workspace too small");
  SPAI_CHECK_ARG(n < (1 << 25) - 1, "spai_residual_lines: n=%d above the 2^25 - 1 lines the index keys hold", n);
  SPAI_CHECK_ARG((int64_t)((nl + kNT - 1) / kNT) * B < ((int64_t)1 << 31), "spai_residual_lines: grid too large");
  const ResidVariant* v = nullptr;
  for (const auto& c : kResid)
    if (W <= c.W && WA <= c.WA && a_dtype == c.a_dtype && m_dtype == c.m_dtype) {
      v = &c;
      break;
    }
  if (v == nullptr) {
    set_error("spai_residual_lines: no kernel for W=%d WA=%d (a_dtype %d, m_dtype %d): widths 5/7/13 x 5/7", W, WA,
              a_dtype, m_dtype);
    return SPAI_ERR_UNSUPPORTED;
  }
  const int32_t nblk = (nl + kNT - 1) / kNT;
  double* partials = static_cast<double*>(workspace);
  v->fn(line_begin, line_end, W, WA, B, nblk, m_idx, idx_bstride, m_val, val_bstride, a_idx, a_val, partials, s);
  SPAI_CHECK_LAUNCH();
  k_resid_reduce<<<B, kNT, 0, s>>>(partials, nblk, res2_out);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
