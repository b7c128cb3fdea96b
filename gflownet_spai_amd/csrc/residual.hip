// Batched ||M_b A - I||_F^2 / ||A M_b - I||_F^2 of B ARBITRARY sparse M_b (gfx950) — the
// generic SpMM residual of PreconditionerEnv.calculate_residual (preconditioner.py:79-93),
// for any M, not only the masked copies / least-squares fills of one candidate pattern.
//
// Every matrix is a set of LINES (rows for M A, columns for A M) in ELL form, W slots per
// line of M (index k_p, value m_p; k_p < 0 = empty slot), WA per line of A.  One line l of
// M contributes
//     || sum_p m_p A_line(k_p) - e_l ||^2 = 1 - 2 sum_p m_p A_line(k_p)[l]
//                                         + sum_{p,q} m_p m_q <A_line(k_p), A_line(k_q)>
// (sparse dot products by index matching over the WA x WA entry pairs, one compare and one
// select each; fp64 accumulation of the products, as k_line).  One thread per (line, sample): it reads the W slots of its line
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
        // an index occurs at most once per line: entry s of line p meets at most one entry of
        // line q, so a select chain in A's own precision (one compare + one select per entry
        // pair) finds its partner's value; padding entries (index -1, value 0) add nothing
        double g = 0.0;
#pragma unroll
        for (int s = 0; s < WA; ++s) {
          TA m = (TA)0;
#pragma unroll
          for (int t = 0; t < WA; ++t) m = ai[p][s] == ai[q][t] ? av[q][t] : m;
          g += (double)av[p][s] * (double)m;
        }
        acc += 2.0 * v[q] * g;
      }
      r2 += v[p] * acc;
    }
  }
  r2 = block_sum<kNT>(r2, sred);
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
  k_resid<W, WA, TA, TV><<<nblk * B, kNT, 0, s>>>(lb, le, wrt, wart, B, nblk, mi, ib, static_cast<const TV*>(mv), vb,
                                                   ai, static_cast<const TA*>(av), partials);
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
