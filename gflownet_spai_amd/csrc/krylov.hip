// Krylov evaluation of a preconditioner on gfx950 (reference:
// GFlowNet100.py:61-93 solve_with_gmres = scipy.sparse.linalg.gmres(A, b, x0=0, M=M, ...)).
// GMRES itself is host-orchestrated (gflownet_spai_amd/gmres.py restates scipy's algorithm
// step for step); its two products per inner iteration, A v and M (A v), run here.
//
//   k_ell_spmv  y = A x over row-ELL lines (the env's Lines layout, -1 padded): one thread per
//               row, fp64 products and sum in slot order (deterministic), fp32 or fp64 values.
//               HBM-bound: per row W (4 + s) bytes of lines + 8 of y, x gathered through L2.
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kSpmvNT = 256;

template <typename VT, int W>
__global__ __launch_bounds__(kSpmvNT) void k_ell_spmv(int32_t n, const int32_t* __restrict__ idx,
                                                      const VT* __restrict__ val, const double* __restrict__ x,
                                                      double* __restrict__ y) {
  const int i = blockIdx.x * kSpmvNT + threadIdx.x;
  if (i >= n) return;
  const int32_t* ri = idx + (int64_t)i * W;
  const VT* rv = val + (int64_t)i * W;
  int32_t c[W];
  VT v[W];
#pragma unroll
  for (int s = 0; s < W; ++s) c[s] = ri[s], v[s] = rv[s];
  double acc = 0.0;
#pragma unroll
  for (int s = 0; s < W; ++s)
    if (c[s] >= 0) acc = fma((double)v[s], x[c[s]], acc);
  y[i] = acc;
}

template <typename VT>
__global__ __launch_bounds__(kSpmvNT) void k_ell_spmv_any(int32_t n, int32_t W, const int32_t* __restrict__ idx,
                                                          const VT* __restrict__ val, const double* __restrict__ x,
                                                          double* __restrict__ y) {
  const int i = blockIdx.x * kSpmvNT + threadIdx.x;
  if (i >= n) return;
  double acc = 0.0;
  for (int s = 0; s < W; ++s) {
    const int32_t c = idx[(int64_t)i * W + s];
    if (c >= 0) acc = fma((double)val[(int64_t)i * W + s], x[c], acc);
  }
  y[i] = acc;
}

template <typename VT>
void launch_spmv(int32_t n, int32_t W, const int32_t* idx, const VT* val, const double* x, double* y, hipStream_t s) {
  const int g = (n + kSpmvNT - 1) / kSpmvNT;
  switch (W) {
#define SPAI_W(w) \
  case w: k_ell_spmv<VT, w><<<g, kSpmvNT, 0, s>>>(n, idx, val, x, y); break;
    SPAI_W(1) SPAI_W(2) SPAI_W(3) SPAI_W(4) SPAI_W(5) SPAI_W(6) SPAI_W(7) SPAI_W(8) SPAI_W(9) SPAI_W(13)
#undef SPAI_W
    default: k_ell_spmv_any<VT><<<g, kSpmvNT, 0, s>>>(n, W, idx, val, x, y);
  }
}

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" int spai_ell_spmv(int32_t n, int32_t W, const int32_t* idx, const void* val, int32_t val_dtype,
                             const double* x, double* y, void* stream) {
  SPAI_CHECK_ARG(n >= 0 && W >= 1, "spai_ell_spmv: bad shape n=%d W=%d", n, W);
  if (n == 0) return SPAI_OK;
  SPAI_CHECK_ARG(idx && val && x && y, "spai_ell_spmv: null pointer");
  SPAI_CHECK_ARG(val_dtype == SPAI_DTYPE_F32 || val_dtype == SPAI_DTYPE_F64, "spai_ell_spmv: bad dtype %d", val_dtype);
  hipStream_t s = (hipStream_t)stream;
  if (val_dtype == SPAI_DTYPE_F32)
    launch_spmv(n, W, idx, static_cast<const float*>(val), x, y, s);
  else
    launch_spmv(n, W, idx, static_cast<const double*>(val), x, y, s);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
