// Accuracy of gfx950's v_rsq_f64 / v_rcp_f64 (the QR fill's reflections use them):
// max and mean relative error against IEEE 1/sqrt and 1/x (correctly rounded sqrt / division)
// over 2^22 log-uniform inputs, with and without one Newton step.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k_probe(int n, const double* x, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = x[i];
  const double r = __builtin_amdgcn_rsq(t);
  const double e = fma(-t * r, r, 1.0);
  const double rn = fma(0.5 * r, e, r);
  const double c = __builtin_amdgcn_rcp(t);
  const double cn = fma(c, fma(-t, c, 1.0), c);
  const double ref_r = 1.0 / sqrt(t), ref_c = 1.0 / t;
  out[4 * i + 0] = fabs(r - ref_r) / ref_r;
  out[4 * i + 1] = fabs(rn - ref_r) / ref_r;
  out[4 * i + 2] = fabs(c - ref_c) / ref_c;
  out[4 * i + 3] = fabs(cn - ref_c) / ref_c;
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    x[i] = std::exp2(-40.0 + 80.0 * (double)(s >> 11) / 9007199254740992.0);
  }
  double *dx, *dout;
  hipMalloc(&dx, n * 8); hipMalloc(&dout, n * 32);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k_probe<<<n / 256, 256>>>(n, dx, dout);
  std::vector<double> o(4 * (size_t)n);
  hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
  const char* nm[4] = {"v_rsq_f64", "v_rsq_f64+newton", "v_rcp_f64", "v_rcp_f64+newton"};
  printf("{");
  for (int k = 0; k < 4; ++k) {
    double mx = 0, mean = 0;
    for (int i = 0; i < n; ++i) { mx = std::fmax(mx, o[4 * i + k]); mean += o[4 * i + k]; }
    printf("%s\"%s\": {\"max_rel\": %.3e, \"mean_rel\": %.3e, \"max_ulp\": %.2f}", k ? ", " : "", nm[k], mx, mean / n,
           mx / 1.1102230246251565e-16);
  }
  printf(", \"n\": %d}\n", n);
  return 0;
}
