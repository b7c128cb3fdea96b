// Host-only harness for the sanitizer builds of the multi-threaded Matrix Market reader
// (gflownet_spai_amd/csrc/mtx.cpp, built here with g++ -fsanitize=address,undefined or
// -fsanitize=thread; no HIP).  Reads one file with the given thread count and prints
// "rows cols nnz checksum" (checksum: fixed-order sum over entries of row * 31 + col * 7 + val)
// for tests/test_ingest_sanitize.py to compare with scipy.io.mmread.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/spai_hip.h"

namespace spai {
static thread_local std::string g_err;
void set_error(const char* fmt, ...) {  // the library's capi.hip definition, restated host-only
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}
}  // namespace spai

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s file.mtx threads\n", argv[0]);
    return 2;
  }
  int64_t dims[4];
  int32_t kinds[4];
  if (spai_mtx_header(argv[1], dims, kinds) != 0) {
    printf("error %s\n", spai::g_err.c_str());
    return 0;
  }
  const int64_t cap = dims[3];
  std::vector<int64_t> r(cap > 0 ? cap : 1), c(cap > 0 ? cap : 1);
  std::vector<double> v(cap > 0 ? cap : 1);
  int64_t nnz = 0;
  if (spai_mtx_read(argv[1], r.data(), c.data(), v.data(), cap, atoi(argv[2]), &nnz) != 0) {
    printf("error %s\n", spai::g_err.c_str());
    return 0;
  }
  double cs = 0.0;
  for (int64_t i = 0; i < nnz; ++i) cs += (double)r[i] * 31.0 + (double)c[i] * 7.0 + v[i];
  printf("%lld %lld %lld %.17g\n", (long long)dims[0], (long long)dims[1], (long long)nnz, cs);
  return 0;
}
