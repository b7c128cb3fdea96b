// Error plumbing for the C ABI: every extern "C" entry point returns a status code and
// records a thread-local message; nothing throws across the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/spai_hip.h"

namespace spai {

void set_error(const char* fmt, ...);

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// Bump allocator over the caller's workspace.
struct Carve {
  char* base;
  size_t off = 0;
  explicit Carve(void* p) : base(static_cast<char*>(p)) {}
  template <typename T>
  T* take(size_t n) {
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off = align_up(off + n * sizeof(T));
    return p;
  }
};

}  // namespace spai

#define SPAI_CHECK_ARG(cond, ...)          \
  do {                                     \
    if (!(cond)) {                         \
      ::spai::set_error(__VA_ARGS__);      \
      return SPAI_ERR_INVALID;             \
    }                                      \
  } while (0)

#define SPAI_CHECK_HIP(expr)                                                             \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      ::spai::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                       \
      return SPAI_ERR_HIP;                                                               \
    }                                                                                    \
  } while (0)

#define SPAI_CHECK_LAUNCH() SPAI_CHECK_HIP(hipGetLastError())
