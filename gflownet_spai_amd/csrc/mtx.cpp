// Matrix Market ingest for the host.  Replaces
//   gflownet/utils.py:54-63  market_matrix_to_sparse_tensor: scipy.io.mmread(path).tocoo()
//   GFlowNet100.py:44-46     load_mtx_file: csr_matrix(mmread(path))
// with a multi-threaded parser over a memory map.  The COO it returns is the one mmread
// returns, entry for entry: the file's entries in file order, then (symmetric and
// skew-symmetric files) the mirror (j, i) of every off-diagonal entry, again in file order,
// negated for skew-symmetric.  That order is what makes the action ids of a drop-in env
// (position in initial_matrix._indices(), preconditioner.py:23-25) match the reference's.
// Values: real -> correctly rounded double (std::from_chars), integer -> exact, pattern -> 1.
//
// Passes, each split over T threads at line boundaries of the body:
//   1. count entry lines per chunk (memchr over '\n') -> chunk offsets (prefix sum, in order)
//   2. parse every chunk into its slice of (row, col, val)
//   3. count off-diagonal entries per chunk -> mirror offsets; write the mirrors
// Host code only (no GPU): the data reaches the device as the caller's tensors.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <charconv>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/spai_hip.h"

namespace spai {
void set_error(const char* fmt, ...);  // capi.hip

namespace {

struct MappedFile {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  ~MappedFile() {
    if (p && n) munmap(const_cast<char*>(p), n);
    if (fd >= 0) close(fd);
  }
  bool open_ro(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      n = 0;
      return false;
    }
    madvise(m, n, MADV_SEQUENTIAL);
    p = static_cast<const char*>(m);
    return true;
  }
};

struct Header {
  int64_t rows = 0, cols = 0, entries = 0;
  int32_t field = 0, symmetry = 0;
  size_t body = 0;  // offset of the first entry line
};

std::string lower(std::string s) {
  for (char& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

const char* skip_ws(const char* s, const char* e) {
  while (s < e && (*s == ' ' || *s == '\t' || *s == '\r')) ++s;
  return s;
}

// whitespace, then an optional '+' (std::from_chars takes only '-')
const char* skip_ws_plus(const char* s, const char* e) {
  s = skip_ws(s, e);
  return (s < e && *s == '+') ? s + 1 : s;
}

bool blank_or_comment(const char* s, const char* e) {
  s = skip_ws(s, e);
  return s == e || *s == '\n' || *s == '%';
}

int parse_header(const MappedFile& f, Header& h) {
  const char* p = f.p;
  const char* end = f.p + f.n;
  const char* nl = p ? static_cast<const char*>(memchr(p, '\n', f.n)) : nullptr;
  if (!nl) {
    set_error("mtx: no header line");
    return SPAI_ERR_INVALID;
  }
  std::vector<std::string> tok;
  {
    std::string line(p, nl);
    size_t i = 0;
    while (i < line.size()) {
      while (i < line.size() && std::isspace((unsigned char)line[i])) ++i;
      size_t j = i;
      while (j < line.size() && !std::isspace((unsigned char)line[j])) ++j;
      if (j > i) tok.push_back(lower(line.substr(i, j - i)));
      i = j;
    }
  }
  if (tok.size() != 5 || tok[0] != "%%matrixmarket" || tok[1] != "matrix") {
    set_error("mtx: not a Matrix Market matrix header");
    return SPAI_ERR_INVALID;
  }
  if (tok[2] != "coordinate") {
    set_error("mtx: format '%s' unsupported (market_matrix_to_sparse_tensor needs coordinate: mmread(...).tocoo())",
              tok[2].c_str());
    return SPAI_ERR_UNSUPPORTED;
  }
  if (tok[3] == "real" || tok[3] == "double")
    h.field = SPAI_MTX_REAL;
  else if (tok[3] == "integer")
    h.field = SPAI_MTX_INTEGER;
  else if (tok[3] == "pattern")
    h.field = SPAI_MTX_PATTERN;
  else {
    set_error("mtx: field '%s' unsupported (the reference converts values to float64)", tok[3].c_str());
    return SPAI_ERR_UNSUPPORTED;
  }
  if (tok[4] == "general")
    h.symmetry = SPAI_MTX_GENERAL;
  else if (tok[4] == "symmetric")
    h.symmetry = SPAI_MTX_SYMMETRIC;
  else if (tok[4] == "skew-symmetric")
    h.symmetry = SPAI_MTX_SKEW;
  else {
    set_error("mtx: symmetry '%s' unsupported", tok[4].c_str());
    return SPAI_ERR_UNSUPPORTED;
  }
  // comments, then the size line
  p = nl + 1;
  while (p < end) {
    const char* e = static_cast<const char*>(memchr(p, '\n', end - p));
    if (!e) e = end;
    if (!blank_or_comment(p, e)) {
      int64_t v[3];
      const char* s = p;
      for (int k = 0; k < 3; ++k) {
        s = skip_ws(s, e);
        auto r = std::from_chars(s, e, v[k]);
        if (r.ec != std::errc()) {
          set_error("mtx: bad size line");
          return SPAI_ERR_INVALID;
        }
        s = r.ptr;
      }
      if (v[0] < 0 || v[1] < 0 || v[2] < 0) {
        set_error("mtx: negative size");
        return SPAI_ERR_INVALID;
      }
      h.rows = v[0], h.cols = v[1], h.entries = v[2];
      if (h.symmetry != SPAI_MTX_GENERAL && h.rows != h.cols) {
        set_error("mtx: %s matrix must be square", tok[4].c_str());
        return SPAI_ERR_INVALID;
      }
      h.body = (size_t)((e < end ? e + 1 : end) - f.p);
      return SPAI_OK;
    }
    p = e + 1;
  }
  set_error("mtx: missing size line");
  return SPAI_ERR_INVALID;
}

// chunk boundaries of [b, e): starts at line starts
std::vector<const char*> split_lines(const char* b, const char* e, int parts) {
  std::vector<const char*> cut(parts + 1, e);
  cut[0] = b;
  const size_t n = (size_t)(e - b);
  for (int k = 1; k < parts; ++k) {
    const char* s = std::max(cut[k - 1], b + n * k / parts);
    if (s > b && s < e && s[-1] != '\n') {
      const char* nl = static_cast<const char*>(memchr(s, '\n', e - s));
      s = nl ? nl + 1 : e;
    }
    cut[k] = s;
  }
  return cut;
}

int64_t count_entries(const char* s, const char* e) {
  int64_t c = 0;
  while (s < e) {
    const char* nl = static_cast<const char*>(memchr(s, '\n', e - s));
    const char* le = nl ? nl : e;
    if (!blank_or_comment(s, le)) ++c;
    s = le + 1;
  }
  return c;
}

// parse the entry lines of [s, e) into rows/cols/vals from index 0; returns a status
int parse_chunk(const char* s, const char* e, const Header& h, int64_t* row, int64_t* col, double* val,
                std::string& err) {
  int64_t k = 0;
  while (s < e) {
    const char* nl = static_cast<const char*>(memchr(s, '\n', e - s));
    const char* le = nl ? nl : e;
    if (!blank_or_comment(s, le)) {
      int64_t i, j;
      const char* q = skip_ws(s, le);
      auto r = std::from_chars(q, le, i);
      if (r.ec != std::errc()) return err = "bad row index", SPAI_ERR_INVALID;
      q = skip_ws(r.ptr, le);
      r = std::from_chars(q, le, j);
      if (r.ec != std::errc()) return err = "bad column index", SPAI_ERR_INVALID;
      if (i < 1 || i > h.rows || j < 1 || j > h.cols) return err = "index out of range", SPAI_ERR_INVALID;
      double v = 1.0;
      if (h.field != SPAI_MTX_PATTERN) {
        q = skip_ws_plus(r.ptr, le);
        if (h.field == SPAI_MTX_INTEGER) {
          int64_t iv;
          auto rv = std::from_chars(q, le, iv);
          if (rv.ec != std::errc()) return err = "bad integer value", SPAI_ERR_INVALID;
          v = (double)iv;
        } else {
          auto rv = std::from_chars(q, le, v);
          if (rv.ec != std::errc()) return err = "bad real value", SPAI_ERR_INVALID;
        }
      }
      row[k] = i - 1;
      col[k] = j - 1;
      val[k] = v;
      ++k;
    }
    s = le + 1;
  }
  return SPAI_OK;
}

template <typename F>
void run_parallel(int T, F&& f) {
  std::vector<std::thread> th;
  th.reserve(T);
  for (int t = 1; t < T; ++t) th.emplace_back(f, t);
  f(0);
  for (auto& x : th) x.join();
}

}  // namespace
}  // namespace spai

using namespace spai;

#define SPAI_CHECK_ARG(cond, ...)   \
  do {                              \
    if (!(cond)) {                  \
      ::spai::set_error(__VA_ARGS__); \
      return SPAI_ERR_INVALID;      \
    }                               \
  } while (0)

extern "C" int spai_mtx_header(const char* path, int64_t* dims, int32_t* kinds) {
  SPAI_CHECK_ARG(path && dims && kinds, "spai_mtx_header: null pointer");
  MappedFile f;
  if (!f.open_ro(path)) {
    set_error("mtx: cannot open '%s'", path);
    return SPAI_ERR_INVALID;
  }
  Header h;
  const int st = parse_header(f, h);
  if (st != SPAI_OK) return st;
  dims[0] = h.rows;
  dims[1] = h.cols;
  dims[2] = h.entries;
  dims[3] = h.symmetry == SPAI_MTX_GENERAL ? h.entries : 2 * h.entries;  // capacity the read needs
  kinds[0] = h.field;
  kinds[1] = h.symmetry;
  return SPAI_OK;
}

extern "C" int spai_mtx_read(const char* path, int64_t* row, int64_t* col, double* val, int64_t capacity,
                             int32_t threads, int64_t* nnz_out) {
  SPAI_CHECK_ARG(path && nnz_out, "spai_mtx_read: null pointer");
  MappedFile f;
  if (!f.open_ro(path)) {
    set_error("mtx: cannot open '%s'", path);
    return SPAI_ERR_INVALID;
  }
  Header h;
  int st = parse_header(f, h);
  if (st != SPAI_OK) return st;
  SPAI_CHECK_ARG(capacity >= h.entries && (h.entries == 0 || (row && col && val)),
                 "spai_mtx_read: capacity %lld < %lld entries", (long long)capacity, (long long)h.entries);
  const char* b = f.p + h.body;
  const char* e = f.p + f.n;
  const int T = std::max(1, std::min<int>(threads > 0 ? threads : (int)std::thread::hardware_concurrency(),
                                          (int)std::max<size_t>(1, (size_t)(e - b) / (1 << 20))));
  auto cut = split_lines(b, e, T);
  std::vector<int64_t> cnt(T + 1, 0);
  run_parallel(T, [&](int t) { cnt[t + 1] = count_entries(cut[t], cut[t + 1]); });
  for (int t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
  if (cnt[T] != h.entries) {
    set_error("mtx: %lld entry lines, header says %lld", (long long)cnt[T], (long long)h.entries);
    return SPAI_ERR_INVALID;
  }
  std::vector<int> sts(T, SPAI_OK);
  std::vector<std::string> errs(T);
  run_parallel(T, [&](int t) {
    sts[t] = parse_chunk(cut[t], cut[t + 1], h, row + cnt[t], col + cnt[t], val + cnt[t], errs[t]);
  });
  for (int t = 0; t < T; ++t)
    if (sts[t] != SPAI_OK) {
      set_error("mtx: %s", errs[t].c_str());
      return sts[t];
    }
  int64_t nnz = h.entries;
  if (h.symmetry != SPAI_MTX_GENERAL) {
    // mirrors of the off-diagonal entries, in file order, after all file entries
    std::vector<int64_t> off(T + 1, 0);
    run_parallel(T, [&](int t) {
      int64_t c = 0;
      for (int64_t k = cnt[t]; k < cnt[t + 1]; ++k) c += row[k] != col[k];
      off[t + 1] = c;
    });
    for (int t = 0; t < T; ++t) off[t + 1] += off[t];
    nnz += off[T];
    SPAI_CHECK_ARG(capacity >= nnz, "spai_mtx_read: capacity %lld < %lld entries after mirroring",
                   (long long)capacity, (long long)nnz);
    const double sgn = h.symmetry == SPAI_MTX_SKEW ? -1.0 : 1.0;
    run_parallel(T, [&](int t) {
      int64_t o = h.entries + off[t];
      for (int64_t k = cnt[t]; k < cnt[t + 1]; ++k)
        if (row[k] != col[k]) {
          row[o] = col[k];
          col[o] = row[k];
          val[o] = sgn * val[k];
          ++o;
        }
    });
  }
  *nnz_out = nnz;
  return SPAI_OK;
}
