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
// select each; fp64 accumulation of the products, as k_line).
//
// W <= 7 (k_resid_shared): one thread per line for ALL B samples.  The Gram of the line's
// slots (the index matching: all of the arithmetic) is formed once per chunk of 8 samples on
// the union of their index sets when they agree slot by slot (sub-patterns of one pattern, the
// GFlowNet candidates), then each sample is a W x W quadratic form; lanes whose samples
// disagree evaluate each sample on its own index set.  A is read once per line for the batch:
// algorithmic bytes per launch = bytes(A) + sum_b bytes(M_b) (SURVEY §8d with A shared by the
// batch).  Consecutive line ranges run on one XCD (bijective XCD remap), so the A halo of
// neighbouring blocks is served by that XCD's L2.
// W = 13, A values exact in fp32 (k_resid_wide): one thread per line for chunks of 8 samples;
// the line's index matching runs once per chunk and each pair's product
// <A_line(k_p), A_line(k_q)> goes straight into the chunk's quadratic forms (the 91-value Gram
// is never held).  W = 13 with fp64 A values (k_resid_row16): sixteen lanes per line, one slot
// each, the pairs matched across lanes by DPP row rotations (C3: round 2's thread per (line,
// sample) 1.76 ms -> chunks of 4 0.54 -> 0.21 ms; fp64 A 0.26 ms).
// Per-block partial sums, then a fixed-order reduction per sample: the result is
// bit-reproducible, and both kernels evaluate a line with the same operations in the same order.
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

// The n slots of one ELL line, p[0 .. n), n = W at compile time when `full` (the stored width
// equals the template width): 16-byte vector loads (4-byte alignment suffices for vector
// memory instructions on gfx950) + a scalar tail — fewer, wider memory instructions for the
// texture address/data units, which bound this kernel (TA/TD busy ~80 % with dword loads).
// Otherwise clamped scalar loads (slot min(q, n - 1)), masked by the caller.
template <int W, bool FULL, typename T>
__device__ __forceinline__ void load_slots(const T* __restrict__ p, int n, T (&out)[W]) {
  constexpr int kPer = 16 / sizeof(T);
  // the vector type carries the ELEMENT's alignment: a line starts at any multiple of
  // sizeof(T), and a type that claimed 16-byte alignment let the compiler widen the scalar tail
  // into a 16-byte load past the line (past the buffer's end on its last line: a fault when
  // the allocation ends at a page)
  typedef T vec_t __attribute__((ext_vector_type(kPer), aligned(sizeof(T))));
  if constexpr (FULL) {
#pragma unroll
    for (int q = 0; q + kPer <= W; q += kPer) {
      const vec_t v = *reinterpret_cast<const vec_t*>(p + q);
#pragma unroll
      for (int e = 0; e < kPer; ++e) out[q + e] = v[e];
    }
#pragma unroll
    for (int q = (W / kPer) * kPer; q < W; ++q) out[q] = p[q];
  } else {
#pragma unroll
    for (int q = 0; q < W; ++q) out[q] = p[min(q, n - 1)];
  }
}

// The W lines of A named by k[0..W) (k < 0: empty, index -1 / value 0).  Every load is
// unconditional from a clamped address (line 0 / the line's last slot) and masked afterwards:
// no branch around a load, so all of them are in flight together.
template <int W, int WA, bool FULL, typename TA>
__device__ __forceinline__ void gather_a_lines(const int (&k)[W], int wart, const int32_t* __restrict__ a_idx,
                                               const TA* __restrict__ a_val, int (&ai)[W][WA], TA (&av)[W][WA]) {
#pragma unroll
  for (int p = 0; p < W; ++p) {
    const int64_t base = (int64_t)max(k[p], 0) * wart;
    int ii[WA];
    TA xx[WA];
    load_slots<WA, FULL, int>(a_idx + base, wart, ii);
    load_slots<WA, FULL, TA>(a_val + base, wart, xx);
#pragma unroll
    for (int s = 0; s < WA; ++s) {
      const bool on = k[p] >= 0 && s < wart;
      ai[p][s] = on ? ii[s] : -1;
      av[p][s] = on ? xx[s] : (TA)0;
    }
  }
}

// <A_line p, A_line q> by index matching: an index occurs at most once per line, so entry s of
// line p meets at most one entry of line q; a select chain in A's own precision (one compare +
// one select per entry pair) finds its partner's value; padding (index -1, value 0) adds
// nothing.  fp64 fma accumulation in slot order.
template <int WA, typename TA>
__device__ __forceinline__ double pair_dot(const int (&ip)[WA], const TA (&xp)[WA], const int (&iq)[WA],
                                           const TA (&xq)[WA]) {
  double g = 0.0;
#pragma unroll
  for (int s = 0; s < WA; ++s) {
    TA m = (TA)0;
#pragma unroll
    for (int t = 0; t < WA; ++t) m = ip[s] == iq[t] ? xq[t] : m;
    g = fma((double)xp[s], (double)m, g);
  }
  return g;
}

// The same with line p's values already widened to fp64 (identical products and order).
template <int WA, typename TA>
__device__ __forceinline__ double pair_dot_w(const int (&ip)[WA], const double (&xp)[WA], const int (&iq)[WA],
                                             const TA (&xq)[WA]) {
  // t outer, s inner: the WA independent select chains advance together, so consecutive
  // compares are independent (their lane masks do not serialise on one SGPR pair)
  TA m[WA];
#pragma unroll
  for (int s = 0; s < WA; ++s) m[s] = (TA)0;
#pragma unroll
  for (int t = 0; t < WA; ++t)
#pragma unroll
    for (int s = 0; s < WA; ++s) m[s] = ip[s] == iq[t] ? xq[t] : m[s];
  double g = 0.0;
#pragma unroll
  for (int s = 0; s < WA; ++s) g = fma(xp[s], (double)m[s], g);
  return g;
}

// Line Gram of M's slots against line j of A-product space:
//   c_p = A_line(k_p)[j],  G_pp = ||A_line(k_p)||^2,  G_pq = <A_line(k_p), A_line(k_q)> (q > p).
// An index occurs at most once per line: entry s of line p meets at most one entry of line q,
// so a select chain in A's own precision (one compare + one select per entry pair) finds its
// partner's value; padding entries (index -1, value 0) add nothing.  fp64 accumulation.
template <int W, int WA, typename TA>
__device__ __forceinline__ void line_gram(const int (&ai)[W][WA], const TA (&av)[W][WA], int j, double (&c)[W],
                                          double (&gd)[W], double (&go)[W * (W - 1) / 2]) {
  int o = 0;
#pragma unroll
  for (int p = 0; p < W; ++p) {
    double cp = 0.0, gpp = 0.0;
#pragma unroll
    for (int s = 0; s < WA; ++s) {
      const double x = (double)av[p][s];
      gpp = fma(x, x, gpp);
      cp += (ai[p][s] == j) ? x : 0.0;
    }
    c[p] = cp;
    gd[p] = gpp;
#pragma unroll
    for (int q = p + 1; q < W; ++q) go[o++] = pair_dot<WA, TA>(ai[p], av[p], ai[q], av[q]);
  }
}

// ||sum_p v_p A_line(k_p) - e_j||^2 = 1 + sum_p v_p (v_p G_pp - 2 c_p + sum_{q>p} v_q (2 G_pq)),
// as explicit fma in this order (every kernel evaluates a line with exactly these operations;
// 2 G_pq is exact, so v_q (2 G_pq) is the product 2 v_q G_pq).
template <int W>
__device__ __forceinline__ double line_res2(const double (&v)[W], const double (&c)[W], const double (&gd)[W],
                                            const double (&go)[W * (W - 1) / 2]) {
  double r2 = 1.0;
  int o = 0;
#pragma unroll
  for (int p = 0; p < W; ++p) {
    double acc = fma(v[p], gd[p], -2.0 * c[p]);
#pragma unroll
    for (int q = p + 1; q < W; ++q) acc = fma(v[q], 2.0 * go[o++], acc);
    r2 = fma(v[p], acc, r2);
  }
  return r2;
}

// Any line of any M_b on its own: gather the A lines it names, Gram, residual.
template <int W, int WA, bool FULL, typename TA>
__device__ __forceinline__ double line_res2_any(const int (&k)[W], const double (&v)[W], int j, int wart,
                                                const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val) {
  int ai[W][WA];
  TA av[W][WA];
  gather_a_lines<W, WA, FULL, TA>(k, wart, a_idx, a_val, ai, av);
  double c[W], gd[W], go[W * (W - 1) / 2];
  line_gram<W, WA, TA>(ai, av, j, c, gd, go);
  return line_res2<W>(v, c, gd, go);
}

// Thread per line, all samples (W <= 7).  The B samples of a batch are mostly sub-patterns of
// ONE line pattern (the GFlowNet candidates: the candidate pattern with removals), so the Gram
// of a line — the index matching, all of the kernel's arithmetic — is formed once per chunk of
// kChunk samples on the union pattern k*_p = max_b k_b[p], and each sample costs a W x W
// quadratic form.  A lane whose samples disagree on a slot (two different valid indices)
// evaluates those samples on their own index sets (line_res2_any), so any M is exact.
// Pass 1 reads the chunk's index slots once (union, per-sample validity bits); pass 2 reads
// the values.  A is read once per line for the whole batch: algorithmic bytes per launch =
// bytes(A) + sum_b bytes(M_b).  Per-sample sums: wave sum, then the kNT/64 wave partials in
// order (a fixed reduction tree), so a sample's result does not depend on the other samples.
#ifndef KCHUNK
#define KCHUNK 8
#endif
constexpr int kChunk = KCHUNK;

template <int W, int WA, bool FULL, typename TA, typename TV>
__device__ __forceinline__ void resid_shared_body(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                  int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                  int64_t idx_bstride, const TV* __restrict__ m_val,
                                                  int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                  const TA* __restrict__ a_val, double* __restrict__ partials,
                                                  double (&sred)[kChunk][kNT / 64]) {
  static_assert(kChunk * W <= 64, "validity bits of a chunk in one u64");
  const int blk = xcd_remap(blockIdx.x, gridDim.x);  // consecutive line ranges on one XCD (A halo in L2)
  const int j = line_begin + blk * kNT + threadIdx.x;
  const bool valid = j < line_end;
  const int jj = valid ? j : line_begin;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int b0 = 0; b0 < B; b0 += kChunk) {
    const int nb = min(kChunk, B - b0);
    int kmax[W], kmin[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      kmax[p] = -1;
      kmin[p] = INT_MAX;
    }
    // every index load of the chunk issued together (one round trip), then the union and the
    // validity bits
    // (unconditional loads from clamped addresses: sample min(b0 + i, B - 1), slot
    // min(p, wrt - 1); masked afterwards)
    int kk[kChunk][W];
#pragma unroll
    for (int i = 0; i < kChunk; ++i) {
      const int32_t* mi = m_idx + (int64_t)min(b0 + i, B - 1) * idx_bstride + (int64_t)jj * wrt;
      int k[W];
      load_slots<W, FULL, int>(mi, wrt, k);
#pragma unroll
      for (int p = 0; p < W; ++p) kk[i][p] = (valid && i < nb && p < wrt) ? k[p] : -1;
    }
    uint64_t bits = 0;
#pragma unroll
    for (int i = 0; i < kChunk; ++i) {
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const int k = kk[i][p];
        if (k >= 0) {
          bits |= (uint64_t)1 << (i * W + p);
          kmax[p] = max(kmax[p], k);
          kmin[p] = min(kmin[p], k);
        }
      }
    }
    bool shared = true;
#pragma unroll
    for (int p = 0; p < W; ++p) shared = shared && (kmax[p] < 0 || kmin[p] == kmax[p]);
    // a lane is either on the shared pattern for the whole chunk (one Gram, quadratic forms)
    // or evaluates every sample on its own index set; the two branches' registers are not
    // live together
    double r2s[kChunk];
#pragma unroll
    for (int i = 0; i < kChunk; ++i) r2s[i] = 0.0;
    if (valid && shared) {
      int ai[W][WA];
      TA av[W][WA];
      double c[W], gd[W], go[W * (W - 1) / 2];
      gather_a_lines<W, WA, FULL, TA>(kmax, wart, a_idx, a_val, ai, av);
      TV vv[kChunk][W];  // the chunk's values, in flight together with the A lines
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        const TV* mv = m_val + (int64_t)min(b0 + i, B - 1) * val_bstride + (int64_t)jj * wrt;
        load_slots<W, FULL, TV>(mv, wrt, vv[i]);  // masked by the validity bits
      }
      line_gram<W, WA, TA>(ai, av, j, c, gd, go);
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        if (i < nb) {
          double v[W];
#pragma unroll
          for (int p = 0; p < W; ++p) v[p] = ((bits >> (i * W + p)) & 1) ? (double)vv[i][p] : 0.0;  // empty: unused
          r2s[i] = line_res2<W>(v, c, gd, go);
        }
      }
    } else if (valid) {
#pragma unroll 1
      for (int i = 0; i < nb; ++i) {  // one sample at a time (registers)
        {
          const int32_t* mi = m_idx + (int64_t)(b0 + i) * idx_bstride + (int64_t)jj * wrt;
          const TV* mv = m_val + (int64_t)(b0 + i) * val_bstride + (int64_t)jj * wrt;
          int k[W], kp[W];
          TV x[W];
          double v[W];
          load_slots<W, FULL, int>(mi, wrt, kp);
          load_slots<W, FULL, TV>(mv, wrt, x);
#pragma unroll
          for (int p = 0; p < W; ++p) {
            const bool on = (bits >> (i * W + p)) & 1;
            k[p] = on ? kp[p] : -1;
            v[p] = on ? (double)x[p] : 0.0;
          }
          const double r2 = line_res2_any<W, WA, FULL, TA>(k, v, j, wart, a_idx, a_val);
#pragma unroll
          for (int u = 0; u < kChunk; ++u) r2s[u] = u == i ? r2 : r2s[u];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kChunk; ++i) {
      if (i < nb) {
        const double r2 = wave_sum_dpp(r2s[i]);
        if (lane == 0) sred[i][w] = r2;
      }
    }
    __syncthreads();
    if (threadIdx.x < nb) {
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < kNT / 64; ++u) s += sred[threadIdx.x][u];
      partials[(int64_t)(b0 + threadIdx.x) * nblk + blk] = s;
    }
    __syncthreads();
  }
}

// WAVES: the occupancy the register allocator must keep (4 waves/SIMD for the fp32 5-wide lines
// of C4 without spills: 117 -> 81 us; the wider / fp64 variants spill there, so 1 = its choice)
template <int W, int WA, typename TA, typename TV, int WAVES>
__global__ __launch_bounds__(kNT, WAVES) void k_resid_shared(int32_t line_begin, int32_t line_end, int32_t wrt,
                                                      int32_t wart, int32_t B, int32_t nblk,
                                                      const int32_t* __restrict__ m_idx, int64_t idx_bstride,
                                                      const TV* __restrict__ m_val, int64_t val_bstride,
                                                      const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val,
                                                      double* __restrict__ partials) {
  __shared__ double sred[kChunk][kNT / 64];
  if (wrt == W && wart == WA)  // stored widths = template widths: 16-byte slot loads
    resid_shared_body<W, WA, true, TA, TV>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                           val_bstride, a_idx, a_val, partials, sred);
  else
    resid_shared_body<W, WA, false, TA, TV>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                            val_bstride, a_idx, a_val, partials, sred);
}

// Thread per line, chunks of C samples, W > 7 (C3's 13-wide lines): the samples' index sets
// are read together; when they agree slot by slot (sub-patterns of one pattern) the A lines of
// the union pattern are gathered once per chunk and every entry pair is matched ONCE for the
// chunk: c_p and G_pp open each sample's row accumulator, each G_pq (q > p) is added to it as
// soon as it is formed (pair_dot), and the row is closed into the sample's sum — exactly
// line_res2's operations in line_res2's order, so a sample gets the same bits as on its own.
// The Gram itself is never stored (91 + 26 fp64 values would not fit beside the A lines).
// Lanes whose samples disagree evaluate each sample on its own index set (line_res2_any).
// The index matching (49 compare + select per entry pair, 78 pairs per 13-wide line) is all of
// the kernel's work, so the chunk is as large as the registers allow: with A's values exact in
// fp32 (the caller passes them narrowed, widened back exactly here; 91 registers for the A
// lines' values) C = 8, one matching per line for the usual batch of 8, at one wave per SIMD
// (the chunk's 8 x 13 fp64 values, the A lines and the row accumulators: ~480 registers).
// fp64 A values would leave room for chunks of 4 only (182 registers of A values): those go to
// k_resid_row16 instead (0.26 vs 0.47 ms at C3).
template <int W, int WA, int C, bool FULL, typename TA, typename TV>
__device__ __forceinline__ void resid_wide_body(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                int64_t idx_bstride, const TV* __restrict__ m_val,
                                                int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                const TA* __restrict__ a_val, double* __restrict__ partials,
                                                double (&sred)[C][kNT / 64]) {
  static_assert(W <= 32, "validity bits of a sample in one u32");
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int j = line_begin + blk * kNT + threadIdx.x;
  const bool valid = j < line_end;
  const int jj = valid ? j : line_begin;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll 1
  for (int b0 = 0; b0 < B; b0 += C) {
    const int nb = min(C, B - b0);
    int kmax[W], kmin[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      kmax[p] = -1;
      kmin[p] = INT_MAX;
    }
    uint32_t bits[C];  // bit p of bits[i]: slot p of sample b0 + i is valid
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const int32_t* mi = m_idx + (int64_t)min(b0 + i, B - 1) * idx_bstride + (int64_t)jj * wrt;
      int k[W];
      load_slots<W, FULL, int>(mi, wrt, k);
      bits[i] = 0u;
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const int kp = (valid && i < nb && p < wrt) ? k[p] : -1;
        if (kp >= 0) {
          bits[i] |= 1u << p;
          kmax[p] = max(kmax[p], kp);
          kmin[p] = min(kmin[p], kp);
        }
      }
    }
    bool shared = true;
#pragma unroll
    for (int p = 0; p < W; ++p) shared = shared && (kmax[p] < 0 || kmin[p] == kmax[p]);
    double r2s[C];
#pragma unroll
    for (int i = 0; i < C; ++i) r2s[i] = 0.0;
    if (valid && shared) {
      int ai[W][WA];
      TA av[W][WA];
      gather_a_lines<W, WA, FULL, TA>(kmax, wart, a_idx, a_val, ai, av);
      double v[C][W];
#pragma unroll
      for (int i = 0; i < C; ++i) {
        TV x[W];
        load_slots<W, FULL, TV>(m_val + (int64_t)min(b0 + i, B - 1) * val_bstride + (int64_t)jj * wrt, wrt, x);
#pragma unroll
        for (int p = 0; p < W; ++p) v[i][p] = ((bits[i] >> p) & 1u) ? (double)x[p] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < C; ++i) r2s[i] = 1.0;
#pragma unroll
      for (int p = 0; p < W; ++p) {
        double cp = 0.0, gpp = 0.0;  // line_gram's c_p and G_pp
#pragma unroll
        for (int s = 0; s < WA; ++s) {
          const double x = (double)av[p][s];
          gpp = fma(x, x, gpp);
          cp += (ai[p][s] == j) ? x : 0.0;
        }
        double acc[C];
#pragma unroll
        for (int i = 0; i < C; ++i) acc[i] = fma(v[i][p], gpp, -2.0 * cp);
#pragma unroll
        for (int q = p + 1; q < W; ++q) {
          const double g2 = 2.0 * pair_dot<WA, TA>(ai[p], av[p], ai[q], av[q]);  // line_gram's 2 G_pq
#pragma unroll
          for (int i = 0; i < C; ++i) acc[i] = fma(v[i][q], g2, acc[i]);
        }
#pragma unroll
        for (int i = 0; i < C; ++i) r2s[i] = fma(v[i][p], acc[i], r2s[i]);
      }
#pragma unroll
      for (int i = 0; i < C; ++i) r2s[i] = i < nb ? r2s[i] : 0.0;
    } else if (valid) {
#pragma unroll 1
      for (int i = 0; i < nb; ++i) {  // one sample at a time on its own index set
        const int32_t* mi = m_idx + (int64_t)(b0 + i) * idx_bstride + (int64_t)jj * wrt;
        const TV* mv = m_val + (int64_t)(b0 + i) * val_bstride + (int64_t)jj * wrt;
        int k[W], kp[W];
        TV x[W];
        double v[W];
        uint32_t bi = 0u;
#pragma unroll
        for (int u = 0; u < C; ++u) bi = u == i ? bits[u] : bi;
        load_slots<W, FULL, int>(mi, wrt, kp);
        load_slots<W, FULL, TV>(mv, wrt, x);
#pragma unroll
        for (int p = 0; p < W; ++p) {
          const bool on = (bi >> p) & 1u;
          k[p] = on ? kp[p] : -1;
          v[p] = on ? (double)x[p] : 0.0;
        }
        const double r2 = line_res2_any<W, WA, FULL, TA>(k, v, j, wart, a_idx, a_val);
#pragma unroll
        for (int u = 0; u < C; ++u) r2s[u] = u == i ? r2 : r2s[u];
      }
    }
#pragma unroll
    for (int i = 0; i < C; ++i) {
      if (i < nb) {
        const double r2 = wave_sum_dpp(r2s[i]);
        if (lane == 0) sred[i][w] = r2;
      }
    }
    __syncthreads();
    if (threadIdx.x < nb) {
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < kNT / 64; ++u) s += sred[threadIdx.x][u];
      partials[(int64_t)(b0 + threadIdx.x) * nblk + blk] = s;
    }
    __syncthreads();
  }
}

template <int W, int WA, typename TA, typename TV>
__global__ __launch_bounds__(kNT) void k_resid_wide(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                    int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                    int64_t idx_bstride, const TV* __restrict__ m_val,
                                                    int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                    const TA* __restrict__ a_val, double* __restrict__ partials) {
  static_assert(sizeof(TA) == 4, "fp64 A values: k_resid_row16");
  constexpr int C = 8;
  __shared__ double sred[C][kNT / 64];
  if (wrt == W && wart == WA)
    resid_wide_body<W, WA, C, true, TA, TV>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                            val_bstride, a_idx, a_val, partials, sred);
  else
    resid_wide_body<W, WA, C, false, TA, TV>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                             val_bstride, a_idx, a_val, partials, sred);
}

// W > 7 with the pattern's Gram cache (spai_residual_lines_gram): the index matching of
// k_resid_wide depends on A and the index sets only, and when a sample's index set is a
// slot-aligned sub-pattern of a pattern whose Gram cache exists (PreconditionerEnv's candidate
// pattern: every slot either the pattern's index or empty) the matching is already done — its
// G_pq, G_pp and c_p are the cache's values (k_gram_build: the same products in the same order
// as line_gram).  The line residual is then line_res2 on the cached values, per sample: one
// thread per line, the cache as its dictionary (spai_line_cache_dict: a handful of distinct
// entries, read from L1/L2 per sample, so no Gram is held in registers), the samples' index sets
// and values streamed with the next sample's loads in flight.  A lane whose sample is not aligned
// evaluates it from A (line_res2_lean).  Same per-sample block sums as k_resid_wide: the same bits.
// line_res2_any with two A lines in registers at a time instead of all W: line q is re-read
// (L1/L2) for every p < q, its address made opaque per use so the compiler cannot keep the W lines
// live; the same operations in the same order (line_gram, then line_res2), so the same bits.
// The unaligned lanes' path of k_resid_gram, which keeps that kernel's registers low.
template <int WA, bool FULL, typename TA>
__device__ __forceinline__ void a_line_opaque(int k, int wart, const int32_t* __restrict__ a_idx,
                                              const TA* __restrict__ a_val, int (&ai)[WA], TA (&av)[WA]) {
  int kk = k;
  asm volatile("" : "+v"(kk));
  const int64_t base = (int64_t)max(kk, 0) * wart;
  int ii[WA];
  TA xx[WA];
  load_slots<WA, FULL, int>(a_idx + base, wart, ii);
  load_slots<WA, FULL, TA>(a_val + base, wart, xx);
#pragma unroll
  for (int s = 0; s < WA; ++s) {
    const bool on = kk >= 0 && s < wart;
    ai[s] = on ? ii[s] : -1;
    av[s] = on ? xx[s] : (TA)0;
  }
}
template <int W>
__device__ __forceinline__ void slot_of(const int (&k)[W], const double (&v)[W], int p, int& kp, double& vp) {
  kp = -1;
  vp = 0.0;
#pragma unroll
  for (int u = 0; u < W; ++u) {  // select chains: no dynamically indexed register arrays (scratch)
    kp = u == p ? k[u] : kp;
    vp = u == p ? v[u] : vp;
  }
}
template <int W, int WA, bool FULL, typename TA>
__device__ __forceinline__ double line_res2_lean(const int (&k)[W], const double (&v)[W], int j, int wart,
                                                 const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val) {
  double r2 = 1.0;
#pragma unroll 1
  for (int p = 0; p < W; ++p) {
    int kp, ip[WA];
    double vp;
    TA xp[WA];
    slot_of<W>(k, v, p, kp, vp);
    a_line_opaque<WA, FULL, TA>(kp, wart, a_idx, a_val, ip, xp);
    double cp = 0.0, gpp = 0.0;
#pragma unroll
    for (int s = 0; s < WA; ++s) {
      const double x = (double)xp[s];
      gpp = fma(x, x, gpp);
      cp += (ip[s] == j) ? x : 0.0;
    }
    double acc = fma(vp, gpp, -2.0 * cp);
#pragma unroll 1
    for (int q = p + 1; q < W; ++q) {
      int kq, iq[WA];
      double vq;
      TA xq[WA];
      slot_of<W>(k, v, q, kq, vq);
      a_line_opaque<WA, FULL, TA>(kq, wart, a_idx, a_val, iq, xq);
      acc = fma(vq, 2.0 * pair_dot<WA, TA>(ip, xp, iq, xq), acc);
    }
    r2 = fma(vp, acc, r2);
  }
  return r2;
}

template <int W, int WA, bool FULL, typename TA, typename TV, typename GT>
__device__ __forceinline__ void resid_gram_body(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                int64_t idx_bstride, const TV* __restrict__ m_val,
                                                int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                const TA* __restrict__ a_val, const int32_t* __restrict__ pat_idx,
                                                const GT* __restrict__ gram, const int32_t* __restrict__ line_entry,
                                                double* __restrict__ partials, double (&sred)[kChunk][kNT / 64]) {
  constexpr int T = W * (W + 1) / 2;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int j = line_begin + blk * kNT + threadIdx.x;
  const bool valid = j < line_end;
  const int jj = valid ? j : line_begin;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int pk[W];  // the cached pattern's indices of the line
  {
    int k[W];
    load_slots<W, FULL, int>(pat_idx + (int64_t)jj * wrt, wrt, k);
#pragma unroll
    for (int p = 0; p < W; ++p) pk[p] = p < wrt ? k[p] : -1;
  }
  const GT* gp = gram + (int64_t)line_entry[jj] * (T + W);
  int kn[W];
  TV xn[W];
  auto load_sample = [&](int b) {
    load_slots<W, FULL, int>(m_idx + (int64_t)b * idx_bstride + (int64_t)jj * wrt, wrt, kn);
    load_slots<W, FULL, TV>(m_val + (int64_t)b * val_bstride + (int64_t)jj * wrt, wrt, xn);
  };
  load_sample(0);
#pragma unroll 1
  for (int b0 = 0; b0 < B; b0 += kChunk) {
    const int nb = min(kChunk, B - b0);
    double r2s[kChunk];
#pragma unroll
    for (int i = 0; i < kChunk; ++i) r2s[i] = 0.0;
#pragma unroll 1
    for (int i = 0; i < nb; ++i) {
      int k[W];
      double v[W];
      bool aligned = true;
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const int kp = (valid && p < wrt) ? kn[p] : -1;
        k[p] = kp >= 0 ? kp : -1;
        v[p] = kp >= 0 ? (double)xn[p] : 0.0;
        aligned = aligned && (kp < 0 || kp == pk[p]);
      }
      if (b0 + i + 1 < B) load_sample(b0 + i + 1);  // in flight while this sample is evaluated
      double r2 = 0.0;
      if (valid && aligned) {  // line_res2 on the cached Gram
        // the entry read as 16-byte pieces (entries are 16-byte aligned: T + W is a multiple of
        // 16 / sizeof(GT); each piece loaded once per sample, a quarter / half of the load
        // instructions of element loads)
        typedef GT gvec_t __attribute__((ext_vector_type(16 / sizeof(GT))));
        constexpr int kPer = 16 / sizeof(GT);
        constexpr bool kVec = (T + W) % kPer == 0;  // 16-byte aligned entries (W = 5, 13; not 7)
        const gvec_t* gv = reinterpret_cast<const gvec_t*>(gp);  // (the compiler keeps the entry in
        // registers across the samples: re-reading it per sample from L1 measured 103 vs 83 us at C3)
        auto G = [&](int q) { return kVec ? (double)gv[q / kPer][q % kPer] : (double)gp[q]; };
        r2 = 1.0;
#pragma unroll
        for (int p = 0; p < W; ++p) {
          const int g0 = p * W - p * (p - 1) / 2;  // G_pp; G_pq at g0 + q - p
          double acc = fma(v[p], G(g0), -2.0 * G(T + p));
#pragma unroll
          for (int q = p + 1; q < W; ++q) acc = fma(v[q], 2.0 * G(g0 + q - p), acc);
          r2 = fma(v[p], acc, r2);
        }
      } else if (valid) {
        r2 = line_res2_lean<W, WA, FULL, TA>(k, v, j, wart, a_idx, a_val);
      }
#pragma unroll
      for (int u = 0; u < kChunk; ++u) r2s[u] = u == i ? r2 : r2s[u];
    }
#pragma unroll
    for (int i = 0; i < kChunk; ++i) {
      if (i < nb) {
        const double r2 = wave_sum_dpp(r2s[i]);
        if (lane == 0) sred[i][w] = r2;
      }
    }
    __syncthreads();
    if (threadIdx.x < nb) {
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < kNT / 64; ++u) s += sred[threadIdx.x][u];
      partials[(int64_t)(b0 + threadIdx.x) * nblk + blk] = s;
    }
    __syncthreads();
  }
}

// (164 registers, 3 waves per SIMD; asking for 4 spills: 137 vs 103 us at C3)
template <int W, int WA, typename TA, typename TV, typename GT>
__global__ __launch_bounds__(kNT) void k_resid_gram(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                    int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                    int64_t idx_bstride, const TV* __restrict__ m_val,
                                                    int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                    const TA* __restrict__ a_val, const int32_t* __restrict__ pat_idx,
                                                    const GT* __restrict__ gram, const int32_t* __restrict__ line_entry,
                                                    double* __restrict__ partials) {
  static_assert(sizeof(TA) == 4, "fp32(-exact) A values (the unaligned lanes' fallback)");
  __shared__ double sred[kChunk][kNT / 64];
  if (wrt == W && wart == WA)
    resid_gram_body<W, WA, true, TA, TV, GT>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                             val_bstride, a_idx, a_val, pat_idx, gram, line_entry, partials, sred);
  else
    resid_gram_body<W, WA, false, TA, TV, GT>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                              val_bstride, a_idx, a_val, pat_idx, gram, line_entry, partials, sred);
}

// Wide lines (8 <= W <= 16, C3's 13-wide lines), SIXTEEN lanes per line: lane p of a 16-lane row
// holds slot p only — the index and values of A line k_p (2 WA registers) and the chunk's 8
// values v_ip — so a line's 78 entry-pair matchings are spread over its lanes at ~100 registers
// per lane (4+ waves per SIMD) instead of one thread holding all 13 A lines at one wave per SIMD.
// Round d = 1..8: every lane takes the slot data of lane p - d (mod 16) by DPP row_ror, matches
// the pair (pair_dot) and adds v_iq * 2 G_pq (d = 8: both lanes of the pair meet, each adds
// v_iq * G_pq) to its per-sample sum; every unordered pair is matched exactly once.  The lane's
// row value v_ip (v_ip G_pp - 2 c_p + sum) is summed over the 16 lanes by a fixed DPP tree.
// A block walks 16 groups of 16 consecutive lines (256 lines, the partials of k_resid_shared).
// Rows whose samples disagree on a slot evaluate each sample on its own index set with the same
// per-sample operations (a sample's value never depends on the other samples of its chunk:
// bit-identical to the sample alone).  Explicit _rn arithmetic: no contraction differences
// between the chunk and the single-sample instantiations.
constexpr int kRowC = 8;  // samples per chunk of the row kernel
// Round D of row_eval: the slot data of lane p - D (mod 16) by DPP row_ror:D, one pair matched.
// (row_ror has a source lane for every lane: bound_ctrl, no "old" operand to preload)
template <int kCtl>
__device__ __forceinline__ int dpp_row_i(int x) {
  return __builtin_amdgcn_mov_dpp(x, kCtl, 0xf, 0xf, true);
}
template <int kCtl>
__device__ __forceinline__ double dpp_row_d(double x) {
  const uint64_t u = __double_as_longlong(x);
  const int lo = dpp_row_i<kCtl>((int)(uint32_t)u), hi = dpp_row_i<kCtl>((int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
template <int D, int C, int WA, typename TA>
__device__ __forceinline__ void row_round(const int (&ai)[WA], const TA (&av)[WA], const double (&xd)[WA],
                                          const double (&v)[C], double (&acc)[C]) {
  constexpr int kCtl = 0x120 + D;  // row_ror:D
  int pi[WA];
  TA pa[WA];
#pragma unroll
  for (int s = 0; s < WA; ++s) {
    pi[s] = dpp_row_i<kCtl>(ai[s]);
    if constexpr (sizeof(TA) == 4)
      pa[s] = __int_as_float(dpp_row_i<kCtl>(__float_as_int(av[s])));
    else
      pa[s] = dpp_row_d<kCtl>(av[s]);
  }
  const double g = pair_dot_w<WA, TA>(ai, xd, pi, pa);
  const double g2 = D < 8 ? 2.0 * g : g;  // D = 8: both lanes of the pair add it
#pragma unroll
  for (int i = 0; i < C; ++i) acc[i] = fma(dpp_row_d<kCtl>(v[i]), g2, acc[i]);
}

// A line k of the lane's slot (k < 0: empty, index -1 / value 0; clamped unconditional loads).
template <int WA, bool FULL, typename TA>
__device__ __forceinline__ void row_load(int k, int wart, const int32_t* __restrict__ a_idx,
                                         const TA* __restrict__ a_val, int (&ai)[WA], TA (&av)[WA]) {
  const int64_t base = (int64_t)max(k, 0) * wart;
  load_slots<WA, FULL, int>(a_idx + base, wart, ai);
  load_slots<WA, FULL, TA>(a_val + base, wart, av);
#pragma unroll
  for (int s = 0; s < WA; ++s) {
    const bool on = k >= 0 && s < wart;
    ai[s] = on ? ai[s] : -1;
    av[s] = on ? av[s] : (TA)0;
  }
}

// The row values v_ip (v_ip G_pp - 2 c_p + sum_q v_iq 2 G_pq) of C samples from the lane's A line.
template <int C, int WA, typename TA>
__device__ __forceinline__ void row_eval(const int (&ai)[WA], const TA (&av)[WA], int j, const double (&v)[C],
                                         double (&row)[C]) {
  double xd[WA];
  double cp = 0.0, gpp = 0.0;
#pragma unroll
  for (int s = 0; s < WA; ++s) {
    xd[s] = (double)av[s];
    gpp = fma(xd[s], xd[s], gpp);
    cp = __dadd_rn(cp, (ai[s] == j) ? xd[s] : 0.0);
  }
  double acc[C];
#pragma unroll
  for (int i = 0; i < C; ++i) acc[i] = 0.0;
  row_round<1, C, WA, TA>(ai, av, xd, v, acc);
  row_round<2, C, WA, TA>(ai, av, xd, v, acc);
  row_round<3, C, WA, TA>(ai, av, xd, v, acc);
  row_round<4, C, WA, TA>(ai, av, xd, v, acc);
  row_round<5, C, WA, TA>(ai, av, xd, v, acc);
  row_round<6, C, WA, TA>(ai, av, xd, v, acc);
  row_round<7, C, WA, TA>(ai, av, xd, v, acc);
  row_round<8, C, WA, TA>(ai, av, xd, v, acc);
#pragma unroll
  for (int i = 0; i < C; ++i) row[i] = __dmul_rn(v[i], __dadd_rn(fma(v[i], gpp, -2.0 * cp), acc[i]));
}

// Sum over the 16 lanes of a row, fixed tree (row_shr 1, 2, 4, 8): lane 15 of the row holds it.
__device__ __forceinline__ double row16_sum(double x) {
  x = __dadd_rn(x, dpp_d<0x111, 0xf>(x));
  x = __dadd_rn(x, dpp_d<0x112, 0xf>(x));
  x = __dadd_rn(x, dpp_d<0x114, 0xf>(x));
  x = __dadd_rn(x, dpp_d<0x118, 0xf>(x));
  return x;
}

template <int W, int WA, bool FULL, typename TA, typename TV>
__device__ __forceinline__ void resid_row16_body(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                 int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                 int64_t idx_bstride, const TV* __restrict__ m_val,
                                                 int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                 const TA* __restrict__ a_val, double* __restrict__ partials,
                                                 double (&sred)[kRowC][kNT / 16]) {
  static_assert(W <= 16, "one slot per lane of a 16-lane row");
  constexpr int kGroups = kNT / 16;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int r = threadIdx.x >> 4, p = threadIdx.x & 15;
  const int rw = (threadIdx.x & 63) >> 4;  // row inside the wave
#pragma unroll 1
  for (int b0 = 0; b0 < B; b0 += kRowC) {
    const int nb = min(kRowC, B - b0);
    double tot[kRowC];  // this row's sum over its 16 lines (valid in lane 15 of the row)
#pragma unroll
    for (int i = 0; i < kRowC; ++i) tot[i] = 0.0;
    // Software pipeline over the block's 16 line groups: while group it is evaluated, the A
    // lines of group it + 1 and the slot indices / values of group it + 2 are in flight, so the
    // dependent gather (indices -> A lines) never stalls a wave.
    int kn[kRowC];  // raw slot indices / values of the group being loaded
    TV xn[kRowC];
    auto load_group = [&](int it) {
      const int j = line_begin + blk * kNT + it * 16 + r;
      const int jj = j < line_end ? j : line_begin;
      const int64_t o = (int64_t)jj * wrt + min(p, wrt - 1);
      // sample bases recomputed here (opaque first sample): 8 x 2 loop-invariant 64-bit bases
      // held across the loop would take 32 SGPRs, and the matching needs SGPR pairs for its masks
      int bs = b0;
      asm volatile("" : "+s"(bs));
#pragma unroll
      for (int i = 0; i < kRowC; ++i) {
        const int b = min(bs + i, B - 1);
        kn[i] = m_idx[(int64_t)b * idx_bstride + o];
        xn[i] = m_val[(int64_t)b * val_bstride + o];
      }
    };
    // a group's masked indices / values, its union index and whether its row is shared
    auto take_group = [&](int it, int (&kk)[kRowC], double (&v)[kRowC], int& ku, bool& shared) {
      const int j = line_begin + blk * kNT + it * 16 + r;
      const bool slot = j < line_end && p < W && p < wrt;
      int kmax = -1, kmin = INT_MAX;
#pragma unroll
      for (int i = 0; i < kRowC; ++i) {
        const int k = kn[i];
        const bool on = slot && i < nb && k >= 0;
        kk[i] = on ? k : -1;
        v[i] = on ? (double)xn[i] : 0.0;
        if (on) {
          kmax = max(kmax, k);
          kmin = min(kmin, k);
        }
      }
      // a row is on the shared path when every lane's valid indices agree across the chunk
      const uint64_t bad = __ballot(!(kmax < 0 || kmin == kmax));
      shared = ((bad >> (rw * 16)) & 0xFFFFull) == 0;
      ku = kmax;
    };
    int kc[kRowC], kuc;
    double vc[kRowC];
    bool shc;
    int aic[WA];
    TA avc[WA];
    load_group(0);
    take_group(0, kc, vc, kuc, shc);
    row_load<WA, FULL, TA>(kuc, wart, a_idx, a_val, aic, avc);
    if (kGroups > 1) load_group(1);
#pragma unroll 1
    for (int it = 0; it < kGroups; ++it) {
      int kx[kRowC], kux = -1;
      double vx[kRowC];
      bool shx = true;
      int aix[WA];
      TA avx[WA];
      if (it + 1 < kGroups) {  // next group: its A lines into flight, then the slots of it + 2
        take_group(it + 1, kx, vx, kux, shx);
        row_load<WA, FULL, TA>(kux, wart, a_idx, a_val, aix, avx);
        if (it + 2 < kGroups) load_group(it + 2);
      }
      const int j = line_begin + blk * kNT + it * 16 + r;
      double row[kRowC];
      if (shc) {
        row_eval<kRowC, WA, TA>(aic, avc, j, vc, row);
      } else {
#pragma unroll 1
        for (int i = 0; i < nb; ++i) {  // one sample at a time on its own index set
          int ki = -1;
          double vi[1] = {0.0}, ri[1];
#pragma unroll
          for (int u = 0; u < kRowC; ++u) {
            ki = u == i ? kc[u] : ki;
            vi[0] = u == i ? vc[u] : vi[0];
          }
          int ai1[WA];
          TA av1[WA];
          row_load<WA, FULL, TA>(ki, wart, a_idx, a_val, ai1, av1);
          row_eval<1, WA, TA>(ai1, av1, j, vi, ri);
#pragma unroll
          for (int u = 0; u < kRowC; ++u) row[u] = u == i ? ri[0] : row[u];
        }
#pragma unroll
        for (int u = 0; u < kRowC; ++u) row[u] = u < nb ? row[u] : 0.0;
      }
      const bool valid = j < line_end;
#pragma unroll
      for (int i = 0; i < kRowC; ++i) {
        const double s = row16_sum(row[i]);
        tot[i] = __dadd_rn(tot[i], valid ? __dadd_rn(1.0, s) : 0.0);
      }
#pragma unroll
      for (int i = 0; i < kRowC; ++i) {
        kc[i] = kx[i];
        vc[i] = vx[i];
      }
#pragma unroll
      for (int s = 0; s < WA; ++s) {
        aic[s] = aix[s];
        avc[s] = avx[s];
      }
      shc = shx;
    }
    if (p == 15) {
#pragma unroll
      for (int i = 0; i < kRowC; ++i) sred[i][r] = tot[i];
    }
    __syncthreads();
    if (threadIdx.x < nb) {
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < kGroups; ++u) s = __dadd_rn(s, sred[threadIdx.x][u]);
      partials[(int64_t)(b0 + threadIdx.x) * nblk + blk] = s;
    }
    __syncthreads();
  }
}

template <int W, int WA, typename TA, typename TV>
__global__ __launch_bounds__(kNT) void k_resid_row16(int32_t line_begin, int32_t line_end, int32_t wrt, int32_t wart,
                                                     int32_t B, int32_t nblk, const int32_t* __restrict__ m_idx,
                                                     int64_t idx_bstride, const TV* __restrict__ m_val,
                                                     int64_t val_bstride, const int32_t* __restrict__ a_idx,
                                                     const TA* __restrict__ a_val, double* __restrict__ partials) {
  __shared__ double sred[kRowC][kNT / 16];
  if (wart == WA)
    resid_row16_body<W, WA, true, TA, TV>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                          val_bstride, a_idx, a_val, partials, sred);
  else
    resid_row16_body<W, WA, false, TA, TV>(line_begin, line_end, wrt, wart, B, nblk, m_idx, idx_bstride, m_val,
                                           val_bstride, a_idx, a_val, partials, sred);
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
  constexpr int kWaves = (W == 5 && sizeof(TA) == 4 && sizeof(TV) == 4) ? 4 : 1;
  if constexpr (W <= 7)
    k_resid_shared<W, WA, TA, TV, kWaves><<<nblk, kNT, 0, s>>>(lb, le, wrt, wart, B, nblk, mi, ib, static_cast<const TV*>(mv),
                                                        vb, ai, static_cast<const TA*>(av), partials);
  else if constexpr (sizeof(TA) == 4)  // C3 exact-A: 0.21 ms vs 0.23 for k_resid_row16
    k_resid_wide<W, WA, TA, TV><<<nblk, kNT, 0, s>>>(lb, le, wrt, wart, B, nblk, mi, ib, static_cast<const TV*>(mv), vb,
                                                      ai, static_cast<const TA*>(av), partials);
  else  // fp64 A: 0.26 ms vs 0.47 for k_resid_wide's chunks of 4 (C3, resid_bench.py --wide --inexact)
    k_resid_row16<W, WA, TA, TV><<<nblk, kNT, 0, s>>>(lb, le, wrt, wart, B, nblk, mi, ib, static_cast<const TV*>(mv), vb,
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

template <int W, int WA, typename TV, typename GT>
void launch_resid_gram(int32_t lb, int32_t le, int32_t wrt, int32_t wart, int32_t B, int32_t nblk, const int32_t* mi,
                       int64_t ib, const void* mv, int64_t vb, const int32_t* ai, const void* av, const int32_t* pat_idx,
                       const void* gram, const int32_t* line_entry, double* partials, hipStream_t s) {
  k_resid_gram<W, WA, float, TV, GT><<<nblk, kNT, 0, s>>>(lb, le, wrt, wart, B, nblk, mi, ib, static_cast<const TV*>(mv),
                                                          vb, ai, static_cast<const float*>(av), pat_idx,
                                                          static_cast<const GT*>(gram), line_entry, partials);
}
using ResidGramFn = decltype(&launch_resid_gram<5, 5, float, float>);
template <int W, int WA>
ResidGramFn pick_resid_gram(bool m32, bool g32) {
  return m32 ? (g32 ? launch_resid_gram<W, WA, float, float> : launch_resid_gram<W, WA, float, double>)
             : (g32 ? launch_resid_gram<W, WA, double, float> : launch_resid_gram<W, WA, double, double>);
}

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" int spai_residual_lines_gram(int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                                        const int32_t* m_idx, int64_t idx_bstride, const void* m_val, int32_t m_dtype,
                                        int64_t val_bstride, int32_t WA, const int32_t* a_idx, const void* a_val,
                                        int32_t a_dtype, const int32_t* pat_idx, const void* gram_dict,
                                        int32_t gram_dtype, const int32_t* line_entry, int32_t B, double* res2_out,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(n >= 1 && line_begin >= 0 && line_end >= line_begin && line_end <= n && W >= 1 && WA >= 1 &&
                     B >= 1 && idx_bstride >= 0 && val_bstride >= 0,
                 "spai_residual_lines_gram: bad shape");
  SPAI_CHECK_ARG(m_idx && m_val && a_idx && a_val && pat_idx && gram_dict && line_entry && res2_out && workspace,
                 "spai_residual_lines_gram: null pointer");
  SPAI_CHECK_ARG(m_dtype == SPAI_DTYPE_F32 || m_dtype == SPAI_DTYPE_F64, "spai_residual_lines_gram: bad m_dtype");
  SPAI_CHECK_ARG(gram_dtype == SPAI_DTYPE_F32 || gram_dtype == SPAI_DTYPE_F64,
                 "spai_residual_lines_gram: bad gram_dtype");
  SPAI_CHECK_ARG(((uintptr_t)gram_dict & 15) == 0, "spai_residual_lines_gram: gram_dict not 16-byte aligned");
  // the cache's width is the pattern's: W exactly 5 (A <= 5 wide), 7 or 13 (A <= 7 wide)
  const bool shape_ok = (W == 5 && WA <= 5) || ((W == 7 || W == 13) && WA <= 7);
  if (!shape_ok || a_dtype != SPAI_DTYPE_F32) {
    set_error("spai_residual_lines_gram: lines of M 5 / 7 / 13 wide over A lines <= 5 / 7 / 7 wide with fp32(-exact) "
              "A values only (W=%d WA=%d a_dtype %d): use spai_residual_lines",
              W, WA, a_dtype);
    return SPAI_ERR_UNSUPPORTED;
  }
  const int32_t nl = line_end - line_begin;
  hipStream_t s = (hipStream_t)stream;
  if (nl == 0) {
    SPAI_CHECK_HIP(hipMemsetAsync(res2_out, 0, sizeof(double) * B, s));
    return SPAI_OK;
  }
  SPAI_CHECK_ARG(workspace_bytes >= spai_residual_workspace_bytes(nl, B),
                 "spai_residual_lines_gram: workspace too small");
  const int32_t nblk = (nl + kNT - 1) / kNT;
  double* partials = static_cast<double*>(workspace);
  const bool m32 = m_dtype == SPAI_DTYPE_F32, g32 = gram_dtype == SPAI_DTYPE_F32;
  const ResidGramFn fn = W == 5 ? pick_resid_gram<5, 5>(m32, g32)
                                : (W == 7 ? pick_resid_gram<7, 7>(m32, g32) : pick_resid_gram<13, 7>(m32, g32));
  fn(line_begin, line_end, W, WA, B, nblk, m_idx, idx_bstride, m_val, val_bstride, a_idx, a_val, pat_idx, gram_dict,
     line_entry, partials, s);
  SPAI_CHECK_LAUNCH();
  k_resid_reduce<<<B, kNT, 0, s>>>(partials, nblk, res2_out);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

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
