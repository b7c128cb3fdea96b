// Least-squares fill of M by Householder QR for gfx950.  The north star's per-column constrained
// least squares
//     m_l = argmin || A[:, J] m - e_l ||_2 ,  J = the kept pattern slots of line l
// solved the way it names: the line's dense block A[I, slots] (I = the union of the rows the
// slots' A lines touch) is staged in LDS once per line and factored by Householder reflections on
// L lanes of a wavefront (a "group"), each lane holding RPL rows of the block; the reflections'
// norms and dot products are group reductions on DPP lane swaps (quad_perm, row_half_mirror,
// row_mirror) — no LDS traffic inside the factorisation.  No normal equations: the conditioning
// is that of A[I, J] itself, not its square (the Gram-cached fill in gram.hip is the
// normal-equations path).
//
// Per block: 256 consecutive lines (the exact-sum invariance unit, LINE_ALIGN), in rounds of NG
// lines (one per group).  Per round:
//   1. per line, on its group of L lanes: the W slots' A lines are staged in LDS and one lane
//      merges them (they are sorted by row index) into the dense block D = A[I, slots], rows of I
//      ascending, with the column norms ||D[:, p]||^2 and the position of row l in I; then the
//      FULL Householder QR of D (all slots, the sample-independent part): R (W x W), the first W
//      entries of Q^T e_l and the tail ||(Q^T e_l)[W..]||^2 (+1 when l is not in I) go to LDS;
//   2. per (line, sample), on ONE lane: the removal bitmap's kept slots J select the columns R_J
//      of R (R_J = Q^T D_J: the same singular values as A[I, J], so the small problem
//      min ||R_J m - Q^T e|| keeps the QR's accuracy, no normal equations), which are
//      re-triangularised by Householder reflections of at most W rows; a slot is dropped when
//      its remaining norm is below 1e-12 ||D[:, p]|| (numerical rank deficiency in fp64; the
//      normal equations of gram.hip already drop a column whose remaining norm is below ~3e-7 of
//      its norm: 1e-13 of the squared norm); back-substitution gives m, and the line residual^2
//      is the tail + (Q^T e) below the pivots (sums of squares: no cancellation).
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <vector>

#include "spai_device.h"
#include "spai_status.h"
#include "spai_timer.h"

namespace spai {
namespace {

constexpr int kQNT = 256;     // threads per block (k_qr_rows; the fill instances choose theirs)
constexpr int kQLines = 256;  // lines per block (= distributed.LINE_ALIGN)
constexpr int kQChunk = 8;    // samples per residual chunk
constexpr int kQTabW = 5;     // widths whose (entry, mask) solutions are tabled per launch (2^W masks)
// a table record: the W solution values in M's type, then the residual^2 (fp64) in the last 8 bytes;
// whole 16-byte pieces (float M, W = 5: 32 bytes)
template <int W, typename TM>
__host__ __device__ constexpr int qr_rec_bytes() { return ((W * (int)sizeof(TM) + 7) / 8 * 8 + 8 + 15) / 16 * 16; }

// Sum over the L lanes of a group (L = 4, 8, 16, 32 consecutive lanes), valid on every lane of
// the group with identical bits (each step adds a commutative pair).
template <int L>
__device__ __forceinline__ double group_sum(double v) {
  v += dpp_d<0xB1, 0xf>(v);  // quad_perm [1, 0, 3, 2]
  v += dpp_d<0x4E, 0xf>(v);  // quad_perm [2, 3, 0, 1]
  if constexpr (L >= 8) v += dpp_d<0x141, 0xf>(v);  // row_half_mirror: quad 0 <-> quad 1
  if constexpr (L >= 16) v += dpp_d<0x140, 0xf>(v);  // row_mirror: half-row 0 <-> 1
  if constexpr (L >= 32) v += __shfl_xor(v, 16, kWave);
  static_assert(L == 4 || L == 8 || L == 16 || L == 32, "group size");
  return v;
}

// Union size of the rows the slots' A lines touch, per line (max over the lines -> *out).
template <int W, int WA>
__global__ __launch_bounds__(kQNT) void k_qr_rows(int32_t n, int32_t wrt, const int32_t* __restrict__ pat_idx,
                                                  int32_t wart, const int32_t* __restrict__ a_idx,
                                                  int32_t* __restrict__ out) {
  const int l = blockIdx.x * kQNT + threadIdx.x;
  int rows = 0;
  if (l < n) {
    int kp[W], h[W], cur[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      kp[p] = p < wrt ? pat_idx[(int64_t)l * wrt + p] : -1;
      h[p] = 0;
      const int a = kp[p] >= 0 ? a_idx[(int64_t)kp[p] * wart] : -1;
      cur[p] = a >= 0 ? a : INT_MAX;
    }
#pragma unroll 1
    for (int it = 0; it < W * WA; ++it) {
      int r = INT_MAX;
#pragma unroll
      for (int p = 0; p < W; ++p) r = min(r, cur[p]);
      if (r == INT_MAX) break;
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (cur[p] == r) {
          ++h[p];
          const int a = h[p] < wart ? a_idx[(int64_t)kp[p] * wart + h[p]] : -1;
          cur[p] = a >= 0 ? a : INT_MAX;
        }
      ++rows;
    }
  }
  rows = max(rows, (int)__shfl_xor(rows, 1, kWave));
#pragma unroll
  for (int o = 2; o < kWave; o <<= 1) rows = max(rows, (int)__shfl_xor(rows, o, kWave));
  if ((threadIdx.x & 63) == 0 && rows > 0) atomicMax(out, rows);
}

// 1/x to ~1 ulp: hardware reciprocal + one Newton step (x finite, non-zero)
__device__ __forceinline__ double qr_rcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}

// A group lives inside one wavefront, and a wave's LDS instructions execute in order: a hand-off
// between the lanes of a group needs only that the compiler keeps the LDS accesses in program
// order (no block barrier, so the waves of a block progress independently).
__device__ __forceinline__ void group_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// LDS row strides chosen against bank conflicts (64 banks of 4 bytes).  The dense blocks: group
// g's block starts at g * qr_group_stride words, and the two access shapes are lane (g, j)
// reading row j (+ L i) of its group's block and the 64 / L group leaders writing during the
// merge; the smallest padding that minimises the worse of the two (e.g. W = 5, R = 16, L = 4:
// 80 -> 84 words per group, 4-way -> conflict-free).  Per-line fp64 rows read by consecutive
// lines in phase 2 get an odd stride in doubles (conflict-free over a half-wave).
__host__ __device__ constexpr int qr_ways(int gs, int rw, int L) {
  int worst = 0;
  for (int b = 0; b < 64; ++b) {
    int n1 = 0, n2 = 0;
    for (int g = 0; g < 64 / L; ++g) {
      n2 += (gs * g) % 64 == b;
      for (int j = 0; j < L; ++j) n1 += (gs * g + rw * j) % 64 == b;
    }
    worst = n1 > worst ? n1 : worst;
    worst = n2 > worst ? n2 : worst;
  }
  return worst;
}
template <int R, int W, int L, typename TA>
__host__ __device__ constexpr int qr_group_stride() {  // in elements of TA
  constexpr int ew = (int)(sizeof(TA) / 4), base = R * W;
  int best = base, bw = 1 << 30;
  for (int pad = 0; pad < 16; ++pad) {
    const int w = qr_ways((base + pad) * ew, W * ew, L);
    if (w < bw) {
      bw = w;
      best = base + pad;
    }
  }
  return best;
}
__host__ __device__ constexpr int odd_up(int x) { return x | 1; }

#ifndef QR_WPE
#define QR_WPE 2  // waves per SIMD of the 5-wide fill instances (175 VGPRs: 2 is what they reach)
#endif

// LDS of the per-line factorisation (phase 1) for NT / L groups of L lanes.
template <int W, int WA, int L, int RPL, int NT, typename TA>
struct QrStage {
  static constexpr int NG = NT / L, R = L * RPL, T = W * (W + 1) / 2;
  static constexpr int GS = qr_group_stride<R, W, L, TA>();
  TA sDb[NG * GS];                 // dense blocks A[I, slots] (rows of I ascending), GS per group
  int sAi[NG][W][WA];              // staged A lines of the slots
  TA sAv[NG][W][WA];
  double sCn[NG][W];               // ||D[:, p]||^2 (the rank floor of the masked solves)
  int sRowL[NG];                   // position of row l in I; -1: not in I; -2: block overflow
  double sRf[NG][odd_up(T)];       // R of the full block (all slots), packed upper triangle
  double sC[NG][odd_up(W + 1)];    // (Q^T e_l)[0..W), then the tail ||(Q^T e_l)[W..)||^2 (+1 if l not in I)
  int sAct[NG][W];                 // action ids of the slots (-1: no slot / empty A line)
};

// Phase 1 for line l on group g (lane j of L): the slots' A lines staged and merged (one lane;
// they are sorted by row index) into D = A[I, slots], then the FULL Householder QR of D on the
// group -> S.sRf[g], S.sC[g], S.sCn[g], S.sAct[g].  Sample-independent: it depends on A and the
// pattern only.  Ends with the group's LDS writes issued (the caller orders them by a barrier).
template <int W, int WA, int L, int RPL, int NT, typename TA>
__device__ __forceinline__ void qr_factor_line(QrStage<W, WA, L, RPL, NT, TA>& S, int g, int j, bool valid, int l,
                                               int32_t wrt, const int32_t* __restrict__ pat_idx,
                                               const int32_t* __restrict__ pat_act, int32_t wart,
                                               const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val) {
  using St = QrStage<W, WA, L, RPL, NT, TA>;
  constexpr int R = St::R, GS = St::GS;
#define SD(g_, r_, p_) S.sDb[(g_) * GS + (r_) * W + (p_)]
  for (int e = j; e < W * WA; e += L) {
    const int p = e / WA, s = e % WA;
    const int kp = (valid && p < wrt) ? pat_idx[(int64_t)l * wrt + p] : -1;
    const int a = (kp >= 0 && s < wart) ? a_idx[(int64_t)kp * wart + s] : -1;
    S.sAi[g][p][s] = a;
    S.sAv[g][p][s] = a >= 0 ? a_val[(int64_t)kp * wart + s] : (TA)0;
  }
  for (int e = j; e < R * W; e += L) S.sDb[g * GS + e] = (TA)0;
  group_sync();
  if (j == 0) {  // merge the sorted A lines into the rows of I (ascending)
    int h[W], cur[W];
    double cn[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      h[p] = 0;
      cn[p] = 0.0;
      const int a = S.sAi[g][p][0];
      cur[p] = a >= 0 ? a : INT_MAX;
    }
    int rowl = -1, rho = 0;
#pragma unroll 1
    for (int it = 0; it <= R; ++it) {
      int rmin = INT_MAX;
#pragma unroll
      for (int p = 0; p < W; ++p) rmin = min(rmin, cur[p]);
      if (rmin == INT_MAX) break;
      if (rho == R) {  // more rows than the instance holds (the caller's max_rows was wrong)
        rowl = -2;
        break;
      }
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (cur[p] == rmin) {
          const TA v = S.sAv[g][p][h[p]];
          SD(g, rho, p) = v;
          cn[p] += (double)v * (double)v;
          ++h[p];
          const int a = h[p] < WA ? S.sAi[g][p][h[p]] : -1;
          cur[p] = a >= 0 ? a : INT_MAX;
        }
      if (rmin == l) rowl = rho;
      ++rho;
    }
#pragma unroll
    for (int p = 0; p < W; ++p) {
      S.sCn[g][p] = cn[p];
      S.sAct[g][p] = (valid && p < wrt && S.sAi[g][p][0] >= 0) ? pat_act[(int64_t)l * wrt + p] : -1;
    }
    S.sRowL[g] = rowl;
  }
  group_sync();
  const int rowl = S.sRowL[g];
  double dv[RPL][W], rhs[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    const int rho = j + L * i;
#pragma unroll
    for (int p = 0; p < W; ++p) dv[i][p] = (double)SD(g, rho, p);
    rhs[i] = rho == rowl ? 1.0 : 0.0;
  }
  // reflection p maps column p onto row p (a column already zero below row p: none)
#pragma unroll
  for (int p = 0; p < W; ++p) {
    double s1 = 0.0, xk = 0.0;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const int rho = j + L * i;
      const double x = dv[i][p];
      s1 = fma(rho >= p ? x : 0.0, x, s1);
      xk += rho == p ? x : 0.0;
    }
    const double sig = group_sum<L>(s1), xkk = group_sum<L>(xk);
    const double sq = sqrt(sig);
    const double alpha = xkk >= 0.0 ? -sq : sq;
    const double tau = sig > 0.0 ? qr_rcp(sig - alpha * xkk) : 0.0;  // H = I - tau v v^T
    double v[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const int rho = j + L * i;
      v[i] = rho >= p ? dv[i][p] - (rho == p ? alpha : 0.0) : 0.0;
    }
    double d[W + 1];  // v . column q (q > p), v . rhs
#pragma unroll
    for (int q = p + 1; q <= W; ++q) {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < RPL; ++i) a = fma(v[i], q < W ? dv[i][q] : rhs[i], a);
      d[q] = a;
    }
#pragma unroll
    for (int q = p + 1; q <= W; ++q) d[q] = group_sum<L>(d[q]) * tau;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
#pragma unroll
      for (int q = p + 1; q < W; ++q) dv[i][q] = fma(-d[q], v[i], dv[i][q]);
      rhs[i] = fma(-d[W], v[i], rhs[i]);
    }
    // row p of R and (Q^T e)_p are final now (later reflections act on rows > p)
    if (j == p % L) {
      const int base = p * W - p * (p - 1) / 2;
      S.sRf[g][base] = sig > 0.0 ? alpha : dv[p / L][p];
#pragma unroll
      for (int q = p + 1; q < W; ++q) S.sRf[g][base + (q - p)] = dv[p / L][q];
      S.sC[g][p] = rhs[p / L];
    }
  }
  double tl = 0.0;  // the tail of Q^T e: rows >= W
#pragma unroll
  for (int i = 0; i < RPL; ++i) tl = fma(j + L * i >= W ? rhs[i] : 0.0, rhs[i], tl);
  tl = group_sum<L>(tl);
  if (j == 0) S.sC[g][W] = rowl == -2 ? __builtin_nan("") : tl + (rowl < 0 ? 1.0 : 0.0);
#undef SD
}

// 1/sqrt(t) to ~1 ulp: hardware reciprocal square root + one Newton step (t > 0, normal)
__device__ __forceinline__ double qr_rsq(double t) {
  const double r = __builtin_amdgcn_rsq(t);
  const double e = fma(-t * r, r, 1.0);  // 1 - t r^2
  return fma(0.5 * r, e, r);
}

// Phase 2 for one (line, sample) on ONE lane: min ||R_J m - c|| over the kept columns J of the
// line's full-block R (R_J = Q^T D_J has the singular values of A[I, J], so the small problem
// keeps the QR's accuracy: no normal equations).  The pivot of a kept column p stays in row p:
// the rows whose own column was removed (or rank-dropped) are "free", and at column p ONE
// Householder reflection over {free rows < p} u {row p} maps column p onto row p (the pivot rows
// < p take no part: their entries of v are 0, so they are left exactly as they are).  Only which
// rows are free depends on the mask — no data-dependent row index anywhere, so the back-
// substitution is the plain triangular one.  Column p pivots when it is kept and its norm outside
// the pivot rows exceeds 1e-12 ||D[:, p]|| (thr[p] = 1e-24 ||D[:, p]||^2: fp64 rank deficiency), else
// m_p = 0 and row p becomes free (no reflection).  Rm (Rm[i][q], i <= q; the rest is never read)
// and c are worked in place; m gets the solution; returns the line residual^2 = tail + sum of
// (Q^T e)^2 over the free rows (sums of squares: no cancellation).
template <int W>
__device__ __forceinline__ double qr_masked_solve(double (&Rm)[W][W], double (&c)[W], double tail,
                                                  const double (&thr)[W], const bool (&keep)[W], double (&m)[W]) {
  bool piv[W];
  double rd[W];
  {  // column 0 has no rows above it: its reflection would only flip row 0's sign (skipped)
    const double x0 = Rm[0][0];
    piv[0] = keep[0] && x0 * x0 > thr[0];
    rd[0] = piv[0] ? qr_rcp(x0) : 0.0;
  }
#pragma unroll
  for (int p = 1; p < W; ++p) {
    double v[W];  // the reflection vector over rows 0..p (0 on the pivot rows)
    const double xp = Rm[p][p];
    double sig = xp * xp;
#pragma unroll
    for (int i = 0; i < p; ++i) {
      v[i] = piv[i] ? 0.0 : Rm[i][p];
      sig = fma(v[i], v[i], sig);
    }
    piv[p] = keep[p] && sig > thr[p];  // |R_pp| after the reflection > 1e-12 ||D[:, p]||
    const double rs = qr_rsq(piv[p] ? sig : 1.0);
    const double sq = sig * rs;                                 // sqrt(sig)
    const double alpha = __builtin_copysign(sq, -xp);           // the new R_pp (sign opposite to x_p)
    const double tau = piv[p] ? qr_rcp(fma(sq, __builtin_fabs(xp), sig)) : 0.0;  // 1 / (sig - alpha x_p)
    v[p] = xp - alpha;
    rd[p] = piv[p] ? __builtin_copysign(rs, -xp) : 0.0;         // 1 / alpha
#pragma unroll
    for (int q = p + 1; q <= W; ++q) {
      double a = v[p] * (q < W ? Rm[p][q] : c[p]);
#pragma unroll
      for (int i = 0; i < p; ++i) a = fma(v[i], q < W ? Rm[i][q] : c[i], a);
      a *= tau;
#pragma unroll
      for (int i = 0; i <= p; ++i) {
        if (q < W) Rm[i][q] = fma(-a, v[i], Rm[i][q]);
        else c[i] = fma(-a, v[i], c[i]);
      }
    }
  }
  double rsum = tail;  // + (Q^T e) over the free rows
#pragma unroll
  for (int i = 0; i < W; ++i) rsum = fma(piv[i] ? 0.0 : c[i], c[i], rsum);
#pragma unroll
  for (int p = W - 1; p >= 0; --p) {
    double a = c[p];
#pragma unroll
    for (int q = p + 1; q < W; ++q) a = fma(-Rm[p][q], m[q], a);  // m_q = 0 for a non-pivot q
    m[p] = a * rd[p];  // 0 for a dropped slot
  }
  return rsum;
}

// The fused fill: phase 1 and phase 2 in one launch, A read every call (no cache).
template <int W, int WA, int L, int RPL, int NT, typename TA, typename TM>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(W <= 5 ? QR_WPE : 2))) void k_qr_fill(int32_t n, int32_t line_begin, int32_t line_end, int32_t wrt,
                                                  const int32_t* __restrict__ pat_idx,
                                                  const int32_t* __restrict__ pat_act, int32_t wart,
                                                  const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val,
                                                  int32_t B, const uint32_t* __restrict__ removed, int32_t words,
                                                  int32_t word_base, TM* __restrict__ m_out,
                                                  double* __restrict__ partials) {
  using St = QrStage<W, WA, L, RPL, NT, TA>;
  constexpr int NG = St::NG, NR = kQLines / NG;  // groups, rounds
  static_assert(kQLines % NG == 0 && W * WA <= 8 * 1024, "shapes");
  __shared__ St S;
  __shared__ double sR2[kQChunk][NG];       // per (sample, group line): the sum over the rounds
  const int t = threadIdx.x, g = t / L, j = t % L, lane = t & 63, wave = t >> 6;
  const int lb = blockIdx.x;
  const int64_t nloc = line_end - line_begin;
  const int blk0 = line_begin + lb * kQLines;
  const int nvl = min(kQLines, line_end - blk0);

#pragma unroll 1
  for (int b0 = 0; b0 < B; b0 += kQChunk) {
    const int nb = min(kQChunk, B - b0);
    for (int i = t; i < kQChunk * NG; i += NT) (&sR2[0][0])[i] = 0.0;  // ordered by the first barrier
#pragma unroll 1
    for (int r = 0; r < NR; ++r) {
      {
        const int li = r * NG + g;
        const bool valid = li < nvl;
        qr_factor_line<W, WA, L, RPL, NT, TA>(S, g, j, valid, blk0 + (valid ? li : 0), wrt, pat_idx, pat_act, wart,
                                              a_idx, a_val);
      }
      __syncthreads();  // R, Q^T e of the round's lines
      {
        const int gl = t % NG;
        const int li = r * NG + gl;
        const bool valid = li < nvl;
        const int l = blk0 + (valid ? li : 0);
        int act[W], wofs[W];
        double thr[W];
#pragma unroll
        for (int p = 0; p < W; ++p) {
          act[p] = S.sAct[gl][p];
          wofs[p] = act[p] >= 0 ? (act[p] >> 5) - word_base : 0;
          thr[p] = 1e-24 * S.sCn[gl][p];
        }
#pragma unroll 1
        for (int s = t / NG; s < nb; s += NT / NG) {
          const int b = b0 + s;
          const uint32_t* rm = removed + (int64_t)b * words;
          bool keep[W];
#pragma unroll
          for (int p = 0; p < W; ++p) keep[p] = act[p] >= 0 && !((rm[wofs[p]] >> (act[p] & 31)) & 1u);
          double Rm[W][W], c[W], m[W];
#pragma unroll
          for (int i = 0; i < W; ++i) {
#pragma unroll
            for (int q = i; q < W; ++q) Rm[i][q] = S.sRf[gl][i * W - i * (i - 1) / 2 + (q - i)];
            c[i] = S.sC[gl][i];
          }
          const double rs = qr_masked_solve<W>(Rm, c, S.sC[gl][W], thr, keep, m);
          if (valid) {
            if (m_out != nullptr) {
              TM* dst = m_out + ((int64_t)b * nloc + (l - line_begin)) * wrt;
#pragma unroll
              for (int p = 0; p < W; ++p)
                if (p < wrt) dst[p] = (TM)m[p];
            }
            sR2[s][gl] += rs;  // one thread per (s, gl): the rounds in order
          }
        }
      }
      __syncthreads();  // the round's LDS is reused by the next round
    }
    // per-sample block sums in a fixed order (the k_gram_fill partial layout)
    static_assert(NG <= 64, "one wave sums a sample's group lines");
    for (int s = wave; s < nb; s += NT / 64) {
      double acc = lane < NG ? sR2[s][lane] : 0.0;
      acc = wave_sum(acc);
      if (lane == 0) partials[(int64_t)(b0 + s) * gridDim.x + lb] = acc;
    }
    __syncthreads();
  }
}

// ---- the R cache: phase 1 once per env (A and the pattern are constant for an env's lifetime,
// preconditioner.py:23-25), phase 2 per rollout from the cache.
// Layout (blocks of 64 lines, structure of arrays as the Gram cache): rcache[l / 64][q][l % 64],
// q < T: R packed upper triangle (row-major, p <= q); T + p: (Q^T e_l)_p; T + W: the tail.
__host__ __device__ constexpr int qr_cache_q(int W) { return W * (W + 1) / 2 + W + 1; }

template <int W, int WA, int L, int RPL, int NT, typename TA>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void k_qr_factor(int32_t n, int32_t wrt,
                                                  const int32_t* __restrict__ pat_idx,
                                                  const int32_t* __restrict__ pat_act, int32_t wart,
                                                  const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val,
                                                  double* __restrict__ rcache) {
  using St = QrStage<W, WA, L, RPL, NT, TA>;
  constexpr int NG = St::NG, NR = kQLines / NG, T = St::T, NQ = qr_cache_q(W);
  __shared__ St S;
  const int t = threadIdx.x, g = t / L, j = t % L;
  const int blk0 = blockIdx.x * kQLines;
  const int nvl = min(kQLines, n - blk0);
#pragma unroll 1
  for (int r = 0; r < NR; ++r) {
    const int li = r * NG + g;
    const bool valid = li < nvl;
    qr_factor_line<W, WA, L, RPL, NT, TA>(S, g, j, valid, blk0 + (valid ? li : 0), wrt, pat_idx, pat_act, wart,
                                          a_idx, a_val);
    __syncthreads();
    for (int e = t; e < NG * NQ; e += NT) {  // consecutive threads: consecutive lines of one entry
      const int gl = e % NG, q = e / NG, li2 = r * NG + gl;
      if (li2 >= nvl) continue;
      const int l = blk0 + li2;
      const double v = q < T ? S.sRf[gl][q] : S.sC[gl][q - T];
      rcache[(int64_t)(l >> 6) * NQ * 64 + q * 64 + (l & 63)] = v;
    }
    __syncthreads();
  }
}

// Phase 2 from the R cache, one thread per line (the k_gram_fill stream): per line the W action
// ids and the NQ cached values once, the column norms ||D[:, p]||^2 = sum_i R_ip^2 recomputed
// (they only set the rank floor), then per sample W mask bits, the masked re-triangularisation and
// back-substitution (qr_masked_solve), M staged through LDS and written with 16-byte `nt` buffer
// stores, the line residuals summed per sample in a fixed order (the k_gram_fill partial layout:
// 256-line blocks, so 256-line-aligned shards sum to one launch's bits).
#ifndef QRS_WPE
#define QRS_WPE 4
#endif
// kDict: rcache is the cache's dictionary (spai_qr_cache_dict: its distinct entries, NQ doubles
// each, contiguous) and line_entry[j] names line j's entry; else the full cache, 64 lines
// interleaved per entry value (coalesced).
template <int W, typename TM, bool kDict>
__global__ __launch_bounds__(kQNT) __attribute__((amdgpu_waves_per_eu(W <= 5 ? QRS_WPE : (W <= 7 ? 2 : 1)))) void k_qr_solve(
    int32_t line_begin, int32_t line_end, int32_t wrt, const int32_t* __restrict__ pat_act,
    const double* __restrict__ rcache, const int32_t* __restrict__ line_entry, int32_t B,
    const uint32_t* __restrict__ removed, int32_t words, int32_t word_base, TM* __restrict__ m_out,
    double* __restrict__ partials) {
  constexpr int T = W * (W + 1) / 2, NQ = qr_cache_q(W);
  static_assert(kQNT == kQLines, "one thread per line of a 256-line block");
  __shared__ double s_r2[kQChunk][kQNT];
#ifndef QRS_WAVE_M
  __shared__ __attribute__((aligned(16))) TM s_m[2][kQNT * W];
#else
  __shared__ __attribute__((aligned(16))) TM s_m[1][kQNT * W];  // per-wave regions
#endif
  // W > 7 (13-wide lines): the line's 91-value R is not held across the samples (with the working
  // copy it would take ~370 registers) but re-read per sample from the cache (its dictionary: L1/L2)
  constexpr bool kHold = W <= 7;
  __shared__ double s_c0[kHold ? W + 1 : 1][kQNT];  // the line's Q^T e and tail (LDS, not registers: 4 waves per SIMD)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lb = blockIdx.x;
  const int j = line_begin + lb * kQNT + t;
  const bool valid = j < line_end;
  const int64_t nloc = line_end - line_begin;
  const int jj = valid ? j : line_begin;  // clamped: loads stay in bounds
  const int nvl = min(kQNT, line_end - (line_begin + lb * kQNT));

  int act[W];
  {
    int av[W];  // every load issued before any is used
#pragma unroll
    for (int p = 0; p < W; ++p) av[p] = pat_act[(int64_t)jj * wrt + min(p, wrt - 1)];
#pragma unroll
    for (int p = 0; p < W; ++p) act[p] = (valid && p < wrt) ? av[p] : -1;
  }
  double R0[kHold ? T : 1];
  float thf[W];  // the rank floors 1e-24 ||D[:, p]||^2 in fp32 (registers: 4 waves per SIMD at W = 5)
  // a dictionary entry is shared by most lanes of a wave (stencil lines): broadcast loads from L2
  constexpr int kStride = kDict ? 1 : 64;
  const double* rp = kDict ? rcache + (int64_t)line_entry[jj] * NQ : rcache + (int64_t)(jj >> 6) * NQ * 64 + (jj & 63);
  auto rval = [&](int q) { return kHold ? R0[q] : rp[q * kStride]; };
  if constexpr (kHold) {
#pragma unroll
    for (int q = 0; q < T; ++q) R0[q] = rp[q * kStride];
#pragma unroll
    for (int p = 0; p <= W; ++p) s_c0[p][t] = rp[(T + p) * kStride];  // read back by this thread only
  }
#pragma unroll
  for (int p = 0; p < W; ++p) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i <= p; ++i) {
      const double x = rval(i * W - i * (i - 1) / 2 + (p - i));
      s = fma(x, x, s);
    }
    thf[p] = (float)(1e-24 * s);  // (0 only below 1e-21: the floor then drops exact zeros only)
  }
  // bitmap word offset of a slot (recomputed where used: no registers held across the samples)
  auto wofs = [&](int p) { return act[p] >= 0 ? (act[p] >> 5) - word_base : 0; };
  uint32_t wd[W];  // the slots' bitmap words of the next sample are loaded while the current one is solved
#pragma unroll
  for (int p = 0; p < W; ++p) wd[p] = removed[wofs(p)];
#pragma unroll 1
  for (int b = 0; b < B; ++b) {
    bool keep[W];
#pragma unroll
    for (int p = 0; p < W; ++p) keep[p] = act[p] >= 0 && !((wd[p] >> (act[p] & 31)) & 1u);
    if (b + 1 < B) {
      const uint32_t* rn = removed + (int64_t)(b + 1) * words;
#pragma unroll
      for (int p = 0; p < W; ++p) wd[p] = rn[wofs(p)];
    }
    double thr[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      float f = thf[p];
      asm volatile("" : "+v"(f));  // widened per sample, not held as fp64 across the loop
      thr[p] = (double)f;
    }
    double Rm[W][W], c[W], m[W], tail;
    if constexpr (kHold) {
#pragma unroll
      for (int i = 0; i < W; ++i) {
#pragma unroll
        for (int q = i; q < W; ++q) Rm[i][q] = R0[i * W - i * (i - 1) / 2 + (q - i)];
        c[i] = s_c0[i][t];
      }
      tail = s_c0[W][t];
    } else {
      const double* rps = rp;
      asm volatile("" : "+v"(rps));  // opaque per sample: re-read, not held across the samples
#pragma unroll
      for (int i = 0; i < W; ++i) {
#pragma unroll
        for (int q = i; q < W; ++q) Rm[i][q] = rps[(i * W - i * (i - 1) / 2 + (q - i)) * kStride];
        c[i] = rps[(T + i) * kStride];
      }
      tail = rps[(T + W) * kStride];
    }
    const double rs = qr_masked_solve<W>(Rm, c, tail, thr, keep, m);
    s_r2[b % kQChunk][t] = valid ? rs : 0.0;
#ifdef QRS_DIRECT  // A/B: M stored from the registers (no LDS staging, no barrier per sample)
    if (m_out != nullptr && valid) {
      TM* dst = m_out + ((int64_t)b * nloc + (j - line_begin)) * wrt;
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (p < wrt) nt_store(dst + p, (TM)m[p]);
    }
#else
#ifndef QRS_WAVE_M  // M staged per block; QRS_WAVE_M (A/B): per wave, no block barrier per sample —
                    // 6 VGPRs spilled at 128, 0.127 vs 0.106 ms at C4 (the Gram fills gain from it)
    {  // M (no branch on m_out: store_m_block drops every store when it is null)
      TM* sm = s_m[b & 1];
      if (valid) {
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p < wrt) sm[t * wrt + p] = (TM)m[p];
      }
      __syncthreads();
      store_m_block<kQNT, W, TM>(m_out ? m_out + ((int64_t)b * nloc + (int64_t)lb * kQNT) * wrt : nullptr, sm,
                                 nvl * wrt);
    }
#else
    {  // M staged per WAVE (its 64 lines are one contiguous run of M): no block barrier per sample
      const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: scalar offsets
      TM* sm = s_m[0] + wv * 64 * W;
      if (valid) {
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p < wrt) sm[lane * wrt + p] = (TM)m[p];
      }
      __builtin_amdgcn_wave_barrier();
      const int nw = min(max(nvl - wv * 64, 0), 64);
      store_m_block<64, W, TM>(m_out ? m_out + ((int64_t)b * nloc + (int64_t)lb * kQNT + wv * 64) * wrt : nullptr,
                               sm, nw * wrt, lane);
      __builtin_amdgcn_wave_barrier();
    }
#endif
#endif
    if (b % kQChunk == kQChunk - 1 || b == B - 1) {  // the chunk's fixed-order block sums
      const int c0b = b - b % kQChunk, nb = b - c0b + 1;
      __syncthreads();
      for (int u = wave; u < nb; u += kQNT / 64) {
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < kQNT / 64; ++q) acc += s_r2[u][q * 64 + lane];
        acc = wave_sum(acc);
        if (lane == 0) partials[(int64_t)(c0b + u) * gridDim.x + lb] = acc;
      }
      __syncthreads();
    }
  }
}

// Every (entry, keep mask) solution of the R cache's dictionary, once per launch of the cached
// fill (k_qr_lookup's table): thread g solves mask g % 2^W of entry g / 2^W with the per-line path's
// arithmetic on the same values (its R, Q^T e and tail from the entry, the rank floors recomputed as
// sum_i R_ip^2 in the same order) and writes the record {m_0 .. m_{W-1}, residual^2} (fp64).
constexpr int kQTabMaxEntries = 4096;  // (table <= 6.3 MB at W = 5; larger dictionaries solve per line)
template <int W, typename TM>
__global__ __launch_bounds__(kQNT) void k_qr_table(int32_t entries, const double* __restrict__ dict,
                                                   char* __restrict__ mtab) {
  constexpr int T = W * (W + 1) / 2, NQ = qr_cache_q(W), kMasks = 1 << W;
  const int g = blockIdx.x * kQNT + threadIdx.x;
  const int e = g / kMasks, mk = g % kMasks;
  if (e >= entries) return;
  const double* re = dict + (int64_t)e * NQ;
  double Rm[W][W], c[W], m[W], thr[W];
  bool keep[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
#pragma unroll
    for (int q = i; q < W; ++q) Rm[i][q] = re[i * W - i * (i - 1) / 2 + (q - i)];
    c[i] = re[T + i];
  }
  const double tail = re[T + W];
#pragma unroll
  for (int p = 0; p < W; ++p) {
    double sq = 0.0;
#pragma unroll
    for (int i = 0; i <= p; ++i) sq = fma(Rm[i][p], Rm[i][p], sq);
    thr[p] = (double)(float)(1e-24 * sq);
    keep[p] = (mk >> p) & 1;
  }
  const double rs = qr_masked_solve<W>(Rm, c, tail, thr, keep, m);
  constexpr int kRec = qr_rec_bytes<W, TM>();
  char* out = mtab + (int64_t)g * kRec;
#pragma unroll
  for (int p = 0; p < W; ++p) reinterpret_cast<TM*>(out)[p] = (TM)m[p];  // (the per-line path's conversion)
  *reinterpret_cast<double*>(out + kRec - 8) = rs;
}

// The cached fill from that table: per line the W action ids and the entry index; per sample the
// W keep bits pick the record {M values, residual^2} (the next sample's record loads while this one
// is stored).  No solve and no per-line R or Q^T e held, so more blocks per CU than k_qr_solve; M
// staged per block and stored, and the residual sums formed, exactly as k_qr_solve does (the same
// bits as solving every (line, sample) on its own lane).
#ifndef QR_LOOKUP_WPE
#define QR_LOOKUP_WPE 6
#endif
template <int W, typename TM>
__global__ __launch_bounds__(kQNT) __attribute__((amdgpu_waves_per_eu(QR_LOOKUP_WPE))) void k_qr_lookup(
    int32_t line_begin, int32_t line_end, int32_t wrt, const int32_t* __restrict__ pat_act,
    const int32_t* __restrict__ line_entry, int32_t B, const uint32_t* __restrict__ removed, int32_t words,
    int32_t word_base, TM* __restrict__ m_out, double* __restrict__ partials, const char* __restrict__ mtab) {
  constexpr int kMasks = 1 << W, kRec = qr_rec_bytes<W, TM>(), kRW = kRec / 16;
  typedef unsigned int u4t __attribute__((ext_vector_type(4)));
  __shared__ double s_r2[kQChunk][kQNT];
  __shared__ __attribute__((aligned(16))) TM s_m[2][kQNT * W];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lb = blockIdx.x;
  const int j = line_begin + lb * kQNT + t;
  const bool valid = j < line_end;
  const int64_t nloc = line_end - line_begin;
  const int jj = valid ? j : line_begin;  // clamped: loads stay in bounds
  const int nvl = min(kQNT, line_end - (line_begin + lb * kQNT));
  int act[W];
  {
    int av[W];
#pragma unroll
    for (int p = 0; p < W; ++p) av[p] = pat_act[(int64_t)jj * wrt + min(p, wrt - 1)];
#pragma unroll
    for (int p = 0; p < W; ++p) act[p] = (valid && p < wrt) ? av[p] : -1;
  }
  const u4t* tab = reinterpret_cast<const u4t*>(mtab) + (int64_t)line_entry[jj] * kMasks * kRW;
  auto wofs = [&](int p) { return act[p] >= 0 ? (act[p] >> 5) - word_base : 0; };
  auto mask_of = [&](const uint32_t (&w)[W]) {
    int mt = 0;
#pragma unroll
    for (int p = 0; p < W; ++p) mt |= (int)(act[p] >= 0 && !((w[p] >> (act[p] & 31)) & 1u)) << p;
    return mt;
  };
  // per group of kG samples: their W * kG bitmap words in flight together, then their kG records
  // in flight together with the next group's bitmap words, so a block waits on ~1 memory round
  // trip per group instead of one per sample
  constexpr int kG = 4;
  static_assert(kQChunk % kG == 0, "whole sample groups per residual chunk");
  uint32_t wv[kG][W];
#pragma unroll
  for (int i = 0; i < kG; ++i)
#pragma unroll
    for (int p = 0; p < W; ++p) wv[i][p] = i < B ? removed[(int64_t)i * words + wofs(p)] : 0u;
#pragma unroll 1
  for (int b0 = 0; b0 < B; b0 += kQChunk) {
    const int nb = min(kQChunk, B - b0);
#pragma unroll
    for (int g0 = 0; g0 < kQChunk; g0 += kG) {
      if (g0 < nb) {
        u4t rc[kG][kRW];
#pragma unroll
        for (int i = 0; i < kG; ++i) {
          const int mt = mask_of(wv[i]);
#pragma unroll
          for (int k = 0; k < kRW; ++k) rc[i][k] = g0 + i < nb ? tab[mt * kRW + k] : (u4t){0u, 0u, 0u, 0u};
        }
        const int bn = b0 + g0 + kG;  // the next group's first sample
#pragma unroll
        for (int i = 0; i < kG; ++i)
#pragma unroll
          for (int p = 0; p < W; ++p) wv[i][p] = bn + i < B ? removed[(int64_t)(bn + i) * words + wofs(p)] : 0u;
#pragma unroll
        for (int i = 0; i < kG; ++i) {
          if (g0 + i < nb) {
            const int b = b0 + g0 + i;
            const TM* mv = reinterpret_cast<const TM*>(&rc[i][0]);
            const double rs = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(&rc[i][0]) + kRec - 8);
            s_r2[g0 + i][t] = valid ? rs : 0.0;
            TM* sm = s_m[b & 1];
            if (valid) {
#pragma unroll
              for (int p = 0; p < W; ++p)
                if (p < wrt) sm[t * wrt + p] = mv[p];
            }
            __syncthreads();
            store_m_block<kQNT, W, TM>(m_out ? m_out + ((int64_t)b * nloc + (int64_t)lb * kQNT) * wrt : nullptr, sm,
                                       nvl * wrt);
          }
        }
      }
    }
    // the chunk's fixed-order block sums (k_qr_solve's)
    __syncthreads();
    for (int u = wave; u < nb; u += kQNT / 64) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kQNT / 64; ++q) acc += s_r2[u][q * 64 + lane];
      acc = wave_sum(acc);
      if (lane == 0) partials[(int64_t)(b0 + u) * gridDim.x + lb] = acc;
    }
    __syncthreads();
  }
}

// (W class, A width class, rows) -> instance
template <int W, int WA, int L, int RPL, int NT, typename TM>
hipError_t launch_qr(bool a32, int32_t n, int32_t lb, int32_t le, int32_t wrt, const int32_t* pi, const int32_t* pa,
                     int32_t wart, const int32_t* ai, const void* av, int32_t B, const uint32_t* rm, int32_t words,
                     int32_t wb, void* mo, double* partials, int32_t nparts, hipStream_t s) {
  if (a32)
    k_qr_fill<W, WA, L, RPL, NT, float, TM><<<nparts, NT, 0, s>>>(n, lb, le, wrt, pi, pa, wart, ai,
                                                                static_cast<const float*>(av), B, rm, words, wb,
                                                                static_cast<TM*>(mo), partials);
  else
    k_qr_fill<W, WA, L, RPL, NT, double, TM><<<nparts, NT, 0, s>>>(n, lb, le, wrt, pi, pa, wart, ai,
                                                                 static_cast<const double*>(av), B, rm, words, wb,
                                                                 static_cast<TM*>(mo), partials);
  return hipGetLastError();
}

template <typename TM>
hipError_t dispatch_qr(int wc, int rows, bool a32, int32_t n, int32_t lb, int32_t le, int32_t wrt, const int32_t* pi,
                       const int32_t* pa, int32_t wart, const int32_t* ai, const void* av, int32_t B,
                       const uint32_t* rm, int32_t words, int32_t wb, void* mo, double* partials, int32_t nparts,
                       hipStream_t s) {
#define SPAI_QR_ARGS a32, n, lb, le, wrt, pi, pa, wart, ai, av, B, rm, words, wb, mo, partials, nparts, s
  if (wc == 5) {
    if (rows <= 16) return launch_qr<5, 5, 4, 4, 256, TM>(SPAI_QR_ARGS);
    return launch_qr<5, 5, 8, 4, 256, TM>(SPAI_QR_ARGS);
  }
  if (wc == 7) {
    if (rows <= 32) return launch_qr<7, 7, 8, 4, 256, TM>(SPAI_QR_ARGS);
    return launch_qr<7, 7, 16, 4, 128, TM>(SPAI_QR_ARGS);
  }
  if (rows <= 64) return launch_qr<13, 7, 16, 4, 128, TM>(SPAI_QR_ARGS);
  return launch_qr<13, 7, 32, 3, 128, TM>(SPAI_QR_ARGS);
#undef SPAI_QR_ARGS
}

// the R cache build: the same (W class, rows) -> instance choice as the fused fill
template <int W, int WA, int L, int RPL, int NT>
hipError_t launch_factor(bool a32, int32_t n, int32_t wrt, const int32_t* pi, const int32_t* pa, int32_t wart,
                         const int32_t* ai, const void* av, double* rc, hipStream_t s) {
  const int grid = (n + kQLines - 1) / kQLines;
  if (a32)
    k_qr_factor<W, WA, L, RPL, NT, float><<<grid, NT, 0, s>>>(n, wrt, pi, pa, wart, ai, static_cast<const float*>(av),
                                                             rc);
  else
    k_qr_factor<W, WA, L, RPL, NT, double><<<grid, NT, 0, s>>>(n, wrt, pi, pa, wart, ai,
                                                              static_cast<const double*>(av), rc);
  return hipGetLastError();
}
hipError_t dispatch_factor(int wc, int rows, bool a32, int32_t n, int32_t wrt, const int32_t* pi, const int32_t* pa,
                           int32_t wart, const int32_t* ai, const void* av, double* rc, hipStream_t s) {
#define SPAI_QF_ARGS a32, n, wrt, pi, pa, wart, ai, av, rc, s
  if (wc == 5) {
    if (rows <= 16) return launch_factor<5, 5, 4, 4, 256>(SPAI_QF_ARGS);
    return launch_factor<5, 5, 8, 4, 256>(SPAI_QF_ARGS);
  }
  if (wc == 7) {
    if (rows <= 32) return launch_factor<7, 7, 8, 4, 256>(SPAI_QF_ARGS);
    return launch_factor<7, 7, 16, 4, 128>(SPAI_QF_ARGS);
  }
  if (rows <= 64) return launch_factor<13, 7, 16, 4, 128>(SPAI_QF_ARGS);
  return launch_factor<13, 7, 32, 3, 128>(SPAI_QF_ARGS);
#undef SPAI_QF_ARGS
}

template <int W, typename TM>
void launch_solve_t(const int32_t* ent, int32_t entries, int32_t lb, int32_t le, int32_t wrt, const int32_t* pa,
                    const double* rc, int32_t B, const uint32_t* rm, int32_t words, int32_t wb, void* mo,
                    double* partials, int32_t nparts, double* mtab, hipStream_t s) {
  KernelTimer kt(SPAI_TIMER_QR, s);  // (the table and the solve: the fill's whole time)
  if constexpr (W <= kQTabW) {
    if (ent && mtab) {  // every (entry, mask) solution once, then the lines read theirs
      const int nt = entries << W;
      k_qr_table<W, TM><<<(nt + kQNT - 1) / kQNT, kQNT, 0, s>>>(entries, rc, reinterpret_cast<char*>(mtab));
      k_qr_lookup<W, TM><<<nparts, kQNT, 0, s>>>(lb, le, wrt, pa, ent, B, rm, words, wb, static_cast<TM*>(mo),
                                                 partials, reinterpret_cast<const char*>(mtab));
      return;
    }
  }
  if (ent)
    k_qr_solve<W, TM, true><<<nparts, kQNT, 0, s>>>(lb, le, wrt, pa, rc, ent, B, rm, words, wb, static_cast<TM*>(mo),
                                                    partials);
  else
    k_qr_solve<W, TM, false><<<nparts, kQNT, 0, s>>>(lb, le, wrt, pa, rc, nullptr, B, rm, words, wb,
                                                     static_cast<TM*>(mo), partials);
}
template <int W>
hipError_t launch_solve(bool f64, const int32_t* ent, int32_t entries, int32_t lb, int32_t le, int32_t wrt,
                        const int32_t* pa, const double* rc, int32_t B, const uint32_t* rm, int32_t words, int32_t wb,
                        void* mo, double* partials, int32_t nparts, double* mtab, hipStream_t s) {
  if (f64)
    launch_solve_t<W, double>(ent, entries, lb, le, wrt, pa, rc, B, rm, words, wb, mo, partials, nparts, mtab, s);
  else
    launch_solve_t<W, float>(ent, entries, lb, le, wrt, pa, rc, B, rm, words, wb, mo, partials, nparts, mtab, s);
  return hipGetLastError();
}

// width class of a (pattern, A) pair: 5 (W <= 5, WA <= 5), 7 (W <= 7, WA <= 7), 13 (W <= 13, WA <= 7)
int qr_class(int32_t W, int32_t WA) {
  if (W <= 5 && WA <= 5) return 5;
  if (W <= 7 && WA <= 7) return 7;
  if (W <= 13 && WA <= 7) return 13;
  return 0;
}
int qr_rows_cap(int wc) { return wc == 5 ? 32 : (wc == 7 ? 64 : 96); }

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" int spai_qr_max_rows(int32_t n, int32_t W, const int32_t* pat_idx, int32_t WA, const int32_t* a_idx,
                                int32_t* max_rows, void* stream) {
  SPAI_CHECK_ARG(n >= 1 && W >= 1 && WA >= 1 && pat_idx && a_idx && max_rows, "spai_qr_max_rows: bad arguments");
  const int wc = qr_class(W, WA);
  if (wc == 0) {
    set_error("spai_qr_max_rows: widths W=%d WA=%d above the compiled 13 / 7", W, WA);
    return SPAI_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  SPAI_CHECK_HIP(hipMemsetAsync(max_rows, 0, sizeof(int32_t), s));
  const int grid = (n + kQNT - 1) / kQNT;
  if (wc == 5)
    k_qr_rows<5, 5><<<grid, kQNT, 0, s>>>(n, W, pat_idx, WA, a_idx, max_rows);
  else if (wc == 7)
    k_qr_rows<7, 7><<<grid, kQNT, 0, s>>>(n, W, pat_idx, WA, a_idx, max_rows);
  else
    k_qr_rows<13, 7><<<grid, kQNT, 0, s>>>(n, W, pat_idx, WA, a_idx, max_rows);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_fill_lines_qr(int32_t n, int32_t line_begin, int32_t line_end, int32_t W, const int32_t* pat_idx,
                                  const int32_t* pat_act, int32_t WA, const int32_t* a_idx, const void* a_val,
                                  int32_t a_dtype, int32_t max_rows, int32_t B, const uint32_t* removed, int32_t words,
                                  int32_t word_base, void* m_out, int32_t m_dtype, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(m_dtype == SPAI_DTYPE_F32 || m_dtype == SPAI_DTYPE_F64, "spai_fill_lines_qr: bad m_dtype");
  SPAI_CHECK_ARG(a_dtype == SPAI_DTYPE_F32 || a_dtype == SPAI_DTYPE_F64, "spai_fill_lines_qr: bad a_dtype");
  SPAI_CHECK_ARG(n >= 1 && line_begin >= 0 && line_end >= line_begin && line_end <= n && W >= 1 && WA >= 1 &&
                     B >= 1 && words >= 1 && word_base >= 0 && max_rows >= 0,
                 "spai_fill_lines_qr: bad shape");
  SPAI_CHECK_ARG(workspace != nullptr, "spai_fill_lines_qr: null workspace");
  const int32_t nl = line_end - line_begin;
  if (nl == 0) return SPAI_OK;
  SPAI_CHECK_ARG(pat_idx && pat_act && a_idx && a_val && removed, "spai_fill_lines_qr: null input");
  const int wc = qr_class(W, WA);
  if (wc == 0 || max_rows > qr_rows_cap(wc)) {
    set_error("spai_fill_lines_qr: widths W=%d WA=%d / %d rows above the compiled 13 / 7 / %d", W, WA, max_rows,
              wc ? qr_rows_cap(wc) : 0);
    return SPAI_ERR_UNSUPPORTED;
  }
  const int32_t nparts = (nl + kQLines - 1) / kQLines;
  SPAI_CHECK_ARG(workspace_bytes >= sizeof(double) * (size_t)nparts * B, "spai_fill_lines_qr: workspace too small");
  double* partials = static_cast<double*>(workspace);
  hipStream_t s = (hipStream_t)stream;
  const bool a32 = a_dtype == SPAI_DTYPE_F32;
  const hipError_t e =
      m_dtype == SPAI_DTYPE_F64
          ? dispatch_qr<double>(wc, max_rows, a32, n, line_begin, line_end, W, pat_idx, pat_act, WA, a_idx, a_val, B,
                                removed, words, word_base, m_out, partials, nparts, s)
          : dispatch_qr<float>(wc, max_rows, a32, n, line_begin, line_end, W, pat_idx, pat_act, WA, a_idx, a_val, B,
                               removed, words, word_base, m_out, partials, nparts, s);
  SPAI_CHECK_HIP(e);
  return SPAI_OK;
}

// ---- the R cache (phase 1 once per env) and the per-rollout solve from it
static int qr_cache_class(int32_t W, int32_t WA) { return qr_class(W, WA); }

extern "C" size_t spai_qr_cache_bytes(int32_t n, int32_t W, int32_t WA) {
  const int wc = qr_cache_class(W, WA);
  if (n <= 0 || wc == 0) return 0;
  return sizeof(double) * (size_t)qr_cache_q(wc) * (size_t)((n + 63) / 64 * 64);
}

extern "C" int spai_qr_factor(int32_t n, int32_t W, const int32_t* pat_idx, const int32_t* pat_act, int32_t WA,
                              const int32_t* a_idx, const void* a_val, int32_t a_dtype, int32_t max_rows,
                              double* rcache, size_t rcache_bytes, void* stream) {
  SPAI_CHECK_ARG(n >= 1 && W >= 1 && WA >= 1 && max_rows >= 0 && pat_idx && pat_act && a_idx && a_val && rcache,
                 "spai_qr_factor: bad arguments");
  SPAI_CHECK_ARG(a_dtype == SPAI_DTYPE_F32 || a_dtype == SPAI_DTYPE_F64, "spai_qr_factor: bad a_dtype");
  const int wc = qr_cache_class(W, WA);
  if (wc == 0 || max_rows > qr_rows_cap(wc)) {
    set_error("spai_qr_factor: widths W=%d WA=%d / %d rows above the compiled 13 / 7 / %d", W, WA, max_rows,
              wc ? qr_rows_cap(wc) : 0);
    return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_ARG(rcache_bytes >= spai_qr_cache_bytes(n, W, WA), "spai_qr_factor: rcache too small");
  SPAI_CHECK_HIP(dispatch_factor(wc, max_rows, a_dtype == SPAI_DTYPE_F32, n, W, pat_idx, pat_act, WA, a_idx, a_val,
                                 rcache, (hipStream_t)stream));
  return SPAI_OK;
}

extern "C" int spai_fill_lines_qr_cached(int32_t n, int32_t line_begin, int32_t line_end, int32_t W, int32_t WA,
                                         const int32_t* pat_act, const double* rcache, const int32_t* line_entry,
                                         int32_t entries, int32_t B, const uint32_t* removed, int32_t words,
                                         int32_t word_base, void* m_out, int32_t m_dtype, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(m_dtype == SPAI_DTYPE_F32 || m_dtype == SPAI_DTYPE_F64, "spai_fill_lines_qr_cached: bad m_dtype");
  SPAI_CHECK_ARG(n >= 1 && line_begin >= 0 && line_end >= line_begin && line_end <= n && W >= 1 && WA >= 1 &&
                     B >= 1 && words >= 1 && word_base >= 0,
                 "spai_fill_lines_qr_cached: bad shape");
  SPAI_CHECK_ARG(workspace != nullptr, "spai_fill_lines_qr_cached: null workspace");
  const int32_t nl = line_end - line_begin;
  if (nl == 0) return SPAI_OK;
  SPAI_CHECK_ARG(pat_act && rcache && removed, "spai_fill_lines_qr_cached: null input");
  const int wc = qr_cache_class(W, WA);
  if (wc != 5 && wc != 7 && wc != 13) {
    set_error("spai_fill_lines_qr_cached: width class %d (W=%d WA=%d): the cached solve is compiled for 5, 7 and 13",
              wc, W, WA);
    return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_ARG(!line_entry || entries >= 1, "spai_fill_lines_qr_cached: a dictionary needs entries >= 1");
  const int32_t nparts = (nl + kQNT - 1) / kQNT;
  SPAI_CHECK_ARG(workspace_bytes >= sizeof(double) * (size_t)nparts * B,
                 "spai_fill_lines_qr_cached: workspace too small");
  double* partials = static_cast<double*>(workspace);
  // the (entry, mask) table after the partials, when the dictionary is small and the workspace has room
  double* mtab = nullptr;
  {
    const size_t off = align_up(sizeof(double) * (size_t)nparts * B);
    const size_t tb = sizeof(double) * (size_t)entries * (1u << kQTabW) * (kQTabW + 1);
    if (line_entry && wc <= kQTabW && entries <= kQTabMaxEntries && workspace_bytes >= off + tb)
      mtab = reinterpret_cast<double*>(static_cast<char*>(workspace) + off);
  }
  hipStream_t s = (hipStream_t)stream;
  const bool f64 = m_dtype == SPAI_DTYPE_F64;
  const hipError_t e =
      wc == 5   ? launch_solve<5>(f64, line_entry, entries, line_begin, line_end, W, pat_act, rcache, B, removed,
                                  words, word_base, m_out, partials, nparts, mtab, s)
      : wc == 7 ? launch_solve<7>(f64, line_entry, entries, line_begin, line_end, W, pat_act, rcache, B, removed,
                                  words, word_base, m_out, partials, nparts, nullptr, s)
                : launch_solve<13>(f64, line_entry, entries, line_begin, line_end, W, pat_act, rcache, B, removed,
                                   words, word_base, m_out, partials, nparts, nullptr, s);
  SPAI_CHECK_HIP(e);
  return SPAI_OK;
}

// ---- the dictionary of a per-line cache (the R cache, the Gram cache): its distinct line
// entries, bitwise, once per env on the host
extern "C" int spai_line_cache_dict(int32_t n, int32_t nq, int32_t elem_bytes, const void* cache, size_t cache_bytes,
                                    int32_t max_entries, void* dict, size_t dict_bytes, int32_t* line_entry,
                                    int32_t* entries_out, void* stream) {
  SPAI_CHECK_ARG(n >= 1 && nq >= 1 && (elem_bytes == 4 || elem_bytes == 8) && max_entries >= 1 && cache && dict &&
                     line_entry && entries_out,
                 "spai_line_cache_dict: bad arguments");
  const size_t groups = (size_t)(n + 63) / 64, eb = (size_t)nq * elem_bytes;
  SPAI_CHECK_ARG(cache_bytes >= groups * 64 * eb, "spai_line_cache_dict: cache too small");
  SPAI_CHECK_ARG(dict_bytes >= (size_t)max_entries * eb, "spai_line_cache_dict: dict too small");
  std::vector<unsigned char> h(groups * 64 * eb);
  hipStream_t s = (hipStream_t)stream;
  SPAI_CHECK_HIP(hipMemcpyAsync(h.data(), cache, h.size(), hipMemcpyDeviceToHost, s));
  SPAI_CHECK_HIP(hipStreamSynchronize(s));
  // open addressing over FNV-1a hashes of the entries' bytes; equal entries compared bitwise
  size_t cap = 1;
  while (cap < 2 * (size_t)std::min<int64_t>(n, (int64_t)max_entries + 1)) cap <<= 1;
  std::vector<int32_t> slot(cap, -1);
  std::vector<unsigned char> uniq, e(eb);
  std::vector<int32_t> ent(n);
  int32_t count = 0;
  for (int32_t j = 0; j < n; ++j) {
    // value q of line j sits at ((j / 64) * nq + q) * 64 + j % 64 (blocks of 64 lines)
    const unsigned char* g = h.data() + ((size_t)(j >> 6) * nq * 64 + (j & 63)) * elem_bytes;
    for (int q = 0; q < nq; ++q) std::memcpy(e.data() + (size_t)q * elem_bytes, g + (size_t)q * 64 * elem_bytes, elem_bytes);
    uint64_t hv = 1469598103934665603ull;
    for (size_t k = 0; k < eb; ++k) hv = (hv ^ e[k]) * 1099511628211ull;
    size_t i = hv & (cap - 1);
    for (;;) {
      const int32_t u = slot[i];
      if (u < 0 || std::memcmp(uniq.data() + (size_t)u * eb, e.data(), eb) == 0) break;
      i = (i + 1) & (cap - 1);
    }
    if (slot[i] < 0) {
      if (count == max_entries) {  // too many distinct entries: the caller keeps the full cache
        *entries_out = max_entries + 1;
        return SPAI_OK;
      }
      slot[i] = count++;
      uniq.insert(uniq.end(), e.begin(), e.end());
    }
    ent[j] = slot[i];
  }
  SPAI_CHECK_HIP(hipMemcpy(dict, uniq.data(), uniq.size(), hipMemcpyHostToDevice));
  SPAI_CHECK_HIP(hipMemcpy(line_entry, ent.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice));
  *entries_out = count;
  return SPAI_OK;
}
