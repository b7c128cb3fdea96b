// Training-side kernels for gfx950 (the TB loss, the backward policy
// and the optimizer step consume the hot path's outputs on the device).
//
// 1. Gradient of the logged forward probabilities w.r.t. the policy logits.
//    The trajectory of sample b lists its removed actions a_0 .. a_{k-1} and then the
//    terminal E; step t is the masked softmax of policy.py:65-73 over the actions still
//    available, so with w_a = exp(l_a - lmax) and R_t = (untouched mass) + sum_{s>=t} w_{a_s}
//        p_t = w_{a_t} / R_t,   d log p_t / d l_a = [a = a_t] - w_a [a available at t] / R_t.
//    Given gp_t = dL/dp_t (the TB loss, gflownet/utils.py:228-278, differentiates
//    log(p + eps)), G_t = gp_t p_t and H_t = G_t / R_t = gp_t p_t^2 / w_{a_t}:
//        dL/dl_{a_t} += G_t - w_{a_t} S_t            S_t = sum_{s<=t} H_s (inclusive)
//        dL/dl_a     += -w_a S_last                 a untouched (never chosen, a < E)
//    because a logged action a_s is available at every step t <= s and an untouched one at
//    every step.  O(T + E) per sample instead of autograd through [B, E+1] temporaries.
//      k_lpg_part    per (4096-position chunk, sample): fixed-order fp64 sum of H
//      k_lpg_scan    per sample: chunk bases (sequential, fixed order) and S_last
//      k_lpg_dense   per action: the untouched terms of every sample (fixed b order)
//      k_lpg_scatter per chunk of one sample (launched per sample in b order when the logits
//                    are shared, so the read-modify-writes never race): S_t and the logged terms
//      k_lpg_out     fp64 accumulator -> fp32 gradient
//
// 2. BackwardPolicy's LSTM (policy.py:75-129: nn.LSTM(input 1, hidden H), input = the action
//    id as a float, packed to each trajectory's n_b entries != -1) — the recurrence is a chain
//    of n_b dependent steps, so one thread runs one sample with the weights in registers;
//    the next 16 inputs are loaded while the current 16 steps compute.  Gate order i, f, g, o
//    (torch).  k_lstm_fwd keeps (h_t, c_t) of every step for k_lstm_bwd, which runs the
//    steps backwards (BPTT) with fp64 gradient accumulators and writes one gradient row per
//    sample (summed over samples by the caller in a fixed order).
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kGNT = 256;
constexpr int kGPer = 16;
constexpr int kGChunk = kGNT * kGPer;  // positions per block (16 consecutive per thread)
constexpr int kScanNT = 64;

// exp(l - lm) to ~1 ulp of fp32: the difference is exact in fp64, exp(hi + lo) = exp(hi)(1 + lo)
__device__ __forceinline__ double weight(float l, float lm) {
  const double d = (double)l - (double)lm;
  const float hi = (float)d, lo = (float)(d - (double)hi);
  const float e = expf(hi);
  return (double)fmaf(e, lo, e);
}

struct LpgArgs {
  const float* logits;
  int64_t bstride;
  int32_t E;
  const float* lmax;
  const int64_t* actions;
  int64_t lda;
  int32_t T;
  const float* p;
  int64_t ldp;
  const float* gp;
  int64_t ldg;
};

// the 16 positions of this thread: H_t (and G_t, w_{a_t}, a_t) in fp64
__device__ __forceinline__ void lpg_terms(const LpgArgs& g, int b, int t0, int64_t* a, double* G, double* H,
                                          double* w) {
  const float lm = g.lmax[b];
  const float* lg = g.logits + (int64_t)b * g.bstride;
#pragma unroll
  for (int i = 0; i < kGPer; ++i) {
    const int t = t0 + i;
    a[i] = t < g.T ? g.actions[(int64_t)b * g.lda + t] : -1;
  }
#pragma unroll
  for (int i = 0; i < kGPer; ++i) {
    const int t = t0 + i;
    G[i] = H[i] = w[i] = 0.0;
    if (a[i] >= 0 && a[i] <= g.E) {
      const double pt = g.p[(int64_t)b * g.ldp + t];
      const double gt = g.gp[(int64_t)b * g.ldg + t];
      const double wt = weight(lg[a[i]], lm);
      G[i] = gt * pt;
      H[i] = wt > 0.0 ? G[i] * pt / wt : 0.0;
      w[i] = wt;
    }
  }
}

__global__ __launch_bounds__(kGNT) void k_lpg_part(LpgArgs g, int32_t nchunk, double* __restrict__ part) {
  const int b = blockIdx.y, c = blockIdx.x;
  int64_t a[kGPer];
  double G[kGPer], H[kGPer], w[kGPer];
  lpg_terms(g, b, c * kGChunk + threadIdx.x * kGPer, a, G, H, w);
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kGPer; ++i) s += H[i];
  __shared__ double sred[kGNT / 64];
  s = block_sum<kGNT>(s, sred);
  if (threadIdx.x == 0) part[(int64_t)b * nchunk + c] = s;
}

// chunk bases in chunk order (one lane per sample; a few hundred chunks)
__global__ __launch_bounds__(kScanNT) void k_lpg_scan(int32_t B, int32_t nchunk, const double* __restrict__ part,
                                                      double* __restrict__ base, double* __restrict__ slast) {
  const int b = blockIdx.x * kScanNT + threadIdx.x;
  if (b >= B) return;
  double s = 0.0;
  for (int c = 0; c < nchunk; ++c) {
    base[(int64_t)b * nchunk + c] = s;
    s += part[(int64_t)b * nchunk + c];
  }
  slast[b] = s;
}

// untouched actions: acc[a] = sum_b -w_{a,b} S_last[b]   (a < E, bit a of sample b clear)
// shared logits: one [E+1] row, samples summed in order; per-sample logits: row b each.
__global__ __launch_bounds__(kGNT) void k_lpg_dense(LpgArgs g, int32_t B, const uint32_t* __restrict__ removed,
                                                    int32_t words, const double* __restrict__ slast,
                                                    double* __restrict__ acc) {
  const int64_t a = (int64_t)blockIdx.x * kGNT + threadIdx.x;
  if (a > g.E) return;
  const int64_t E1 = (int64_t)g.E + 1;
  if (g.bstride == 0) {
    const float l = g.logits[a];
    double s = 0.0;
    for (int b = 0; b < B; ++b) {
      const bool untouched = a < g.E && !((removed[(int64_t)b * words + (a >> 5)] >> (a & 31)) & 1u);
      if (untouched) s -= weight(l, g.lmax[b]) * slast[b];
    }
    acc[a] = s;
  } else {
    for (int b = 0; b < B; ++b) {
      const bool untouched = a < g.E && !((removed[(int64_t)b * words + (a >> 5)] >> (a & 31)) & 1u);
      acc[(int64_t)b * E1 + a] = untouched ? -weight(g.logits[(int64_t)b * g.bstride + a], g.lmax[b]) * slast[b] : 0.0;
    }
  }
}

// logged actions of sample b0 + blockIdx.y: acc[row + a_t] += G_t - w_{a_t} S_t
__global__ __launch_bounds__(kGNT) void k_lpg_scatter(LpgArgs g, int32_t b0, int32_t nchunk,
                                                      const double* __restrict__ base, double* __restrict__ acc) {
  const int b = b0 + blockIdx.y, c = blockIdx.x;
  int64_t a[kGPer];
  double G[kGPer], H[kGPer], w[kGPer];
  lpg_terms(g, b, c * kGChunk + threadIdx.x * kGPer, a, G, H, w);
  double loc = 0.0;
#pragma unroll
  for (int i = 0; i < kGPer; ++i) loc += H[i];
  // exclusive scan of the thread sums (fixed order)
  double incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(incl, o, kWave);
    if ((threadIdx.x & 63) >= o) incl += y;
  }
  __shared__ double sw[kGNT / 64];
  if ((threadIdx.x & 63) == 63) sw[threadIdx.x >> 6] = incl;
  __syncthreads();
  double s = base[(int64_t)b * nchunk + c];
#pragma unroll
  for (int q = 0; q < kGNT / 64; ++q)
    if (q < (int)(threadIdx.x >> 6)) s += sw[q];
  s += incl - loc;
  double* row = acc + (g.bstride == 0 ? 0 : (int64_t)b * ((int64_t)g.E + 1));
#pragma unroll
  for (int i = 0; i < kGPer; ++i) {
    s += H[i];
    if (a[i] >= 0 && a[i] <= g.E) row[a[i]] += G[i] - w[i] * s;
  }
}

__global__ __launch_bounds__(kGNT) void k_lpg_out(int64_t n, const double* __restrict__ acc, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kGNT + threadIdx.x;
  if (i < n) out[i] = (float)acc[i];
}

// ------------------------------------------------------------------ LSTM
constexpr int kLstmNT = 64;
constexpr int kLstmPre = 16;  // inputs loaded ahead of the recurrence

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

template <int H>
struct LstmW {
  float wih[4 * H], whh[4 * H][H], bias[4 * H];
  __device__ __forceinline__ void load(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh) {
#pragma unroll
    for (int r = 0; r < 4 * H; ++r) {
      wih[r] = w_ih[r];
      bias[r] = b_ih[r] + b_hh[r];
#pragma unroll
      for (int k = 0; k < H; ++k) whh[r][k] = w_hh[r * H + k];
    }
  }
  // activated gates (i, f, g, o) for input x and previous h
  __device__ __forceinline__ void gates(float x, const float* h, float* gt) const {
#pragma unroll
    for (int r = 0; r < 4 * H; ++r) {
      float v = fmaf(wih[r], x, bias[r]);
#pragma unroll
      for (int k = 0; k < H; ++k) v = fmaf(whh[r][k], h[k], v);
      gt[r] = (r >= 2 * H && r < 3 * H) ? tanhf(v) : sigm(v);
    }
  }
};

template <int H>
__global__ __launch_bounds__(kLstmNT) void k_lstm_fwd(int32_t B, const int64_t* __restrict__ traj, int64_t ldt,
                                                      const int32_t* __restrict__ lengths, int32_t T,
                                                      const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                                      const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                      float* __restrict__ h_last, float* __restrict__ states) {
  const int b = blockIdx.x * kLstmNT + threadIdx.x;
  if (b >= B) return;
  LstmW<H> W;
  W.load(w_ih, w_hh, b_ih, b_hh);
  const int n = min(lengths[b], T);
  const int64_t* tr = traj + (int64_t)b * ldt;
  float h[H], c[H];
#pragma unroll
  for (int k = 0; k < H; ++k) h[k] = c[k] = 0.0f;
  int64_t cur[kLstmPre], nxt[kLstmPre];
#pragma unroll
  for (int i = 0; i < kLstmPre; ++i) cur[i] = i < n ? tr[i] : 0;
  for (int t0 = 0; t0 < n; t0 += kLstmPre) {
#pragma unroll
    for (int i = 0; i < kLstmPre; ++i) nxt[i] = t0 + kLstmPre + i < n ? tr[t0 + kLstmPre + i] : 0;
#pragma unroll
    for (int i = 0; i < kLstmPre; ++i) {
      if (t0 + i >= n) break;
      float gt[4 * H];
      W.gates((float)cur[i], h, gt);
#pragma unroll
      for (int k = 0; k < H; ++k) {
        c[k] = fmaf(gt[H + k], c[k], gt[k] * gt[2 * H + k]);
        h[k] = gt[3 * H + k] * tanhf(c[k]);
      }
      if (states != nullptr) {
        float* st = states + ((int64_t)b * T + t0 + i) * 2 * H;
#pragma unroll
        for (int k = 0; k < H; ++k) {
          st[k] = h[k];
          st[H + k] = c[k];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kLstmPre; ++i) cur[i] = nxt[i];
  }
#pragma unroll
  for (int k = 0; k < H; ++k) h_last[(int64_t)b * H + k] = h[k];
}

// grad row per sample: d w_ih [4H] | d w_hh [4H][H] | d bias [4H] (= d b_ih = d b_hh), fp64.
// One 64-lane block per sample: the lanes stage the next kBwdC steps (inputs, (h, c)) from
// HBM into LDS while lane 0 runs the current kBwdC steps backwards from the other buffer,
// leaving the gate gradients of each step in LDS; then every lane folds the chunk into its
// share of the fp64 weight-gradient accumulators (off the serial chain).
constexpr int kBwdC = 64;
template <int H>
__global__ __launch_bounds__(kLstmNT) void k_lstm_bwd(int32_t B, const int64_t* __restrict__ traj, int64_t ldt,
                                                      const int32_t* __restrict__ lengths, int32_t T,
                                                      const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                                      const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                      const float* __restrict__ states,
                                                      const float* __restrict__ dh_last, double* __restrict__ grad) {
  constexpr int R = 4 * H, S = 2 * H, NG = 2 * R + R * H;
  constexpr int kPer = (kBwdC * S + kLstmNT - 1) / kLstmNT;  // state floats staged per lane
  constexpr int kAcc = (NG + kLstmNT - 1) / kLstmNT;         // gradient entries per lane
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n = min(lengths[b], T);
  const int64_t* tr = traj + (int64_t)b * ldt;
  const float* st = states + (int64_t)b * T * S;
  // buffer q holds steps [t0 - 1, t0 + kBwdC): x of the kBwdC steps and (h, c) of kBwdC + 1
  __shared__ float s_x[2][kBwdC];
  __shared__ float s_st[2][(kBwdC + 1) * S];
  __shared__ float s_da[kBwdC][R];
  auto load = [&](int t0, float& xr, float* sr) {  // lane's share of chunk [t0, t0 + kBwdC)
    const int t = t0 + lane;
    xr = (t >= 0 && t < n) ? (float)tr[t] : 0.0f;
#pragma unroll
    for (int i = 0; i < kPer + 1; ++i) {
      const int e = i * kLstmNT + lane;  // element of the (kBwdC + 1) * S window starting at step t0 - 1
      const int ts = t0 - 1 + e / S;
      sr[i] = (e < (kBwdC + 1) * S && ts >= 0 && ts < n) ? st[(int64_t)ts * S + e % S] : 0.0f;
    }
  };
  auto store = [&](int q, float xr, const float* sr) {
    s_x[q][lane] = xr;
#pragma unroll
    for (int i = 0; i < kPer + 1; ++i) {
      const int e = i * kLstmNT + lane;
      if (e < (kBwdC + 1) * S) s_st[q][e] = sr[i];
    }
  };
  const int nchunk = (n + kBwdC - 1) / kBwdC;
  float xr, sr[kPer + 1];
  if (nchunk > 0) {
    load((nchunk - 1) * kBwdC, xr, sr);
    store(0, xr, sr);
  }
  __syncthreads();
  LstmW<H> W;
  W.load(w_ih, w_hh, b_ih, b_hh);
  float dh[H], dc[H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    dh[k] = dh_last[(int64_t)b * H + k];
    dc[k] = 0.0f;
  }
  double acc[kAcc];
#pragma unroll
  for (int i = 0; i < kAcc; ++i) acc[i] = 0.0;
  for (int j = nchunk - 1; j >= 0; --j) {
    const int q = (nchunk - 1 - j) & 1;
    const int t0 = j * kBwdC, cnt = min(n, t0 + kBwdC) - t0;
    if (j > 0) load((j - 1) * kBwdC, xr, sr);  // in flight while lane 0 computes
    if (lane == 0) {
      for (int o = cnt - 1; o >= 0; --o) {  // step t0 + o: (h, c)_{t-1} at window row o, (h, c)_t at row o + 1
        const float x = s_x[q][o];
        float hp[H], cp[H], ct[H];
#pragma unroll
        for (int k = 0; k < H; ++k) {
          hp[k] = s_st[q][o * S + k];
          cp[k] = s_st[q][o * S + H + k];
          ct[k] = s_st[q][(o + 1) * S + H + k];
        }
        float gt[R];
        W.gates(x, hp, gt);
        float da[R];
#pragma unroll
        for (int k = 0; k < H; ++k) {
          const float ig = gt[k], fg = gt[H + k], gg = gt[2 * H + k], og = gt[3 * H + k];
          const float tc = tanhf(ct[k]);
          const float dcc = dc[k] + dh[k] * og * (1.0f - tc * tc);
          da[k] = dcc * gg * ig * (1.0f - ig);
          da[H + k] = dcc * cp[k] * fg * (1.0f - fg);
          da[2 * H + k] = dcc * ig * (1.0f - gg * gg);
          da[3 * H + k] = dh[k] * tc * og * (1.0f - og);
          dc[k] = dcc * fg;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) s_da[o][r] = da[r];
#pragma unroll
        for (int k = 0; k < H; ++k) {
          float v = 0.0f;
#pragma unroll
          for (int r = 0; r < R; ++r) v = fmaf(W.whh[r][k], da[r], v);
          dh[k] = v;
        }
      }
    }
    __syncthreads();
    // entry e: d w_ih[r] (e < R), d w_hh[r][k] (R <= e < R + R H), d bias[r]; steps in descending order
#pragma unroll
    for (int i = 0; i < kAcc; ++i) {
      const int e = i * kLstmNT + lane;
      if (e < NG) {
        const int r = e < R ? e : (e < R + R * H ? (e - R) / H : e - R - R * H);
        const int k = (e - R) % H;
        for (int o = cnt - 1; o >= 0; --o) {
          const float in = e < R ? s_x[q][o] : (e < R + R * H ? s_st[q][o * S + k] : 1.0f);
          acc[i] += (double)s_da[o][r] * (double)in;
        }
      }
    }
    __syncthreads();
    if (j > 0) store(q ^ 1, xr, sr);
    __syncthreads();
  }
  double* g = grad + (int64_t)b * NG;
#pragma unroll
  for (int i = 0; i < kAcc; ++i) {
    const int e = i * kLstmNT + lane;
    if (e < NG) g[e] = acc[i];
  }
}

// ------------------------------------------------------------------ LSTM, H = 4 (the reference's size)
// A step of one sample is 16 gate rows: one wave runs 4 samples, one 16-lane DPP row each.
// Lane r of a row owns gate row q*H + k (unit k = r >> 2, gate type q = r & 3), so a unit's
// four gates sit in one quad: quad_perm broadcasts hand i, f, g, o to the quad, which then
// updates (c_k, h_k) redundantly; the recurrent product needs the other units' h, fetched
// by row rotations (row_ror 4, 8, 12) against weights pre-rotated per lane at load time.
// ~25 VALU instructions on the serial chain per step instead of ~1000 for a scalar step.
// The rotation direction of row_ror is probed once (lane id through row_ror:1).
constexpr int kH4 = 4;
constexpr int kPre4 = 16;  // steps of inputs prefetched ahead

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fsig(float y) { return frcp(1.0f + __expf(-y)); }
__device__ __forceinline__ float ftanh(float y) { return fmaf(2.0f, fsig(2.0f * y), -1.0f); }

struct Lane4 {
  int r, k, q, d;  // lane in row, unit, gate type, row_ror:1 source offset (1 or 15)
  __device__ __forceinline__ void init() {
    r = threadIdx.x & 15;
    k = r >> 2;
    q = r & 3;
    const int probe = __builtin_amdgcn_update_dpp(0, r, 0x121, 0xF, 0xF, false);  // row_ror:1
    d = (r - probe) & 15;
  }
  // unit whose h row_ror(4m) brings to this lane
  __device__ __forceinline__ int unit_rot(int m) const { return (k - m * d) & 3; }
  // lane whose value row_ror(m) brings to this lane
  __device__ __forceinline__ int lane_rot(int m) const { return (r - m * d) & 15; }
};

__device__ __forceinline__ float gate_act(float z, int q) {
  const float s = fsig(q == 2 ? 2.0f * z : z);
  return q == 2 ? fmaf(2.0f, s, -1.0f) : s;
}

// pre-activation of this lane's gate row from x and the quad-resident h
__device__ __forceinline__ float gate_z(float wx, float bb, const float* wr, float x, float h) {
  float z = fmaf(wx, x, bb);
  z = fmaf(wr[0], h, z);
  z = fmaf(wr[1], dppf<0x124>(h), z);  // row_ror:4
  z = fmaf(wr[2], dppf<0x128>(h), z);  // row_ror:8
  z = fmaf(wr[3], dppf<0x12C>(h), z);  // row_ror:12
  return z;
}

__global__ __launch_bounds__(64) void k_lstm_fwd4(int32_t B, const int64_t* __restrict__ traj, int64_t ldt,
                                                  const int32_t* __restrict__ lengths, int32_t T,
                                                  const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                                  const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                  float* __restrict__ h_last, float* __restrict__ states) {
  constexpr int H = kH4;
  Lane4 L;
  L.init();
  const int b = blockIdx.x * 4 + (threadIdx.x >> 4);
  const bool live = b < B;
  const int bb = live ? b : B - 1;
  const int row = L.q * H + L.k;
  const float wx = w_ih[row], bs = b_ih[row] + b_hh[row];
  float wr[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) wr[m] = w_hh[row * H + L.unit_rot(m)];
  const int n = live ? min(lengths[bb], T) : 0;
  int nmax = n;  // the wave runs to its longest row; finished rows hold their state
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o, kWave));
  const int64_t* tr = traj + (int64_t)bb * ldt;
  float* st = states ? states + (int64_t)bb * T * 2 * H : nullptr;
  float h = 0.0f, c = 0.0f;
  float xc[kPre4], xn[kPre4];
#pragma unroll
  for (int i = 0; i < kPre4; ++i) xc[i] = i < n ? (float)tr[i] : 0.0f;
  for (int t0 = 0; t0 < nmax; t0 += kPre4) {
#pragma unroll
    for (int i = 0; i < kPre4; ++i) xn[i] = t0 + kPre4 + i < n ? (float)tr[t0 + kPre4 + i] : 0.0f;
#pragma unroll
    for (int i = 0; i < kPre4; ++i) {
      const int t = t0 + i;
      const float a = gate_act(gate_z(wx, bs, wr, xc[i], h), L.q);
      const float ig = dppf<0x00>(a), fg = dppf<0x55>(a), gg = dppf<0xAA>(a), og = dppf<0xFF>(a);  // quad_perm
      const float cn = fmaf(fg, c, ig * gg);
      const float hn = og * ftanh(cn);
      const bool act = t < n;
      c = act ? cn : c;
      h = act ? hn : h;
      if (st != nullptr && act && L.q < 2) st[(int64_t)t * 2 * H + L.q * H + L.k] = L.q == 0 ? h : c;
    }
#pragma unroll
    for (int i = 0; i < kPre4; ++i) xc[i] = xn[i];
  }
  if (live && L.q == 0) h_last[(int64_t)b * H + L.k] = h;
}

__global__ __launch_bounds__(64) void k_lstm_bwd4(int32_t B, const int64_t* __restrict__ traj, int64_t ldt,
                                                  const int32_t* __restrict__ lengths, int32_t T,
                                                  const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                                  const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                  const float* __restrict__ states,
                                                  const float* __restrict__ dh_last, double* __restrict__ grad) {
  constexpr int H = kH4, R = 4 * H, NG = 2 * R + R * H;
  Lane4 L;
  L.init();
  const int b = blockIdx.x * 4 + (threadIdx.x >> 4);
  const bool live = b < B;
  const int bb = live ? b : B - 1;
  const int row = L.q * H + L.k;
  const float wx = w_ih[row], bs = b_ih[row] + b_hh[row];
  float wr[4], wt[16];
#pragma unroll
  for (int m = 0; m < 4; ++m) wr[m] = w_hh[row * H + L.unit_rot(m)];
#pragma unroll
  for (int m = 0; m < 16; ++m) {  // W_hh[row of the lane row_ror(m) reads][k]
    const int lr = L.lane_rot(m);
    wt[m] = w_hh[((lr & 3) * H + (lr >> 2)) * H + L.k];
  }
  const int n = live ? min(lengths[bb], T) : 0;
  int nmax = n;
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o, kWave));
  const int64_t* tr = traj + (int64_t)bb * ldt;
  const float* st = states + (int64_t)bb * T * 2 * H;
  float dh = live ? dh_last[(int64_t)b * H + L.k] : 0.0f, dc = 0.0f;
  double gx = 0.0, gbias = 0.0, gh[4] = {0.0, 0.0, 0.0, 0.0};
  // step t needs x_t, (h, c)_{t-1} of unit k, c_t of unit k; t descends from nmax - 1
  auto ld = [&](int t, float& x, float& hp, float& cp) {
    x = (t >= 0 && t < n) ? (float)tr[t] : 0.0f;
    hp = (t >= 1 && t - 1 < n) ? st[(int64_t)(t - 1) * 2 * H + L.k] : 0.0f;
    cp = (t >= 1 && t - 1 < n) ? st[(int64_t)(t - 1) * 2 * H + H + L.k] : 0.0f;
  };
  float ct = (nmax - 1 < n && nmax >= 1) ? st[(int64_t)(nmax - 1) * 2 * H + H + L.k] : 0.0f;
  float xc[kPre4], hc[kPre4], cc[kPre4], xn[kPre4], hn[kPre4], cn[kPre4];
#pragma unroll
  for (int i = 0; i < kPre4; ++i) ld(nmax - 1 - i, xc[i], hc[i], cc[i]);
  for (int t0 = nmax - 1; t0 >= 0; t0 -= kPre4) {
#pragma unroll
    for (int i = 0; i < kPre4; ++i) ld(t0 - kPre4 - i, xn[i], hn[i], cn[i]);
#pragma unroll
    for (int i = 0; i < kPre4; ++i) {
      const int t = t0 - i;
      if (t < 0) break;  // wave-uniform
      const float x = xc[i], hp = hc[i], cp = cc[i];
      const float a = gate_act(gate_z(wx, bs, wr, x, hp), L.q);
      const float ig = dppf<0x00>(a), fg = dppf<0x55>(a), gg = dppf<0xAA>(a), og = dppf<0xFF>(a);
      const float tc = ftanh(ct);
      const float dcc = fmaf(dh * og, 1.0f - tc * tc, dc);
      const float P = L.q == 0 ? dcc * gg : (L.q == 1 ? dcc * cp : (L.q == 2 ? dcc * ig : dh * tc));
      const float D = L.q == 2 ? 1.0f - a * a : a * (1.0f - a);
      const bool act = t < n;
      const float da = act ? P * D : 0.0f;
      // dh_{t-1}[k] = sum over the 16 gate rows of W_hh[row][k] * da_row
      float v = wt[0] * da;
      v = fmaf(wt[1], dppf<0x121>(da), v);
      v = fmaf(wt[2], dppf<0x122>(da), v);
      v = fmaf(wt[3], dppf<0x123>(da), v);
      v = fmaf(wt[4], dppf<0x124>(da), v);
      v = fmaf(wt[5], dppf<0x125>(da), v);
      v = fmaf(wt[6], dppf<0x126>(da), v);
      v = fmaf(wt[7], dppf<0x127>(da), v);
      v = fmaf(wt[8], dppf<0x128>(da), v);
      v = fmaf(wt[9], dppf<0x129>(da), v);
      v = fmaf(wt[10], dppf<0x12A>(da), v);
      v = fmaf(wt[11], dppf<0x12B>(da), v);
      v = fmaf(wt[12], dppf<0x12C>(da), v);
      v = fmaf(wt[13], dppf<0x12D>(da), v);
      v = fmaf(wt[14], dppf<0x12E>(da), v);
      v = fmaf(wt[15], dppf<0x12F>(da), v);
      const float h1 = dppf<0x124>(hp), h2 = dppf<0x128>(hp), h3 = dppf<0x12C>(hp);
      const double dd = (double)da;
      gx = fma(dd, (double)x, gx);
      gbias += dd;
      gh[0] = fma(dd, (double)hp, gh[0]);
      gh[1] = fma(dd, (double)h1, gh[1]);
      gh[2] = fma(dd, (double)h2, gh[2]);
      gh[3] = fma(dd, (double)h3, gh[3]);
      dc = act ? dcc * fg : dc;
      dh = act ? v : dh;
      ct = act || t - 1 < n ? cp : ct;
    }
#pragma unroll
    for (int i = 0; i < kPre4; ++i) {
      xc[i] = xn[i];
      hc[i] = hn[i];
      cc[i] = cn[i];
    }
  }
  if (live) {
    double* g = grad + (int64_t)b * NG;
    g[row] = gx;
#pragma unroll
    for (int m = 0; m < 4; ++m) g[R + row * H + L.unit_rot(m)] = gh[m];
    g[R + R * H + row] = gbias;
  }
}

}  // namespace
}  // namespace spai

using namespace spai;

static int nchunks(int32_t T) { return (T + kGChunk - 1) / kGChunk; }

extern "C" size_t spai_logp_grad_workspace_bytes(int32_t E, int32_t T, int32_t B, int32_t per_sample) {
  if (E < 0 || T <= 0 || B <= 0) return 0;
  Carve c(nullptr);
  const int nc = nchunks(T);
  c.take<double>((size_t)B * nc);                                 // part
  c.take<double>((size_t)B * nc);                                 // base
  c.take<double>(B);                                              // slast
  c.take<double>((size_t)(per_sample ? B : 1) * ((size_t)E + 1));  // accumulator
  return c.off;
}

extern "C" int spai_logp_grad(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                              const int64_t* actions, int64_t lda, int32_t T, const float* probs, int64_t ldp,
                              const float* gprobs, int64_t ldg, const uint32_t* removed, int32_t words,
                              float* grad_out, void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(logits && lmax && actions && probs && gprobs && removed && grad_out, "spai_logp_grad: null pointer");
  SPAI_CHECK_ARG(E >= 0 && B > 0 && T > 0, "spai_logp_grad: bad shape E=%d B=%d T=%d", E, B, T);
  SPAI_CHECK_ARG(lda >= T && ldp >= T && ldg >= T, "spai_logp_grad: leading dimensions must be >= T");
  SPAI_CHECK_ARG(bstride == 0 || bstride >= (int64_t)E + 1, "spai_logp_grad: bstride must be 0 or >= E+1");
  SPAI_CHECK_ARG(words >= (E + 31) / 32, "spai_logp_grad: removal bitmap has %d words < ceil(E/32)", words);
  const int per_sample = bstride != 0;
  SPAI_CHECK_ARG(workspace && workspace_bytes >= spai_logp_grad_workspace_bytes(E, T, B, per_sample),
                 "spai_logp_grad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int nc = nchunks(T);
  Carve c(workspace);
  double* part = c.take<double>((size_t)B * nc);
  double* base = c.take<double>((size_t)B * nc);
  double* slast = c.take<double>(B);
  const int64_t nacc = (int64_t)(per_sample ? B : 1) * ((int64_t)E + 1);
  double* acc = c.take<double>((size_t)nacc);
  LpgArgs g{logits, bstride, E, lmax, actions, lda, T, probs, ldp, gprobs, ldg};
  k_lpg_part<<<dim3(nc, B), kGNT, 0, s>>>(g, nc, part);
  k_lpg_scan<<<(B + kScanNT - 1) / kScanNT, kScanNT, 0, s>>>(B, nc, part, base, slast);
  k_lpg_dense<<<(int)(((int64_t)E + 1 + kGNT - 1) / kGNT), kGNT, 0, s>>>(g, B, removed, words, slast, acc);
  if (per_sample) {
    k_lpg_scatter<<<dim3(nc, B), kGNT, 0, s>>>(g, 0, nc, base, acc);
  } else {
    for (int b = 0; b < B; ++b) k_lpg_scatter<<<dim3(nc, 1), kGNT, 0, s>>>(g, b, nc, base, acc);
  }
  k_lpg_out<<<(int)((nacc + kGNT - 1) / kGNT), kGNT, 0, s>>>(nacc, acc, grad_out);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_lstm_forward(int32_t B, int32_t H, const int64_t* traj, int64_t ldt, const int32_t* lengths,
                                 int32_t T, const float* w_ih, const float* w_hh, const float* b_ih,
                                 const float* b_hh, float* h_last, float* states, void* stream) {
  SPAI_CHECK_ARG(traj && lengths && w_ih && w_hh && b_ih && b_hh && h_last, "spai_lstm_forward: null pointer");
  SPAI_CHECK_ARG(B > 0 && T > 0 && ldt >= T, "spai_lstm_forward: bad shape B=%d T=%d ldt=%lld", B, T, (long long)ldt);
  hipStream_t s = (hipStream_t)stream;
  const int g = (B + kLstmNT - 1) / kLstmNT;
  switch (H) {
    case 2: k_lstm_fwd<2><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, h_last, states); break;
    case 4: k_lstm_fwd4<<<(B + 3) / 4, 64, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, h_last, states); break;
    case 8: k_lstm_fwd<8><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, h_last, states); break;
    default:
      set_error("spai_lstm_forward: hidden_dim %d not compiled (2, 4, 8)", H);
      return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_lstm_backward(int32_t B, int32_t H, const int64_t* traj, int64_t ldt, const int32_t* lengths,
                                  int32_t T, const float* w_ih, const float* w_hh, const float* b_ih,
                                  const float* b_hh, const float* states, const float* dh_last, double* grad,
                                  void* stream) {
  SPAI_CHECK_ARG(traj && lengths && w_ih && w_hh && b_ih && b_hh && states && dh_last && grad,
                 "spai_lstm_backward: null pointer");
  SPAI_CHECK_ARG(B > 0 && T > 0 && ldt >= T, "spai_lstm_backward: bad shape B=%d T=%d", B, T);
  hipStream_t s = (hipStream_t)stream;
  const int g = B;  // one block per sample
  switch (H) {
    case 2: k_lstm_bwd<2><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, dh_last, grad); break;
    case 4: k_lstm_bwd4<<<(B + 3) / 4, 64, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, dh_last, grad); break;
    case 8: k_lstm_bwd<8><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, dh_last, grad); break;
    default:
      set_error("spai_lstm_backward: hidden_dim %d not compiled (2, 4, 8)", H);
      return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
