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
// The recurrence is a chain of n_b dependent steps per sample, so the forward and the BPTT
// adjoint chain each run one sample per wave on a 16-lane DPP row (exec = lanes 0-15) and
// carry nothing else; all off-chain work runs as parallel passes over 16-step blocks.
//
// Forward (k_lstm_fwd4): lane r owns gate row q*H + k (unit k = r >> 2, gate q = r & 3), so a
// unit's four gates sit in one quad: quad_perm broadcasts i, f, g, o to the quad, which
// updates (c_k, h_k) redundantly; W_hh h takes the other units' h through row_ror 4, 8, 12
// against weights pre-rotated per lane.  The activation's pre-scale (-log2 e, twice that
// for tanh) is folded into the weights, so a gate is a two-deep fma tree -> v_exp -> v_rcp; the
// quad receives the raw sigmoids and applies g = 2 s_g - 1 and tanh inside two fmas (cell4, hid4).
// Only a checkpoint (h, c) per 16-step block is stored ("states" = [B][ceil(T/16)][2H]);
// the inputs are prefetched three blocks ahead.  Fwd4Step restates a step for one thread
// with the same instructions in the same order (bit-identical states), so the backward
// passes recompute any block from its checkpoint.
//
// Backward: the adjoint s_t = (dh_t, dc+_t) of BPTT obeys a LINEAR recurrence whose
// coefficients depend only on the forward states:
//    dc_t = dc+_t + gamma dh_t,  gamma = o (1 - tanh^2 c_t)
//    dz_{q,k} = A_{q,k} dh_t[k] + B_{q,k} dc+_t[k]   (A = alpha gamma, B = alpha for i, f, g;
//                                                    A = tanh(c_t) o (1 - o), B = 0 for o)
//    dc+_{t-1} = f gamma dh_t + f dc+_t,   dh_{t-1} = W_hh^T dz
//  k_lstm_coef4  (parallel, one thread per block) recomputes the block's states and folds
//                W_hh into per-lane chain coefficients;
//  k_lstm_adj4   runs the chain: per step 1 load, 2 fma, 3 row-rotated adds, 1 quad
//                broadcast, 2 fma; it stores the adjoint once per block;
//  k_lstm_grad4  (parallel, one thread per block) recomputes states and the adjoint inside
//                the block from the two checkpoints, sums the gradient in fp64 in a fixed
//                order; k_lstm_gsum4 adds the per-block partial rows in order.
// Chain lane (k, j) [r = 4k + j] carries the partial of target unit u = (k - j) & 3:
//    p = a1 dh[k] + a2 dc[k],  a1 = sum_q W_hh[q,k][u] A_{q,k},  a2 = sum_q W_hh[q,k][u] B_{q,k};
// lane 4u collects lanes (4u + 5m) mod 16, m = 1..3 (one per other quad) by row_ror, and a
// quad_perm broadcast returns dh_{t-1}[u] to its quad.  The row_ror direction is probed once
// per kernel (ror_sign).
constexpr int kH4 = 4;
constexpr int kBlk4 = 16;        // steps per block (checkpoint interval, prefetch unit)
constexpr int kGrad4NT = 256;    // k_lstm_grad4 threads per block
constexpr int kGrad4Blocks = 64; // k_lstm_grad4 blocks per sample
constexpr int kNG4 = 8 * kH4 + 4 * kH4 * kH4;  // 96 gradient entries per sample
constexpr float kLog2e = 1.4426950408889634f;

// DPP move within a row whose 16 lanes are all active (row_ror, quad_perm): every source is
// valid, so the old value is never read and need not be materialised
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// sigmoid of y given -log2(e) y
__device__ __forceinline__ float fsig_pre(float ny) { return frcp(1.0f + fexp2(ny)); }
__device__ __forceinline__ float ftanh(float y) { return fmaf(2.0f, fsig_pre((-2.0f * kLog2e) * y), -1.0f); }

// +1 if row_ror:N hands lane i the value of lane i + N, -1 if that of lane i - N.  Lane 0 must
// be active; the DPP result goes straight to readfirstlane (no arithmetic it could fold into).
__device__ __forceinline__ int ror_sign() {
  const int src = __builtin_amdgcn_update_dpp(0, (int)(threadIdx.x & 15), 0x121, 0xF, 0xF, false);  // row_ror:1
  return __builtin_amdgcn_readfirstlane(src) == 1 ? 1 : -1;
}

__device__ __forceinline__ int nblocks4(int n) { return (n + kBlk4 - 1) / kBlk4; }

// a gate row's scaled weights, as the forward lane (q, k) holds them
struct Row4 {
  float wx, bs, wr[4];
  __device__ __forceinline__ void load(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                                       int q, int k, int sg) {
    const int row = q * kH4 + k;
    const float sc = (q == 2 ? -2.0f : -1.0f) * kLog2e;
    wx = w_ih[row] * sc;
    bs = (b_ih[row] + b_hh[row]) * sc;
#pragma unroll
    for (int m = 0; m < 4; ++m) wr[m] = w_hh[row * kH4 + ((k + m * sg) & 3)] * sc;  // unit row_ror(4m) brings
  }
  // sigmoid of the (pre-scaled) gate pre-activation: sigma(z) for i, f, o; sigma(2z) for g.
  // Two-deep tree: (own unit, +2sg) and (+sg, +3sg), the units row_ror 4, 8, 12 bring.
  __device__ __forceinline__ float sig(float x, float h0, float h1, float h2, float h3) const {
    float z1 = fmaf(wr[0], h0, fmaf(wx, x, bs));
    float z2 = wr[1] * h1;
    z1 = fmaf(wr[2], h2, z1);
    z2 = fmaf(wr[3], h3, z2);
    return fsig_pre(z1 + z2);
  }
};

// the cell update from the four gate sigmoids (s_g = sigma(2 z_g), so g = 2 s_g - 1):
//   c' = f c + i (2 s_g - 1) = fma(2i, s_g, fma(f, c, -i)),  h' = o tanh(c') = fma(2o, sigma(2c'), -o)
__device__ __forceinline__ float cell4(float si, float sf, float sgg, float c) {
  return fmaf(si + si, sgg, fmaf(sf, c, -si));
}
__device__ __forceinline__ float hid4(float so, float c) {
  return fmaf(so + so, fsig_pre((-2.0f * kLog2e) * c), -so);
}

// one thread's bit-identical restatement of k_lstm_fwd4's step (all 16 rows)
struct Fwd4Step {
  Row4 row[16];  // [q * 4 + k]
  __device__ __forceinline__ void load(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                                       int sg) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) row[q * 4 + k].load(w_ih, w_hh, b_ih, b_hh, q, k, sg);
  }
  // gate values g[q][k] (i, f, g = tanh, o) and the step update of h, c
  __device__ __forceinline__ void step(float x, float* h, float* c, float (*g)[4], int sg) const {
    float hn[4], cn[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float sq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        sq[q] = row[q * 4 + k].sig(x, h[k], h[(k + sg) & 3], h[(k + 2 * sg) & 3], h[(k + 3 * sg) & 3]);
      cn[k] = cell4(sq[0], sq[1], sq[2], c[k]);
      hn[k] = hid4(sq[3], cn[k]);
      g[0][k] = sq[0], g[1][k] = sq[1], g[2][k] = fmaf(2.0f, sq[2], -1.0f), g[3][k] = sq[3];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) h[k] = hn[k], c[k] = cn[k];
  }
};

__global__ __launch_bounds__(64) void k_lstm_fwd4(const int64_t* __restrict__ traj, int64_t ldt,
                                                  const int32_t* __restrict__ lengths, int32_t T,
                                                  const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                                  const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                  float* __restrict__ h_last, float* __restrict__ states) {
  if (threadIdx.x >= 16) return;
  const int r = threadIdx.x, k = r >> 2, q = r & 3, sg = ror_sign();
  const int b = blockIdx.x;
  Row4 R;
  R.load(w_ih, w_hh, b_ih, b_hh, q, k, sg);
  const int n = min(lengths[b], T);
  const int32_t* x32 = reinterpret_cast<const int32_t*>(traj + (int64_t)b * ldt);  // ids < 2^31: low words
  float* ck = states ? states + (int64_t)b * nblocks4(T) * 2 * kH4 + (q & 1) * kH4 + k : nullptr;
  float h = 0.0f, c = 0.0f;
  auto step = [&](int32_t xi) {
    const float a = R.sig((float)xi, h, dppf<0x124>(h), dppf<0x128>(h), dppf<0x12C>(h));  // row_ror 4, 8, 12
    const float si = dppf<0x00>(a), sf = dppf<0x55>(a), sgg = dppf<0xAA>(a), so = dppf<0xFF>(a);  // quad_perm
    c = cell4(si, sf, sgg, c);
    h = hid4(so, c);
  };
  auto ckpt = [&](int m) {
    if (ck) ck[(int64_t)m * 2 * kH4] = (q & 1) ? c : h;
  };
  const int nb = n / kBlk4;
  auto ldblk = [&](int32_t* dst, int m) {
    if (nb == 0) return;  // no full block: nothing in the ring is read
    const int32_t* p = x32 + 2 * kBlk4 * min(m, nb - 1);
#pragma unroll
    for (int i = 0; i < kBlk4; ++i) dst[i] = p[2 * i];
  };
  auto runblk = [&](const int32_t* xs, int m) {
    ckpt(m);
#pragma unroll
    for (int i = 0; i < kBlk4; ++i) step(xs[i]);
  };
  int32_t x0[kBlk4], x1[kBlk4], x2[kBlk4];
  ldblk(x0, 0);
  ldblk(x1, 1);
  ldblk(x2, 2);
  int m = 0;
  for (; m + 3 <= nb; m += 3) {
    runblk(x0, m);
    ldblk(x0, m + 3);
    runblk(x1, m + 1);
    ldblk(x1, m + 4);
    runblk(x2, m + 2);
    ldblk(x2, m + 5);
  }
  if (m < nb) runblk(x0, m);
  if (m + 1 < nb) runblk(x1, m + 1);
  if (nb * kBlk4 < n) {
    ckpt(nb);
    for (int t = nb * kBlk4; t < n; ++t) step(x32[2 * t]);
  }
  if (q == 0) h_last[(int64_t)b * kH4 + k] = h;
}

__device__ __forceinline__ void load_ckpt4(const float* ck, float* h, float* c) {
  const float4 h4 = reinterpret_cast<const float4*>(ck)[0], c4 = reinterpret_cast<const float4*>(ck)[1];
  h[0] = h4.x, h[1] = h4.y, h[2] = h4.z, h[3] = h4.w;
  c[0] = c4.x, c[1] = c4.y, c[2] = c4.z, c[3] = c4.w;
}

// per step, A and B of each gate row: dz_{q,k} = A dh[k] + B dc+[k]; gamma of each unit
__device__ __forceinline__ void adj_coef4(const float (*g)[4], const float* cp, const float* ct, float* A, float* Bc,
                                          float* gam) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float i = g[0][k], f = g[1][k], gg = g[2][k], o = g[3][k];
    const float tc = ftanh(ct[k]);
    gam[k] = o * (1.0f - tc * tc);
    const float ai = gg * i * (1.0f - i), af = cp[k] * f * (1.0f - f), ag = i * (1.0f - gg * gg);
    A[0 * 4 + k] = ai * gam[k];
    A[1 * 4 + k] = af * gam[k];
    A[2 * 4 + k] = ag * gam[k];
    A[3 * 4 + k] = tc * o * (1.0f - o);
    Bc[0 * 4 + k] = ai;
    Bc[1 * 4 + k] = af;
    Bc[2 * 4 + k] = ag;
    Bc[3 * 4 + k] = 0.0f;
  }
}

// coef [B][T][16 lanes] float4 (a1, a2, f gamma, f) for chain lane (k, j), target u = (k - j) & 3
__global__ __launch_bounds__(256) void k_lstm_coef4(const int64_t* __restrict__ traj, int64_t ldt,
                                                    const int32_t* __restrict__ lengths, int32_t T,
                                                    const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                                    const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                    const float* __restrict__ states, float4* __restrict__ coef) {
  const int sg = ror_sign();  // before any lane leaves
  const int b = blockIdx.y;
  const int n = min(lengths[b], T);
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nblocks4(n)) return;
  Fwd4Step F;
  F.load(w_ih, w_hh, b_ih, b_hh, sg);
  float whh[64];
#pragma unroll
  for (int e = 0; e < 64; ++e) whh[e] = w_hh[e];
  float h[4], c[4];
  load_ckpt4(states + ((int64_t)b * nblocks4(T) + m) * 8, h, c);
  const int32_t* x32 = reinterpret_cast<const int32_t*>(traj + (int64_t)b * ldt);
  float4* out = coef + ((int64_t)b * T + (int64_t)m * kBlk4) * 16;
  const int steps = min(kBlk4, n - m * kBlk4);
  for (int i = 0; i < steps; ++i) {
    float cp[4] = {c[0], c[1], c[2], c[3]}, g[4][4];
    F.step((float)x32[2 * (m * kBlk4 + i)], h, c, g, sg);
    float A[16], Bc[16], gam[4];
    adj_coef4(g, cp, c, A, Bc, gam);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = r >> 2, u = (k - (r & 3)) & 3;
      float a1 = 0.0f, a2 = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float wqu = whh[(q * 4 + k) * 4 + u];
        a1 = fmaf(wqu, A[q * 4 + k], a1);
        a2 = fmaf(wqu, Bc[q * 4 + k], a2);
      }
      out[i * 16 + r] = make_float4(a1, a2, g[1][k] * gam[k], g[1][k]);
    }
  }
}

// the adjoint chain; cka [B][ceil(T/16)][8] = (dh, dc+) entering step min(16m + 15, n - 1)
template <bool PLUS>  // PLUS: row_ror:N hands lane i the value of lane i + N
__device__ __forceinline__ void adj_chain4(const float4* __restrict__ cf, float* __restrict__ ck, int n, int r,
                                           float dh, float dc) {
  constexpr int N1 = PLUS ? 5 : 11, N2 = PLUS ? 10 : 6, N3 = PLUS ? 15 : 1;
  const int j = r & 3;
  float* ckl = ck + (j & 1) * 4 + (r >> 2);
  // carried: s with dh = quad_perm[0,0,0,0](s) (dh itself at the start: equal across the quad)
  float s = dh;
  auto step = [&](const float4 c) {
    const float d = dppf<0x00>(s);
    const float p = fmaf(c.x, d, c.y * dc);
    dc = fmaf(c.z, d, c.w * dc);
    // two-deep sum: the three rotations read p independently (no DPP hazard between them)
    s = (p + dppf<0x120 + N1>(p)) + (dppf<0x120 + N2>(p) + dppf<0x120 + N3>(p));
  };
  auto ckpt = [&](int m) { ckl[(int64_t)m * 8] = (j & 1) ? dc : dppf<0x00>(s); };
  const int nb = n / kBlk4;
  if (nb * kBlk4 < n) {  // the partial top block first
    ckpt(nb);
    for (int t = n - 1; t >= nb * kBlk4; --t) step(cf[(int64_t)t * 16]);
  }
  auto ldblk = [&](float4* dst, int m) {  // coefficients of steps 16m + 15 .. 16m
    if (nb == 0) return;
    const float4* p = cf + (int64_t)max(m, 0) * kBlk4 * 16;
#pragma unroll
    for (int i = 0; i < kBlk4; ++i) dst[i] = p[(kBlk4 - 1 - i) * 16];
  };
  auto runblk = [&](const float4* cs, int m) {
    ckpt(m);
#pragma unroll
    for (int i = 0; i < kBlk4; ++i) step(cs[i]);
  };
  float4 c0[kBlk4], c1[kBlk4], c2[kBlk4];
  ldblk(c0, nb - 1);
  ldblk(c1, nb - 2);
  ldblk(c2, nb - 3);
  int m = nb - 1;
  for (; m >= 2; m -= 3) {
    runblk(c0, m);
    ldblk(c0, m - 3);
    runblk(c1, m - 1);
    ldblk(c1, m - 4);
    runblk(c2, m - 2);
    ldblk(c2, m - 5);
  }
  if (m >= 0) runblk(c0, m);
  if (m >= 1) runblk(c1, m - 1);
}

__global__ __launch_bounds__(64) void k_lstm_adj4(const int32_t* __restrict__ lengths, int32_t T,
                                                  const float* __restrict__ dh_last, const float4* __restrict__ coef,
                                                  float* __restrict__ cka) {
  if (threadIdx.x >= 16) return;
  const int r = threadIdx.x, b = blockIdx.x;
  const int n = min(lengths[b], T);
  const float4* cf = coef + (int64_t)b * T * 16 + r;
  float* ck = cka + (int64_t)b * nblocks4(T) * 8;
  const float dh = dh_last[(int64_t)b * kH4 + (r >> 2)];
  if (ror_sign() == 1)
    adj_chain4<true>(cf, ck, n, r, dh, 0.0f);
  else
    adj_chain4<false>(cf, ck, n, r, dh, 0.0f);
}

// gradient partial rows [B][kGrad4Blocks][96]: block-strided threads, fp64 sums, fixed-order reductions
__global__ __launch_bounds__(kGrad4NT) void k_lstm_grad4(const int64_t* __restrict__ traj, int64_t ldt,
                                                         const int32_t* __restrict__ lengths, int32_t T,
                                                         const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                                                         const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                         const float* __restrict__ states,
                                                         const float* __restrict__ cka, double* __restrict__ part) {
  __shared__ double red[kGrad4NT / kWave][kNG4];
  const int sg = ror_sign();
  const int b = blockIdx.y;
  const int n = min(lengths[b], T);
  Fwd4Step F;
  F.load(w_ih, w_hh, b_ih, b_hh, sg);
  float whh[64];
#pragma unroll
  for (int e = 0; e < 64; ++e) whh[e] = w_hh[e];
  const int32_t* x32 = reinterpret_cast<const int32_t*>(traj + (int64_t)b * ldt);
  const int nbt = nblocks4(T);
  double gi[16], gb[16], gh[64];
#pragma unroll
  for (int e = 0; e < 16; ++e) gi[e] = gb[e] = 0.0;
#pragma unroll
  for (int e = 0; e < 64; ++e) gh[e] = 0.0;
  for (int m = blockIdx.x * kGrad4NT + threadIdx.x; m < nblocks4(n); m += kGrad4Blocks * kGrad4NT) {
    const int t0 = m * kBlk4, steps = min(kBlk4, n - t0);
    float hs[kBlk4 + 1][4], cs[kBlk4 + 1][4], xs[kBlk4];
    load_ckpt4(states + ((int64_t)b * nbt + m) * 8, hs[0], cs[0]);
#pragma unroll
    for (int i = 0; i < kBlk4; ++i) {
      if (i < steps) {
        float g[4][4];
        xs[i] = (float)x32[2 * (t0 + i)];
#pragma unroll
        for (int k = 0; k < 4; ++k) hs[i + 1][k] = hs[i][k], cs[i + 1][k] = cs[i][k];
        F.step(xs[i], hs[i + 1], cs[i + 1], g, sg);
      }
    }
    float dh[4], dc[4];
    load_ckpt4(cka + ((int64_t)b * nbt + m) * 8, dh, dc);
#pragma unroll
    for (int i = kBlk4 - 1; i >= 0; --i) {
      if (i < steps) {
        float hh[4] = {hs[i][0], hs[i][1], hs[i][2], hs[i][3]}, cc[4] = {cs[i][0], cs[i][1], cs[i][2], cs[i][3]};
        float g[4][4];
        F.step(xs[i], hh, cc, g, sg);  // gates of step t0 + i (h, c of step t0 + i - 1 in)
        float A[16], Bc[16], gam[4];
        adj_coef4(g, cs[i], cs[i + 1], A, Bc, gam);
        float dz[16];
#pragma unroll
        for (int row = 0; row < 16; ++row) {
          const int k = row & 3;
          dz[row] = fmaf(A[row], dh[k], Bc[row] * dc[k]);
          const double dd = (double)dz[row];
          gi[row] = fma(dd, (double)xs[i], gi[row]);
          gb[row] += dd;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) gh[row * 4 + jj] = fma(dd, (double)hs[i][jj], gh[row * 4 + jj]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float v = 0.0f;
#pragma unroll
          for (int row = 0; row < 16; ++row) v = fmaf(whh[row * 4 + k], dz[row], v);
          dc[k] = fmaf(g[1][k] * gam[k], dh[k], g[1][k] * dc[k]);
          dh[k] = v;
        }
      }
    }
  }
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  auto wsum = [&](double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
  };
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const double a = wsum(gi[e]), c = wsum(gb[e]);
    if (lane == 0) red[wv][e] = a, red[wv][80 + e] = c;
  }
#pragma unroll
  for (int e = 0; e < 64; ++e) {
    const double a = wsum(gh[e]);
    if (lane == 0) red[wv][16 + e] = a;
  }
  __syncthreads();
  if (threadIdx.x < kNG4) {
    double s = 0.0;
#pragma unroll
    for (int v = 0; v < kGrad4NT / kWave; ++v) s += red[v][threadIdx.x];
    part[((int64_t)b * kGrad4Blocks + blockIdx.x) * kNG4 + threadIdx.x] = s;
  }
}

__global__ __launch_bounds__(128) void k_lstm_gsum4(const double* __restrict__ part, double* __restrict__ grad) {
  const int b = blockIdx.x, e = threadIdx.x;
  if (e >= kNG4) return;
  double s = 0.0;
  for (int i = 0; i < kGrad4Blocks; ++i) s += part[((int64_t)b * kGrad4Blocks + i) * kNG4 + e];
  grad[(int64_t)b * kNG4 + e] = s;
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

extern "C" size_t spai_lstm_states_floats(int32_t B, int32_t H, int32_t T) {
  if (B <= 0 || T <= 0 || H <= 0) return 0;
  return H == kH4 ? (size_t)B * ((T + kBlk4 - 1) / kBlk4) * 2 * H : (size_t)B * T * 2 * H;
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
    case 4: k_lstm_fwd4<<<B, 64, 0, s>>>(traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, h_last, states); break;
    case 8: k_lstm_fwd<8><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, h_last, states); break;
    default:
      set_error("spai_lstm_forward: hidden_dim %d not compiled (2, 4, 8)", H);
      return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

// H = 4 backward workspace: chain coefficients, adjoint checkpoints, per-block gradient rows
static size_t lstm4_ws(int32_t B, int32_t T, float4** coef, float** adj, double** part, void* base) {
  Carve c(base);
  float4* cf = c.take<float4>((size_t)B * T * 16);
  float* ad = c.take<float>((size_t)B * ((T + kBlk4 - 1) / kBlk4) * 8);
  double* pt = c.take<double>((size_t)B * kGrad4Blocks * kNG4);
  if (coef) *coef = cf, *adj = ad, *part = pt;
  return c.off;
}

extern "C" size_t spai_lstm_backward_workspace_bytes(int32_t B, int32_t H, int32_t T) {
  if (H != kH4 || B <= 0 || T <= 0) return 0;
  return lstm4_ws(B, T, nullptr, nullptr, nullptr, nullptr);
}

extern "C" int spai_lstm_backward(int32_t B, int32_t H, const int64_t* traj, int64_t ldt, const int32_t* lengths,
                                  int32_t T, const float* w_ih, const float* w_hh, const float* b_ih,
                                  const float* b_hh, const float* states, const float* dh_last, double* grad,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(traj && lengths && w_ih && w_hh && b_ih && b_hh && states && dh_last && grad,
                 "spai_lstm_backward: null pointer");
  SPAI_CHECK_ARG(B > 0 && T > 0 && ldt >= T, "spai_lstm_backward: bad shape B=%d T=%d", B, T);
  hipStream_t s = (hipStream_t)stream;
  const int g = B;  // one block per sample
  switch (H) {
    case 2: k_lstm_bwd<2><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, dh_last, grad); break;
    case 4: {
      SPAI_CHECK_ARG(workspace && workspace_bytes >= spai_lstm_backward_workspace_bytes(B, H, T),
                     "spai_lstm_backward: workspace too small");
      float4* coef;
      float* adj;
      double* part;
      lstm4_ws(B, T, &coef, &adj, &part, workspace);
      k_lstm_coef4<<<dim3((T + 255) / 256, B), 256, 0, s>>>(traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, coef);
      k_lstm_adj4<<<B, 64, 0, s>>>(lengths, T, dh_last, coef, adj);
      k_lstm_grad4<<<dim3(kGrad4Blocks, B), kGrad4NT, 0, s>>>(traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states,
                                                              adj, part);
      k_lstm_gsum4<<<B, 128, 0, s>>>(part, grad);
      break;
    }
    case 8: k_lstm_bwd<8><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, dh_last, grad); break;
    default:
      set_error("spai_lstm_backward: hidden_dim %d not compiled (2, 4, 8)", H);
      return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
