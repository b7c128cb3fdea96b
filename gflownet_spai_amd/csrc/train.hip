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
    case 4: k_lstm_fwd<4><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, h_last, states); break;
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
    case 4: k_lstm_bwd<4><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, dh_last, grad); break;
    case 8: k_lstm_bwd<8><<<g, kLstmNT, 0, s>>>(B, traj, ldt, lengths, T, w_ih, w_hh, b_ih, b_hh, states, dh_last, grad); break;
    default:
      set_error("spai_lstm_backward: hidden_dim %d not compiled (2, 4, 8)", H);
      return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
