// ForwardPolicy logits for gfx950 (reference: policy.py:14-73, BasePolicy + ForwardPolicy):
//     logits = fc(mean_pool(relu(GATv2_2(relu(GATv2_1(x))))))[:E+1]
// with the GATv2Conv semantics of PyG (heads 4 then 1, edge_dim 1, negative slope 0.2,
// self loops replaced by loops whose attribute is the mean of the node's incoming
// attributes, softmax over each target's incoming edges, concat heads, + bias):
//     s_ij^h   = att_h . leaky_relu(W_l x_j + W_r x_i + W_e a_ij)_h
//     alpha_ij = softmax_j(s_ij^h)            (over the incoming edges of target i)
//     out_i^h  = sum_j alpha_ij^h (W_l x_j + b_l)_h + bias_h
// The graph arrives as a CSR by target with the self loops already in place (built once
// per state graph by the host, gflownet_spai_amd/policy.py), so each target's softmax is
// a single pass over its row with an online (running max) normaliser.
//
//   k_gat1  one thread per node (hid <= 8; else per (node, head), 4 lanes per node):
//           layer-1 attention in registers; epilogue relu + the layer-2 input transforms
//           W_l2 h, W_r2 h (per-head partial products summed across a node's lanes in a
//           fixed order) -> [n][2*hid] fp32.
//   k_gat2  one thread per node: layer-2 attention over the gathered W_l2 h_j rows; epilogue
//           relu + the block's fp64 pooled sum.  k_pool sums the block partials in block
//           order (deterministic) into h = mean.
//   k_fc    one thread per action: logit_a = b_a + W_a . h (W row-major [actions][hid],
//           16-byte loads), the block max; k_max writes lmax.
// Cross-block reductions are separate one-block kernels, not last-block-done counters: on
// gfx950 a device-scope fence writes back the XCD's L2, which costs far more than a launch.
// Every kernel is bound by HBM / L2 gathers; the only products are hid-wide dot products
// per node or action (K <= 128, M = 1 for the fc), so there is no MFMA tile to fill.
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kNT = 256;
constexpr int kH1 = 4;  // BasePolicy.in_head (policy.py:20)

// Offsets of the packed GATv2 parameter blocks (host packs them in this order):
//   W_l [HC][F], b_l [HC], W_r [HC][F], b_r [HC], W_e [HC], att [HC], bias [HC]
__host__ __device__ constexpr int gat_params(int HC, int F) { return 2 * HC * F + 5 * HC; }

__device__ __forceinline__ float leaky(float v) { return v > 0.0f ? v : 0.2f * v; }

constexpr int kEdgeChunk = 8;  // edges of one target whose loads are issued together
constexpr int kCh1 = 4;        // k_gat1 chunk: fewer registers than kEdgeChunk (occupancy 6 waves/SIMD at hid 4)
constexpr int kRedNT = 1024;   // one-block reductions

// Online softmax step: fold score s with value row v[0..C) into (m, den, acc).
template <int C>
__device__ __forceinline__ void online_step(float s, const float* v, float& m, float& den, float* acc) {
  if (s > m) {  // rescale what was accumulated under the old maximum
    const float r = __expf(m - s);
    den = fmaf(den, r, 1.0f);
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = fmaf(acc[c], r, v[c]);
    m = s;
  } else {
    const float p = __expf(s - m);
    den += p;
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = fmaf(p, v[c], acc[c]);
  }
}

// Layer 1.  HPT heads per thread (4 for hid <= 8: one thread per node; 1 above: one thread
// per (node, head), the node's 4 lanes adjacent).  Per target: the edge ids, attributes
// and source features of up to kCh1 edges are loaded before any is used (one memory
// round trip per chunk instead of three per edge).  Latency-bound gathers: occupancy is the
// lever (hid 4, fin 1: 80 VGPRs, 6 waves/SIMD; 76 -> 57 us at C4).
template <int F, int C, int HPT>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(C <= 4 && F == 1 ? 6 : 1)))
void k_gat1(int32_t n, const float* __restrict__ x, const int32_t* __restrict__ rp,
                                              const int32_t* __restrict__ src, const float* __restrict__ ea,
                                              const float* __restrict__ p1, const float* __restrict__ p2,
                                              float* __restrict__ xlr2) {
  constexpr int HC = kH1 * C;  // layer-1 width (heads concatenated)
  constexpr int P1 = gat_params(HC, F);
  constexpr int L = kH1 / HPT;  // lanes per node
  constexpr int W2 = 2 * C * HC + 2 * C;  // W_l2, b_l2, W_r2, b_r2
  __shared__ float s1[P1];
  __shared__ float s2[W2];
  for (int i = threadIdx.x; i < P1; i += kNT) s1[i] = p1[i];
  for (int i = threadIdx.x; i < W2; i += kNT) s2[i] = p2[i];
  __syncthreads();
  const float* Wl = s1;
  const float* bl = Wl + HC * F;
  const float* Wr = bl + HC;
  const float* br = Wr + HC * F;
  const float* We = br + HC;
  const float* att = We + HC;
  const float* bias = att + HC;
  // the per-edge weights straight from the kernel argument: uniform addresses -> scalar
  // loads, SGPR operands (the LDS copies would be hoisted into ~50 VGPRs and cost occupancy)
  const float* gWl = p1;
  const float* gWe = p1 + 2 * HC * F + 2 * HC;
  const float* gatt = gWe + HC;

  const int64_t t = (int64_t)blockIdx.x * kNT + threadIdx.x;
  const int node = (int)(t / L), lane_h = (int)(t % L);
  const int hb = lane_h * HPT;  // first head of this thread
  const bool live = node < n;
  const int i = live ? node : n - 1;
  const int e0 = rp[i], e1 = rp[i + 1];
  float xi[F];
#pragma unroll
  for (int f = 0; f < F; ++f) xi[f] = x[(int64_t)i * F + f];
  float xr[HPT][C], acc[HPT][C], m[HPT], den[HPT];
#pragma unroll
  for (int q = 0; q < HPT; ++q) {
    m[q] = -INFINITY;
    den[q] = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int o = (hb + q) * C + c;
      float v = br[o];
#pragma unroll
      for (int f = 0; f < F; ++f) v = fmaf(Wr[o * F + f], xi[f], v);
      xr[q][c] = v;
      acc[q][c] = 0.0f;
    }
  }
  // Per chunk: all scores first, one maximum per head, then the weights: no data-dependent
  // rescaling branch per edge.  The aggregation is affine in the source features,
  //     sum_j p_j (W_l x_j + b_l) = W_l (sum_j p_j x_j) + b_l sum_j p_j,
  // so a head accumulates F weighted features and the weight sum instead of C products.
  float kc[HPT][C];  // b_l + W_r x_i: the per-target constant of every channel
#pragma unroll
  for (int q = 0; q < HPT; ++q)
#pragma unroll
    for (int c = 0; c < C; ++c) kc[q][c] = bl[(hb + q) * C + c] + xr[q][c];
  float sx[HPT][F];
#pragma unroll
  for (int q = 0; q < HPT; ++q)
#pragma unroll
    for (int f = 0; f < F; ++f) sx[q][f] = 0.0f;
  for (int eb = e0; eb < e1; eb += kCh1) {
    int js[kCh1];
    float as[kCh1], xj[kCh1][F];
#pragma unroll
    for (int k = 0; k < kCh1; ++k) {
      const int e = min(eb + k, e1 - 1);  // clamped: every load is in bounds, extras unused
      js[k] = src[e];
      as[k] = ea[e];
    }
#pragma unroll
    for (int k = 0; k < kCh1; ++k)
#pragma unroll
      for (int f = 0; f < F; ++f) xj[k][f] = x[(int64_t)js[k] * F + f];
    const int nv = min(kCh1, e1 - eb);
    float sc[kCh1][HPT];
    float mc[HPT];
#pragma unroll
    for (int q = 0; q < HPT; ++q) mc[q] = m[q];
#pragma unroll
    for (int k = 0; k < kCh1; ++k) {
#pragma unroll
      for (int q = 0; q < HPT; ++q) {
        float v = -INFINITY;
        if (k < nv) {
          v = 0.0f;
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const int o = (hb + q) * C + c;
            float z = fmaf(gWe[o], as[k], kc[q][c]);
#pragma unroll
            for (int f = 0; f < F; ++f) z = fmaf(gWl[o * F + f], xj[k][f], z);
            v = fmaf(gatt[o], leaky(z), v);
          }
        }
        sc[k][q] = v;
        mc[q] = fmaxf(mc[q], v);
      }
    }
#pragma unroll
    for (int q = 0; q < HPT; ++q) {  // rescale what earlier chunks accumulated (exp(-inf) = 0 first)
      const float r = __expf(m[q] - mc[q]);
      den[q] *= r;
#pragma unroll
      for (int f = 0; f < F; ++f) sx[q][f] *= r;
      m[q] = mc[q];
    }
#pragma unroll
    for (int k = 0; k < kCh1; ++k) {
      if (k < nv) {
#pragma unroll
        for (int q = 0; q < HPT; ++q) {
          const float pk = __expf(sc[k][q] - m[q]);
          den[q] += pk;
#pragma unroll
          for (int f = 0; f < F; ++f) sx[q][f] = fmaf(pk, xj[k][f], sx[q][f]);
        }
      }
    }
  }
  // acc[q][c] = sum_j p_j xl_j[c] from the affine form
#pragma unroll
  for (int q = 0; q < HPT; ++q)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int o = (hb + q) * C + c;
      float v = bl[o] * den[q];
#pragma unroll
      for (int f = 0; f < F; ++f) v = fmaf(Wl[o * F + f], sx[q][f], v);
      acc[q][c] = v;
    }
  // epilogue: relu(out) of this thread's heads, then its slice of W_l2 h1 and W_r2 h1
  const float* Wl2 = s2;
  const float* bl2 = Wl2 + C * HC;
  const float* Wr2 = bl2 + C;
  const float* br2 = Wr2 + C * HC;
  float out[2 * C];
#pragma unroll
  for (int o = 0; o < 2 * C; ++o) out[o] = 0.0f;
#pragma unroll
  for (int q = 0; q < HPT; ++q) {
    const float inv = den[q] > 0.0f ? 1.0f / den[q] : 0.0f;  // no incoming edge: out = bias (PyG)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int k = (hb + q) * C + c;
      const float h1 = fmaxf(fmaf(acc[q][c], inv, bias[k]), 0.0f);
#pragma unroll
      for (int o = 0; o < C; ++o) {
        out[o] = fmaf(Wl2[o * HC + k], h1, out[o]);
        out[C + o] = fmaf(Wr2[o * HC + k], h1, out[C + o]);
      }
    }
  }
  if constexpr (L == 4) {
    // sum over the node's 4 lanes by xor shuffles, (h0+h1)+(h2+h3) in every lane
#pragma unroll
    for (int k = 0; k < 2 * C; ++k) {
      const float a1 = __shfl_xor(out[k], 1, kWave);
      const float lo = (lane_h & 1) ? a1 + out[k] : out[k] + a1;
      const float a2 = __shfl_xor(lo, 2, kWave);
      out[k] = (lane_h & 2) ? a2 + lo : lo + a2;
    }
  }
  if (live) {
    float* dst = xlr2 + (int64_t)node * 2 * C;
    constexpr int per = 2 * C / L;  // components written by each lane of the node
#pragma unroll
    for (int k = 0; k < 2 * C; ++k)
      if (k / per == lane_h) dst[k] = out[k] + (k < C ? bl2[k] : br2[k - C]);
  }
}

// Layer 2 (one head), one thread per node: gathered W_l2 h_j rows (C floats, 16-byte
// loads), chunked like layer 1; epilogue relu + the block's fp64 pooled sum.
#ifndef GAT2_WPE4
#define GAT2_WPE4 7  // waves/SIMD of k_gat2 at hid 4 (66 VGPRs, no spills)
#endif
template <int C>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(C <= 4 ? GAT2_WPE4 : 1))) void k_gat2(int32_t n, const int32_t* __restrict__ rp,
                                              const int32_t* __restrict__ src, const float* __restrict__ ea,
                                              const float* __restrict__ p2, const float* __restrict__ xlr2,
                                              double* __restrict__ part) {
  constexpr int HC = kH1 * C;
  constexpr int CH = C <= 8 ? kEdgeChunk : 4;  // gathered rows held in registers per chunk
  const float* We = p2 + 2 * C * HC + 2 * C;
  const float* att = We + C;
  const float* bias = att + C;
  const int node = blockIdx.x * kNT + threadIdx.x;
  const bool live = node < n;
  const int i = live ? node : n - 1;
  const int e0 = rp[i], e1 = rp[i + 1];
  float xr[C], acc[C];
#pragma unroll
  for (int c4 = 0; c4 < C / 4; ++c4) {
    const float4 v = reinterpret_cast<const float4*>(xlr2 + (int64_t)i * 2 * C + C)[c4];
    xr[4 * c4] = v.x;
    xr[4 * c4 + 1] = v.y;
    xr[4 * c4 + 2] = v.z;
    xr[4 * c4 + 3] = v.w;
  }
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.0f;
  float m = -INFINITY, den = 0.0f;
  for (int eb = e0; eb < e1; eb += CH) {
    int js[CH];
    float as[CH], xl[CH][C];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int e = min(eb + k, e1 - 1);
      js[k] = src[e];
      as[k] = ea[e];
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const float4* row = reinterpret_cast<const float4*>(xlr2 + (int64_t)js[k] * 2 * C);
#pragma unroll
      for (int c4 = 0; c4 < C / 4; ++c4) {
        const float4 v = row[c4];
        xl[k][4 * c4] = v.x;
        xl[k][4 * c4 + 1] = v.y;
        xl[k][4 * c4 + 2] = v.z;
        xl[k][4 * c4 + 3] = v.w;
      }
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if (eb + k >= e1) break;
      float sc = 0.0f;
#pragma unroll
      for (int c = 0; c < C; ++c) sc = fmaf(att[c], leaky(xl[k][c] + xr[c] + We[c] * as[k]), sc);
      online_step<C>(sc, xl[k], m, den, acc);
    }
  }
  const float inv = den > 0.0f ? 1.0f / den : 0.0f;
  __shared__ double sred[kNT / 64][C];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    double v = live ? (double)fmaxf(fmaf(acc[c], inv, bias[c]), 0.0f) : 0.0;
    v = wave_sum(v);
    if (lane == 0) sred[wv][c] = v;
  }
  __syncthreads();
  if (threadIdx.x < C) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < kNT / 64; ++k) v += sred[k][threadIdx.x];
    part[(int64_t)blockIdx.x * C + threadIdx.x] = v;
  }
}

// pooled mean over all n nodes from the k_gat2 block partials [nblk][C]: thread t sums a
// contiguous run of blocks, then a fixed-order tree over the threads (deterministic)
template <int C>
__global__ __launch_bounds__(kRedNT) void k_pool(int32_t n, int32_t nblk, const double* __restrict__ part,
                                                 float* __restrict__ hpool) {
  const int per = (nblk + kRedNT - 1) / kRedNT;
  const int b0 = threadIdx.x * per, b1 = min(b0 + per, nblk);
  double v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) v[c] = 0.0;
#pragma unroll 8
  for (int b = b0; b < b1; ++b)
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] += part[(int64_t)b * C + c];
  __shared__ double sred[kRedNT / 64][C];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const double w = wave_sum(v[c]);
    if (lane == 0) sred[wv][c] = w;
  }
  __syncthreads();
  if (threadIdx.x < C) {
    double r = 0.0;
#pragma unroll
    for (int k = 0; k < kRedNT / 64; ++k) r += sred[k][threadIdx.x];
    hpool[threadIdx.x] = (float)(r / (double)n);
  }
}

#ifndef KFCPER
#define KFCPER 4
#endif
constexpr int kFcPer = KFCPER;  // actions per thread of k_fc (strided by kNT inside a block)

// The pooled embedding of the constant-row closed form (k_const_pool's arithmetic, same fmaf
// order): h1 = relu(W_l1 x0 + b_l1 + bias1), h = relu(W_l2 h1 + b_l2 + bias2).  Uniform loads
// (scalar unit); k_fc evaluates it in every thread instead of a separate one-block launch.
template <int F, int C>
__device__ __forceinline__ void const_pool(const float* __restrict__ x0, const float* __restrict__ p1,
                                           const float* __restrict__ p2, float (&hv)[C]) {
  constexpr int HC = kH1 * C;
  const float* bl = p1 + HC * F;
  const float* bias1 = p1 + 2 * HC * F + 5 * HC - HC;
  float h1[HC];
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    float v = bl[k];
#pragma unroll
    for (int f = 0; f < F; ++f) v = fmaf(p1[k * F + f], x0[f], v);
    h1[k] = fmaxf(v + bias1[k], 0.0f);
  }
  const float* bl2 = p2 + C * HC;
  const float* bias2 = p2 + 2 * C * HC + 5 * C - C;
#pragma unroll
  for (int o = 0; o < C; ++o) {
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < HC; ++k) v = fmaf(p2[o * HC + k], h1[k], v);
    hv[o] = fmaxf((v + bl2[o]) + bias2[o], 0.0f);
  }
}

template <int F, int C, bool kConst>
__global__ __launch_bounds__(kNT) void k_fc(int32_t na, const float* __restrict__ W, const float* __restrict__ b,
                                            const float* __restrict__ hpool, const float* __restrict__ x0,
                                            const float* __restrict__ p1, const float* __restrict__ p2,
                                            float* __restrict__ logits, float* __restrict__ pmax) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  float hv[C];
  if constexpr (kConst) {
    const_pool<F, C>(x0, p1, p2, hv);
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) hv[c] = hpool[c];
  }
  float l = -INFINITY;
  f4v q[kFcPer][C / 4];
  float bv[kFcPer];
  const int base = blockIdx.x * (kNT * kFcPer) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kFcPer; ++k) {  // all loads first: W is streamed once per rollout
    const int a = min(base + k * kNT, na - 1);
    const f4v* row = reinterpret_cast<const f4v*>(W + (int64_t)a * C);
#pragma unroll
    for (int c4 = 0; c4 < C / 4; ++c4) q[k][c4] = __builtin_nontemporal_load(row + c4);
    bv[k] = __builtin_nontemporal_load(b + a);
  }
#pragma unroll
  for (int k = 0; k < kFcPer; ++k) {
    const int a = base + k * kNT;
    float v = bv[k];
#pragma unroll
    for (int c4 = 0; c4 < C / 4; ++c4) {
      v = fmaf(q[k][c4].x, hv[4 * c4], v);
      v = fmaf(q[k][c4].y, hv[4 * c4 + 1], v);
      v = fmaf(q[k][c4].z, hv[4 * c4 + 2], v);
      v = fmaf(q[k][c4].w, hv[4 * c4 + 3], v);
    }
    if (a < na) {
      logits[a] = v;
      l = fmaxf(l, v);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) l = fmaxf(l, __shfl_xor(l, o, kWave));
  __shared__ float sm[kNT / 64];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = sm[0];
#pragma unroll
    for (int k = 1; k < kNT / 64; ++k) v = fmaxf(v, sm[k]);
    pmax[blockIdx.x] = v;
  }
}

// lmax[0..B-1] = max of the k_fc block maxima (a max: independent of the order)
__global__ __launch_bounds__(kRedNT) void k_max(int32_t nblk, const float* __restrict__ pmax,
                                                float* __restrict__ lmax, int32_t B) {
  __shared__ float sm[kRedNT / 64];
  float v = -INFINITY;
  for (int k = threadIdx.x; k < nblk; k += kRedNT) v = fmaxf(v, pmax[k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = sm[0];
#pragma unroll
  for (int k = 1; k < kRedNT / 64; ++k) r = fmaxf(r, sm[k]);
  for (int bb = threadIdx.x; bb < B; bb += kRedNT) lmax[bb] = r;
}

// ------------------------------------------------------------------ constant node features
// state_to_data builds x = ones(2N, 1) (gflownet.py:247): every source a target aggregates
// carries the same W_l x_j + b_l, and the softmax weights of a target sum to 1 (its self
// loop guarantees an in-edge), so each layer's output is the same for every node:
//     h1 = relu(W_l1 x0 + b_l1 + bias1),  h2 = relu(W_l2 h1 + b_l2 + bias2),  pool = h2.
// The whole GATv2 stack then collapses to these two small products (one block), and only
// the fc GEMV streams memory.  The general kernels above remain the path for any other x.

// flag stays 1 iff every row of x [n][F] equals row 0 (a benign race: writers only store 0).
__global__ __launch_bounds__(kNT) void k_rows_const(int32_t n, int32_t F, const float* __restrict__ x,
                                                    int32_t* __restrict__ flag) {
  const int64_t total = (int64_t)n * F;
  bool same = true;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT)
    same &= x[i] == x[i % F];
  if (__any(!same) && (threadIdx.x & 63) == 0) *flag = 0;
}

struct PolicyWs {
  float* xlr2;
  double* part;
  float* hpool;
  float* pmax;
};

int fc_blocks(int32_t na) { return (na + kNT * kFcPer - 1) / (kNT * kFcPer); }

size_t policy_ws(int32_t n, int32_t hid, int32_t na, void* base, PolicyWs* w) {
  Carve c(base);
  const int g2 = (n + kNT - 1) / kNT;
  w->xlr2 = c.take<float>((size_t)n * 2 * hid);
  w->part = c.take<double>((size_t)g2 * hid);
  w->hpool = c.take<float>(hid);
  w->pmax = c.take<float>(fc_blocks(na));
  return c.off;
}

template <int F, int C>
void launch_policy(int32_t n, const float* x, const int32_t* rp, const int32_t* src, const float* ea, const float* p1,
                   const float* p2, const float* fw, const float* fb, int32_t na, float* logits, float* lmax,
                   int32_t B, const PolicyWs& w, hipStream_t s, bool const_rows) {
  constexpr int HPT = C <= 8 ? kH1 : 1;
  const int64_t t1 = (int64_t)n * (kH1 / HPT);
  const int g2 = (n + kNT - 1) / kNT, gf = fc_blocks(na);
  if (const_rows) {  // the pooled embedding is computed inside k_fc (const_pool)
    k_fc<F, C, true><<<gf, kNT, 0, s>>>(na, fw, fb, w.hpool, x, p1, p2, logits, w.pmax);
  } else {
    k_gat1<F, C, HPT><<<(int)((t1 + kNT - 1) / kNT), kNT, 0, s>>>(n, x, rp, src, ea, p1, p2, w.xlr2);
    k_gat2<C><<<g2, kNT, 0, s>>>(n, rp, src, ea, p2, w.xlr2, w.part);
    k_pool<C><<<1, kRedNT, 0, s>>>(n, g2, w.part, w.hpool);
    k_fc<F, C, false><<<gf, kNT, 0, s>>>(na, fw, fb, w.hpool, x, p1, p2, logits, w.pmax);
  }
  if (B > 0) k_max<<<1, kRedNT, 0, s>>>(gf, w.pmax, lmax, B);  // B == 0: the caller reduces w.pmax (= lmax)
}

template <int F>
bool dispatch_hid(int32_t hid, int32_t n, const float* x, const int32_t* rp, const int32_t* src, const float* ea,
                  const float* p1, const float* p2, const float* fw, const float* fb, int32_t na, float* logits,
                  float* lmax, int32_t B, const PolicyWs& w, hipStream_t s, bool cr) {
  switch (hid) {
    case 4: launch_policy<F, 4>(n, x, rp, src, ea, p1, p2, fw, fb, na, logits, lmax, B, w, s, cr); return true;
    case 8: launch_policy<F, 8>(n, x, rp, src, ea, p1, p2, fw, fb, na, logits, lmax, B, w, s, cr); return true;
    case 16: launch_policy<F, 16>(n, x, rp, src, ea, p1, p2, fw, fb, na, logits, lmax, B, w, s, cr); return true;
    case 32: launch_policy<F, 32>(n, x, rp, src, ea, p1, p2, fw, fb, na, logits, lmax, B, w, s, cr); return true;
    default: return false;
  }
}

#include "policy_bwd.inc"

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" size_t spai_policy_params(int32_t layer, int32_t fin, int32_t hid) {
  if (layer == 1) return (size_t)gat_params(kH1 * hid, fin);
  if (layer == 2) return (size_t)gat_params(hid, kH1 * hid);
  return 0;
}

extern "C" size_t spai_policy_workspace_bytes(int32_t n_nodes, int32_t hid, int32_t num_actions) {
  PolicyWs w;
  return policy_ws(n_nodes, hid, num_actions, nullptr, &w);
}

extern "C" int spai_policy_rows_constant(int32_t n_nodes, int32_t fin, const float* x, int32_t* flag, void* stream) {
  SPAI_CHECK_ARG(x && flag && n_nodes > 0 && fin > 0, "spai_policy_rows_constant: bad argument");
  hipStream_t s = (hipStream_t)stream;
  // *flag = 1 (0x00000001) by a byte memset of its low byte after zeroing: no pageable host
  // source, so the call is capturable in a HIP graph and never stages through the host
  SPAI_CHECK_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
  SPAI_CHECK_HIP(hipMemsetAsync(flag, 1, 1, s));
  const int64_t total = (int64_t)n_nodes * fin;
  const int grid = (int)std::min<int64_t>(2048, (total + kNT - 1) / kNT);
  k_rows_const<<<grid, kNT, 0, s>>>(n_nodes, fin, x, flag);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int32_t spai_policy_lmax_parts(int32_t num_actions) { return num_actions > 0 ? fc_blocks(num_actions) : 0; }

extern "C" int spai_policy_logits(int32_t n_nodes, int32_t fin, int32_t hid, const float* x, const int32_t* rowptr,
                                  const int32_t* src, const float* eattr, const float* gat1, const float* gat2,
                                  const float* fc_w, const float* fc_b, int32_t num_actions, float* logits,
                                  float* lmax, int32_t B, int32_t const_rows, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  SPAI_CHECK_ARG(x && gat1 && gat2 && fc_w && fc_b && logits && lmax && (const_rows || (rowptr && src && eattr)),
                 "spai_policy_logits: null pointer");
  SPAI_CHECK_ARG(n_nodes > 0 && num_actions > 0 && B >= 0, "spai_policy_logits: bad shape");
  SPAI_CHECK_ARG(((uintptr_t)fc_w & 15) == 0, "spai_policy_logits: fc weight must be 16-byte aligned");
  SPAI_CHECK_ARG(workspace && workspace_bytes >= spai_policy_workspace_bytes(n_nodes, hid, num_actions),
                 "spai_policy_logits: workspace too small");
  PolicyWs w;
  policy_ws(n_nodes, hid, num_actions, workspace, &w);
  if (B == 0) w.pmax = lmax;  // deferred maximum: the fc block maxima go to the caller's buffer
  hipStream_t s = (hipStream_t)stream;
  bool ok = false;
  switch (fin) {
    case 1: ok = dispatch_hid<1>(hid, n_nodes, x, rowptr, src, eattr, gat1, gat2, fc_w, fc_b, num_actions, logits,
                                 lmax, B, w, s, const_rows != 0); break;
    case 2: ok = dispatch_hid<2>(hid, n_nodes, x, rowptr, src, eattr, gat1, gat2, fc_w, fc_b, num_actions, logits,
                                 lmax, B, w, s, const_rows != 0); break;
    case 4: ok = dispatch_hid<4>(hid, n_nodes, x, rowptr, src, eattr, gat1, gat2, fc_w, fc_b, num_actions, logits,
                                 lmax, B, w, s, const_rows != 0); break;
    default: break;
  }
  if (!ok) {
    set_error("spai_policy_logits: no kernel for node_features=%d hidden_dim=%d (compiled: 1/2/4 x 4/8/16/32)", fin,
              hid);
    return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" size_t spai_policy_backward_workspace_bytes(int32_t n_nodes, int32_t n_edges, int32_t fin, int32_t hid,
                                                       int32_t num_actions) {
  PolicyWs w;
  PolicyBwdWs v;
  const size_t a = align_up(policy_ws(n_nodes, hid, num_actions, nullptr, &w));
  return a + policy_bwd_ws(n_nodes, n_edges, fin, hid, num_actions, nullptr, &v);
}

extern "C" int spai_policy_backward(int32_t n_nodes, int32_t n_edges, int32_t fin, int32_t hid, const float* x,
                                    const int32_t* rowptr, const int32_t* src, const float* eattr,
                                    const int32_t* rev_ptr, const int32_t* rev_eid, const float* gat1,
                                    const float* gat2, const float* fc_w, int32_t num_actions, const float* dlogits,
                                    float* g_gat1, float* g_gat2, float* g_fc_w, float* g_fc_b, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  SPAI_CHECK_ARG(x && rowptr && src && eattr && rev_ptr && rev_eid && gat1 && gat2 && fc_w && dlogits && g_gat1 &&
                     g_gat2 && g_fc_w && g_fc_b,
                 "spai_policy_backward: null pointer");
  SPAI_CHECK_ARG(n_nodes > 0 && n_edges >= 0 && num_actions > 0, "spai_policy_backward: bad shape");
  if ((fin != 1 && fin != 2 && fin != 4) || (hid != 4 && hid != 8)) {
    set_error("spai_policy_backward: no kernel for node_features=%d hidden_dim=%d (compiled: 1/2/4 x 4/8)", fin, hid);
    return SPAI_ERR_UNSUPPORTED;
  }
  SPAI_CHECK_ARG(workspace && workspace_bytes >= spai_policy_backward_workspace_bytes(n_nodes, n_edges, fin, hid,
                                                                                      num_actions),
                 "spai_policy_backward: workspace too small");
  PolicyWs w;
  PolicyBwdWs v;
  const size_t a = align_up(policy_ws(n_nodes, hid, num_actions, workspace, &w));
  policy_bwd_ws(n_nodes, n_edges, fin, hid, num_actions, static_cast<char*>(workspace) + a, &v);
  hipStream_t s = (hipStream_t)stream;
  switch (fin) {
    case 1: dispatch_bwd<1>(hid, n_nodes, x, rowptr, src, eattr, rev_ptr, rev_eid, gat1, gat2, fc_w, num_actions,
                            dlogits, g_gat1, g_gat2, g_fc_w, g_fc_b, w, v, s); break;
    case 2: dispatch_bwd<2>(hid, n_nodes, x, rowptr, src, eattr, rev_ptr, rev_eid, gat1, gat2, fc_w, num_actions,
                            dlogits, g_gat1, g_gat2, g_fc_w, g_fc_b, w, v, s); break;
    default: dispatch_bwd<4>(hid, n_nodes, x, rowptr, src, eattr, rev_ptr, rev_eid, gat1, gat2, fc_w, num_actions,
                             dlogits, g_gat1, g_gat2, g_fc_w, g_fc_b, w, v, s); break;
  }
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
