// The columns split's bitmap exchange for gfx950 (distributed.py).
//
// Rank q fills the lines of its 256-line-aligned column shard for every candidate, so it needs,
// per candidate, the removal bits of exactly the actions its lines hold.  Action ids are raw COO
// positions (preconditioner.py:23-25), so for a matrix whose raw order is not banded (thermal2's
// file order, any permuted numbering) those bits are scattered over the whole bitmap.  The send
// buffer is therefore built by gathering, per destination q, the bits of q's action ids in
// LINE-MAJOR order (the order q's fill visits them) and packing them 32 to a word: every rank
// receives exactly nnz(shard) bits per candidate whatever the numbering; the receiving fill reads
// them through a shard-local action table (the same line-major positions).
#include "spai_device.h"
#include "spai_status.h"

namespace spai {
namespace {

constexpr int kPackNT = 256;

// One thread per packed bit j of destination q (blockIdx.y); a wave's 64 bits are two whole
// words (j0 is a multiple of 64), formed by one ballot per candidate.  Layout of q's block at
// out + out_off[q]: [bl][wq + 1] words = the wq packed words, then the candidate's removal count.
__global__ __launch_bounds__(kPackNT) void k_bitmap_pack(int32_t bl, const uint32_t* __restrict__ removed,
                                                         int32_t words, const int32_t* __restrict__ counts,
                                                         const int32_t* __restrict__ ids,
                                                         const int64_t* __restrict__ seg,
                                                         const int64_t* __restrict__ out_off,
                                                         uint32_t* __restrict__ out) {
  const int q = blockIdx.y, lane = threadIdx.x & 63;
  const int64_t s0 = seg[q], m = seg[q + 1] - s0, wq = (m + 31) / 32;
  const int64_t j = (int64_t)blockIdx.x * kPackNT + threadIdx.x;
  if ((int64_t)blockIdx.x * kPackNT >= m && blockIdx.x != 0) return;  // block-uniform
  uint32_t* o = out + out_off[q];
  const int a = j < m ? ids[s0 + j] : -1;
  const int64_t w = (j - lane) >> 5;  // the wave's first word
  const uint32_t* rw = removed + (a >= 0 ? (a >> 5) : 0);
  const uint32_t sh = (uint32_t)a & 31u;
  // candidates in chunks of 8: the chunk's 8 words in flight at once (one memory round trip per chunk
  // instead of one per candidate), then one ballot and two word stores per candidate
  constexpr int kC = 8;
#pragma unroll 1
  for (int b0 = 0; b0 < bl; b0 += kC) {
    uint32_t v[kC];
#pragma unroll
    for (int i = 0; i < kC; ++i) v[i] = (a >= 0 && b0 + i < bl) ? rw[(int64_t)(b0 + i) * words] : 0u;
#pragma unroll
    for (int i = 0; i < kC; ++i) {
      if (b0 + i >= bl) break;  // (uniform)
      const uint64_t mask = __ballot((v[i] >> sh) & 1u);
      uint32_t* ob = o + (int64_t)(b0 + i) * (wq + 1);
      if (lane == 0 && w < wq) ob[w] = (uint32_t)mask;
      if (lane == 32 && w + 1 < wq) ob[w + 1] = (uint32_t)(mask >> 32);
    }
  }
  if (j == 0)
    for (int b = 0; b < bl; ++b) o[(int64_t)b * (wq + 1) + wq] = (uint32_t)counts[b];
}

// Window layout: destination q's block is [bl][span[q] + 1] words = the removal words
// removed[b][lo[q] .. lo[q] + span[q]) (contiguous: coalesced reads, no gather), then counts[b].
// One thread per output word.
__global__ __launch_bounds__(kPackNT) void k_window_pack(int32_t bl, const uint32_t* __restrict__ removed,
                                                         int32_t words, const int32_t* __restrict__ counts,
                                                         const int64_t* __restrict__ lo,
                                                         const int64_t* __restrict__ span,
                                                         const int64_t* __restrict__ out_off,
                                                         uint32_t* __restrict__ out) {
  const int q = blockIdx.y;
  const int64_t sp = span[q], row = sp + 1;
  const int64_t i = (int64_t)blockIdx.x * kPackNT + threadIdx.x;
  if (i >= (int64_t)bl * row) return;
  const int64_t b = i / row, t = i - b * row;
  out[out_off[q] + i] = t < sp ? removed[b * words + lo[q] + t] : (uint32_t)counts[b];
}

}  // namespace
}  // namespace spai

using namespace spai;

extern "C" int spai_bitmap_pack(int32_t P, int32_t bl, const uint32_t* removed, int32_t words, const int32_t* counts,
                                const int32_t* ids, const int64_t* seg, const int64_t* out_off, int64_t max_seg,
                                uint32_t* out, void* stream) {
  SPAI_CHECK_ARG(P >= 1 && bl >= 1 && words >= 1 && max_seg >= 0 && removed && counts && seg && out_off && out &&
                     (ids || max_seg == 0),
                 "spai_bitmap_pack: bad arguments");
  SPAI_CHECK_ARG(P <= 65535, "spai_bitmap_pack: P=%d above 65535", P);
  const int64_t gx = (max_seg + kPackNT - 1) / kPackNT;
  SPAI_CHECK_ARG(gx <= 0x7fffffff, "spai_bitmap_pack: segment too long");
  dim3 grid((unsigned)(gx > 0 ? gx : 1), (unsigned)P);
  k_bitmap_pack<<<grid, kPackNT, 0, (hipStream_t)stream>>>(bl, removed, words, counts, ids, seg, out_off, out);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}

extern "C" int spai_window_pack(int32_t P, int32_t bl, const uint32_t* removed, int32_t words, const int32_t* counts,
                                const int64_t* lo, const int64_t* span, const int64_t* out_off, int64_t max_span,
                                uint32_t* out, void* stream) {
  SPAI_CHECK_ARG(P >= 1 && bl >= 1 && words >= 1 && max_span >= 0 && max_span <= words && removed && counts && lo &&
                     span && out_off && out,
                 "spai_window_pack: bad arguments");
  SPAI_CHECK_ARG(P <= 65535, "spai_window_pack: P=%d above 65535", P);
  const int64_t gx = ((int64_t)bl * (max_span + 1) + kPackNT - 1) / kPackNT;
  SPAI_CHECK_ARG(gx <= 0x7fffffff, "spai_window_pack: window too long");
  dim3 grid((unsigned)gx, (unsigned)P);
  k_window_pack<<<grid, kPackNT, 0, (hipStream_t)stream>>>(bl, removed, words, counts, lo, span, out_off, out);
  SPAI_CHECK_LAUNCH();
  return SPAI_OK;
}
