// cairo_amd/csrc/precode.hip -- the entropy precode on the GPU (SURVEY.md
// §8(f) F2): the exact feed-bit sequence serialize_slice builds before its
// arithmetic coder (serialize.cpp:10-340, stream.cpp:550-581,
// golomb.cpp:8-91), so the host runs only the ABAC loop over it.
//
// The feed of a frame, LSB-first, sections in the reference's order:
//   block types (3 bits per MB), prediction targets (log2 R bits per non-intra
//   MB), motion x then motion y deltas (se, motion MBs), sub-pel flag / amount
//   / index (motion MBs), quality deltas (se, non-copy MBs), then the
//   coefficients of the non-copy MBs: Y as four 8x8 blocks per MB (TL, TR, BL,
//   BR), then U, then V, each block ue(run) + se(zig-zag coefficients) with a
//   delta DC.
//
// Three kernels per launch, on the launch's stream after the engine:
//   k_feed_len    one wave per 8x8 coefficient block: its bits (zig-zag in
//                 lanes, the run from a ballot, exp-Golomb lengths summed)
//   k_feed_scan   one 1024-thread workgroup per frame: the block-table sections
//                 (lengths, segmented "previous value" scans, codes), the
//                 exclusive scan of the block lengths into bit offsets, the
//                 section capacity check, zeroing of the feed words
//   k_feed_write  one wave per block again: codes OR-ed in at their offsets
//   k_feed_copy   the used words (and the header) to the frame's mapped
//                 pinned host buffer
// A coefficient section longer than the feed stream's 32 Mbit capacity
// (common.cpp:147: the reference then drops whole writes, bitstream.cpp:206-216)
// is flagged instead (`overflow`): the host codes that frame from the block
// table and coefficients itself, with the reference's drop rule.
#include "precode.h"

namespace cairo {

namespace {

typedef const __attribute__((address_space(4))) FrameArgs FA;

__constant__ uint8_t kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// exp-Golomb of val >= 1 in stream order (LSB first): (bits-1) zeros, then
// val MSB first (golomb.cpp:31-84).
__device__ __forceinline__ uint32_t eg_len(uint32_t val) { return 2u * (32u - __clz(val)) - 1u; }
__device__ __forceinline__ uint32_t eg_code(uint32_t val) {
  const uint32_t bits = 32u - __clz(val);
  return (__brev(val) >> (32u - bits)) << (bits - 1u);
}
// Signed mapping (stream.cpp / egtables.h): 0 -> 1, v > 0 -> 2|v|, v < 0 ->
// 2|v| + 1, with |-32768| = 32767 (math.h abs).
__device__ __forceinline__ uint32_t se_val(int v) {
  if (v == 0) return 1u;
  const int a = v < 0 ? (v == -32768 ? 32767 : -v) : v;
  return ((uint32_t)a << 1) | (uint32_t)(v < 0);
}

__device__ __forceinline__ const BlockDesc& desc_at(FA& a, int mb) { return a.table[mb]; }

// Bits of `len` (<= 32) at bit position p of the zeroed word buffer.
__device__ __forceinline__ void or_bits(uint32_t* w, uint64_t p, uint32_t code, uint32_t len) {
  if (!len) return;
  const uint32_t sh = (uint32_t)(p & 31);
  atomicOr(&w[p >> 5], code << sh);
  if (sh + len > 32) atomicOr(&w[(p >> 5) + 1], code >> (32 - sh));
}

// Coefficient block idx of a frame (feed order: Y blocks mb*4+sub, then U,
// then V): plane pointer, pitch, origin, delta-DC reference (serialize.cpp:35-123).
struct Blk {
  const int16_t* p;
  int pitch;
  int16_t last_dc;
  bool copy;
};

__device__ __forceinline__ Blk block_of(FA& a, int idx) {
  const int mbs = a.wmb * a.hmb;
  Blk b;
  int mb, sub = 0, pl;
  if (idx < 4 * mbs) {
    mb = idx >> 2, sub = idx & 3, pl = 0;
  } else {
    mb = idx - 4 * mbs, pl = 1;
    if (mb >= mbs) mb -= mbs, pl = 2;
  }
  const int mx = mb % a.wmb, my = mb / a.wmb;
  b.copy = (desc_at(a, mb).block_type & kCopy) != 0;
  if (pl == 0) {
    const int16_t* y = a.coef.y;
    const int w = a.wa;
    const int x0 = 16 * mx, y0 = 16 * my;
    b.pitch = w;
    b.p = y + (size_t)(y0 + 8 * (sub >> 1)) * w + x0 + 8 * (sub & 1);
    if (sub == 0)
      b.last_dc = mx > 0 ? y[(size_t)y0 * w + x0 - 8] : (my > 0 ? y[(size_t)(y0 - 8) * w + x0] : 0);
    else if (sub == 3)
      b.last_dc = y[(size_t)(y0 + 8) * w + x0];
    else
      b.last_dc = y[(size_t)y0 * w + x0];
  } else {
    const int16_t* c = pl == 1 ? a.coef.u : a.coef.v;
    const int w = a.wa >> 1;
    const int x0 = 8 * mx, y0 = 8 * my;
    b.pitch = w;
    b.p = c + (size_t)y0 * w + x0;
    b.last_dc = mx > 0 ? c[(size_t)y0 * w + x0 - 8] : (my > 0 ? c[(size_t)(y0 - 8) * w + x0] : 0);
  }
  return b;
}

// This lane's zig-zag coefficient (lane k of the wave = scan position k),
// the block's run (last nonzero + 1) and this lane's code length.
__device__ __forceinline__ int lane_coef(const Blk& b, int lane, int& run) {
  const int r = kZig[lane];
  int c = b.p[(size_t)(r >> 3) * b.pitch + (r & 7)];
  if (lane == 0) c = (int16_t)(c - b.last_dc);
  const uint64_t nz = __ballot(c != 0);
  run = nz ? 64 - __clzll(nz) : 0;
  return c;
}

__global__ __launch_bounds__(256) void k_feed_len(FeedArgs f) {
  FA& a = ((FA*)f.fa)[blockIdx.y];
  const int mbs = a.wmb * a.hmb, lane = threadIdx.x & 63;
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (idx >= 6 * mbs) return;
  const Blk b = block_of(a, idx);
  int32_t* lens = f.lens + (size_t)f.slot[blockIdx.y] * f.lens_stride;
  if (b.copy) {
    if (lane == 0) lens[idx] = 0;
    return;
  }
  int run;
  const int c = lane_coef(b, lane, run);
  uint32_t len = lane < run ? eg_len(se_val(c)) : 0u;
  for (int o = 32; o; o >>= 1) len += __shfl_xor(len, o);
  if (lane == 0) lens[idx] = (int32_t)(len + eg_len((uint32_t)run + 1u));
}

constexpr int kScanT = 1024;

// Block-wide exclusive scan of one 64-bit value per thread; returns the
// prefix, *total the sum.
__device__ uint64_t block_scan(uint64_t v, uint64_t* sh, uint64_t* total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint64_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  if (t == 0) {
    uint64_t s = 0;
    for (int i = 0; i < kScanT / 64; i++) {
      const uint64_t u = sh[i];
      sh[i] = s;
      s += u;
    }
    sh[kScanT / 64] = s;
  }
  __syncthreads();
  const uint64_t r = sh[w] + x - v;
  *total = sh[kScanT / 64];
  __syncthreads();
  return r;
}

// Segmented "latest present value" over threads: the value of the last
// present item before this thread's run (0 if none) -- the reference's
// `last` carried across the raster loop.
__device__ int block_last(bool has, int last, int* sh_has, int* sh_val) {
  const int t = threadIdx.x;
  sh_has[t] = has ? t : -1;
  sh_val[t] = last;
  __syncthreads();
  // inclusive max-scan of the index of the latest thread with an item
  for (int o = 1; o < kScanT; o <<= 1) {
    const int v = t >= o ? sh_has[t - o] : -1;
    __syncthreads();
    if (v > sh_has[t]) sh_has[t] = v;
    __syncthreads();
  }
  const int src = t > 0 ? sh_has[t - 1] : -1;
  const int r = src >= 0 ? sh_val[src] : 0;
  __syncthreads();
  return r;
}

// The table lists, in feed order.
enum { kTypes, kTargets, kMvx, kMvy, kSpPred, kSpAmount, kSpIndex, kQuality, kLists };

// Item of list L for MB d: present?, and (for the delta lists) its value.
__device__ __forceinline__ bool item(int L, const BlockDesc& d, int& value) {
  const bool intra = d.block_type & kIntra, motion = d.block_type & kMotion, copy = d.block_type & kCopy;
  switch (L) {
    case kTypes: value = (int)(d.block_type & 7u); return true;
    case kTargets: value = d.prediction_target; return !intra;
    case kMvx: value = d.motion_x; return motion;
    case kMvy: value = d.motion_y; return motion;
    case kSpPred: value = d.sp_pred & 1; return motion;
    case kSpAmount: value = d.sp_amount & 1; return motion && d.sp_pred;
    case kSpIndex: value = d.sp_index & 7; return motion && d.sp_pred;
    default: value = d.q_index; return !copy;
  }
}

// Code of an item given the previous present value of its list.
__device__ __forceinline__ uint32_t item_code(int L, int value, int prev, int tbits, uint32_t* len) {
  switch (L) {
    case kTypes: *len = 3; return (uint32_t)value;
    case kTargets: *len = (uint32_t)tbits; return (uint32_t)value & ((1u << tbits) - 1u);
    case kSpPred:
    case kSpAmount: *len = 1; return (uint32_t)value;
    case kSpIndex: *len = 3; return (uint32_t)value;
    default: {  // motion / quality deltas: se, int16 arithmetic as in the reference
      const uint32_t v = se_val((int16_t)(value - prev));
      *len = eg_len(v);
      return eg_code(v);
    }
  }
}

__global__ __launch_bounds__(kScanT) void k_feed_scan(FeedArgs f) {
  __shared__ uint64_t sh[kScanT / 64 + 1];
  __shared__ int sh_has[kScanT], sh_val[kScanT];
  __shared__ uint64_t list_base[kLists + 1];
  FA& a = ((FA*)f.fa)[blockIdx.x];
  const int slot = f.slot[blockIdx.x];
  const int t = threadIdx.x, mbs = a.wmb * a.hmb;
  const int per = (mbs + kScanT - 1) / kScanT, m0 = min(t * per, mbs), m1 = min(m0 + per, mbs);
  const int tbits = 31 - __clz(max(a.ring & 0xFF, 1));  // log2((uint8)R), serialize.cpp:179
  uint32_t* feed = f.feed + (size_t)slot * f.feed_stride;
  uint32_t* hdr = f.hdr + (size_t)slot * kFeedHdrWords;
  int32_t* lens = f.lens + (size_t)slot * f.lens_stride;

  // ---- table lists: carry-in of the delta lists, lengths, offsets ----
  int carry[kLists];
  uint64_t off[kLists];
  uint64_t base = 0;
  for (int L = 0; L < kLists; L++) {
    int last = 0;
    bool has = false;
    uint64_t bits = 0;
    if (L == kMvx || L == kMvy || L == kQuality) {
      for (int m = m0; m < m1; m++) {
        int v;
        if (item(L, desc_at(a, m), v)) has = true, last = v;
      }
      carry[L] = block_last(has, last, sh_has, sh_val);
    } else {
      carry[L] = 0;
    }
    int prev = carry[L];
    for (int m = m0; m < m1; m++) {
      int v;
      if (!item(L, desc_at(a, m), v)) continue;
      uint32_t len;
      item_code(L, v, prev, tbits, &len);
      bits += len;
      prev = v;
    }
    uint64_t total;
    off[L] = base + block_scan(bits, sh, &total);
    if (t == 0) list_base[L] = base;
    base += total;
  }
  const uint64_t table_bits = base;

  // ---- coefficient blocks: exclusive scan of the lengths, sections Y, U, V ----
  const int nb = 6 * mbs, bper = (nb + kScanT - 1) / kScanT;
  const int b0 = min(t * bper, nb), b1 = min(b0 + bper, nb);
  uint64_t s = 0;
  for (int i = b0; i < b1; i++) s += (uint32_t)lens[i];
  uint64_t total;
  uint64_t o = table_bits + block_scan(s, sh, &total);
  for (int i = b0; i < b1; i++) {  // lengths -> offsets, in place (as int32 offsets from table_bits)
    const uint32_t l = (uint32_t)lens[i];
    lens[i] = (int32_t)(o - table_bits);
    o += l;
  }
  __syncthreads();
  const uint64_t all = table_bits + total;
  // section sizes: Y = blocks [0, 4 mbs), U = [4 mbs, 5 mbs), V = the rest
  __shared__ uint64_t sec[3];
  if (t == 0) {
    const uint64_t u0 = (uint64_t)(uint32_t)lens[4 * mbs], v0 = (uint64_t)(uint32_t)lens[5 * mbs];
    sec[0] = u0, sec[1] = v0 - u0, sec[2] = total - v0;
  }
  __syncthreads();
  const bool overflow = sec[0] > kFeedCapacityBits || sec[1] > kFeedCapacityBits || sec[2] > kFeedCapacityBits ||
                        all + 64 > (uint64_t)f.feed_stride * 32;
  if (t == 0) {
    hdr[0] = (uint32_t)all;
    hdr[1] = (uint32_t)(all >> 32);
    hdr[2] = overflow ? 1u : 0u;
    hdr[3] = (uint32_t)table_bits;
  }
  if (overflow) return;  // the host codes this frame itself (k_feed_write / k_feed_copy see the flag)
  // ---- zero the words, then write the table lists ----
  const uint64_t words = (all + 31) / 32 + 1;
  for (uint64_t i = t; i < words; i += kScanT) feed[i] = 0;
  __syncthreads();
  for (int L = 0; L < kLists; L++) {
    int prev = carry[L];
    uint64_t p = off[L];
    for (int m = m0; m < m1; m++) {
      int v;
      if (!item(L, desc_at(a, m), v)) continue;
      uint32_t len;
      const uint32_t code = item_code(L, v, prev, tbits, &len);
      or_bits(feed, p, code, len);
      p += len;
      prev = v;
    }
  }
}

__global__ __launch_bounds__(256) void k_feed_write(FeedArgs f) {
  FA& a = ((FA*)f.fa)[blockIdx.y];
  const int slot = f.slot[blockIdx.y];
  if (f.hdr[(size_t)slot * kFeedHdrWords + 2]) return;  // overflow: the host codes this frame
  const int mbs = a.wmb * a.hmb, lane = threadIdx.x & 63;
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (idx >= 6 * mbs) return;
  const Blk b = block_of(a, idx);
  if (b.copy) return;
  int run;
  const int c = lane_coef(b, lane, run);
  const uint32_t val = se_val(c);
  const uint32_t len = lane < run ? eg_len(val) : 0u;
  uint32_t x = len;  // inclusive prefix of the lane lengths
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  const uint64_t base = (uint64_t)f.hdr[(size_t)slot * kFeedHdrWords + 3] +
                        (uint32_t)f.lens[(size_t)slot * f.lens_stride + idx];
  uint32_t* feed = f.feed + (size_t)slot * f.feed_stride;
  const uint32_t ul = eg_len((uint32_t)run + 1u);
  if (lane == 0) or_bits(feed, base, eg_code((uint32_t)run + 1u), ul);
  if (lane < run) or_bits(feed, base + ul + (x - len), eg_code(val), len);
}

__global__ __launch_bounds__(256) void k_feed_copy(FeedArgs f) {
  const int j = blockIdx.y, slot = f.slot[j];
  const uint32_t* hdr = f.hdr + (size_t)slot * kFeedHdrWords;
  uint32_t* host = f.host[j];
  const uint64_t all = (uint64_t)hdr[0] | ((uint64_t)hdr[1] << 32);
  const uint64_t words = hdr[2] ? 0 : (all + 31) / 32;
  const uint32_t* feed = f.feed + (size_t)slot * f.feed_stride;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256)
    host[kFeedHdrWords + i] = feed[i];
  if (blockIdx.x == 0 && threadIdx.x < kFeedHdrWords) host[threadIdx.x] = hdr[threadIdx.x];
}

}  // namespace

hipError_t launch_precode(const FeedArgs& f, int mbs, hipStream_t s) {
  const dim3 blocks((6 * mbs + 3) / 4, f.nframes);
  hipLaunchKernelGGL(k_feed_len, blocks, dim3(256), 0, s, f);
  hipLaunchKernelGGL(k_feed_scan, dim3(f.nframes), dim3(kScanT), 0, s, f);
  hipLaunchKernelGGL(k_feed_write, blocks, dim3(256), 0, s, f);
  hipLaunchKernelGGL(k_feed_copy, dim3(64, f.nframes), dim3(256), 0, s, f);
  return hipGetLastError();
}

}  // namespace cairo
