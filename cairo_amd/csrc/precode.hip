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
// Six kernels per launch, on the launch's stream after the engine:
//   k_feed_len    one wave per macroblock: the bits of its six 8x8 blocks
//                 (zig-zag in lanes, the run from a ballot, exp-Golomb
//                 lengths summed)
//   k_feed_agg / k_feed_carry / k_feed_scan   the scan over chunks of 256
//                 macroblocks (chunk aggregates in parallel, the chunks' carries
//                 in order per frame, then the chunks in parallel again): the
//                 table items' codes (segmented "previous value" scans for the
//                 delta lists) and the exclusive scans of the eleven lists'
//                 lengths, the section capacity check, zeroing of the feed words
//   k_feed_write  one wave per macroblock again: codes OR-ed in at their offsets
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

// The six 8x8 blocks of macroblock mb (Y TL, TR, BL, BR, U, V): this lane's
// zig-zag coefficient of each (lane k = scan position k), with the delta DC
// on lane 0 (serialize.cpp:35-123: the left neighbour's block at x - 8, or
// the one above at y - 8 in the first column; stale output_cache values of
// copy macroblocks included).
// Lanes 0..47 load the macroblock's 768 bytes as
// 16-byte rows (luma 16 rows x 2 halves, then 8 U and 8 V rows) into the
// wave's buffer (luma 16x16, U 8x8, V 8x8), then every lane reads its
// zig-zag element of each block: one wide load per lane instead of six
// scattered 2-byte loads.
__device__ __forceinline__ void mb_coefs(FA& a, int mb, int lane, int16_t* buf, int c[6]) {
  const int mx = mb % a.wmb, my = mb / a.wmb;
  const int w = a.wa, cw = a.wa >> 1;
  const int x0 = 16 * mx, y0 = 16 * my, cx = 8 * mx, cy = 8 * my;
  if (lane < 48) {
    const int16_t* src;
    int dst;
    if (lane < 32) {
      src = a.coef.y + (size_t)(y0 + (lane >> 1)) * w + x0 + 8 * (lane & 1);
      dst = (lane >> 1) * 16 + 8 * (lane & 1);
    } else {
      const int r = lane & 7;
      src = (lane < 40 ? a.coef.u : a.coef.v) + (size_t)(cy + r) * cw + cx;
      dst = (lane < 40 ? 256 : 320) + 8 * r;
    }
    *(uint4*)&buf[dst] = *(const uint4*)src;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int r = kZig[lane], ry = r >> 3, rx = r & 7;
#pragma unroll
  for (int b = 0; b < 4; b++) c[b] = buf[(8 * (b >> 1) + ry) * 16 + 8 * (b & 1) + rx];
  c[4] = buf[256 + r];
  c[5] = buf[320 + r];
  if (lane == 0) {
    const int16_t* y = a.coef.y;
    const int16_t* u = a.coef.u;
    const int16_t* v = a.coef.v;
    const int16_t dy = mx > 0 ? y[(size_t)y0 * w + x0 - 8] : (my > 0 ? y[(size_t)(y0 - 8) * w + x0] : 0);
    const int16_t du = mx > 0 ? u[(size_t)cy * cw + cx - 8] : (my > 0 ? u[(size_t)(cy - 8) * cw + cx] : 0);
    const int16_t dv = mx > 0 ? v[(size_t)cy * cw + cx - 8] : (my > 0 ? v[(size_t)(cy - 8) * cw + cx] : 0);
    const int16_t d0 = (int16_t)c[0], d2 = (int16_t)c[2];  // this MB's TL and BL DCs (lane 0 holds them)
    c[0] = (int16_t)(c[0] - dy);
    c[1] = (int16_t)(c[1] - d0);
    c[2] = (int16_t)(c[2] - d0);
    c[3] = (int16_t)(c[3] - d2);
    c[4] = (int16_t)(c[4] - du);
    c[5] = (int16_t)(c[5] - dv);
  }
}

__device__ __forceinline__ int run_of(int c) {
  const uint64_t nz = __ballot(c != 0);
  return nz ? 64 - __clzll(nz) : 0;
}

// Wave scans by DPP (gfx9 row shifts and row broadcasts: six dependent VALU
// steps instead of six LDS permutes).  dpp_src: lane i's source value, 0 where
// the control selects none (bound_ctrl off: the old value, 0, stays).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_src(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xF, false);
}
// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += dpp_src<0x111, 0xF>(x);  // row_shr:1
  x += dpp_src<0x112, 0xF>(x);  // row_shr:2
  x += dpp_src<0x114, 0xF>(x);  // row_shr:4
  x += dpp_src<0x118, 0xF>(x);  // row_shr:8
  x += dpp_src<0x142, 0xA>(x);  // row_bcast:15 into rows 1 and 3
  x += dpp_src<0x143, 0xC>(x);  // row_bcast:31 into rows 2 and 3
  return x;
}
// The wave's total (uniform).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(v), 63);
}
// Segmented "last present value" scan (inclusive): (h, v) of the latest lane
// <= this one with h set.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void last_step(int& h, int& v) {
  const int h2 = (int)dpp_src<kCtrl, kRowMask>((uint32_t)h), v2 = (int)dpp_src<kCtrl, kRowMask>((uint32_t)v);
  if (!h) h = h2, v = v2;
}
__device__ __forceinline__ void wave_last_present(int& h, int& v) {
  last_step<0x111, 0xF>(h, v);
  last_step<0x112, 0xF>(h, v);
  last_step<0x114, 0xF>(h, v);
  last_step<0x118, 0xF>(h, v);
  last_step<0x142, 0xA>(h, v);
  last_step<0x143, 0xC>(h, v);
}
// Lane i - 1's value (0 on lane 0): wave_shr:1.
__device__ __forceinline__ int wave_prev(int v) { return (int)dpp_src<0x138, 0xF>((uint32_t)v); }

// Phase 1: one wave per macroblock, the bits of its six blocks.
__global__ __launch_bounds__(256) void k_feed_len(FeedArgs f) {
  FA& a = ((FA*)f.fa)[blockIdx.y];
  const int mbs = a.wmb * a.hmb, lane = threadIdx.x & 63;
  const int mb = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (mb >= mbs) return;
  uint32_t* blen = f.scratch + (size_t)f.slot[blockIdx.y] * f.scratch_stride;  // [6][mbs]
  if (a.table[mb].block_type & kCopy) {
    if (lane < 6) blen[(size_t)lane * mbs + mb] = 0;
    return;
  }
  __shared__ __attribute__((aligned(16))) int16_t cbuf[4][384];
  int c[6];
  mb_coefs(a, mb, lane, cbuf[threadIdx.x >> 6], c);
  uint32_t mine = 0;
#pragma unroll
  for (int b = 0; b < 6; b++) {
    const int run = run_of(c[b]);
    const uint32_t t = wave_sum(lane < run ? eg_len(se_val(c[b])) : 0u) + eg_len((uint32_t)run + 1u);
    if (lane == b) mine = t;
  }
  if (lane < 6) blen[(size_t)lane * mbs + mb] = mine;
}

// The table lists (serialize.cpp:156-286), then the three coefficient
// sections, in feed order.
enum { kTypes, kTargets, kMvx, kMvy, kSpPred, kSpAmount, kSpIndex, kQuality, kSecY, kSecU, kSecV, kLists };
constexpr int kTabLists = kSecY;

// Item of table list L for MB d: present?, and its value.
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

// Code of an item given the previous present value of its list (delta lists).
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

__device__ __forceinline__ bool delta_list(int L) { return L == kMvx || L == kMvy || L == kQuality; }

constexpr int kScanT = kFeedChunk, kScanW = kScanT / 64;  // small workgroups fit beside the persistent engine
static_assert(kFeedChunkWords >= kLists + 9, "chunk record: 11 sums / offsets, 3 x (has, first, last)");
constexpr int kDeltaLists[3] = {kMvx, kMvy, kQuality};

// The table items and lengths of this thread's macroblock (chunk c, thread t)
// and the delta lists' "previous present value" inside its wave
// (segmented scans); shared by the aggregate and the final pass of the scan.
struct ChunkItems {
  bool valid;
  BlockDesc d;
  int val[kTabLists];
  bool has[kTabLists];
  int prev[3];  // 0x7FFFFFFF: no present item earlier in the wave
  uint32_t len[kLists];
};

__device__ __forceinline__ void chunk_items(FA& a, const uint32_t* blen, int mbs, int mb, int lane, int hv_out[3],
                                            int vv_out[3], ChunkItems& it) {
  it.valid = mb < mbs;
  if (it.valid) {
    it.d = a.table[mb];
  } else {
    memset(&it.d, 0, sizeof(it.d));
    it.d.block_type = kCopy;  // no items, no blocks
  }
#pragma unroll
  for (int L = 0; L < kTabLists; L++) it.has[L] = it.valid && item(L, it.d, it.val[L]);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int L = kDeltaLists[k];
    int hv = it.has[L], vv = it.val[L];  // inclusive within the wave
    wave_last_present(hv, vv);
    hv_out[k] = hv, vv_out[k] = vv;
    const int he = wave_prev(hv), ve = wave_prev(vv);  // exclusive within the wave
    it.prev[k] = lane > 0 && he ? ve : 0x7FFFFFFF;             // 0x7FFFFFFF: look further back
  }
#pragma unroll
  for (int L = 0; L < kTabLists; L++) it.len[L] = 0;
  it.len[kSecY] = it.valid ? blen[mb] + blen[mbs + mb] + blen[2 * (size_t)mbs + mb] + blen[3 * (size_t)mbs + mb] : 0;
  it.len[kSecU] = it.valid ? blen[4 * (size_t)mbs + mb] : 0;
  it.len[kSecV] = it.valid ? blen[5 * (size_t)mbs + mb] : 0;
}

__device__ __forceinline__ uint32_t* chunk_record(const FeedArgs& f, int slot, int mbs, int c) {
  return f.scratch + (size_t)slot * f.scratch_stride + (size_t)kFeedScratchPerMB * mbs + (size_t)c * kFeedChunkWords;
}

// The scan of the table lists and sections (serialize.cpp:156-286) runs in
// three passes over chunks of kFeedChunk macroblocks, so that the chunks of
// a frame run in parallel (one workgroup per frame walking its 127 chunks of a
// 4K frame took 0.83 ms of the gap between two engine launches):
//   k_feed_agg    per chunk: each list's summed lengths, except the delta
//                 lists' first present item (its code depends on the value
//                 before the chunk), and that item's value and the chunk's
//                 last present value;
//   k_feed_carry  per frame: the chunks in order -- the first items'
//                 lengths, each chunk's offset within every list and its
//                 delta carries; the list bases, capacity check and header;
//   k_feed_scan   per chunk: the items' codes and positions (as before, from
//                 the chunk's carry-ins), and its share of zeroing the feed.
__global__ __launch_bounds__(kScanT) void k_feed_agg(FeedArgs f) {
  __shared__ uint32_t wsum[kScanW][kLists];
  __shared__ int whas[kScanW][3], wval[kScanW][3], wfh[kScanW][3], wfv[kScanW][3];
  FA& a = ((FA*)f.fa)[blockIdx.y];
  const int slot = f.slot[blockIdx.y];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, mbs = a.wmb * a.hmb;
  const int tbits = 31 - __clz(max(a.ring & 0xFF, 1));
  const uint32_t* blen = f.scratch + (size_t)slot * f.scratch_stride;
  const int mb = blockIdx.x * kScanT + t;
  ChunkItems it;
  int hv[3], vv[3];
  chunk_items(a, blen, mbs, mb, lane, hv, vv, it);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int L = kDeltaLists[k];
    const uint64_t b = __ballot(it.has[L]);  // the wave's first present item
    const int fl = b ? (int)__ffsll((unsigned long long)b) - 1 : 0;
    const int fv = __shfl(it.val[L], fl);
    if (lane == 63) whas[w][k] = hv[k], wval[w][k] = vv[k], wfh[w][k] = b != 0, wfv[w][k] = fv;
  }
  __syncthreads();
  bool first[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int L = kDeltaLists[k];
    int pv = it.prev[k];
    first[k] = false;
    if (pv == 0x7FFFFFFF) {  // the last present value of an earlier wave of the chunk, if any
      for (int i = w - 1; i >= 0; i--)
        if (whas[i][k]) {
          pv = wval[i][k];
          break;
        }
      if (pv == 0x7FFFFFFF) first[k] = it.has[L];  // the chunk's first present item: done by k_feed_carry
    }
    if (it.has[L] && !first[k]) (void)item_code(L, it.val[L], pv, tbits, &it.len[L]);
  }
#pragma unroll
  for (int L = 0; L < kTabLists; L++)
    if (it.has[L] && !delta_list(L)) (void)item_code(L, it.val[L], 0, tbits, &it.len[L]);
#pragma unroll
  for (int L = 0; L < kLists; L++) {
    const uint32_t x = wave_sum(it.len[L]);
    if (lane == 0) wsum[w][L] = x;
  }
  __syncthreads();
  uint32_t* rec = chunk_record(f, slot, mbs, blockIdx.x);
  if (t < kLists) {
    uint32_t s = 0;
    for (int i = 0; i < kScanW; i++) s += wsum[i][t];
    rec[t] = s;
  } else if (t < kLists + 3) {  // per delta list: any present item, the first's value, the last's value
    const int k = t - kLists;
    int has = 0, fv = 0, lv = 0;
    for (int i = 0; i < kScanW; i++) {
      if (wfh[i][k] && !has) fv = wfv[i][k];
      if (whas[i][k]) has = 1, lv = wval[i][k];
    }
    rec[kLists + k] = has, rec[kLists + 3 + k] = fv, rec[kLists + 6 + k] = lv;
  }
}

// One wave per frame: lane L walks list L's chunk records in order (staged
// through LDS 64 at a time), replacing each record's sums by the chunk's
// offset within the list and, for the delta lists, its carry-in (any
// present value before the chunk, and the last one).
__global__ __launch_bounds__(64) void k_feed_carry(FeedArgs f) {
  constexpr int kTile = 64;
  __shared__ uint32_t tile[kTile * kFeedChunkWords];
  FA& a = ((FA*)f.fa)[blockIdx.x];
  const int slot = f.slot[blockIdx.x];
  const int lane = threadIdx.x, mbs = a.wmb * a.hmb, nch = (mbs + kFeedChunk - 1) / kFeedChunk;
  uint32_t* rec0 = chunk_record(f, slot, mbs, 0);
  uint32_t* hdr = f.hdr + (size_t)slot * kFeedHdrWords;
  const int k = lane == kMvx ? 0 : (lane == kMvy ? 1 : (lane == kQuality ? 2 : -1));
  uint64_t run = 0;
  int ch = 0, cv = 0;
  for (int c0 = 0; c0 < nch; c0 += kTile) {
    const int n = min(kTile, nch - c0);
    for (int i = lane; i < n * kFeedChunkWords; i += 64) tile[i] = rec0[(size_t)c0 * kFeedChunkWords + i];
    __syncthreads();
    if (lane < kLists) {
      for (int c = 0; c < n; c++) {
        uint32_t* r = &tile[c * kFeedChunkWords];
        uint32_t sum = r[lane];
        if (k >= 0) {
          const int has = (int)r[kLists + k], fv = (int)r[kLists + 3 + k], lv = (int)r[kLists + 6 + k];
          if (has) sum += eg_len(se_val((int16_t)(fv - (ch ? cv : 0))));
          r[kLists + k] = (uint32_t)ch, r[kLists + 3 + k] = (uint32_t)cv;  // carry-in
          if (has) ch = 1, cv = lv;
        }
        r[lane] = (uint32_t)run;  // offsets within a list stay below 2^26 (else overflow, below)
        run += sum;
      }
    }
    __syncthreads();
    for (int i = lane; i < n * kFeedChunkWords; i += 64) rec0[(size_t)c0 * kFeedChunkWords + i] = tile[i];
    __syncthreads();
  }
  // list bases, capacity, header
  uint64_t base = run;  // lane L: list L's total -> exclusive prefix over the lists
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(base, o);
    if (lane >= o) base += y;
  }
  base -= run;
  const uint64_t all = __shfl(base + run, kLists - 1);
  const bool sec_over = lane >= kSecY && lane < kLists && run > kFeedCapacityBits;
  const bool o = __ballot(sec_over) != 0 || all + 64 > (uint64_t)f.feed_stride * 32;
  if (lane < kLists) hdr[4 + lane] = (uint32_t)base;
  if (lane == 0) hdr[0] = (uint32_t)all, hdr[1] = (uint32_t)(all >> 32), hdr[2] = o ? 1u : 0u, hdr[3] = 0u;
}

// Per chunk: the table items' codes and positions within their lists, and
// the blocks' offsets within their sections, from the chunk's carry-ins
// (k_feed_carry); then the chunk's share of zeroing the words k_feed_write
// ORs into.
__global__ __launch_bounds__(kScanT) void k_feed_scan(FeedArgs f) {
  __shared__ uint32_t wsum[kScanW][kLists];
  __shared__ int whas[kScanW][3], wval[kScanW][3];
  __shared__ uint32_t carry_bits[kLists];
  __shared__ int carry_has[3], carry_val[3];
  FA& a = ((FA*)f.fa)[blockIdx.y];
  const int slot = f.slot[blockIdx.y];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, mbs = a.wmb * a.hmb;
  const int tbits = 31 - __clz(max(a.ring & 0xFF, 1));  // log2((uint8)R), serialize.cpp:179
  uint32_t* sc = f.scratch + (size_t)slot * f.scratch_stride;
  const uint32_t* blen = sc;                  // [6][mbs]
  uint32_t* tcode = sc + 6 * (size_t)mbs;     // [8][mbs]
  uint32_t* tpos = tcode + 8 * (size_t)mbs;   // [8][mbs]: len << 26 | offset in list
  uint32_t* boff = tpos + 8 * (size_t)mbs;    // [3][mbs]: offset of the MB's first block in its section
  const uint32_t* hdr = f.hdr + (size_t)slot * kFeedHdrWords;
  const uint32_t* rec = chunk_record(f, slot, mbs, blockIdx.x);
  if (t < kLists) carry_bits[t] = rec[t];
  if (t < 3) carry_has[t] = (int)rec[kLists + t], carry_val[t] = (int)rec[kLists + 3 + t];
  const int mb = blockIdx.x * kScanT + t;
  ChunkItems it;
  int hv[3], vv[3];
  chunk_items(a, blen, mbs, mb, lane, hv, vv, it);
#pragma unroll
  for (int k = 0; k < 3; k++)
    if (lane == 63) whas[w][k] = hv[k], wval[w][k] = vv[k];
  __syncthreads();  // whas / wval and the carry-ins complete
  if (t < 3) {  // waves' carries, in order: the last present value before each wave
    int h = carry_has[t], v = carry_val[t];
    for (int i = 0; i < kScanW; i++) {
      const int h2 = whas[i][t], v2 = wval[i][t];
      whas[i][t] = h, wval[i][t] = v;
      if (h2) h = 1, v = v2;
    }
  }
  __syncthreads();
  uint32_t code[kTabLists];
#pragma unroll
  for (int L = 0; L < kTabLists; L++) code[L] = 0;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int L = kDeltaLists[k];
    if (it.prev[k] == 0x7FFFFFFF) it.prev[k] = whas[w][k] ? wval[w][k] : 0;
    if (it.has[L]) code[L] = item_code(L, it.val[L], it.prev[k], tbits, &it.len[L]);
  }
#pragma unroll
  for (int L = 0; L < kTabLists; L++)
    if (it.has[L] && !delta_list(L)) code[L] = item_code(L, it.val[L], 0, tbits, &it.len[L]);
  // exclusive scans of the eleven lengths
  uint32_t inc[kLists];
#pragma unroll
  for (int L = 0; L < kLists; L++) {
    const uint32_t x = wave_incl_sum(it.len[L]);
    inc[L] = x;
    if (lane == 63) wsum[w][L] = x;
  }
  __syncthreads();
  if (t < kLists) {  // wave prefixes, plus the chunk's offset within the list
    uint32_t s = carry_bits[t];
    for (int i = 0; i < kScanW; i++) {
      const uint32_t u = wsum[i][t];
      wsum[i][t] = s;
      s += u;
    }
  }
  __syncthreads();
  if (it.valid) {
#pragma unroll
    for (int L = 0; L < kTabLists; L++) {
      const uint32_t off = wsum[w][L] + inc[L] - it.len[L];
      tcode[(size_t)L * mbs + mb] = code[L];
      tpos[(size_t)L * mbs + mb] = it.has[L] ? (it.len[L] << 26) | (off & 0x3FFFFFFu) : 0u;
    }
#pragma unroll
    for (int k = 0; k < 3; k++)
      boff[(size_t)k * mbs + mb] = wsum[w][kSecY + k] + inc[kSecY + k] - it.len[kSecY + k];
  }
  // this chunk's share of the words the writer ORs into (none on overflow:
  // the host codes that frame from its planes)
  if (hdr[2]) return;
  const uint64_t all_bits = (uint64_t)hdr[0] | ((uint64_t)hdr[1] << 32);
  const uint64_t words = (all_bits + 31) / 32 + 1, per = (words + gridDim.x - 1) / gridDim.x;
  uint32_t* feed = f.feed + (size_t)slot * f.feed_stride;
  const uint64_t w0 = (uint64_t)blockIdx.x * per, w1 = min(words, w0 + per);
  for (uint64_t i = w0 + t; i < w1; i += kScanT) feed[i] = 0;
}

// Words an 8x8 block's codes can span: ue(65) (13 bits) + 64 codes of at
// most 31 bits, from any bit of a word.
constexpr int kBlockWords = (13 + 64 * 31 + 31) / 32 + 1;

// Phase 3: one wave per macroblock: its table items (lanes 0..7) and its
// six blocks' codes, OR-ed in at their offsets.
__global__ __launch_bounds__(256) void k_feed_write(FeedArgs f) {
  FA& a = ((FA*)f.fa)[blockIdx.y];
  const int slot = f.slot[blockIdx.y];
  const uint32_t* hdr = f.hdr + (size_t)slot * kFeedHdrWords;
  if (hdr[2]) return;  // overflow: the host codes this frame
  const int mbs = a.wmb * a.hmb, lane = threadIdx.x & 63;
  const int mb = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (mb >= mbs) return;
  const uint32_t* sc = f.scratch + (size_t)slot * f.scratch_stride;
  const uint32_t* tcode = sc + 6 * (size_t)mbs;
  const uint32_t* tpos = tcode + 8 * (size_t)mbs;
  const uint32_t* boff = tpos + 8 * (size_t)mbs;
  uint32_t* feed = f.feed + (size_t)slot * f.feed_stride;
  // Bounds guard: every word written lies below the frame's feed end (the
  // words k_feed_scan zeroed, inside the slot's buffer).  A write past it
  // would be a precode bug: it is dropped and counted in hdr[3], which the
  // host reports as a hardware failure of the frame (backend.hip
  // frame_result) instead of coding wrong bits.
  const uint64_t all_bits = (uint64_t)hdr[0] | ((uint64_t)hdr[1] << 32);
  const uint64_t limit = min((uint64_t)f.feed_stride, (all_bits + 31) / 32 + 1);
  uint32_t* const bad = const_cast<uint32_t*>(hdr) + 3;
  if (lane < kTabLists) {
    const uint32_t p = tpos[(size_t)lane * mbs + mb];
    const uint64_t at = (uint64_t)hdr[4 + lane] + (p & 0x3FFFFFFu);
    if (((at + (p >> 26) + 31) >> 5) > limit) atomicAdd(bad, 1u);
    else or_bits(feed, at, tcode[(size_t)lane * mbs + mb], p >> 26);
  }
  if (a.table[mb].block_type & kCopy) return;
  // A block's codes are assembled in LDS words, then stored: the words inside
  // its bit range belong to it alone (plain stores); only its first and last
  // word are shared with the neighbouring blocks (global atomic OR).
  __shared__ uint32_t stage[4][kBlockWords];
  __shared__ __attribute__((aligned(16))) int16_t cbuf[4][384];
  uint32_t* sw = stage[threadIdx.x >> 6];
  int c[6];
  mb_coefs(a, mb, lane, cbuf[threadIdx.x >> 6], c);
  uint64_t pos = (uint64_t)hdr[4 + kSecY] + boff[mb];
#pragma unroll
  for (int b = 0; b < 6; b++) {
    if (b == 4) pos = (uint64_t)hdr[4 + kSecU] + boff[(size_t)mbs + mb];
    if (b == 5) pos = (uint64_t)hdr[4 + kSecV] + boff[2 * (size_t)mbs + mb];
    const int run = run_of(c[b]);
    if (run == 0) {  // (wave-uniform) an all-zero block is the one-bit ue(1): one atomic, no staging
      if (lane == 0) or_bits(feed, pos, 1u, 1u);
      pos += 1;
      continue;
    }
    const uint32_t val = se_val(c[b]);
    const uint32_t len = lane < run ? eg_len(val) : 0u;
    const uint32_t x = wave_incl_sum(len);  // inclusive prefix of the lane lengths
    const uint32_t ul = eg_len((uint32_t)run + 1u);
    const uint64_t end = pos + ul + (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    const uint64_t w0 = pos >> 5;
    const int nw = (int)(((end + 31) >> 5) - w0);  // <= kBlockWords
    if (w0 + nw > limit || nw > kBlockWords) {  // (wave-uniform) the guard above
      if (lane == 0) atomicAdd(bad, 1u);
      return;
    }
    for (int i = lane; i < nw; i += 64) sw[i] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t rel = (uint32_t)(pos & 31);
    if (lane == 0) or_bits(sw, rel, eg_code((uint32_t)run + 1u), ul);
    if (lane < run) or_bits(sw, rel + ul + (x - len), eg_code(val), len);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < nw; i += 64) {
      if (i == 0 || i == nw - 1)
        atomicOr(&feed[w0 + i], sw[i]);
      else
        feed[w0 + i] = sw[i];
    }
    __builtin_amdgcn_wave_barrier();
    pos = end;
  }
}

// Phase 4: the used words and the header into the frame's mapped pinned
// buffer; the frame's block table and the context's timeout words into its
// mapped pinned stage (what the host entropy stage and the status check read:
// no per-frame D2H copy, whose shader blit would wait for a workgroup slot of
// the persistent engine).
__global__ __launch_bounds__(256) void k_feed_copy(FeedArgs f) {
  const int j = blockIdx.y, slot = f.slot[j];
  const uint32_t* hdr = f.hdr + (size_t)slot * kFeedHdrWords;
  uint32_t* host = f.host[j];
  const uint64_t all = (uint64_t)hdr[0] | ((uint64_t)hdr[1] << 32);
  const uint64_t words = hdr[2] ? 0 : (all + 31) / 32;
  const uint32_t* feed = f.feed + (size_t)slot * f.feed_stride;
  const uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, di = (uint64_t)gridDim.x * 256;
  for (uint64_t i = i0; i < words; i += di) host[kFeedHdrWords + i] = feed[i];
  if (blockIdx.x == 0 && threadIdx.x < kFeedHdrWords) host[threadIdx.x] = hdr[threadIdx.x];
  if (uint4* th = f.table_host[j]) {
    const uint4* tb = (const uint4*)((FA*)f.fa)[j].table;
    for (uint64_t i = i0; i < (uint64_t)f.table_words; i += di) th[i] = tb[i];
  }
  if (f.err_host[j] && blockIdx.x == 0 && threadIdx.x < 64) {
    // the timeout record: its kind first (acquire: it is stored last, with
    // release, kernels.hip report_timeout), then the payload -- a record
    // seen complete, or no record
    const int32_t* sticky = ((FA*)f.fa)[j].sticky;
    const int32_t kind = __shfl(
        threadIdx.x == 0 ? __hip_atomic_load(sticky + TimeoutInfo::kKind, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                         : 0,
        0);
    if (threadIdx.x < TimeoutInfo::kWords)
      f.err_host[j][threadIdx.x] =
          threadIdx.x == TimeoutInfo::kKind
              ? kind
              : (kind ? __hip_atomic_load(sticky + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0);
  }
}

}  // namespace

hipError_t launch_precode(const FeedArgs& f, int mbs, hipStream_t s) {
  const dim3 blocks((mbs + 3) / 4, f.nframes);
  hipLaunchKernelGGL(k_feed_len, blocks, dim3(256), 0, s, f);
  const int nch = (mbs + kFeedChunk - 1) / kFeedChunk;
  hipLaunchKernelGGL(k_feed_agg, dim3(nch, f.nframes), dim3(kScanT), 0, s, f);
  hipLaunchKernelGGL(k_feed_carry, dim3(f.nframes), dim3(64), 0, s, f);
  hipLaunchKernelGGL(k_feed_scan, dim3(nch, f.nframes), dim3(kScanT), 0, s, f);
  hipLaunchKernelGGL(k_feed_write, blocks, dim3(256), 0, s, f);
  return hipGetLastError();
}

// Phase 4 alone: PCIe-bound writes into mapped host memory, so it can run
// on another stream than the engine launches (backend.hip flush).
hipError_t launch_feed_copy(const FeedArgs& f, hipStream_t s) {
  hipLaunchKernelGGL(k_feed_copy, dim3(64, f.nframes), dim3(256), 0, s, f);
  return hipGetLastError();
}

}  // namespace cairo
