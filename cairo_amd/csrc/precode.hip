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
// Four kernels per launch, on the launch's stream after the engine:
//   k_feed_len    one wave per macroblock: the bits of its six 8x8 blocks
//                 (zig-zag in lanes, the run from a ballot, exp-Golomb
//                 lengths summed)
//   k_feed_scan   one 256-thread workgroup per frame over chunks of 256
//                 macroblocks: the table items' codes (segmented "previous
//                 value" scans for the delta lists) and the exclusive scans of
//                 the eleven lists' lengths, the section capacity check,
//                 zeroing of the feed words
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
// copy macroblocks included).  All six loads are issued together.
__device__ __forceinline__ void mb_coefs(FA& a, int mb, int lane, int c[6]) {
  const int mx = mb % a.wmb, my = mb / a.wmb;
  const int r = kZig[lane], ry = r >> 3, rx = r & 7;
  const int16_t* y = a.coef.y;
  const int16_t* u = a.coef.u;
  const int16_t* v = a.coef.v;
  const int w = a.wa, cw = a.wa >> 1;
  const int x0 = 16 * mx, y0 = 16 * my, cx = 8 * mx, cy = 8 * my;
#pragma unroll
  for (int b = 0; b < 4; b++) c[b] = y[(size_t)(y0 + 8 * (b >> 1) + ry) * w + x0 + 8 * (b & 1) + rx];
  c[4] = u[(size_t)(cy + ry) * cw + cx + rx];
  c[5] = v[(size_t)(cy + ry) * cw + cx + rx];
  if (lane == 0) {
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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

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
  int c[6];
  mb_coefs(a, mb, lane, c);
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

constexpr int kScanT = 256, kScanW = kScanT / 64;  // small workgroups fit beside the persistent engine

// Phase 2: one 256-thread workgroup per frame walks the macroblocks in
// chunks of 256 (one per thread, coalesced; a workgroup that small fits
// beside the persistent engine's, so it runs in the slots a finishing launch
// frees): the table items' codes, the
// delta lists' previous values (segmented scans), and the exclusive scans of
// all eleven lists' lengths with carries across chunks.  Offsets are stored
// relative to their list's start; the list bases follow from the totals.
__global__ __launch_bounds__(kScanT) void k_feed_scan(FeedArgs f) {
  __shared__ uint32_t wsum[kScanW][kLists];
  __shared__ int whas[kScanW][3], wval[kScanW][3];
  __shared__ uint64_t carry_bits[kLists];
  __shared__ int carry_has[3], carry_val[3];
  FA& a = ((FA*)f.fa)[blockIdx.x];
  const int slot = f.slot[blockIdx.x];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, mbs = a.wmb * a.hmb;
  const int tbits = 31 - __clz(max(a.ring & 0xFF, 1));  // log2((uint8)R), serialize.cpp:179
  uint32_t* sc = f.scratch + (size_t)slot * f.scratch_stride;
  const uint32_t* blen = sc;                  // [6][mbs]
  uint32_t* tcode = sc + 6 * (size_t)mbs;     // [8][mbs]
  uint32_t* tpos = tcode + 8 * (size_t)mbs;   // [8][mbs]: len << 26 | offset in list
  uint32_t* boff = tpos + 8 * (size_t)mbs;    // [3][mbs]: offset of the MB's first block in its section
  uint32_t* hdr = f.hdr + (size_t)slot * kFeedHdrWords;
  if (t < kLists) carry_bits[t] = 0;
  if (t < 3) carry_has[t] = 0, carry_val[t] = 0;
  __syncthreads();
  for (int c0 = 0; c0 < mbs; c0 += kScanT) {
    const int mb = c0 + t;
    const bool valid = mb < mbs;
    BlockDesc d;
    if (valid) {
      d = a.table[mb];
    } else {
      memset(&d, 0, sizeof(d));
      d.block_type = kCopy;  // no items, no blocks
    }
    // the delta lists' previous values: segmented "last present" scans
    int val[kTabLists], prev[3];
    bool has[kTabLists];
#pragma unroll
    for (int L = 0; L < kTabLists; L++) has[L] = valid && item(L, d, val[L]);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int L = k == 0 ? kMvx : (k == 1 ? kMvy : kQuality);
      int hv = has[L], vv = val[L];  // inclusive within the wave
      for (int o = 1; o < 64; o <<= 1) {
        const int h2 = __shfl_up(hv, o), v2 = __shfl_up(vv, o);
        if (lane >= o && !hv) hv = h2, vv = v2;
      }
      if (lane == 63) whas[w][k] = hv, wval[w][k] = vv;
      const int he = __shfl_up(hv, 1), ve = __shfl_up(vv, 1);  // exclusive within the wave
      prev[k] = lane > 0 && he ? ve : 0x7FFFFFFF;                // 0x7FFFFFFF: look further back
    }
    // the lengths
    uint32_t len[kLists], code[kTabLists];
#pragma unroll
    for (int L = 0; L < kTabLists; L++) len[L] = 0, code[L] = 0;
    len[kSecY] = valid ? blen[mb] + blen[mbs + mb] + blen[2 * (size_t)mbs + mb] + blen[3 * (size_t)mbs + mb] : 0;
    len[kSecU] = valid ? blen[4 * (size_t)mbs + mb] : 0;
    len[kSecV] = valid ? blen[5 * (size_t)mbs + mb] : 0;
    __syncthreads();  // whas / wval complete
    if (t < 3) {  // waves' carries, in order: the last present value before each wave
      int hv = carry_has[t], vv = carry_val[t];
      for (int i = 0; i < kScanW; i++) {
        const int h2 = whas[i][t], v2 = wval[i][t];
        whas[i][t] = hv, wval[i][t] = vv;
        if (h2) hv = 1, vv = v2;
      }
      carry_has[t] = hv, carry_val[t] = vv;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int L = k == 0 ? kMvx : (k == 1 ? kMvy : kQuality);
      if (prev[k] == 0x7FFFFFFF) prev[k] = whas[w][k] ? wval[w][k] : 0;
      if (has[L]) code[L] = item_code(L, val[L], prev[k], tbits, &len[L]);
    }
#pragma unroll
    for (int L = 0; L < kTabLists; L++)
      if (has[L] && !delta_list(L)) code[L] = item_code(L, val[L], 0, tbits, &len[L]);
    // exclusive scans of the eleven lengths
    uint32_t inc[kLists];
#pragma unroll
    for (int L = 0; L < kLists; L++) {
      uint32_t x = len[L];
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
      }
      inc[L] = x;
      if (lane == 63) wsum[w][L] = x;
    }
    __syncthreads();
    if (t < kLists) {  // wave prefixes, plus the running carry of the list
      uint64_t s = carry_bits[t];
      for (int i = 0; i < kScanW; i++) {
        const uint32_t u = wsum[i][t];
        wsum[i][t] = (uint32_t)s;  // offsets within a list stay below 2^26 (else overflow, below)
        s += u;
      }
      carry_bits[t] = s;
    }
    __syncthreads();
    if (valid) {
#pragma unroll
      for (int L = 0; L < kTabLists; L++) {
        const uint32_t off = wsum[w][L] + inc[L] - len[L];
        tcode[(size_t)L * mbs + mb] = code[L];
        tpos[(size_t)L * mbs + mb] = has[L] ? (len[L] << 26) | (off & 0x3FFFFFFu) : 0u;
      }
#pragma unroll
      for (int k = 0; k < 3; k++) boff[(size_t)k * mbs + mb] = wsum[w][kSecY + k] + inc[kSecY + k] - len[kSecY + k];
    }
    __syncthreads();  // wsum / whas reused by the next chunk
  }
  // list bases, capacity, header; then zero the words the writer ORs into
  __shared__ uint64_t all_bits;
  __shared__ int over;
  if (t == 0) {
    uint64_t b = 0;
    for (int L = 0; L < kLists; L++) {
      hdr[4 + L] = (uint32_t)b;
      b += carry_bits[L];
    }
    const bool o = carry_bits[kSecY] > kFeedCapacityBits || carry_bits[kSecU] > kFeedCapacityBits ||
                   carry_bits[kSecV] > kFeedCapacityBits || b + 64 > (uint64_t)f.feed_stride * 32;
    hdr[0] = (uint32_t)b;
    hdr[1] = (uint32_t)(b >> 32);
    hdr[2] = o ? 1u : 0u;
    all_bits = b;
    over = o;
  }
  __syncthreads();
  if (over) return;  // the host codes this frame from its planes
  uint32_t* feed = f.feed + (size_t)slot * f.feed_stride;
  const uint64_t words = (all_bits + 31) / 32 + 1;
  for (uint64_t i = t; i < words; i += kScanT) feed[i] = 0;
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
  if (lane < kTabLists) {
    const uint32_t p = tpos[(size_t)lane * mbs + mb];
    or_bits(feed, (uint64_t)hdr[4 + lane] + (p & 0x3FFFFFFu), tcode[(size_t)lane * mbs + mb], p >> 26);
  }
  if (a.table[mb].block_type & kCopy) return;
  // A block's codes are assembled in LDS words, then stored: the words inside
  // its bit range belong to it alone (plain stores); only its first and last
  // word are shared with the neighbouring blocks (global atomic OR).
  __shared__ uint32_t stage[4][kBlockWords];
  uint32_t* sw = stage[threadIdx.x >> 6];
  int c[6];
  mb_coefs(a, mb, lane, c);
  uint64_t pos = (uint64_t)hdr[4 + kSecY] + boff[mb];
#pragma unroll
  for (int b = 0; b < 6; b++) {
    if (b == 4) pos = (uint64_t)hdr[4 + kSecU] + boff[(size_t)mbs + mb];
    if (b == 5) pos = (uint64_t)hdr[4 + kSecV] + boff[2 * (size_t)mbs + mb];
    const int run = run_of(c[b]);
    const uint32_t val = se_val(c[b]);
    const uint32_t len = lane < run ? eg_len(val) : 0u;
    uint32_t x = len;  // inclusive prefix of the lane lengths
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    const uint32_t ul = eg_len((uint32_t)run + 1u);
    const uint64_t end = pos + ul + __shfl(x, 63);
    const uint64_t w0 = pos >> 5;
    const int nw = (int)(((end + 31) >> 5) - w0);  // <= kBlockWords
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
  hipLaunchKernelGGL(k_feed_scan, dim3(f.nframes), dim3(kScanT), 0, s, f);
  hipLaunchKernelGGL(k_feed_write, blocks, dim3(256), 0, s, f);
  hipLaunchKernelGGL(k_feed_copy, dim3(64, f.nframes), dim3(256), 0, s, f);
  return hipGetLastError();
}

}  // namespace cairo
