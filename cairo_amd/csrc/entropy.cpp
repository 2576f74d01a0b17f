// cairo_amd/csrc/entropy.cpp -- host entropy stage (stays on the CPU by design).
//
// serialize_slice (reference serialize.cpp:319-340): block-table sections,
// delta-DC zig-zag run-length coefficients, exp-Golomb precode, adaptive
// binary arithmetic coder (abac.cpp).  The coder is bit-serial by
// construction (one adaptive model per frame), so the speed comes from a
// short serial chain: the precode is built first as one packed feed (table-
// driven exp-Golomb codes), then a single loop codes it with the coder state
// in registers, no division and no data-dependent branch per symbol; frames
// are spread over host threads by the caller (pipeline.cpp).
#include <immintrin.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/cairo_amd.h"
#include "entropy.h"
#include "evx_defs.h"

namespace cairo {

namespace {

// EVX_MACROBLOCK_8x8_ZIGZAG (scan.h:60-70): raster index of scan position k.
constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18,
                                 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                                 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43,
                                 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
                                 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Bit reversal of a byte.
struct Rev8 {
  uint8_t v[256];
  constexpr Rev8() : v() {
    for (int i = 0; i < 256; i++) {
      int r = 0;
      for (int b = 0; b < 8; b++) r |= ((i >> b) & 1) << (7 - b);
      v[i] = (uint8_t)r;
    }
  }
  constexpr uint8_t operator[](uint32_t i) const { return v[i]; }
};
constexpr Rev8 kRev8;

// exp-Golomb code of v >= 1 in stream order (LSB first): (bits-1) zeros then v
// MSB first (golomb.cpp:31-84; egtables.h holds the same codes for |v| < 256).
inline uint64_t golomb(uint32_t v, uint32_t* len) {
  const uint32_t bits = 32u - (uint32_t)__builtin_clz(v);
  uint32_t rev = 0;
  for (uint32_t x = v; x; x >>= 1) rev = (rev << 1) | (x & 1u);
  *len = 2 * bits - 1;
  return (uint64_t)rev << (bits - 1);
}

struct CodeTables {
  uint32_t se_code[65536];
  uint8_t se_len[65536];
  uint32_t ue_code[65];
  uint8_t ue_len[65];
  CodeTables() {
    for (int i = 0; i < 65536; i++) {
      const int16_t v = (int16_t)i;
      uint32_t len;
      const uint32_t val = v == 0 ? 1u : (((uint32_t)iabs(v) << 1) | (uint32_t)((v >> 15) & 1));
      const uint64_t c = golomb(val, &len);
      se_code[i] = (uint32_t)c;  // |v| = 32768 would need 33 bits; never produced
      se_len[i] = (uint8_t)(len > 32 ? 32 : len);
    }
    for (int r = 0; r <= 64; r++) {
      uint32_t len;
      ue_code[r] = (uint32_t)golomb((uint32_t)r + 1, &len);
      ue_len[r] = (uint8_t)len;
    }
  }
};
const CodeTables kCodes;

// Adaptive binary arithmetic coder, 16-bit precision (abac.cpp:28-348), run
// over the whole feed of a slice with its state in registers.  The coder is
// one serial chain per slice; everything here is about making that chain
// short (about 14 dependent operations per symbol) and keeping the rest off
// it.
//
// resolve_model's split floor(range * h0 / n), n = h0 + h1 (abac.cpp:78-93),
// without a division on the chain: the model counts depend only on the
// symbols, so the fixed-point ratio M = h0 * 2^47 / n (rounded up by 1..3
// units) is precomputed for a block of symbols (vectorized), and the split is
// one multiply: floor(range * M / 2^47).  Exact while 3 * 2^16 * n < 2^47
// (n < 7e8; a slice has at most 8 feed sections of 32 Mbit, n < 2^28): the
// overshoot range * (M - h0 2^47 / n) / 2^47 stays below 1/n, the smallest
// nonzero fractional part of range * h0 / n, and M >= h0 2^47 / n keeps exact
// quotients.  The double estimate of h0 2^47 / n is within 2^-4 of the true
// value, so floor(estimate) + 2 overshoots by 1..2.0625.
//
// The symbol: b is known in advance, so both outcomes are formed from the
// state at the start of the step and one select (cmov) picks each value:
//   b = 0: l1 = low,     h1 = mid,   r' = t              (mid = low + t)
//   b = 1: l1 = mid + 1, h1 = high,  r' = r - t - 1      (r = high - low)
// resolve_encode_scaling (abac.cpp:178-224) in closed form, without a
// data-dependent branch per symbol:
//  * E1/E2 shift-out: k = clz16(l1 ^ h1) common leading bits leave MSB first;
//    pending underflow bits (e3 copies of the opposite of the first one)
//    follow the first of them;
//  * E3 (underflow): then, while low = 01.. and high = 10.., bit 14 is removed
//    from both: the run of (l = 1, h = 0) just below the first differing bit,
//    i.e. the leading zeros of ~((l1 & ~h1) << 1) shifted by 16 + k.  The
//    reference's bound is high <= 0xBFFD, not 0xBFFF: high = 0xBFFE at the
//    first step, or bits 13..0 of high all ones once its trailing ones reach
//    them, stops the run early.  That needs many trailing ones (about one
//    symbol in 10^4), so it is a predicted branch off the chain.
//  * with s = k + E3 steps in all, low' = (l1 << s) & 0x7FFF and the range
//    is ((r' + 1) << s) - 1: the shifted-out bits of h1 and l1 differ by
//    exactly one unit of 2^15 (common bits cancel; the first differing bit
//    1/0 and the E3 run 0../1.. leave 1).  high = low + range is derived off
//    the chain.
//
// Output bits (b0, the e3 run of !b0, b1..b(k-1) = W + 2^(len-1) - 2^(k-1)
// for W = the top k bits of l1) collect MSB first in a 64-bit accumulator; a
// 32-bit word is stored every step (the store pointer advances when it is
// full, no branch) and the words are bit-reversed into bit_stream order (LSB
// first, bitstream.cpp:181-245) at the end.  `s0` bits of the caller's first
// byte are preloaded.  Returns the number of bits in `buf` (including the s0
// preloaded ones; the buffer holds them rounded up to 4 bytes), or ~0 once
// the output passes `limit`.
inline uint32_t rev32(uint32_t x) {
  x = __builtin_bswap32(x);
  x = ((x & 0x0F0F0F0Fu) << 4) | ((x >> 4) & 0x0F0F0F0Fu);
  x = ((x & 0x33333333u) << 2) | ((x >> 2) & 0x33333333u);
  return ((x & 0x55555555u) << 1) | ((x >> 1) & 0x55555555u);
}

constexpr uint32_t kSplitBlock = 4096;  // symbols whose split ratios are precomputed together

// M for symbols i = 0..len-1 of a block: h0 before symbol i is h[i], n = n0 + i.
inline uint64_t split_ratio(int32_t h0, uint32_t n) {
  return (uint64_t)(int64_t)((double)h0 * (140737488355328.0 / (double)(int32_t)n)) + 2;  // 2^47
}
void splits_scalar(const int32_t* h, uint32_t n0, uint32_t len, uint64_t* out) {
  for (uint32_t i = 0; i < len; i++) out[i] = split_ratio(h[i], n0 + i);
}
__attribute__((target("avx512f,avx512dq"))) void splits_avx512(const int32_t* h, uint32_t n0, uint32_t len,
                                                                uint64_t* out) {
  const __m512d two47 = _mm512_set1_pd(140737488355328.0);
  const __m512d iota = _mm512_setr_pd(0, 1, 2, 3, 4, 5, 6, 7);
  const __m512i two = _mm512_set1_epi64(2);
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {  // the same IEEE operations as split_ratio, 8 at a time
    const __m512d nd = _mm512_add_pd(_mm512_set1_pd((double)(n0 + i)), iota);
    const __m512d hd = _mm512_cvtepi32_pd(_mm256_loadu_si256((const __m256i*)(h + i)));
    const __m512d q = _mm512_mul_pd(hd, _mm512_div_pd(two47, nd));
    _mm512_storeu_si512((__m512i*)(out + i), _mm512_add_epi64(_mm512_cvttpd_epi64(q), two));
  }
  splits_scalar(h + i, n0 + i, len - i, out + i);
}
const bool kHaveAvx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq");

uint64_t abac_encode(const uint64_t* feed, uint64_t nbits, uint8_t first, uint32_t s0, uint8_t* buf,
                     const uint8_t* limit) {
  uint32_t low = 0, high = 0xFFFF, r = 0xFFFF, e3 = 0, h0 = 1, n = 2;
  uint32_t low1 = 1, nlow = ~0u, nlowm1 = ~0u - 1;  // low + 1, ~low, ~low - 1
  uint64_t macc = 0;  // pending output, MSB first: the oldest of the mn bits is bit mn-1
  uint32_t mn = 0;
  uint32_t* p = reinterpret_cast<uint32_t*>(buf);  // 32-bit words, MSB-first until the final reversal
  const uint32_t* const plimit = reinterpret_cast<const uint32_t*>(buf + ((limit - buf) & ~(ptrdiff_t)3));
  alignas(64) int32_t hbuf[kSplitBlock];
  alignas(64) uint64_t mbuf[kSplitBlock];
  auto put1 = [&](uint32_t bit) {
    macc = (macc << 1) | bit;
    if (++mn >= 32) {
      mn -= 32;
      *p++ = (uint32_t)(macc >> mn);
    }
  };
  for (uint32_t i = 0; i < s0; i++) put1((first >> i) & 1u);
  for (uint64_t c0 = 0; c0 < nbits; c0 += kSplitBlock) {
    const uint32_t clen = nbits - c0 < kSplitBlock ? (uint32_t)(nbits - c0) : kSplitBlock;
    const uint64_t* fw = feed + (c0 >> 6);
    {
      uint32_t hh = h0;
      for (uint32_t i = 0; i < clen; i++) {
        hbuf[i] = (int32_t)hh;
        hh += (uint32_t)((~fw[i >> 6] >> (i & 63)) & 1u);
      }
      if (kHaveAvx512)
        splits_avx512(hbuf, n, clen, mbuf);
      else
        splits_scalar(hbuf, n, clen, mbuf);
      h0 = hh;
      n += clen;
    }
    for (uint32_t i = 0; i < clen; i++) {
      if ((i & 63) == 0 && p >= plimit) return ~0ull;  // 64 symbols emit at most 64 * 32 bits: the slack absorbs it
      const uint32_t b = (uint32_t)(fw[i >> 6] >> (i & 63)) & 1u;
      const uint32_t t = (uint32_t)(((uint64_t)r * mbuf[i]) >> 47);  // resolve_model: mid = low + t
      uint32_t l1 = low, h1 = low + t, rp1 = t + 1, ny = 2 * (h1 | nlow) + 1;  // ny = ~((l1 & ~h1) << 1)
      const uint32_t l1b = low1 + t, rp1b = r - t, nyb = 2 * (high | (nlowm1 - t)) + 1;
      asm("test %[b], %[b]\n\tcmovnz %[l1b], %[l1]\n\tcmovnz %[hb], %[h1]\n\tcmovnz %[rb], %[rp]\n\tcmovnz %[nb], %[ny]"
          : [l1] "+&r"(l1), [h1] "+&r"(h1), [rp] "+&r"(rp1), [ny] "+&r"(ny)
          : [b] "r"(b), [l1b] "r"(l1b), [hb] "r"(high), [rb] "r"(rp1b), [nb] "r"(nyb)
          : "cc");
      const uint32_t k16 = _lzcnt_u32(l1 ^ h1);  // 16 + k, k = 0..16
      const uint32_t k = k16 - 16;
      uint32_t s = k16 + _lzcnt_u32(ny << (k16 & 31)) - 16;  // k + the E3 run
      {  // the 0xBFFD bound (rare)
        uint32_t tz = _tzcnt_u32(~h1);
        tz = h1 == 0xBFFEu ? 14u : tz;
        const int32_t bound = 14 - (int32_t)tz;
        const uint32_t X = (int32_t)k > bound ? k : (uint32_t)bound;
        if (__builtin_expect(X < s, 0)) s = X;
      }
      if (__builtin_expect(e3 > 16, 0)) {  // a long pending run: bit by bit
        for (uint32_t j = 0; j < k; j++) {
          const uint32_t bit = (l1 >> (15 - j)) & 1u;
          put1(bit);
          for (; j == 0 && e3; e3--) {
            put1(bit ^ 1u);
            if (p >= plimit) return ~0ull;
          }
        }
      } else {
        const uint32_t nrun = e3 & (0u - (uint32_t)(k != 0));
        const uint32_t len = k + nrun;  // <= 32
        const uint64_t W = l1 >> (16 - k);
        macc = (macc << len) | (W + (1ull << ((len - 1) & 63)) - (1ull << ((k - 1) & 63)));
        mn += len;
        e3 -= nrun;
        const uint32_t full = mn >= 32;
        *p = (uint32_t)(macc >> ((mn - 32) & 63));
        p += full;
        mn -= full << 5;
      }
      e3 += s - k;
      r = (rp1 << s) - 1;
      low = (l1 << s) & 0x7FFFu;
      high = low + r;
      low1 = low + 1;
      nlow = ~low;
      nlowm1 = nlow - 1;
    }
  }
  // flush_encoder (abac.cpp:279-310)
  e3++;
  const uint32_t fb = low < 0x3FFFu ? 0u : 1u;
  put1(fb);
  for (; e3; e3--) {
    put1(fb ^ 1u);
    if (p >= plimit) return ~0ull;
  }
  const uint64_t total = (uint64_t)(p - reinterpret_cast<uint32_t*>(buf)) * 32 + mn;
  *p = mn ? (uint32_t)(macc << (32 - mn)) : 0u;
  for (uint32_t* q = reinterpret_cast<uint32_t*>(buf); q <= p; q++) *q = rev32(*q);
  return total;
}

// The feed: the exp-Golomb precode of a slice, LSB first, all sections
// concatenated (the coder never restarts between them).  The feed stream
// bounds each section to 32 Mbit between empty() calls (common.cpp:147); a
// write that would exceed it is dropped whole (bitstream.cpp:206-216) and the
// callers ignore the error (stream.cpp:573-578).
struct Feed {
  std::vector<uint64_t>* words;
  uint64_t cur = 0;
  uint32_t ncur = 0;
  uint32_t used = 0;
  uint64_t nbits = 0;
  inline void empty() { used = 0; }
  inline void bits(uint32_t code, uint32_t len) {  // len <= 32
    if (used + len > kFeedCapacityBits) return;
    used += len;
    nbits += len;
    cur |= (uint64_t)code << ncur;
    if (ncur + len >= 64) {
      words->push_back(cur);
      cur = (uint64_t)code >> (64 - ncur);  // ncur > 32 here
      ncur = ncur + len - 64;
    } else {
      ncur += len;
    }
  }
  void close() {
    if (ncur) words->push_back(cur);
  }
  inline void se(int16_t v) {
    const uint32_t i = (uint16_t)v;
    bits(kCodes.se_code[i], kCodes.se_len[i]);
  }
  inline void ue_run(uint32_t r) { bits(kCodes.ue_code[r], kCodes.ue_len[r]); }
};

inline const BlockDesc& desc(const uint8_t* table, uint32_t i) {
  return reinterpret_cast<const BlockDesc*>(table)[i];
}

// serialize_block_8x8 + entropy_rle_stream_encode_8x8 (serialize.cpp:10-23,
// stream.cpp:550-581).
inline void block_8x8(Feed& f, const int16_t* src, uint32_t pitch, int16_t last_dc) {
  int16_t c[64];
  for (int j = 0; j < 8; j++) memcpy(c + j * 8, src + (size_t)j * pitch, 16);
  c[0] = (int16_t)(c[0] - last_dc);
  int run = 63;
  while (run >= 0 && c[kZigzag[run]] == 0) run--;
  run++;
  f.ue_run((uint32_t)run);
  for (int k = 0; k < run; k++) f.se(c[kZigzag[k]]);
}

// serialize_image_blocks_16x16 / _8x8 (serialize.cpp:25-123).
void plane_blocks(Feed& f, const int16_t* img, uint32_t width, uint32_t height, uint32_t blk,
                  const uint8_t* table) {
  uint16_t bi = 0;
  f.empty();
  for (uint32_t j = 0; j < height; j += blk)
    for (uint32_t i = 0; i < width; i += blk) {
      const BlockDesc& d = desc(table, bi++);
      if (d.block_type & kCopy) continue;
      int16_t last_dc = 0;
      if (i >= blk)
        last_dc = img[(size_t)j * width + (i - 8)];
      else if (j >= blk)
        last_dc = img[(size_t)(j - 8) * width + i];
      const int16_t* b = img + (size_t)j * width + i;
      if (blk == 16) {
        block_8x8(f, b, width, last_dc);
        block_8x8(f, b + 8, width, b[0]);
        block_8x8(f, b + 8 * width, width, b[0]);
        block_8x8(f, b + 8 * width + 8, width, b[8 * width]);
      } else {
        block_8x8(f, b, width, last_dc);
      }
    }
}

}  // namespace

namespace {

// Code nbits of feed into out at *bit_pos (bits of the first byte below it
// preserved, bits beyond the end untouched).
int code_feed(const uint64_t* feed, uint64_t nbits, uint8_t* out, uint64_t out_bits_capacity, uint64_t* bit_pos) {
  const uint64_t pos0 = *bit_pos;
  if (pos0 > out_bits_capacity) return 7;  // EVX_ERROR_CAPACITY_LIMIT
  // Code the feed into scratch (bit 0 = bit 0 of the caller's byte pos0 / 8,
  // with its bits below pos0 preloaded), then copy; bits beyond the end stay
  // untouched.
  const uint64_t byte0 = pos0 >> 3, cap_bytes = (out_bits_capacity + 7) / 8 - byte0;
  constexpr uint64_t kSlack = 512;  // > the output of one 64-symbol feed word
  // scratch for the coder's word stores: grown without zero-filling (a 4K
  // caller's bit_stream may offer 66 MB; only the pages written are touched)
  thread_local std::unique_ptr<uint32_t[]> scratch;
  thread_local uint64_t scratch_bytes = 0;
  if (scratch_bytes < cap_bytes + kSlack) {
    scratch_bytes = (cap_bytes + kSlack + 4095) & ~(uint64_t)4095;
    scratch.reset(new uint32_t[scratch_bytes / 4]);
  }
  uint8_t* const buf = reinterpret_cast<uint8_t*>(scratch.get());
  const uint32_t s0 = (uint32_t)(pos0 & 7);
  const uint64_t total = abac_encode(feed, nbits, s0 ? out[byte0] : 0, s0, buf, buf + cap_bytes);
  if (total == ~0ull || byte0 * 8 + total > out_bits_capacity) return 7;  // EVX_ERROR_CAPACITY_LIMIT
  const uint64_t n = total - s0;
  const size_t whole = (size_t)(total >> 3);
  memcpy(out + byte0, buf, whole);
  if (total & 7) {
    const uint8_t mask = (uint8_t)((1u << (total & 7)) - 1u);
    out[byte0 + whole] = (uint8_t)((out[byte0 + whole] & ~mask) | (buf[whole] & mask));
  }
  *bit_pos = pos0 + n;
  return 0;
}

}  // namespace

int serialize_feed(const uint32_t* feed, uint64_t feed_bits, uint8_t* out, uint64_t out_bits_capacity,
                   uint64_t* bit_pos) {
  // the 32-bit feed words, LSB-first, are the coder's 64-bit words on a
  // little-endian host; bits of the last word beyond feed_bits (the buffer
  // has slack) are never coded
  thread_local std::vector<uint64_t> words;
  const size_t n64 = (size_t)((feed_bits + 63) / 64);
  const uint64_t n32 = (feed_bits + 31) / 32;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(feed);
  // unaligned, or an odd count of 32-bit words (the last 64-bit read would
  // pass the caller's buffer by 4 bytes): copy
  if (((uintptr_t)feed & 7) || (n32 & 1)) {
    words.assign(n64, 0);
    memcpy(words.data(), feed, (size_t)n32 * 4);
    w = words.data();
  }
  return code_feed(w, feed_bits, out, out_bits_capacity, bit_pos);
}

int serialize_result(cairo_ctx* ctx, int ticket, cairo_frame_result* res, uint32_t ring, uint8_t* out,
                     uint64_t out_bits_capacity, uint64_t* bit_pos) {
  if (res->feed_status == CAIRO_FEED_VALID)
    return serialize_feed(res->feed, res->feed_bits, out, out_bits_capacity, bit_pos);
  if (!res->coef_y) {
    const int r = cairo_ctx_fetch_coef(ctx, ticket, res);
    if (r) return r;
  }
  return serialize_slice(res->block_table, res->wmb, res->hmb, ring, res->coef_y, res->coef_u, res->coef_v, out,
                         out_bits_capacity, bit_pos);
}

// The precode of a slice into `words` (LSB-first feed); returns its bit count.
uint64_t precode_slice(const uint8_t* table, uint32_t wmb, uint32_t hmb, uint32_t ring, const int16_t* cy,
                       const int16_t* cu, const int16_t* cv, std::vector<uint64_t>& feed_words) {
  feed_words.clear();
  Feed f{&feed_words};
  const uint32_t count = (uint16_t)(wmb * hmb);  // uint16 block_count, serialize.cpp:321
  const uint32_t tbits = log2_u32(ring & 0xFF);  // log2((uint8)R), serialize.cpp:179

  f.empty();  // serialize_block_types (serialize.cpp:125-135)
  for (uint32_t i = 0; i < count; i++) f.bits(desc(table, i).block_type & 7u, 3);

  f.empty();  // serialize_prediction_targets (serialize.cpp:137-154)
  for (uint32_t i = 0; i < count; i++) {
    const BlockDesc& d = desc(table, i);
    if (!(d.block_type & kIntra)) f.bits(d.prediction_target & ((1u << tbits) - 1u), tbits);
  }

  f.empty();  // serialize_motion_vectors (serialize.cpp:156-191)
  int16_t last = 0;
  for (uint32_t i = 0; i < count; i++) {
    const BlockDesc& d = desc(table, i);
    if (!(d.block_type & kMotion)) continue;
    f.se((int16_t)(d.motion_x - last));
    last = d.motion_x;
  }
  last = 0;
  for (uint32_t i = 0; i < count; i++) {
    const BlockDesc& d = desc(table, i);
    if (!(d.block_type & kMotion)) continue;
    f.se((int16_t)(d.motion_y - last));
    last = d.motion_y;
  }

  f.empty();  // serialize_subpixel_motion_params (serialize.cpp:193-241)
  for (uint32_t i = 0; i < count; i++) {
    const BlockDesc& d = desc(table, i);
    if (d.block_type & kMotion) f.bits(d.sp_pred & 1u, 1);
  }
  for (uint32_t i = 0; i < count; i++) {
    const BlockDesc& d = desc(table, i);
    if ((d.block_type & kMotion) && d.sp_pred) f.bits(d.sp_amount & 1u, 1);
  }
  for (uint32_t i = 0; i < count; i++) {
    const BlockDesc& d = desc(table, i);
    if ((d.block_type & kMotion) && d.sp_pred) f.bits(d.sp_index & 7u, 3);
  }

  f.empty();  // serialize_block_quality (serialize.cpp:243-261)
  int16_t lq = 0;
  for (uint32_t i = 0; i < count; i++) {
    const BlockDesc& d = desc(table, i);
    if (d.block_type & kCopy) continue;
    f.se((int16_t)(d.q_index - lq));
    lq = d.q_index;
  }

  const uint32_t wa = wmb * 16, ha = hmb * 16;  // serialize_macroblocks (serialize.cpp:125-155)
  plane_blocks(f, cy, wa, ha, 16, table);
  plane_blocks(f, cu, wa / 2, ha / 2, 8, table);
  plane_blocks(f, cv, wa / 2, ha / 2, 8, table);

  f.close();
  return f.nbits;
}

int serialize_slice(const uint8_t* table, uint32_t wmb, uint32_t hmb, uint32_t ring,
                    const int16_t* cy, const int16_t* cu, const int16_t* cv, uint8_t* out,
                    uint64_t out_bits_capacity, uint64_t* bit_pos) {
  if (*bit_pos > out_bits_capacity) return 7;  // EVX_ERROR_CAPACITY_LIMIT
  thread_local std::vector<uint64_t> feed_words;
  const uint64_t nbits = precode_slice(table, wmb, hmb, ring, cy, cu, cv, feed_words);
  return code_feed(feed_words.data(), nbits, out, out_bits_capacity, bit_pos);
}

}  // namespace cairo

extern "C" int cairo_serialize_feed(const uint32_t* feed, uint64_t feed_bits, uint8_t* out, uint32_t out_bytes,
                                    uint32_t* bit_pos) {
  if (!feed || !out || !bit_pos) return 1;
  uint64_t pos = *bit_pos;
  int r = cairo::serialize_feed(feed, feed_bits, out, (uint64_t)out_bytes * 8u, &pos);
  *bit_pos = (uint32_t)pos;
  return r;
}

extern "C" int cairo_precode_slice(const uint8_t* block_table, uint32_t wmb, uint32_t hmb, uint32_t ring,
                                   const int16_t* cy, const int16_t* cu, const int16_t* cv, uint32_t* feed,
                                   uint64_t feed_words, uint64_t* feed_bits) {
  if (!block_table || !cy || !cu || !cv || !feed_bits) return 1;
  std::vector<uint64_t> words;
  const uint64_t nbits = cairo::precode_slice(block_table, wmb, hmb, ring, cy, cu, cv, words);
  *feed_bits = nbits;
  const uint64_t need = (nbits + 31) / 32;
  if (!feed || feed_words < need) return 7;  // EVX_ERROR_CAPACITY_LIMIT: *feed_bits says how much is needed
  memcpy(feed, words.data(), (size_t)need * 4);
  return 0;
}

extern "C" int cairo_serialize_slice(const uint8_t* block_table, uint32_t wmb, uint32_t hmb,
                                     uint32_t ring, const int16_t* cy, const int16_t* cu,
                                     const int16_t* cv, uint8_t* out, uint32_t out_bytes,
                                     uint32_t* bit_pos) {
  if (!block_table || !cy || !cu || !cv || !out || !bit_pos) return 1;
  uint64_t pos = *bit_pos;
  int r = cairo::serialize_slice(block_table, wmb, hmb, ring, cy, cu, cv, out,
                                 (uint64_t)out_bytes * 8u, &pos);
  *bit_pos = (uint32_t)pos;
  return r;
}
