// cairo_amd/csrc/entropy.cpp -- host entropy stage (stays on the CPU by design).
//
// serialize_slice (reference serialize.cpp:319-340): block-table sections,
// delta-DC zig-zag run-length coefficients, exp-Golomb precode, adaptive
// binary arithmetic coder (abac.cpp).  The coder is bit-serial by
// construction (one adaptive model per frame), so the speed comes from a
// tight loop: table-driven exp-Golomb codes fed straight into the coder (no
// intermediate feed buffer), a 64-bit output accumulator, and frames spread
// over host threads by the caller.
#include <cstdint>
#include <cstring>

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

// LSB-first bit writer into the caller's buffer (bit_stream semantics,
// bitstream.cpp:181-245: bits beyond write_index are left untouched).
struct BitWriter {
  uint8_t* data;
  uint64_t cap_bits;
  uint64_t pos;     // bits committed to data
  uint64_t acc = 0; // pending bits, LSB first
  uint32_t nacc = 0;
  bool overflow = false;

  inline void put(uint32_t b) {
    acc |= (uint64_t)(b & 1u) << nacc;
    if (++nacc == 56) flush();
  }
  inline void put_run(uint32_t b, uint32_t n) {
    while (n) {
      uint32_t k = n < 56 - nacc ? n : 56 - nacc;
      if (b) acc |= ((k == 64 ? ~0ull : ((1ull << k) - 1)) << nacc);
      nacc += k;
      n -= k;
      if (nacc == 56) flush();
    }
  }
  void flush() {
    if (!nacc) return;
    if (pos + nacc > cap_bits) {
      overflow = true;
      nacc = 0;
      acc = 0;
      return;
    }
    uint32_t n = nacc;
    uint64_t v = acc;
    while (n) {
      const uint32_t byte = (uint32_t)(pos >> 3), sh = (uint32_t)(pos & 7);
      const uint32_t take = (8 - sh) < n ? (8 - sh) : n;
      const uint32_t mask = ((1u << take) - 1u) << sh;
      data[byte] = (uint8_t)((data[byte] & ~mask) | (((uint32_t)v << sh) & mask));
      v >>= take;
      n -= take;
      pos += take;
    }
    acc = 0;
    nacc = 0;
  }
};

// Adaptive binary arithmetic coder, 16-bit precision (abac.cpp:28-348).
struct Abac {
  uint32_t low = 0, high = 0xFFFF, e3 = 0, h0 = 1, h1 = 1;
  BitWriter* out;

  inline void code(uint32_t bit) {
    const uint64_t range = high - low;
    const uint32_t mid = low + (uint32_t)((range * h0) / (h0 + h1));  // resolve_model
    if (bit) {
      low = mid + 1;
      h1++;
    } else {
      high = mid;
      h0++;
    }
    for (;;) {  // resolve_encode_scaling
      if (((high ^ low) & 0x8000u) == 0) {
        const uint32_t msb = high >> 15;
        low -= msb << 15;
        high -= msb << 15;
        out->put(msb);
        if (e3) {
          out->put_run(msb ^ 1u, e3);
          e3 = 0;
        }
      } else if (high <= 0xBFFDu && low > 0x3FFFu) {
        high -= 0x4000u;
        low -= 0x4000u;
        e3++;
      } else {
        break;
      }
      high = ((high << 1) & 0xFFFFu) | 1u;
      low = (low << 1) & 0xFFFFu;
    }
  }
  void finish() {  // flush_encoder (abac.cpp:279-310)
    e3++;
    const uint32_t b = low < 0x3FFFu ? 0u : 1u;
    out->put(b);
    out->put_run(b ^ 1u, e3);
    e3 = 0;
  }
};

// The feed stream bounds each section to 32 Mbit of precode between empty()
// calls (common.cpp:147); a write that would exceed it is dropped whole
// (bitstream.cpp:206-216) and the callers ignore the error (stream.cpp:573-578).
struct Feed {
  Abac* coder;
  uint32_t used = 0;
  inline void empty() { used = 0; }
  inline void bits(uint32_t code, uint32_t len) {
    if (used + len > kFeedCapacityBits) return;
    used += len;
    for (uint32_t k = 0; k < len; k++) coder->code((code >> k) & 1u);
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

int serialize_slice(const uint8_t* table, uint32_t wmb, uint32_t hmb, uint32_t ring,
                    const int16_t* cy, const int16_t* cu, const int16_t* cv, uint8_t* out,
                    uint64_t out_bits_capacity, uint64_t* bit_pos) {
  BitWriter w{out, out_bits_capacity, *bit_pos};
  Abac a;
  a.out = &w;
  Feed f{&a};
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

  a.finish();
  w.flush();
  *bit_pos = w.pos;
  return w.overflow ? 7 /* EVX_ERROR_CAPACITY_LIMIT */ : 0;
}

}  // namespace cairo

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
