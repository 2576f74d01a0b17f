// cairo_amd/csrc/unserialize.cpp -- host entropy decode of one frame
// (unserialize_slice, reference unserialize.cpp:8-342), the inverse of
// entropy.cpp.
//
// The adaptive binary arithmetic decoder (abac.cpp:123-151, 226-278, 350-420)
// feeds exp-Golomb / raw-bit readers (stream.cpp:292-431, 583-606) that fill
// the persistent block table and the persistent coefficient planes (the
// decoder's input_cache).  Fields the stream does not carry for a block (e.g.
// the motion vector of a non-motion block, the coefficients of a copy block)
// keep their previous values, as in the reference.  Like the reference, the
// decoder reads the caller's bit_stream from its read index and keeps
// shifting bits in after the stream is exhausted (the last bit read repeats
// within a scaling step, abac.cpp:257-263).
#include <cstdint>
#include <cstring>

#include "../../include/cairo_amd.h"
#include "evx_defs.h"

namespace cairo {

namespace {

constexpr int kOk = 0, kInvalidResource = 8;

// EVX_MACROBLOCK_8x8_ZIGZAG (scan.h:60-70): raster index of scan position k.
constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18,
                                 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                                 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43,
                                 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
                                 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// The caller's bit_stream between its read and write indices (LSB-first).
struct Source {
  const uint8_t* data;
  uint32_t rd, wr;
  bool empty() const { return rd == wr; }  // bitstream.cpp:141-144
  uint32_t bit() {
    const uint32_t b = (data[rd >> 3] >> (rd & 7)) & 1u;
    rd++;
    return b;
  }
};

// The feed stream between the decoder and the readers (common.cpp:147): a
// FIFO of decoded bits, emptied per section, 32 Mbit per section.
struct Feed {
  uint64_t bits = 0;
  uint32_t count = 0, used = 0;
  void empty() { bits = 0, count = 0, used = 0; }
  void write(uint32_t b) {
    if (used >= kFeedCapacityBits || count >= 64) return;  // write_bit fails, bit dropped
    used++;
    bits |= (uint64_t)b << count;
    count++;
  }
  // read_bits: n bits LSB-first into the low bits of *v, the others kept;
  // fails (and reads nothing) when fewer than n bits are pending.
  bool read(uint32_t n, uint32_t* v) {
    if (count < n) return false;
    const uint32_t m = (1u << n) - 1u;
    *v = (*v & ~m) | (uint32_t)(bits & m);
    bits >>= n;
    count -= n;
    return true;
  }
};

// Adaptive binary arithmetic decoder, 16-bit precision.
struct Decoder {
  Source* src;
  Feed* feed;
  uint32_t low = 0, high = 0xFFFF, value = 0, h0 = 1, h1 = 1;

  void start() {  // clear() + start_decode (abac.cpp:58-78, 396-420)
    low = 0, high = 0xFFFF, value = 0, h0 = 1, h1 = 1;
    uint32_t b = 0;
    for (int i = 0; i < 16; i++) {
      if (!src->empty()) b = src->bit();
      value = (value << 1) | b;
    }
  }
  // decode(1): one symbol into the feed (decode_symbol + resolve_decode_scaling)
  void symbol() {
    const uint32_t mid = low + (uint32_t)(((uint64_t)(high - low) * h0) / (h0 + h1));  // resolve_model
    if (value >= low && value <= mid) {
      high = mid;
      h0++;
      feed->write(0);
    } else if (value > mid && value <= high) {
      low = mid + 1;
      h1++;
      feed->write(1);
    }
    uint32_t b = 0;
    for (;;) {
      if (high <= 0x7FFFu) {
      } else if (low > 0x7FFFu) {
        high -= 0x8000u, low -= 0x8000u, value -= 0x8000u;
      } else if (high <= 0xBFFDu && low > 0x3FFFu) {  // E3
        high -= 0x4000u, low -= 0x4000u, value -= 0x4000u;
      } else {
        break;
      }
      if (!src->empty()) b = src->bit();
      high = ((high << 1) & 0xFFFFu) | 1u;
      low = (low << 1) & 0xFFFFu;
      value = ((value << 1) & 0xFFFFu) | b;
    }
  }
  // decode(n) then read_bits(n) into the low bits of *v
  bool bits(uint32_t n, uint32_t* v) {
    for (uint32_t i = 0; i < n; i++) symbol();
    return feed->read(n, v);
  }
  // exp-Golomb value (entropy_stream_decode_value, stream.cpp:292-431): the
  // code as it is read (zero prefix, then zero_count + 1 bits MSB first) and
  // the total bit count; false on a runaway prefix (a corrupt stream).
  bool golomb(uint32_t* code, uint32_t* zeros) {
    uint32_t bv = 0;
    symbol();
    feed->read(1, &bv);
    uint32_t z = 0;
    while (!(bv & 0xFFu)) {
      if (++z > 40) return false;
      symbol();
      feed->read(1, &bv);
    }
    uint32_t r = 0;
    for (uint32_t i = 0; i <= z; i++) {
      r = (r << 1) | (bv & 1u);
      if (i < z) {
        symbol();
        feed->read(1, &bv);
      }
    }
    *code = r;
    *zeros = z;
    return true;
  }
  bool ue(uint16_t* out) {
    uint32_t r, z;
    if (!golomb(&r, &z)) return false;
    *out = (uint16_t)(r - 1u);
    return true;
  }
  bool se(int16_t* out) {
    uint32_t r, z;
    if (!golomb(&r, &z)) return false;
    const int16_t res = (int16_t)r;  // the reference accumulates in an int16
    const int32_t sign = 1 - 2 * (res & 1);
    int16_t v = (int16_t)(sign * ((res >> 1) & 0x7FFF));
    if (2 * z + 1 > 0x20) v = (int16_t)(v | 0x8000);  // stream.cpp:424-431
    *out = v;
    return true;
  }
};

// unserialize_block_8x8 (unserialize.cpp:8-21) with the RLE decode
// (stream.cpp:583-606).
bool block_8x8(Decoder& d, int16_t last_dc, int16_t* dst, uint32_t pitch) {
  int16_t c[64];
  memset(c, 0, sizeof(c));
  uint16_t run = 0;
  if (!d.ue(&run) || run > 64) return false;
  for (uint32_t k = 0; k < run; k++)
    if (!d.se(&c[kZigzag[k]])) return false;
  c[0] = (int16_t)(c[0] + last_dc);
  for (int j = 0; j < 8; j++) memcpy(dst + (size_t)j * pitch, c + j * 8, 16);
  return true;
}

// unserialize_image_blocks_16x16 / _8x8 (unserialize.cpp:34-130).
bool plane_blocks(Decoder& d, int16_t* img, uint32_t width, uint32_t height, uint32_t blk,
                  const BlockDesc* table) {
  uint16_t bi = 0;
  d.feed->empty();
  for (uint32_t j = 0; j < height; j += blk)
    for (uint32_t i = 0; i < width; i += blk) {
      const BlockDesc& b = table[bi++];
      if (b.block_type & kCopy) continue;
      int16_t last_dc = 0;
      if (i >= blk)
        last_dc = img[(size_t)j * width + (i - 8)];
      else if (j >= blk)
        last_dc = img[(size_t)(j - 8) * width + i];
      int16_t* p = img + (size_t)j * width + i;
      if (blk == 16) {
        if (!block_8x8(d, last_dc, p, width) || !block_8x8(d, p[0], p + 8, width) ||
            !block_8x8(d, p[0], p + 8 * width, width) ||
            !block_8x8(d, p[8 * width], p + 8 * width + 8, width))
          return false;
      } else if (!block_8x8(d, last_dc, p, width)) {
        return false;
      }
    }
  return true;
}

}  // namespace

// unserialize_slice (unserialize.cpp:321-342): the payload at *read_index of
// data (up to write_index) -> table (wmb*hmb descs) and coefficient planes,
// both persistent across frames.
int unserialize_slice(const uint8_t* data, uint32_t* read_index, uint32_t write_index, uint32_t wmb,
                      uint32_t hmb, uint32_t ring, BlockDesc* table, int16_t* cy, int16_t* cu,
                      int16_t* cv) {
  Source src{data, *read_index, write_index};
  Feed feed;
  Decoder d{&src, &feed};
  const uint32_t count = (uint16_t)(wmb * hmb);  // uint16 block_count, unserialize.cpp:323
  const uint32_t tbits = log2_u32(ring & 0xFF);   // log2((uint8)R), unserialize.cpp:178
  d.start();

  feed.empty();  // block types (unserialize.cpp:150-162)
  for (uint32_t i = 0; i < count; i++) d.bits(3, &table[i].block_type);

  feed.empty();  // prediction targets (:164-181)
  for (uint32_t i = 0; i < count; i++) {
    if (table[i].block_type & kIntra) continue;
    uint32_t v = table[i].prediction_target;
    if (tbits) d.bits(tbits, &v);
    table[i].prediction_target = (uint8_t)v;
  }

  feed.empty();  // motion vectors (:183-221)
  int16_t last = 0;
  for (uint32_t i = 0; i < count; i++) {
    if (!(table[i].block_type & kMotion)) continue;
    int16_t v = 0;
    if (!d.se(&v)) return kInvalidResource;
    table[i].motion_x = (int16_t)(last + v);
    last = table[i].motion_x;
  }
  last = 0;
  for (uint32_t i = 0; i < count; i++) {
    if (!(table[i].block_type & kMotion)) continue;
    int16_t v = 0;
    if (!d.se(&v)) return kInvalidResource;
    table[i].motion_y = (int16_t)(last + v);
    last = table[i].motion_y;
  }

  feed.empty();  // sub-pixel parameters (:223-267)
  for (uint32_t i = 0; i < count; i++) {
    if (!(table[i].block_type & kMotion)) continue;
    uint32_t v = table[i].sp_pred;
    d.bits(1, &v);
    table[i].sp_pred = (uint8_t)v;
  }
  for (uint32_t i = 0; i < count; i++) {
    if (!(table[i].block_type & kMotion) || !table[i].sp_pred) continue;
    uint32_t v = table[i].sp_amount;
    d.bits(1, &v);
    table[i].sp_amount = (uint8_t)v;
  }
  for (uint32_t i = 0; i < count; i++) {
    if (!(table[i].block_type & kMotion) || !table[i].sp_pred) continue;
    uint32_t v = table[i].sp_index;
    d.bits(3, &v);
    table[i].sp_index = (uint8_t)v;
  }

  feed.empty();  // block quality (:269-287)
  int16_t lq = 0;
  for (uint32_t i = 0; i < count; i++) {
    if (table[i].block_type & kCopy) continue;
    int16_t v = 0;
    if (!d.se(&v)) return kInvalidResource;
    table[i].q_index = (uint8_t)(v + lq);
    lq = table[i].q_index;
  }

  const uint32_t wa = wmb * 16, ha = hmb * 16;  // unserialize_macroblocks (:132-160)
  if (!plane_blocks(d, cy, wa, ha, 16, table) || !plane_blocks(d, cu, wa / 2, ha / 2, 8, table) ||
      !plane_blocks(d, cv, wa / 2, ha / 2, 8, table))
    return kInvalidResource;
  *read_index = src.rd;
  return kOk;
}

}  // namespace cairo

extern "C" int cairo_unserialize_slice(const uint8_t* data, uint32_t* read_index, uint32_t write_index,
                                       uint32_t wmb, uint32_t hmb, uint32_t ring, uint8_t* block_table,
                                       int16_t* coef_y, int16_t* coef_u, int16_t* coef_v) {
  if (!data || !read_index || !block_table || !coef_y || !coef_u || !coef_v || *read_index > write_index)
    return 1;  // EVX_ERROR_INVALIDARG
  return cairo::unserialize_slice(data, read_index, write_index, wmb, hmb, ring,
                                  reinterpret_cast<cairo::BlockDesc*>(block_table), coef_y, coef_u, coef_v);
}
