// cairo_amd/csrc/encoder.cpp -- the drop-in evx1_encoder (reference
// evx1enc.cpp:13-168, evx1.cpp:8-63) on top of the GPU backend.
//
// encode(): lazy init (header), frame descriptor, GPU hot path
// (cairo_ctx_submit/wait: convert, inter + intra search, transform, VAQ,
// quantize, reconstruct, deblock, and the entropy precode), the arithmetic
// coder on the host appended to the caller's bit_stream, then the
// reference's frame-state update.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/cairo_amd.h"
#include "../../include/evx1.h"
#include "entropy.h"
#include "evx_defs.h"
#include "stream_format.h"

namespace evx {

namespace {

constexpr uint32 kDefaultRing = 4;         // EVX_REFERENCE_FRAME_COUNT, config.h:39
constexpr uint16 kDefaultQuality = 8;      // EVX_DEFAULT_QUALITY_LEVEL, config.h:40
constexpr uint32 kPeriodicIntra = 3600;    // EVX_PERIODIC_INTRA_RATE, config.h:41

int clip_quality(int q) { return q < 1 ? 1 : (q > 31 ? 31 : q); }

// EVX_CONVERT_PIXEL_YUV_TO_RGB with saturate (convert.cpp:16-19; saturate
// narrows to int16 before clipping, math.h:218-221).
inline uint8 sat(int32 v) {
  const int16 s = (int16)v;
  return (uint8)(s < 0 ? 0 : (s > 255 ? 255 : s));
}

}  // namespace

class gpu_encoder : public evx1_encoder {
 public:
  gpu_encoder() { reset_frame(); }
  ~gpu_encoder() override { clear(); }

  evx_status clear() override {  // evx1enc.cpp:27-40
    if (!initialized_) return EVX_SUCCESS;
    reset_frame();
    cairo_ctx_destroy(ctx_);
    ctx_ = nullptr;
    free(last_table_);
    last_table_ = nullptr;
    initialized_ = false;
    return EVX_SUCCESS;
  }
  evx_status insert_intra() override {  // evx1enc.cpp:42-51
    frame_.type = 0;
    return EVX_SUCCESS;
  }
  evx_status set_quality(uint8 quality) override {  // evx1enc.cpp:53-64
    frame_.quality = (uint16)clip_quality(quality);
    return EVX_SUCCESS;
  }

  evx_status encode(void *image, uint32 width, uint32 height, bit_stream *output) override {
    if (!image || !output || !width || !height) return EVX_ERROR_INVALIDARG;
    if (!initialized_) {  // evx1enc.cpp:104-117
      if (initialize(width, height) != EVX_SUCCESS) return EVX_ERROR_EXECUTION_FAILURE;
      header_t h;
      memset(&h, 0, sizeof(h));  // byte 7 is an unwritten pad in the reference; 0 here
      h.magic[0] = 'E';
      h.magic[1] = 'V';
      h.magic[2] = 'X';
      h.magic[3] = '1';
      h.size = sizeof(header_t);
      h.ref_count = (uint8)ring_;
      h.version = kVersionWord;
      h.frame_width = (uint16)width;
      h.frame_height = (uint16)height;
      if (evx_failed(output->write_bytes(&h, sizeof(h)))) return EVX_ERROR_EXECUTION_FAILURE;
    }
    if (width != width_ || height != height_) return EVX_ERROR_INVALID_RESOURCE;
    frame_t f = frame_;
    if (evx_failed(output->write_bytes(&f, sizeof(f)))) return EVX_ERROR_EXECUTION_FAILURE;

    const auto t0 = std::chrono::steady_clock::now();
    int ticket = -1;
    int r = cairo_ctx_submit(ctx_, (const uint8_t *)image, 0, frame_.index, frame_.type,
                             frame_.quality, &ticket);
    if (r) return EVX_ERROR_EXECUTION_FAILURE;
    cairo_frame_result res;
    r = cairo_ctx_wait(ctx_, ticket, &res);
    if (r) {
      cairo_ctx_release(ctx_, ticket);
      return EVX_ERROR_EXECUTION_FAILURE;
    }
    const auto t1 = std::chrono::steady_clock::now();
    uint64_t pos = output->query_write_index();
    r = cairo::serialize_result(ctx_, ticket, &res, ring_, output->query_data(), output->query_capacity(), &pos);
    if (trace_) {  // CAIRO_ENCODE_TRACE=1: where a synchronous encode() spends its time
      const auto t2 = std::chrono::steady_clock::now();
      fprintf(stderr, "[cairo_amd] encode frame %u: gpu+transfers %.3f ms, host coder %.3f ms (feed %s)\n",
              frame_.index, std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(t2 - t1).count(),
              res.feed_status == CAIRO_FEED_VALID ? "gpu" : "host");
    }
    memcpy(last_table_, res.block_table, (size_t)res.wmb * res.hmb * 16);
    cairo_ctx_release(ctx_, ticket);
    if (r) return EVX_ERROR_EXECUTION_FAILURE;
    output->advance_write_index((uint32)(pos - output->query_write_index()));

    frame_.type = 1;  // evx1enc.cpp:138-153
    if (((frame_.index + 1) % kPeriodicIntra) == 0) insert_intra();
    frame_.index++;
    return EVX_SUCCESS;
  }

  // Debug views (evx1enc.cpp:170-305); DESTINATION is the slot of the last frame.
  evx_status peek(EVX_PEEK_STATE state, void *output) override {
    if (!output) return EVX_ERROR_INVALIDARG;
    if (!initialized_) return EVX_SUCCESS;
    uint8 *out = (uint8 *)output;
    const uint32 wa = (width_ + 15) & ~15u, ha = (height_ + 15) & ~15u, wmb = wa / 16;
    if (state == EVX_PEEK_SOURCE || state == EVX_PEEK_DESTINATION) {
      const size_t ny = (size_t)wa * ha, nc = ny / 4;
      int16 *buf = (int16 *)malloc((ny + 2 * nc) * 2);
      if (!buf) return EVX_ERROR_OUTOFMEMORY;
      const int which =
          state == EVX_PEEK_SOURCE ? 0 : 2 + (int)((frame_.index + ring_ - 1) % ring_);
      if (cairo_ctx_read_planes(ctx_, which, buf, buf + ny, buf + ny + nc)) {
        free(buf);
        return EVX_ERROR_HARDWAREFAIL;
      }
      for (uint32 j = 0; j < height_; j++)
        for (uint32 i = 0; i < width_; i++) {  // convert.cpp:162-223
          const int32 y = buf[(size_t)j * wa + i] - 16;
          const int32 u = buf[ny + (size_t)(j / 2) * (wa / 2) + i / 2] - 128;
          const int32 v = buf[ny + nc + (size_t)(j / 2) * (wa / 2) + i / 2] - 128;
          uint8 *p = out + ((size_t)j * width_ + i) * 3;
          p[0] = sat((256 * y + 358 * v + 128) >> 8);
          p[1] = sat((256 * y - 88 * u - 182 * v + 128) >> 8);
          p[2] = sat((256 * y + 452 * u + 128) >> 8);
        }
      free(buf);
      return EVX_SUCCESS;
    }
    const cairo::BlockDesc *t = (const cairo::BlockDesc *)last_table_;
    for (uint32 j = 0; j < height_; j++)
      for (uint32 i = 0; i < width_; i++) {
        const cairo::BlockDesc &d = t[(i / 16) + (j / 16) * wmb];
        uint8 *p = out + ((size_t)j * width_ + i) * 3;
        const bool copy = (d.block_type & cairo::kCopy) != 0;
        switch (state) {
          case EVX_PEEK_BLOCK_TABLE:
            p[2] = 255 * copy;
            p[1] = 255 * ((d.block_type & cairo::kMotion) != 0);
            p[0] = 255 * ((d.block_type & cairo::kIntra) != 0);
            break;
          case EVX_PEEK_QUANT_TABLE:
            if (!copy) p[0] = p[1] = p[2] = (uint8)(255 - 15 * d.q_index);
            else p[0] = 255, p[1] = 0, p[2] = 0;
            break;
          case EVX_PEEK_BLOCK_VARIANCE:
            if (!copy) {
              int16 v = (int16)(d.variance / 30);
              v = v < 0 ? 0 : (v > 255 ? 255 : v);
              p[0] = p[1] = p[2] = (uint8)v;
            } else {
              p[0] = 255, p[1] = 0, p[2] = 0;
            }
            break;
          case EVX_PEEK_SPMP_TABLE:
            if (!d.sp_pred) p[0] = p[1] = p[2] = 0;
            else p[0] = 0, p[1] = (uint8)(255 * d.sp_amount), p[2] = (uint8)(255 * !d.sp_amount);
            break;
          default:
            return EVX_ERROR_NOTIMPL;
        }
      }
    return EVX_SUCCESS;
  }

  // libcairo_amd configuration (before the first encode).
  evx_status set_ring(uint32 ring) {
    if (initialized_ || ring < 2 || ring > (uint32)cairo::kMaxRing) return EVX_ERROR_INVALIDARG;
    ring_ = ring;
    return EVX_SUCCESS;
  }
  evx_status set_device(int device) {
    if (initialized_) return EVX_ERROR_INVALIDARG;
    device_ = device;
    return EVX_SUCCESS;
  }

 private:
  void reset_frame() {  // clear_frame, common.cpp:50-65
    frame_.type = 0;
    frame_.index = 0;
    frame_.quality = kDefaultQuality;
  }
  evx_status initialize(uint32 width, uint32 height) {  // evx1enc.cpp:66-90
    if (width > 0xFFFF || height > 0xFFFF) return EVX_ERROR_INVALIDARG;
    // one frame in flight: two staging slots (the previous frame's output_cache
    // stays in the other one, for the copy-macroblock chain)
    if (cairo_ctx_create_ex(width, height, ring_, device_, 2, &ctx_)) return EVX_ERROR_HARDWAREFAIL;
    // the GPU precodes the entropy feed; only the arithmetic coder runs here
    if (cairo_ctx_set_outputs(ctx_, CAIRO_OUT_FEED)) return EVX_ERROR_HARDWAREFAIL;
    const size_t mbs = (size_t)((width + 15) / 16) * ((height + 15) / 16);
    last_table_ = (uint8 *)calloc(mbs, 16);
    if (!last_table_) return EVX_ERROR_OUTOFMEMORY;
    width_ = width;
    height_ = height;
    initialized_ = true;
    return EVX_SUCCESS;
  }

  bool initialized_ = false;
  const bool trace_ = getenv("CAIRO_ENCODE_TRACE") != nullptr;
  frame_t frame_;
  uint32 width_ = 0, height_ = 0;
  uint32 ring_ = kDefaultRing;
  int device_ = 0;
  cairo_ctx *ctx_ = nullptr;
  uint8 *last_table_ = nullptr;
};

evx_status create_encoder(evx1_encoder **output) {
  if (!output) return EVX_ERROR_INVALIDARG;
  *output = new (std::nothrow) gpu_encoder;
  return *output ? EVX_SUCCESS : EVX_ERROR_OUTOFMEMORY;
}

evx_status destroy_encoder(evx1_encoder *input) {
  if (!input) return EVX_ERROR_INVALIDARG;
  delete static_cast<gpu_encoder *>(input);
  return EVX_SUCCESS;
}

}  // namespace evx

extern "C" {

int evx_encoder_create(void **enc) {
  evx::evx1_encoder *e = nullptr;
  const int r = evx::create_encoder(&e);
  *enc = e;
  return r;
}
int evx_encoder_destroy(void *enc) { return evx::destroy_encoder((evx::evx1_encoder *)enc); }
int evx_encoder_clear(void *enc) { return ((evx::evx1_encoder *)enc)->clear(); }
int evx_encoder_insert_intra(void *enc) { return ((evx::evx1_encoder *)enc)->insert_intra(); }
int evx_encoder_set_quality(void *enc, uint8_t q) { return ((evx::evx1_encoder *)enc)->set_quality(q); }
int evx_encoder_encode(void *enc, const void *rgb, uint32_t w, uint32_t h, void *bs) {
  return ((evx::evx1_encoder *)enc)->encode((void *)rgb, w, h, (evx::bit_stream *)bs);
}
int evx_encoder_peek(void *enc, int state, void *rgb) {
  return ((evx::evx1_encoder *)enc)->peek((evx::EVX_PEEK_STATE)state, rgb);
}
int evx_encoder_set_ring(void *enc, uint32_t ring) {
  return static_cast<evx::gpu_encoder *>((evx::evx1_encoder *)enc)->set_ring(ring);
}
int evx_encoder_set_device(void *enc, int device) {
  return static_cast<evx::gpu_encoder *>((evx::evx1_encoder *)enc)->set_device(device);
}

// band4 generator: deterministic synthetic content.
void cairo_make_band4(uint8_t *rgb, uint32_t w, uint32_t h, uint32_t t, uint32_t seed) {
  uint32_t s = seed * 2654435761u + t * 40503u;
  for (uint32_t y = 0; y < h; y++) {
    const uint32_t band = (y * 4) / h;
    uint8_t *row = rgb + (size_t)y * w * 3;
    for (uint32_t x = 0; x < w; x++) {
      uint32_t r, g, b, n = 0;
      if (band == 0) {
        r = 90, g = 140, b = 200;
      } else if (band == 1) {
        const uint32_t bx = x + 2 * t;
        r = (bx / 2) & 255;
        g = ((bx / 32) & 1) ? 200 : 60;
        b = 100;
      } else if (band == 2) {
        const uint32_t bx = x + 2 * t, by = y + t;
        r = (bx * 7 + by * 3) & 255;
        g = (((bx >> 3) ^ (by >> 3)) & 1) * 160 + 40;
        b = ((bx * bx + by * by) >> 6) & 255;
      } else {
        const uint32_t bx = x + 3 * t, by = y + t;
        s = s * 1664525u + 1013904223u;
        n = (s >> 27) & 7;
        r = (bx * 5) & 255;
        g = (by * 3) & 255;
        b = ((bx ^ by) & 63) * 4;
      }
      row[3 * x] = (uint8_t)((r + n) & 255);
      row[3 * x + 1] = (uint8_t)((g + n) & 255);
      row[3 * x + 2] = (uint8_t)((b + n) & 255);
    }
  }
}

}  // extern "C"
