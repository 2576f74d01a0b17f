// cairo_amd/csrc/decoder.cpp -- the drop-in evx1_decoder (reference
// evx1dec.cpp:13-136, evx1.cpp:28-81, decode.cpp:146-198) on top of the GPU
// backend.
//
// decode(): lazy init from the stream header, frame descriptor, host entropy
// decode (unserialize_slice, into the persistent block table and coefficient
// planes), then the GPU hot path (cairo_ctx_decode_frame: the decode-mode
// engine reconstructs and deblocks the frame into its ring slot, and
// convert_image writes RGB888), then the reference's frame-state update.
// Like the reference, decode consumes the caller's bit_stream and empties it.
#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/cairo_amd.h"
#include "../../include/evx1.h"
#include "evx_defs.h"
#include "stream_format.h"

namespace cairo {
int unserialize_slice(const uint8_t* data, uint32_t* read_index, uint32_t write_index, uint32_t wmb,
                      uint32_t hmb, uint32_t ring, BlockDesc* table, int16_t* cy, int16_t* cu, int16_t* cv);
}

namespace evx {

namespace {

// decode_block's switch (decode.cpp:14-142) accepts these seven types.
inline bool legal_type(uint32 t) { return t <= 7 && t != 5; }

// frac_index -> direction (motion.cpp:61-109); sp_index 0..7.
inline void frac_dir(uint32 idx, int32 *dx, int32 *dy) {
  static const int8_t kDx[8] = {-1, 0, 1, -1, 1, -1, 0, 1};
  static const int8_t kDy[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
  *dx = kDx[idx & 7];
  *dy = kDy[idx & 7];
}

}  // namespace

class gpu_decoder : public evx1_decoder {
 public:
  gpu_decoder() { frame_index_ = 0; }
  ~gpu_decoder() override { clear(); }

  evx_status clear() override {  // evx1dec.cpp:27-41
    if (!initialized_) return EVX_SUCCESS;
    cairo_ctx_destroy(ctx_);
    ctx_ = nullptr;
    free(table_);
    free(coef_);
    table_ = nullptr;
    coef_ = nullptr;
    frame_index_ = 0;
    initialized_ = false;
    return EVX_SUCCESS;
  }

  evx_status decode(bit_stream *input, void *output) override {  // evx1dec.cpp:90-124
    if (!input || !output) return EVX_ERROR_INVALIDARG;
    if (!initialized_ && initialize(input) != EVX_SUCCESS) return EVX_ERROR_EXECUTION_FAILURE;
    frame_t f;  // read_frame_desc (evx1dec.cpp:75-88)
    if (input->read_bytes(&f, sizeof(f)) != EVX_SUCCESS || f.index != frame_index_)
      return EVX_ERROR_EXECUTION_FAILURE;
    uint32 rd = input->query_read_index();
    const size_t ny = (size_t)wa_ * ha_, nc = ny / 4;
    if (cairo::unserialize_slice(input->query_data(), &rd, input->query_write_index(), wmb_, hmb_,
                                 ring_, table_, coef_, coef_ + ny, coef_ + ny + nc))
      return EVX_ERROR_EXECUTION_FAILURE;
    input->set_read_index(rd);
    if (!valid_table()) return EVX_ERROR_EXECUTION_FAILURE;
    if (cairo_ctx_decode_frame(ctx_, reinterpret_cast<const uint8_t *>(table_), coef_, f.index,
                               static_cast<uint8_t *>(output)))
      return EVX_ERROR_EXECUTION_FAILURE;
    frame_index_++;
    input->empty();
    return EVX_SUCCESS;
  }

  evx_status set_device(int device) {
    if (initialized_) return EVX_ERROR_INVALIDARG;
    device_ = device;
    return EVX_SUCCESS;
  }

 private:
  // initialize (evx1dec.cpp:43-73) with verify_header (common.cpp:25-43).  The
  // reference compiles its ring size in; this decoder takes it from the
  // header (2..4, the sizes the encoder supports).
  evx_status initialize(bit_stream *input) {
    header_t h;
    memset(&h, 0, sizeof(h));
    input->read_bytes(&h, sizeof(h));
    if (h.magic[0] != 'E' || h.magic[1] != 'V' || h.magic[2] != 'X' || h.magic[3] != '1' ||
        h.version != kVersionWord || h.size != sizeof(header_t) || h.ref_count < 2 ||
        h.ref_count > (uint8)cairo::kMaxRing || !h.frame_width || !h.frame_height ||
        (h.frame_width & 1) || (h.frame_height & 1))  // convert_image needs even sizes (convert.cpp:195-199)
      return EVX_ERROR_INVALID_RESOURCE;
    width_ = h.frame_width;
    height_ = h.frame_height;
    ring_ = h.ref_count;
    wa_ = (width_ + 15) & ~15u;
    ha_ = (height_ + 15) & ~15u;
    wmb_ = wa_ / 16;
    hmb_ = ha_ / 16;
    if (cairo_ctx_create_ex(width_, height_, ring_, device_, 2, &ctx_)) return EVX_ERROR_HARDWAREFAIL;  // synchronous: 2 slots
    table_ = (cairo::BlockDesc *)calloc((size_t)wmb_ * hmb_, sizeof(cairo::BlockDesc));
    coef_ = (int16 *)calloc((size_t)wa_ * ha_ * 3 / 2, sizeof(int16));
    if (!table_ || !coef_) {
      free(table_);
      free(coef_);
      cairo_ctx_destroy(ctx_);
      ctx_ = nullptr;
      table_ = nullptr;
      coef_ = nullptr;
      return EVX_ERROR_OUTOFMEMORY;
    }
    frame_index_ = 0;
    initialized_ = true;
    return EVX_SUCCESS;
  }

  // The GPU reconstruction trusts the table; a corrupt stream must not send
  // it outside the frame or the intra window.  Every stream the reference
  // encoder writes passes: its candidates are in frame (motion.cpp:225-275)
  // and the intra search reaches at most 32 px sideways and 48 px up / 16 px
  // down, sub-pel neighbour included.  q_index and sp_index ranges are the
  // quantizer's and the sub-pel direction table's.  (Any prediction target is
  // safe: the slot is (index + R - target) mod R.)
  bool valid_table() const {
    const int32 xmax = (int32)wa_ - 16, ymax = (int32)ha_ - 16;
    for (uint32 by = 0; by < hmb_; by++)
      for (uint32 bx = 0; bx < wmb_; bx++) {
        const cairo::BlockDesc &d = table_[by * wmb_ + bx];
        const uint32 t = d.block_type & 0xFFu;
        if (!legal_type(d.block_type)) return false;
        if (!(t & cairo::kCopy) && d.q_index > 31) return false;
        if (!(t & cairo::kMotion)) continue;
        if (d.sp_pred > 1 || (d.sp_pred && (d.sp_index > 7 || d.sp_amount > 1))) return false;
        const int32 px = (int32)bx * 16, py = (int32)by * 16;
        int32 x0 = px + d.motion_x, y0 = py + d.motion_y, x1 = x0, y1 = y0;
        if (d.sp_pred) {
          int32 dx, dy;
          frac_dir(d.sp_index, &dx, &dy);
          x1 += dx, y1 += dy;
        }
        for (int k = 0; k < 2; k++) {
          const int32 x = k ? x1 : x0, y = k ? y1 : y0;
          if (x < 0 || x > xmax || y < 0 || y > ymax) return false;
          if ((t & cairo::kIntra) && (x < px - 32 || x > px + 32 || y < py - 48 || y > py + 16)) return false;
        }
      }
    return true;
  }

  bool initialized_ = false;
  uint32 frame_index_;
  uint32 width_ = 0, height_ = 0, wa_ = 0, ha_ = 0, wmb_ = 0, hmb_ = 0, ring_ = 0;
  int device_ = 0;
  cairo_ctx *ctx_ = nullptr;
  cairo::BlockDesc *table_ = nullptr;
  int16 *coef_ = nullptr;
};

evx_status create_decoder(evx1_decoder **output) {  // evx1.cpp:28-45
  if (!output) return EVX_ERROR_INVALIDARG;
  *output = new (std::nothrow) gpu_decoder;
  return *output ? EVX_SUCCESS : EVX_ERROR_OUTOFMEMORY;
}

evx_status destroy_decoder(evx1_decoder *input) {  // evx1.cpp:65-81
  if (!input) return EVX_ERROR_INVALIDARG;
  delete static_cast<gpu_decoder *>(input);
  return EVX_SUCCESS;
}

}  // namespace evx

extern "C" {

int evx_decoder_create(void **dec) {
  evx::evx1_decoder *d = nullptr;
  const int r = evx::create_decoder(&d);
  *dec = d;
  return r;
}
int evx_decoder_destroy(void *dec) { return evx::destroy_decoder((evx::evx1_decoder *)dec); }
int evx_decoder_clear(void *dec) { return ((evx::evx1_decoder *)dec)->clear(); }
int evx_decoder_decode(void *dec, void *bs, void *rgb) {
  return ((evx::evx1_decoder *)dec)->decode((evx::bit_stream *)bs, rgb);
}
int evx_decoder_set_device(void *dec, int device) {
  return static_cast<evx::gpu_decoder *>((evx::evx1_decoder *)dec)->set_device(device);
}

}  // extern "C"
