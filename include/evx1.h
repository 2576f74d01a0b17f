/*
 * include/evx1.h -- drop-in replacement for the reference's public API
 * (hinike/cairo evx1.h:55-123), implemented by libcairo_amd.so on MI355X.
 *
 * Same namespace, class names, virtual-function order (Itanium vtable:
 * destructor pair, clear, insert_intra, set_quality, encode, peek) and free
 * functions, so existing callers recompile (and link) unchanged:
 *
 *   evx::bit_stream bs(64 * 1024 * 1024);
 *   evx::evx1_encoder *enc;
 *   evx::create_encoder(&enc);
 *   enc->set_quality(16);
 *   enc->encode(rgb, width, height, &bs);
 *   evx::destroy_encoder(enc);
 *
 * The hot path of encode() runs on the GPU (cairo_amd/csrc/kernels.hip); the
 * entropy stage stays on the host.  Output is bit-exact with the reference.
 */
#ifndef CAIRO_EVX1_H
#define CAIRO_EVX1_H

#include "evx_base.h"
#include "bitstream.h"

namespace evx {

/* evx1.h:55-64 */
enum EVX_PEEK_STATE {
  EVX_PEEK_SOURCE = 0,     /* padded input image (YUV420 -> RGB)   */
  EVX_PEEK_PREDICTION,     /* not implemented in the reference     */
  EVX_PEEK_BLOCK_TABLE,    /* block types as colours               */
  EVX_PEEK_QUANT_TABLE,    /* per-block q index                    */
  EVX_PEEK_SPMP_TABLE,     /* sub-pixel prediction flags           */
  EVX_PEEK_BLOCK_VARIANCE, /* pre-quantization variance            */
  EVX_PEEK_DESTINATION,    /* reconstruction of the last frame     */
};

/* evx1.h:66-94 */
class evx1_encoder {
 protected:
  virtual ~evx1_encoder() {}

 public:
  virtual evx_status clear() = 0;
  virtual evx_status insert_intra() = 0;
  virtual evx_status set_quality(uint8 quality) = 0;
  virtual evx_status encode(void *image, uint32 width, uint32 height, bit_stream *output) = 0;
  virtual evx_status peek(EVX_PEEK_STATE peek_state, void *output) = 0;
};

/* evx1.h:96-113 */
class evx1_decoder {
 protected:
  virtual ~evx1_decoder() {}

 public:
  virtual evx_status clear() = 0;
  virtual evx_status decode(bit_stream *input, void *output) = 0;
};

/* evx1.h:115-121, evx1.cpp:8-63 */
evx_status create_encoder(evx1_encoder **output);
evx_status create_decoder(evx1_decoder **output);
evx_status destroy_encoder(evx1_encoder *input);
evx_status destroy_decoder(evx1_decoder *input);

}  // namespace evx

#endif
