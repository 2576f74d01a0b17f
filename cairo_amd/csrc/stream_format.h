// cairo_amd/csrc/stream_format.h -- the EVX-1 stream records written by the
// encoder and read by the decoder (reference common.h:50-72, version.h:37-41).
#pragma once
#include "../../include/evx_base.h"

namespace evx {

constexpr uint16 kVersionWord = (2 << 8) | 47;  // EVX_VERSION_WORD(2, 47), version.h:37-41

#pragma pack(push, 2)
struct header_t {  // evx_header, common.h:50-62 (byte 7 is an unwritten pad)
  uint8 magic[4];
  uint16 size;
  uint8 ref_count;
  uint16 version;
  uint16 frame_width;
  uint16 frame_height;
};
struct frame_t {  // evx_frame, common.h:66-72
  uint32 type;
  uint32 index;
  uint16 quality;
};
#pragma pack(pop)
static_assert(sizeof(header_t) == 14, "evx_header is 14 bytes");
static_assert(sizeof(frame_t) == 10, "evx_frame is 10 bytes");

}  // namespace evx
