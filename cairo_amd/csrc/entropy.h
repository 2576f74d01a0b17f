// cairo_amd/csrc/entropy.h -- host entropy stage (serialize.cpp:319-340).
#pragma once
#include <cstdint>

#include "../../include/cairo_amd.h"

namespace cairo {

// Append the ABAC payload of one frame at *bit_pos of out (LSB-first), given
// the block table (16-B descs) and the output_cache planes.  Returns an
// evx_status (0, or 7 = EVX_ERROR_CAPACITY_LIMIT when out is too small).
int serialize_slice(const uint8_t* table, uint32_t wmb, uint32_t hmb, uint32_t ring,
                    const int16_t* coef_y, const int16_t* coef_u, const int16_t* coef_v,
                    uint8_t* out, uint64_t out_bits_capacity, uint64_t* bit_pos);

// The same payload from the feed bits the GPU precode produced
// (CAIRO_OUT_FEED, precode.hip): only the arithmetic coder runs on the host.
int serialize_feed(const uint32_t* feed, uint64_t feed_bits, uint8_t* out, uint64_t out_bits_capacity,
                   uint64_t* bit_pos);

// A frame's payload from a context's outputs: the GPU feed when it is valid,
// else the block table and coefficient planes (fetched from the staging slot
// with cairo_ctx_fetch_coef when the context does not copy them).
int serialize_result(cairo_ctx* ctx, int ticket, cairo_frame_result* res, uint32_t ring, uint8_t* out,
                     uint64_t out_bits_capacity, uint64_t* bit_pos);

}  // namespace cairo
