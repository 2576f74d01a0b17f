// cairo_amd/csrc/entropy.h -- host entropy stage (serialize.cpp:319-340).
#pragma once
#include <cstdint>

namespace cairo {

// Append the ABAC payload of one frame at *bit_pos of out (LSB-first), given
// the block table (16-B descs) and the output_cache planes.  Returns an
// evx_status (0, or 7 = EVX_ERROR_CAPACITY_LIMIT when out is too small).
int serialize_slice(const uint8_t* table, uint32_t wmb, uint32_t hmb, uint32_t ring,
                    const int16_t* coef_y, const int16_t* coef_u, const int16_t* coef_v,
                    uint8_t* out, uint64_t out_bits_capacity, uint64_t* bit_pos);

}  // namespace cairo
