// cairo_amd/csrc/evx_defs.h
//
// Constants and exact integer semantics of the EVX-1 encode path, shared by
// the HIP kernels and the host code of libcairo_amd.  Each item cites the
// reference file:line whose behaviour it restates (hinike/cairo).
#pragma once

#include <stdint.h>

#if defined(__HIP__)
#define EVX_HD __host__ __device__ __forceinline__
#else
#define EVX_HD static inline
#endif

namespace cairo {

constexpr int kMB = 16;               // EVX_MACROBLOCK_SIZE, macroblock.h:56
constexpr int kSadGate = 8192;        // EVX_MOTION_SAD_THRESHOLD, motion.cpp:19
constexpr int kRadius = 16;           // EVX_MOTION_SEARCH_RADIUS, motion.cpp:24
constexpr int kQScale = 16;           // EVX_QUANTIZER_SCALE_FACTOR, quantize.cpp:9
constexpr int kMaxRing = 4;           // ring sizes 1..4 (reference: compile-time 4; R=5 is broken there)
constexpr uint32_t kFeedCapacityBits = 32u * 1024u * 1024u;  // common.cpp:147

// Block-type bits, types.h:68-87.
constexpr uint32_t kIntra = 1, kMotion = 2, kCopy = 4;

// evx_block_desc, common.h:78-95 (#pragma pack(2): 16 bytes).
struct BlockDesc {
  uint32_t block_type;
  uint8_t prediction_target;
  uint8_t pad;
  int16_t motion_x;
  int16_t motion_y;
  uint8_t sp_pred;
  uint8_t sp_amount;
  uint8_t sp_index;
  uint8_t q_index;
  int16_t variance;
};
static_assert(sizeof(BlockDesc) == 16, "evx_block_desc is 16 bytes");

// rounded_div, math.h:189-197: half away from zero, sign test on bit 31.
// Restated with wrapping add/sub (the reference is int32 throughout).
EVX_HD int32_t rdiv(int32_t n, int32_t d) {
  if (((uint32_t)n ^ (uint32_t)d) & 0x80000000u)
    return (int32_t)((uint32_t)n - (uint32_t)(d / 2)) / d;
  return (int32_t)((uint32_t)n + (uint32_t)(d / 2)) / d;
}
// evx_round_out, math.h:60.
EVX_HD int32_t round_out(int32_t n, int32_t a) { return n < 0 ? n - a : n + a; }
// abs(int32), math.h:159-165 (MIN -> MAX).
EVX_HD int32_t iabs(int32_t v) { return v == INT32_MIN ? INT32_MAX : (v < 0 ? -v : v); }
// sign(int16), math.h:128-133.
EVX_HD int32_t sign16(int16_t v) { return (v > 0) - (v < 0); }
// LUT log2 over u32, math.h:69-113 (floor(log2 v), 0 for 0).
EVX_HD uint32_t log2_u32(uint32_t v) { return v ? 31u - (uint32_t)__builtin_clz(v) : 0u; }

// luma/chroma DC scale, quantize.cpp:37-55.
EVX_HD int32_t luma_dc_scale(int32_t qp) {
  return qp < 5 ? 8 : qp < 9 ? (qp << 1) : qp < 25 ? qp + 8 : (qp << 1) - 16;
}
EVX_HD int32_t chroma_dc_scale(int32_t qp) {
  return qp < 5 ? 8 : qp < 25 ? ((qp + 13) >> 1) : qp - 6;
}

// query_block_quantization_parameter, quantize.cpp:60-77 (VAQ).
EVX_HD uint32_t vaq_from_variance(uint32_t quality, int32_t variance2) {
  int32_t idx = (int32_t)(log2_u32((uint32_t)variance2) >> 1);
  idx = idx < 1 ? 1 : (idx > 31 ? 31 : idx);
  int32_t q = (int32_t)quality, r = q;
  if (idx > q) r = q + ((idx - q) >> 1);
  else if (idx < q) r = q - ((q - idx) >> 1);
  return (uint32_t)(r < 1 ? 1 : (r > 31 ? 31 : r));
}

// compute_motion_frac_index_from_direction / ..._direction_from_frac_index,
// motion.cpp:61-109.
EVX_HD int32_t frac_index(int32_t i, int32_t j) {
  return j < 0 ? i + 1 : (j == 0 ? (i < 0 ? 3 : 4) : i + 6);
}
EVX_HD void frac_dir(int32_t idx, int32_t* dx, int32_t* dy) {
  if (idx <= 2) { *dy = -1; *dx = idx - 1; }
  else if (idx == 3) { *dx = -1; *dy = 0; }
  else if (idx == 4) { *dx = 1; *dy = 0; }
  else { *dy = 1; *dx = idx - 6; }
}

}  // namespace cairo
