// cairo_amd/csrc/kernels.h -- launch interface of the gfx950 encode-path kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "evx_defs.h"

namespace cairo {

// One plane set in HBM: int16 planes, pitch == plane width (image.cpp:55-68).
struct PlaneSet {
  int16_t* y;
  int16_t* u;
  int16_t* v;
};

// Plane set of ring slot k inside one contiguous allocation.
__host__ __device__ inline PlaneSet ring_slot(int16_t* base, size_t slot_elems, int wa, int ha,
                                              int k) {
  PlaneSet p;
  p.y = base + (size_t)k * slot_elems;
  p.u = p.y + (size_t)wa * ha;
  p.v = p.u + (size_t)(wa / 2) * (ha / 2);
  return p;
}

// Per-frame kernel arguments (passed by value).
struct FrameArgs {
  int wa, ha;          // frame size aligned to 16 (evx1enc.cpp:79-80)
  int w, h;            // nominal frame size (RGB input)
  int wmb, hmb;        // macroblocks per row / column
  int ring;            // R = ring size (EVX_REFERENCE_FRAME_COUNT)
  int index;           // frame index (common.cpp:192-195 ring addressing)
  int inter;           // frame type: 0 intra, 1 inter
  int quality;         // frame quality 1..31
  const uint8_t* rgb;  // RGB888, pitch 3*w
  PlaneSet in;         // input_cache
  PlaneSet coef;       // output_cache (quantized coefficients, persistent)
  int16_t* ring_base;       // R contiguous plane sets (Y, U, V each), slot k at
  size_t slot_elems;        //   ring_base + k * slot_elems
  BlockDesc* table;        // block table [wmb*hmb]
  BlockDesc* inter_desc;   // [(off-1)*mbs + mb]
  int32_t* inter_sad;      // [(off-1)*mbs + mb]
  int32_t* sync;           // SyncLayout words, zeroed before every frame
  int32_t* sticky;         // timeout flag that is never cleared (reported by the host)
  uint64_t* stamps;        // diagnostic: per-MB phase timestamps (nullptr = off)
  uint64_t* granules;      // K2 hand-off: 192 {tag, 2 px} granules per macroblock
  uint32_t epoch;          // granule tag of this frame (per-context submission count)
  int row_workers;         // k_mb_rows: workgroups [0, row_workers) code rows, the rest deblock
};

// Granule hand-off of a reconstructed macroblock (MI355X_MICROARCH.md, R2 form):
// 8-byte {high: tag = FrameArgs::epoch, low: two int16 pixels}, each written by
// ONE sc1 store; the reader polls the data itself.  Layout per macroblock:
// 128 luma dwords (row r, pair d at r*8+d), then 32 U and 32 V (row r, pair d
// at r*4+d).
constexpr int kGranulesPerMB = 192;

// Phase boundaries recorded per macroblock by k_mb_rows when stamps != nullptr.
constexpr int kStampPhases = 12;  // 10 real-time stamps + 2 shader-clock stamps
// ...followed by kDbStamps per MB row: deblock worker phases 0..7, and 8 = the
// row worker's "row coded" publish.
constexpr int kDbStamps = 9;

// Words of FrameArgs::sync (all int32, zeroed per frame).
struct SyncLayout {
  static constexpr int kErr = 0;         // nonzero: a bounded wait timed out
  static constexpr int kRowTicket = 1;   // K2 row dequeue
  static constexpr int kDbTicket = 2;    // deblock row dequeue
  static constexpr int kRowCoded = 8;    // [hmb]: MB row r coded (release/acquire)
  __host__ __device__ static int deblocked(int hmb) { return kRowCoded + hmb; }  // [hmb]
  __host__ __device__ static int words(int hmb) { return kRowCoded + 2 * hmb + 8; }
};

// Deblock workers appended to the row workers of k_mb_rows.
constexpr int kDeblockWorkers = 4;

hipError_t launch_convert(const FrameArgs& a, hipStream_t s);
hipError_t launch_inter_search(const FrameArgs& a, hipStream_t s);
hipError_t launch_mb_rows(const FrameArgs& a, int workgroups, hipStream_t s);
// Debug: rebuild the pre-deblock reconstruction of the last frame from the
// K2 granules into plane set dst.
hipError_t launch_unpack_granules(const FrameArgs& a, PlaneSet dst, hipStream_t s);

// Known-answer entry points: apply the device transform / quantizer code to
// a batch of macroblocks (6 blocks of 64 int16 each, block-major).
hipError_t launch_kat_transform(const int16_t* src, const int16_t* pred, int16_t* coef,
                                int16_t* recon, const uint8_t* qtype, int32_t* qvar,
                                int count, hipStream_t s);

}  // namespace cairo
