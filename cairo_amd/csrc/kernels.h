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

// Plane set k inside one contiguous allocation of plane sets.
__host__ __device__ inline PlaneSet ring_slot(int16_t* base, size_t slot_elems, int wa, int ha,
                                              int k) {
  PlaneSet p;
  p.y = base + (size_t)k * slot_elems;
  p.u = p.y + (size_t)wa * ha;
  p.v = p.u + (size_t)(wa / 2) * (ha / 2);
  return p;
}

// Granule hand-off of a reconstructed macroblock (MI355X_MICROARCH.md, R2 form):
// 8-byte {high: tag = frame epoch, low: two int16 pixels}, each written by
// ONE sc1 store; the reader polls the data itself.  Layout per macroblock:
// 128 luma dwords (row r, pair d at r*8+d), then 32 U and 32 V (row r, pair d
// at r*4+d).
constexpr int kGranulesPerMB = 192;

// Phase boundaries recorded per macroblock by the row code when stamps != nullptr.
constexpr int kStampPhases = 12;  // 10 real-time stamps + 2 shader-clock stamps
// ...followed by kDbStamps per MB row: deblock phases 0..7, and 8 = the row
// coder's "row coded" publish; then 2 words: engine entry (min) / exit (max).
constexpr int kDbStamps = 9;

// Frames per engine launch.
constexpr int kMaxBatch = 16;

// One frame of a batch (host-filled, kernarg).
struct FrameDesc {
  const uint8_t* rgb;  // RGB888, pitch 3*w (device memory)
  int index;           // frame index (common.cpp:192-195 ring addressing)
  int inter;           // 0 intra, 1 inter (references 1..R-1)
  int quality;         // 1..31
  uint32_t epoch;      // granule tag (per-context submission count, never 0)
  int slot;            // staging slot: this frame's source / coefficient / table / granule buffers
  int prev_slot;       // staging slot of the previous frame (output_cache chain)
};

// Per-frame view of the engine's state (built on the device from EngineArgs).
struct FrameArgs {
  int wa, ha;          // frame size aligned to 16 (evx1enc.cpp:79-80)
  int w, h;            // nominal frame size (RGB input)
  int wmb, hmb;        // macroblocks per row / column
  int ring;            // R = ring size (EVX_REFERENCE_FRAME_COUNT)
  int index, inter, quality;
  uint32_t epoch;
  PlaneSet in;         // input_cache of this frame
  PlaneSet coef;       // output_cache of this frame (persistent semantics: copy MBs carry coef_prev)
  PlaneSet coef_prev;  // output_cache of the previous frame
  int16_t* ring_base;  // R contiguous reconstruction slots
  size_t slot_elems;
  BlockDesc* table;    // [wmb*hmb]
  BlockDesc* inter_desc;  // [(off-1)*mbs + mb]
  int32_t* inter_sad;     // [(off-1)*mbs + mb]
  uint64_t* granules;  // [mbs * kGranulesPerMB]
  int32_t* err;        // batch error word (a bounded wait timed out)
  int32_t* sticky;     // timeout flag that is never cleared (reported by the host)
  int32_t* inter_done; // [hmb] inter-search tasks finished per MB row
  int32_t* coded;      // [hmb] MB row coded (slot + table + coefficients written)
  int32_t* deblocked;  // [hmb] MB row deblocked
  uint64_t* stamps;    // diagnostic (nullptr = off)
};

// Words of the batch sync area (int32, zeroed per batch).
struct SyncLayout {
  static constexpr int kErr = 0;
  static constexpr int kTicketInter = 1;
  static constexpr int kTicketRows = 2;
  static constexpr int kTicketDeblock = 3;
  static constexpr int kFlags = 8;  // then per frame j: inter_done, coded, deblocked [hmb each]
  __host__ __device__ static int inter_done(int hmb, int j) { return kFlags + 3 * hmb * j; }
  __host__ __device__ static int coded(int hmb, int j) { return kFlags + 3 * hmb * j + hmb; }
  __host__ __device__ static int deblocked(int hmb, int j) { return kFlags + 3 * hmb * j + 2 * hmb; }
  __host__ __device__ static int words(int hmb) { return kFlags + 3 * hmb * kMaxBatch + 8; }
};

// One engine launch: up to kMaxBatch consecutive frames, pipelined.
struct EngineArgs {
  int wa, ha, w, h, wmb, hmb, ring;
  int nframes;
  FrameDesc fr[kMaxBatch];
  // per-slot buffers: base + slot * stride
  int16_t* src_base;    // plane sets, stride plane_elems
  int16_t* coef_base;   // plane sets, stride plane_elems
  size_t plane_elems;
  BlockDesc* table_base;   // stride mbs
  BlockDesc* idesc_base;   // stride nref * mbs
  int32_t* isad_base;      // stride nref * mbs
  uint64_t* gran_base;     // stride mbs * kGranulesPerMB
  int16_t* ring_base;      // R reconstruction slots, stride plane_elems
  int32_t* sync;           // SyncLayout words
  int32_t* sticky;
  uint64_t* stamps;
  int n_inter, n_rows, n_deblock;  // worker pools (workgroups), in blockIdx order
};

// RGB -> YUV of every frame of the batch into its slot's source planes.
hipError_t launch_convert_batch(const EngineArgs& e, hipStream_t s);
// The pipelined encode engine: inter search, macroblock rows (intra search,
// classify, transform, quantize, reconstruct) and in-loop deblock.
hipError_t launch_engine(const EngineArgs& e, hipStream_t s);
// Debug: rebuild the pre-deblock reconstruction of frame j of the batch from
// its granules into plane set dst.
hipError_t launch_unpack_granules(const EngineArgs& e, int j, PlaneSet dst, hipStream_t s);

// Known-answer entry points: apply the device transform / quantizer code to
// a batch of macroblocks (6 blocks of 64 int16 each, block-major).
hipError_t launch_kat_transform(const int16_t* src, const int16_t* pred, int16_t* coef,
                                int16_t* recon, const uint8_t* qtype, int32_t* qvar,
                                int count, hipStream_t s);

}  // namespace cairo
