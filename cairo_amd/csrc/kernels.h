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
// 8-byte {high: tag = frame epoch, low: payload}, each written by ONE sc1
// store; the reader polls the data itself.  Per macroblock: 128 luma dwords
// (row r, pair d at r*8+d), 32 U and 32 V (row r, pair d at r*4+d), then one
// info granule (copy << 8 | q_index) for the deblock.
constexpr int kGranulesPerMB = 192;   // pixel granules
constexpr int kGranuleStride = 193;   // + info granule

// Inter-search records (one per macroblock and reference offset) as two
// tagged granules in the 16 bytes of an evx_block_desc slot: {epoch, packed
// desc} and {epoch, SAD}.  The row coder polls them by tag (no drain and no
// counter on the helper's side).  The packed desc holds what an inter record
// can carry: type (3 bits), target (2), sp_pred, sp_amount, sp_index (4), and
// the motion vector (7 bits each: |mv| <= 31, the search's reach).  Intra
// and decoded frames count their helpers' carrier tasks in inter_done instead.
__host__ __device__ inline uint32_t pack_inter_desc(const BlockDesc& d) {
  return (d.block_type & 7u) | ((uint32_t)(d.prediction_target & 3) << 3) | ((uint32_t)(d.sp_pred & 1) << 5) |
         ((uint32_t)(d.sp_amount & 1) << 6) | ((uint32_t)(d.sp_index & 15) << 7) |
         (((uint32_t)d.motion_x & 0x7Fu) << 11) | (((uint32_t)d.motion_y & 0x7Fu) << 18);
}
__host__ __device__ inline BlockDesc unpack_inter_desc(uint32_t w) {
  BlockDesc d;
  d.block_type = w & 7u;
  d.prediction_target = (uint8_t)((w >> 3) & 3);
  d.pad = 0;
  d.sp_pred = (uint8_t)((w >> 5) & 1);
  d.sp_amount = (uint8_t)((w >> 6) & 1);
  d.sp_index = (uint8_t)((w >> 7) & 15);
  d.motion_x = (int16_t)((int32_t)(w << 14) >> 25);  // bits 11..17, sign-extended
  d.motion_y = (int16_t)((int32_t)(w << 7) >> 25);   // bits 18..24
  d.q_index = 0;
  d.variance = 0;
  return d;
}

// Phase boundaries recorded per macroblock by the row code when stamps != nullptr.
constexpr int kStampPhases = 12;  // 10 real-time stamps + 2 shader-clock stamps
// ...followed by kDbStamps per MB row: the deblock's publish time of each
// column chunk; then 2 words: engine entry (min) / exit (max).
constexpr int kDbStamps = 256;
// ...and per (frame, row, inter group) kIStamps words: dequeue, ready, done,
// zero-MV checked, window staged, level-2 wait start / end, level-2 count,
// then (reference offset 1) step 16 done, integer steps done, sub-pel done.
constexpr int kIStamps = 12;
// Stamps of frame j of a batch start at j * stamp_frame_words; the 2 engine
// words follow the kMaxBatch frames.
__host__ __device__ inline size_t stamp_frame_words(int wmb, int hmb) {
  return (size_t)wmb * hmb * kStampPhases + (size_t)hmb * kDbStamps;
}

// Timeout diagnostics: the context's sticky words (int32, cleared only by a
// reset).  Every in-kernel wait is bounded (2 s); the first one that gives up
// records what it waited for, so a failed run (a cross-device group above all)
// names the member, frame, row and word instead of only EVX_ERROR_HARDWAREFAIL.
struct TimeoutInfo {
  static constexpr int kKind = 0;    // TimeoutKind (0: no timeout)
  static constexpr int kEpoch = 1;   // the waiting frame's epoch (granule tag)
  static constexpr int kIndex = 2;   // its stream index
  static constexpr int kRow = 3;     // the waiting task's MB row
  static constexpr int kMember = 4;  // group rank of the waiting context (0 alone)
  static constexpr int kNeed = 5;    // what it needed: columns, a count or a tag
  static constexpr int kOn = 6;      // what it waited on: kind-specific (see TimeoutKind)
  static constexpr int kSeenLo = 7;  // the last value it observed, low and high words
  static constexpr int kSeenHi = 8;
  // Device writers claim the record on kClaim (a CAS), write words 1..8, then
  // publish kKind last with a release store: a reader that sees kKind set
  // sees the whole record.
  static constexpr int kClaim = 9;
  static constexpr int kWords = 16;
};
enum TimeoutKind : int32_t {
  kWaitRecords = 1,       // row coder: inter_done of group kOn < kNeed (= nref) records
  kWaitGranule = 2,       // a granule of macroblock kOn (index in the frame) not tagged kNeed
  kWaitPrevProgress = 3,  // row helper: frame epoch-back's progress word of row kOn & 0xFFFF
                          // (back = kOn >> 16) below tagged(epoch - back, kNeed)
  kWaitRowAbove = 4,      // deblock: row kRow-1's progress of this frame below kNeed columns
  kWaitBatch = 5,         // k_batch_wait: kSeenLo of kNeed tasks finished
  kWaitInjected = 6,      // test hook (cairo_ctx_set_debug 16): a helper's progress wait,
                          // recorded as kWaitPrevProgress would be, without waiting
  kWaitHostMark = 9,      // test hook (cairo_ctx_set_debug 8): marked by the host
};

// Time accounting (CAIRO_ACCT=1 builds, cairo_ctx_set_debug 32): where the
// workers' time goes in the steady state, summed over all tasks.
#ifndef CAIRO_ACCT
#define CAIRO_ACCT 0
#endif
constexpr int kAcctShards = 64, kAcctWords = 40;
struct Acct {
  // row coders
  static constexpr int kCoderTasks = 0, kCoderTotal = 1, kCoderGroupWait = 2, kCoderWindow = 3, kCoderSearch = 4,
                       kCoderInter = 5, kCoderDequeue = 6, kCoderMBs = 7;
  // row helpers
  static constexpr int kHelperTasks = 8, kHelperTotal = 9, kHelperWait = 10, kHelperDeblock = 11, kHelperSearch = 12,
                       kHelperCatchup = 13, kHelperDequeue = 14, kHelperChunks = 15;
  // traffic of the staging and the polls (bytes requested, nominal)
  static constexpr int kWinBytes = 16, kWinSpecUnused = 17, kZeroMvBytes = 18, kGranPollBytes = 19,
                       kRecPollBytes = 20, kWinStages = 21, kSearchedTasks = 22, kInterTasks = 23;
  // row coders, after the searches: residual .. reconstruction (classify
  // excluded), publish (granule stores, window update, table), drain (the
  // coefficient drain, the barrier, the info granule)
  static constexpr int kCoderXform = 24, kCoderPublish = 25, kCoderDrain = 26;
  // before the search: the vmcnt(0) after the window (wave 0), the inter
  // records and predictions issued inside a group, the barrier
  static constexpr int kCoderVm0 = 27, kCoderRecords = 28, kCoderPreBarrier = 29;
  static constexpr int kCoderStoreTail = 30;  // CAIRO_ACCT_STORE_TAIL diagnostic builds
  // inside the intra search (thread 0's wave, summed over a macroblock's
  // integer stages / its sub-pel step): candidate evaluation and the result
  // stores to LDS, the barrier, the LDS reads and the ordered replay
  static constexpr int kSrchEval = 31, kSrchBarrier = 32, kSrchSelect = 33, kSubEval = 34, kSubBarrier = 35,
                       kSubSelect = 36;
  // inside the helper's deblock chunk: inputs (granules, block info, the rows
  // above; to the first barrier), the filters, the write-out (stores, drain,
  // progress word)
  static constexpr int kDbInputs = 37, kDbFilter = 38, kDbWrite = 39;
};

// Frames per engine launch.
#ifndef CAIRO_MAX_BATCH
#define CAIRO_MAX_BATCH 48
#endif
constexpr int kMaxBatch = CAIRO_MAX_BATCH;
// Members of a frame-interleaved group (cairo_ctx_join_group).
constexpr int kMaxGroup = 16;
// Members a frame's reconstruction is pushed to (its R-1 referencing frames
// and the stale-row reader R frames later live on at most R other members).
constexpr int kMaxPush = kMaxRing;

// One frame of a batch (host-filled, kernarg).
struct FrameDesc {
  const uint8_t* rgb;  // RGB888, pitch 3*w (device memory)
  const uint8_t* host_rgb;  // host source to upload into rgb at launch (nullptr: already on device)
  int index;           // frame index (common.cpp:192-195 ring addressing)
  int inter;           // 0 intra, 1 inter (references 1..R-1)
  int quality;         // 1..31
  uint32_t epoch;      // granule tag (per-context submission count, never 0)
  int slot;            // staging slot: this frame's source / coefficient / table / granule buffers
  int decode;          // 1: reconstruct from the slot's table + coefficients (the decoder), no search
  // Cross-frame state, resolved by the host (one context: its ring and
  // staging slots; a frame-interleaved group: the owners' buffers, kernels.h
  // FrameArgs):
  PlaneSet recon[kMaxRing];  // [0] this frame's reconstruction, [off] the reference at offset off
  PlaneSet stale;            // frame index-R's deblocked output (the rows below the intra search)
  PlaneSet coef;             // this frame's output_cache (its staging slot's)
  PlaneSet push[kMaxPush];   // FrameArgs::push
  int npush;
  PlaneSet coef_prev;        // the previous frame's output_cache (copy-macroblock chain)
  uint64_t* progress;        // this frame's deblock progress words [hmb]
  const uint64_t* prev_progress;  // the previous frame's (nullptr: none, first frame after a reset)
  const uint64_t* prev2_progress;  // frame index-2's (nullptr: none)
  int sys;                   // FrameArgs::sys
  int member;                // FrameArgs::member
  const BlockDesc* host_table;  // decode: the frame's block table and coefficient planes (y, u, v
  const int16_t* host_coef;     //   contiguous), uploaded at launch
};

// Per-frame view of the engine's state, built by the host for every frame of
// a launch and read by the kernels from device memory (never copied into
// private memory).
struct FrameArgs {
  int wa, ha;          // frame size aligned to 16 (evx1enc.cpp:79-80)
  int w, h;            // nominal frame size (RGB input)
  int wmb, hmb;        // macroblocks per row / column
  int ring;            // R = ring size (EVX_REFERENCE_FRAME_COUNT)
  int index, inter, quality;
  int decode;          // decode mode (FrameDesc::decode): table and coef are inputs
  uint32_t epoch;
  PlaneSet in;         // input_cache of this frame
  PlaneSet coef;       // output_cache of this frame (persistent semantics: copy MBs carry coef_prev)
  PlaneSet coef_prev;  // output_cache of the previous frame
  // Reconstruction buffers: [0] this frame's (written only by its deblock),
  // [off] = frame index-off for off = 1..R-1 (inter references; zero images
  // before the stream start).  In one context these are ring slots
  // (index-off) % R (common.cpp:192-195).
  PlaneSet recon[kMaxRing];
  // The rows below an intra search: frame index-R's deblocked output (zeros
  // for the first R frames).  The reference reuses that slot in place, so this
  // equals recon[0] whenever the group's slot arithmetic does too.
  PlaneSet stale;
  // Mirrors of recon[0] on the members that read this frame (a group on
  // several devices or processes): the deblock stores every written word to
  // each of them as well, before the progress word that declares it final,
  // so the readers' searches read local memory instead of a peer's over xGMI.
  PlaneSet push[kMaxPush];
  int npush;
  BlockDesc* table;    // [wmb*hmb]
  BlockDesc* inter_desc;  // [(off-1)*mbs + mb]: two tagged granules (desc, SAD) per record
  // (unused: holds the field offsets -- and so the kernels' scalar-load
  // merging of this struct -- as measured; dropping it cost 1.3 % at 4K)
  void* reserved0;
  uint64_t* granules;  // [mbs * kGranuleStride]
  int32_t* err;        // batch error word (a bounded wait timed out)
  int32_t* sticky;     // TimeoutInfo words, never cleared by a launch (reported by the host)
  int member;          // group rank of the encoding context (0 alone): timeout diagnostics
  int inject;          // test hook: 1 = row helpers of row min(1, hmb-1) record an injected timeout
  int ng;              // inter-search groups (4 MBs) per row
  int nref;            // inter-search tasks per group (references; 1 carrier task for intra frames)
  int32_t* inter_done; // [hmb][ng] inter-search tasks finished
  // Deblock progress per MB row, tagged: (epoch << 32) | final luma columns.
  // Frame epochs of a stream are consecutive, so the previous frame's words
  // are compared against (epoch - 1) << 32 | need; a staging slot's words are
  // never cleared between frames (a later frame's larger tag also means the
  // earlier frame is final there), so no launch ordering guards them.
  uint64_t* progress;             // [hmb] this frame's
  const uint64_t* prev_progress;  // [hmb] the previous frame's (nullptr: none)
  // [hmb] frame index-2's (nullptr: none): the searches of the older
  // references (offsets 2..R-1) wait on it instead of the previous frame
  const uint64_t* prev2_progress;
  // 1: the cross-frame buffers are shared with other devices or processes (a
  // frame-interleaved group): progress words are stored and polled at system
  // scope, with a system-scope release before each store and a system-scope
  // acquire after each wait on another frame's data.
  int sys;
  int db_shift;        // deblock chunk width, log2 luma columns (4..6: 1, 2 or 4 macroblocks)
  uint64_t* stamps;    // diagnostic (nullptr = off)
  uint64_t* acct;      // diagnostic time accounting (EngineArgs::acct)
  uint64_t* istamps;   // diagnostic: per (row, group) of the inter search, kIStamps stamps (see kernels.hip)
  const uint8_t* rgb;  // RGB888 input, pitch 3*w (device memory)
};

// Build the view of frame j of a launch (host side; kernels.h layout rules).
struct EngineArgs;
FrameArgs make_frame_view(const EngineArgs& e, const FrameDesc& f, int j);

// Words of the batch sync area (int32, zeroed per batch, read only by the
// launch itself).  ng = inter-search groups per MB row ((wmb + 3) / 4).
struct SyncLayout {
  static constexpr int kErr = 0;
  static constexpr int kDone = 4;  // finished tasks (helpers + coders) of the batch
  static constexpr int kLabelOff = 5;  // 1 + the label offset the launch's workers agreed on (0: not yet)
  static constexpr int kTicketRows = 8;      // + label: next ticket of each label's coder queue
  static constexpr int kTicketHelpers = 16;  // + label: of each label's helper queue
  static constexpr int kFlags = 24;
  // per frame j: inter_done[hmb][ng] (tasks finished per group)
  __host__ __device__ static int frame_words(int hmb, int ng) { return hmb * ng; }
  __host__ __device__ static int inter_done(int hmb, int ng, int j) { return kFlags + frame_words(hmb, ng) * j; }
  __host__ __device__ static int words(int hmb, int ng) { return kFlags + frame_words(hmb, ng) * kMaxBatch + 8; }
};

// One engine launch: up to kMaxBatch consecutive frames, pipelined.
struct EngineArgs {
  int wa, ha, w, h, wmb, hmb, ring;
  int nframes;
  const FrameArgs* fa;     // [nframes] per-frame views, device memory
  // per-slot buffers: base + slot * stride
  int16_t* src_base;    // plane sets, stride plane_elems
  size_t plane_elems;
  BlockDesc* table_base;   // stride mbs
  BlockDesc* idesc_base;   // stride nref * mbs
  void* reserved0;         // (unused: keeps the kernel-argument offsets, see FrameArgs::reserved0)
  uint64_t* gran_base;     // stride mbs * kGranuleStride
  int32_t* sync;           // SyncLayout words of this launch
  int32_t* sticky;         // TimeoutInfo words
  int inject;              // FrameArgs::inject
  uint64_t* stamps;
  // Diagnostic time accounting of a build with CAIRO_ACCT=1 (nullptr = off):
  // [kAcctShards][kAcctWords] u64, 10 ns ticks summed per role and phase over
  // every task of the steady state (Acct), sharded by workgroup index.
  uint64_t* acct;
  int n_helpers, n_rows;   // worker pools (workgroups), spread over the block indices (is_helper)
  int32_t* trace;          // diagnostic: [blockIdx][4] live state in mapped host memory (nullptr = off)
  // Per pool (0 helpers, 1 row coders): [nframes * hmb] task order, (frame << 16 | row)
  // sorted by (row + kOrderSlope * frame, frame), then stably partitioned by label
  // (nlab == kLabels); label l's queue is order[seg[l] .. seg[l+1]).
  const int32_t* order[2];
  const int32_t* seg[2];   // [kLabels + 1] each
  int nlab[2];             // 1, or kLabels: one queue per XCD (label = XCD when the dispatcher
                           // deals blocks round-robin; see task_label)
  int decode;              // the launch decodes (every frame has FrameDesc::decode set)
  // The previous launch (still running, or done): its remaining tasks come
  // first for this launch's workers too, so the two co-resident launches
  // share their pools (ptotal = 0: none).
  const FrameArgs* pfa;
  const int32_t* porder[2];
  const int32_t* pseg[2];
  int32_t* psync;
  int ptotal;
  int slope;               // of both task orders (kOrderSlope; 3N + 2 for a member of an N-GPU group)
};

// Frame-row task order of the engine pools.  A task of frame f, row r waits
// at most on frame f-1, row r+3, so any slope > 3 keeps every wait pointing
// to an earlier key (deadlock-free), while frames interleave in the pools
// instead of queueing behind each other.
constexpr int kOrderSlope = 5;  // (4 and 6 slower in rounds 2-3; within 0.3 % in round 5, profiles/r05/ab_4k_order_slope.txt)

// Large frames (more macroblocks than this): the helpers get SIMD issue
// priority (kernels.hip k_engine) and a larger share of a launch's workers
// (backend.hip, 200 of 384: measured best at 4K and 1080p, 0.6 % behind the
// even split at 720p, profiles/r05/sweep_helpers.txt).
constexpr int kPrioFrameMBs = 4000;

// XCD-banded queues: on a frame of at least kBandMinRows macroblock rows each
// pool keeps one queue per label (kLabels), and a worker serves the queue of
// its label (kernels.hip next_task: unless another label's head is more than
// kSteal keys earlier): the workgroups b with one value of b % 8 share an XCD
// (the observed round-robin deal), and the launch agrees on one offset so
// that a label is an XCD.  Row r of every frame has label r * kLabels / hmb
// (contiguous bands): the helpers of neighbouring rows, whose search windows
// overlap by 64 of 80 lines, and the coders of the rows they feed share an
// L2.  Correctness does not rest on the placement: labels partition the block
// indices, each label has workers of both pools, and each label's queue is a
// subsequence of the task order (deadlock freedom as for one queue).
// 4K A/B: 5387-5391 -> 5483-5486 Mpix/s, engine reads -29 %;
// at 1080p (68 rows) -1.2 %, so not below kBandMinRows.
constexpr int kLabels = 8;
constexpr int kBandMinRows = 100;
constexpr int kBandPools = 3;  // bit 0: the helpers' queues are per label, bit 1: the coders'
// Contiguous bands of hmb / kLabels rows (rotating 4- or 8-row bands read
// fewer bytes but ran 0.4-0.8 % slower: profiles/r04/band_traffic_4k.json, ab_4k_k.txt).
__host__ __device__ inline int task_label(int frame, int row, int hmb) {
  (void)frame;
  return row * kLabels / hmb;
}

// A launch's preparation, done by the convert kernel that precedes its
// engine on the stream (no runtime copy or fill kernels, which would compete
// with the co-resident engine launch for workgroup slots): RGB -> YUV of every
// frame (pointers here, so the convert reads nothing from the frame views),
// the frame views from mapped pinned host memory to the device, and the zeroed
// sync area.
struct ConvertArgs {
  int w, h, wa, nframes;
  const uint8_t* rgb[kMaxBatch];  // nullptr: nothing to convert (a decoded frame)
  PlaneSet in[kMaxBatch];
  const uint4* fa_host;  // [fa_chunks] the frame views (device-visible pinned host memory)
  uint4* fa_dev;
  int fa_chunks;
  int32_t* sync;  // [sync_words], zeroed
  int sync_words;
};
// RGB -> YUV of every frame of the batch into its slot's source planes, plus
// the views and sync area above (grid slice z = nframes).
hipError_t launch_convert_batch(const ConvertArgs& c, hipStream_t s);
// The pipelined encode engine: inter search, macroblock rows (intra search,
// classify, transform, quantize, reconstruct) and in-loop deblock.
hipError_t launch_engine(const EngineArgs& e, hipStream_t s);
// Until every task of the batch (sync area `sync`, `tasks` of them, run by
// this launch or the next) has finished; bounded like every wait.
hipError_t launch_batch_wait(int32_t* sync, int tasks, int32_t* sticky, hipStream_t s);
// Engine workgroups resident per CU (occupancy of k_engine: 3 on gfx950).
hipError_t engine_blocks_per_cu(int* n);
// Debug: rebuild the pre-deblock reconstruction of frame j of the batch from
// its granules into plane set dst.
hipError_t launch_unpack_granules(const EngineArgs& e, int j, PlaneSet dst, hipStream_t s);

// convert_image YUV -> RGB (convert.cpp:16-19, 162-223) of plane set src into
// RGB888 rgb (w x h, pitch 3*w).
hipError_t launch_yuv_to_rgb(PlaneSet src, int wa, int w, int h, uint8_t* rgb, hipStream_t s);

// Known-answer entry points: apply the device transform / quantizer code to
// a batch of macroblocks (6 blocks of 64 int16 each, block-major).
hipError_t launch_kat_transform(const int16_t* src, const int16_t* pred, int16_t* coef,
                                int16_t* recon, const uint8_t* qtype, int32_t* qvar,
                                int count, hipStream_t s);

}  // namespace cairo
