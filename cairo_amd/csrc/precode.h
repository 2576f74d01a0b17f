// cairo_amd/csrc/precode.h -- launch interface of the GPU entropy precode
// (precode.hip).
#pragma once

#include "kernels.h"

namespace cairo {

// Header words of a frame's feed (device and mapped host copies): total
// feed bits (lo, hi), overflow flag (a coefficient section exceeds the feed
// stream's 32 Mbit: the host codes the frame itself), then the start bit of
// each of the 11 lists (8 block-table lists, the Y, U and V sections).
constexpr int kFeedHdrWords = 16;
// Per-slot scratch words per macroblock: block lengths [6], table codes [8],
// table positions [8], section offsets [3]; then one record per chunk of
// kFeedChunk macroblocks (the scan's chunk aggregates / carry-ins).
constexpr int kFeedScratchPerMB = 25;
constexpr int kFeedChunk = 256, kFeedChunkWords = 20;
inline size_t feed_scratch_words(size_t mbs) {
  return kFeedScratchPerMB * mbs + kFeedChunkWords * ((mbs + kFeedChunk - 1) / kFeedChunk);
}

// Feed capacity per staging slot, in 32-bit words: the table lists (at most
// 103 bits per macroblock with 31-bit exp-Golomb codes) plus three
// coefficient sections of at most 32 Mbit each, plus slack.
inline size_t feed_words_per_slot(size_t mbs) {
  return ((103 * mbs + 3 * (size_t)kFeedCapacityBits) / 32 + 64 + 15) & ~(size_t)15;  // 64-byte multiple
}

struct FeedArgs {
  int nframes;
  const FrameArgs* fa;            // the launch's frame views (device)
  int slot[kMaxBatch];            // staging slot of frame j
  uint32_t* host[kMaxBatch];      // frame j's mapped pinned host buffer: header, then words
  uint32_t* scratch;              // per slot: feed_scratch_words(mbs) words
  size_t scratch_stride;
  uint32_t* feed;                 // per slot: feed words (device)
  size_t feed_stride;
  uint32_t* hdr;                  // per slot: kFeedHdrWords
  // k_feed_copy also hands over frame j's block table (table_words uint4 from
  // its view's table) and the context's timeout words (TimeoutInfo) into
  // mapped pinned host memory (nullptr: skip)
  uint4* table_host[kMaxBatch];
  int32_t* err_host[kMaxBatch];
  int table_words;
};

// k_feed_len -> k_feed_agg -> k_feed_carry -> k_feed_scan -> k_feed_write ->
// k_feed_copy for every frame of a launch.
hipError_t launch_precode(const FeedArgs& f, int mbs, hipStream_t s);  // phases 1-3 (len, scan, write)
hipError_t launch_feed_copy(const FeedArgs& f, hipStream_t s);          // phase 4 (copy to the host)

}  // namespace cairo
