// cairo_amd/csrc/precode.h -- launch interface of the GPU entropy precode
// (precode.hip).
#pragma once

#include "kernels.h"

namespace cairo {

// Header words of a frame's feed (device and mapped host copies): total
// feed bits (lo, hi), overflow flag (a coefficient section exceeds the feed
// stream's 32 Mbit: the host codes the frame itself), bits of the table lists.
constexpr int kFeedHdrWords = 4;

// Feed capacity per staging slot, in 32-bit words: the table lists (at most
// 103 bits per macroblock with 31-bit exp-Golomb codes) plus three
// coefficient sections of at most 32 Mbit each, plus slack.
inline size_t feed_words_per_slot(size_t mbs) {
  return (103 * mbs + 3 * (size_t)kFeedCapacityBits) / 32 + 64;
}

struct FeedArgs {
  int nframes;
  const FrameArgs* fa;            // the launch's frame views (device)
  int slot[kMaxBatch];            // staging slot of frame j
  uint32_t* host[kMaxBatch];      // frame j's mapped pinned host buffer: header, then words
  int32_t* lens;                  // per slot: 6 * mbs block lengths, then bit offsets
  size_t lens_stride;
  uint32_t* feed;                 // per slot: feed words (device)
  size_t feed_stride;
  uint32_t* hdr;                  // per slot: kFeedHdrWords
};

// k_feed_len -> k_feed_scan -> k_feed_write -> k_feed_copy for every frame of a launch.
hipError_t launch_precode(const FeedArgs& f, int mbs, hipStream_t s);

}  // namespace cairo
