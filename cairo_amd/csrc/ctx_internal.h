// cairo_amd/csrc/ctx_internal.h -- hooks of the device context used by the
// frame pipeline (pipeline.cpp); not part of the C ABI.
#pragma once
#include <atomic>
#include <cstdint>

#include "../../include/cairo_amd.h"

namespace cairo {

// Like cairo_ctx_wait, but never launches the pending batch itself: blocks
// until another thread's submit (a full batch) or flush launched the frame,
// or until *stop becomes true (then kInvalidResource; wake the waiter with
// ctx_wake after setting it).
int ctx_wait_launched(cairo_ctx* c, int ticket, const std::atomic<bool>* stop,
                      cairo_frame_result* out);
// Launch the pending (partial) batch; with ticket >= 0 only if that frame is
// part of it (not yet launched).
int ctx_flush(cairo_ctx* c, int ticket = -1);
void ctx_wake(cairo_ctx* c);
// Macroblock grid, ring size and the ticket the next submit will get.
int ctx_geometry(cairo_ctx* c, uint32_t* wmb, uint32_t* hmb, uint32_t* ring, int* next_ticket);

}  // namespace cairo
