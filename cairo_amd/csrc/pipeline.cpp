// cairo_amd/csrc/pipeline.cpp -- the multi-threaded frame pipeline
// (SURVEY.md §8(f) F1): GPU hot path + host entropy for a stream of frames.
//
// The reference encodes one frame per encode() call, serially
// (evx1enc.cpp:119-168: engine_encode_frame, then serialize_slice).  The
// hot path here runs a batch of frames per engine launch, so the host
// entropy stage (serialize_slice, serialize.cpp:319-340; bit-serial ABAC per
// frame) becomes the bottleneck unless frames are entropy-coded in parallel.
// Frames are entropy-independent: the coder and its adaptive model restart
// per slice (serialize.cpp:323, arith_coder.clear()), and all inputs of a
// frame -- its block table and output_cache snapshot -- are copied to its
// own pinned staging slot by the device context.
//
//   caller thread     cairo_stream_submit  -> cairo_ctx_submit (launches full batches)
//   completion thread waits for each frame's D2H (in ticket order) -> job queue
//   entropy workers   the arithmetic coder over the frame's GPU-precoded feed
//                     (serialize_slice from the planes if the feed overflowed)
//                     into its payload buffer, release the staging slot
//   caller thread     cairo_stream_collect -> payload bits appended in place
//
// Payload bits are the exact serialize_slice output of the frame, so
// appending frame descriptors and payloads in ticket order reproduces the
// reference stream (tests/test_gpu_parity.py::test_stream_*).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/cairo_amd.h"
#include "ctx_internal.h"
#include "entropy.h"

namespace {

constexpr int kSuccess = 0, kInvalidArg = 1, kCapacityLimit = 7, kInvalidResource = 8;  // evx_status (base.h:150-172)

double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Per-frame timeline (us, steady clock): submitted, outputs on the host
// (completion thread), entropy start, entropy end, collected.
enum { kTSubmit, kTOutputs, kTEntropy0, kTEntropy1, kTCollect, kTimes };

struct Frame {
  enum State { kFree, kSubmitted, kDone };
  double t[kTimes] = {};
  int ticket = -1;
  State state = kFree;
  int status = kSuccess;
  std::vector<uint8_t> bits;  // payload, LSB-first from bit 0
  uint64_t nbits = 0;
};

struct Job {
  int ticket;
  cairo_frame_result res;
};

}  // namespace

struct cairo_stream {
  cairo_ctx* ctx = nullptr;
  int stages = 0;
  uint32_t wmb = 0, hmb = 0, ring = 0;
  int next = 0;            // ticket of the next submit
  std::vector<Frame> fr;   // [2 * stages], by ticket
  std::mutex m;
  std::condition_variable cv;  // any frame state / queue change
  std::deque<int> todo;        // submitted, waiting for their outputs (ticket order)
  std::deque<Job> jobs;        // outputs on the host, waiting for a worker
  std::atomic<bool> stop{false};
  std::thread completer;
  std::vector<std::thread> workers;
  bool skip_entropy = false;  // diagnostic (CAIRO_STREAM_SKIP_ENTROPY=1): plumbing only, empty payloads

  Frame& at(int t) { return fr[(size_t)t % fr.size()]; }
  void finish(int t, int status, uint64_t nbits) {
    {
      std::lock_guard<std::mutex> lk(m);
      Frame& f = at(t);
      f.status = status;
      f.nbits = nbits;
      f.state = Frame::kDone;
    }
    cv.notify_all();
  }

  void completion_loop() {
    for (;;) {
      int t;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop.load() || !todo.empty(); });
        if (todo.empty()) return;
        t = todo.front();
        todo.pop_front();
      }
      Job j{t, {}};
      const int r = cairo::ctx_wait_launched(ctx, t, &stop, &j.res);
      if (r) {  // hardware failure (or shutdown): the frame completes with the error
        cairo_ctx_release(ctx, t);
        finish(t, r, 0);
        continue;
      }
      {
        std::lock_guard<std::mutex> lk(m);
        at(t).t[kTOutputs] = now_us();
        jobs.push_back(j);
      }
      cv.notify_all();
    }
  }

  void worker_loop() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop.load() || !jobs.empty(); });
        if (jobs.empty()) return;
        j = jobs.front();
        jobs.pop_front();
      }
      Frame& f = at(j.ticket);  // owned by this worker until kDone
      f.t[kTEntropy0] = now_us();
      cairo_frame_result& o = j.res;
      if (f.bits.empty()) f.bits.resize(std::max<size_t>((size_t)o.wa * o.ha / 2, 1 << 16));
      uint64_t pos = 0;
      int r;
      for (;;) {
        pos = 0;
        if (skip_entropy) {
          r = kSuccess;
          break;
        }
        r = cairo::serialize_result(ctx, j.ticket, &j.res, ring, f.bits.data(), (uint64_t)f.bits.size() * 8, &pos);
        // a frame's precode is bounded by the feed capacity per section, so
        // the payload is too; grow until it fits
        if (r != kCapacityLimit || f.bits.size() >= ((size_t)1 << 31)) break;
        f.bits.resize(f.bits.size() * 2);
      }
      f.t[kTEntropy1] = now_us();
      cairo_ctx_release(ctx, j.ticket);
      finish(j.ticket, r, pos);
    }
  }
};

extern "C" {

// Append n bits of src (LSB-first from bit 0) at bit *pos of dst (capacity
// cap_bits), leaving the bits of dst beyond the new position untouched
// (bit_stream semantics, bitstream.cpp:181-245).
int cairo_bits_append(uint8_t* dst, uint64_t cap_bits, uint64_t* pos, const uint8_t* src,
                      uint64_t n) {
  if (!dst || !pos || (!src && n)) return kInvalidArg;
  if (*pos + n > cap_bits) return kCapacityLimit;
  uint64_t p = *pos;
  const uint32_t sh = (uint32_t)(p & 7);
  uint8_t* d = dst + (p >> 3);
  const uint64_t whole = n >> 3;  // full source bytes
  if (sh == 0) {
    memcpy(d, src, whole);
  } else {
    uint32_t carry = d[0] & ((1u << sh) - 1u);  // bits already in the first byte
    for (uint64_t i = 0; i < whole; i++) {
      const uint32_t v = carry | ((uint32_t)src[i] << sh);
      d[i] = (uint8_t)v;
      carry = v >> 8;
    }
    // carry holds sh bits for byte d[whole]: merge below preserves the rest
    const uint32_t keep = ~((1u << sh) - 1u) & 0xFFu;
    d[whole] = (uint8_t)((d[whole] & keep) | carry);
  }
  const uint32_t rest = (uint32_t)(n & 7);
  if (rest) {  // last partial source byte at bit p + 8*whole
    const uint64_t q = p + whole * 8;
    const uint32_t v = src[whole] & ((1u << rest) - 1u);
    const uint32_t s2 = (uint32_t)(q & 7);
    uint8_t* e = dst + (q >> 3);
    const uint32_t lo = std::min<uint32_t>(rest, 8 - s2);
    const uint32_t m0 = ((1u << lo) - 1u) << s2;
    e[0] = (uint8_t)((e[0] & ~m0) | ((v << s2) & m0));
    if (rest > lo) {
      const uint32_t m1 = (1u << (rest - lo)) - 1u;
      e[1] = (uint8_t)((e[1] & ~m1) | ((v >> lo) & m1));
    }
  }
  *pos = p + n;
  return kSuccess;
}

int cairo_stream_create(cairo_ctx* ctx, int threads, cairo_stream** out) {
  if (!ctx || !out) return kInvalidArg;
  cairo_stream* s = new (std::nothrow) cairo_stream;
  if (!s) return 3;
  s->ctx = ctx;
  s->stages = cairo_ctx_stages(ctx);
  // the GPU precodes each frame's entropy feed; the workers run only the
  // arithmetic coder
  int ro = cairo_ctx_set_outputs(ctx, CAIRO_OUT_FEED);
  if (ro) {
    delete s;
    return ro;
  }
  int r = cairo::ctx_geometry(ctx, &s->wmb, &s->hmb, &s->ring, &s->next);
  if (r) {
    delete s;
    return r;
  }
  s->fr.resize((size_t)2 * s->stages);
  const char* skip = getenv("CAIRO_STREAM_SKIP_ENTROPY");
  s->skip_entropy = skip && skip[0] == '1';
  if (threads <= 0) {
    const unsigned hw = std::thread::hardware_concurrency();
    threads = (int)std::min(15u, hw > 1 ? hw - 1 : 1u);
  }
  s->completer = std::thread([s] { s->completion_loop(); });
  for (int i = 0; i < threads; i++) s->workers.emplace_back([s] { s->worker_loop(); });
  *out = s;
  return kSuccess;
}

int cairo_stream_submit(cairo_stream* s, const uint8_t* rgb, int rgb_on_device, uint32_t index,
                        uint32_t type, uint32_t quality, int* ticket) {
  if (!s || !rgb || !ticket) return kInvalidArg;
  const int t = s->next;
  {
    std::unique_lock<std::mutex> lk(s->m);
    if (s->at(t).state != Frame::kFree) return kInvalidResource;  // ticket t - 2*stages not collected
    // ticket t reuses the staging slot of ticket t - stages: wait for its
    // entropy worker to release it (it is in an already launched batch)
    const int o = t - s->stages;
    s->cv.wait(lk, [&] {
      const Frame& g = s->at(o);
      return o < 0 || g.ticket != o || g.state != Frame::kSubmitted;
    });
  }
  int tk = -1;
  const int r = cairo_ctx_submit(s->ctx, rgb, rgb_on_device, index, type, quality, &tk);
  if (r) return r;
  {
    std::lock_guard<std::mutex> lk(s->m);
    Frame& f = s->at(tk);
    f.ticket = tk;
    f.t[kTSubmit] = now_us();
    f.state = Frame::kSubmitted;
    f.status = kSuccess;
    f.nbits = 0;
    s->todo.push_back(tk);
  }
  s->cv.notify_all();
  s->next = tk + 1;
  *ticket = tk;
  return kSuccess;
}

int cairo_stream_collect(cairo_stream* s, int ticket, uint8_t* out, uint64_t out_bytes,
                         uint64_t* bit_pos) {
  if (!s || ticket < 0 || !bit_pos) return kInvalidArg;
  Frame& f = s->at(ticket);
  bool pending;
  {
    std::lock_guard<std::mutex> lk(s->m);
    if (f.ticket != ticket || f.state == Frame::kFree) return kInvalidResource;
    pending = f.state == Frame::kSubmitted;
  }
  if (pending) {  // launch its batch if it is still the pending one
    const int r = cairo::ctx_flush(s->ctx, ticket);
    if (r) return r;
  }
  {
    std::unique_lock<std::mutex> lk(s->m);
    s->cv.wait(lk, [&] { return f.state == Frame::kDone; });
  }
  int r = f.status;
  if (r == kSuccess) {
    if (out)
      r = cairo_bits_append(out, out_bytes * 8, bit_pos, f.bits.data(), f.nbits);
    else
      *bit_pos += f.nbits;  // count only
    // the caller's buffer is too small: keep the payload, so a collect with a
    // larger buffer (cairo_stream_payload_bits tells how large) still gets it
    if (r == kCapacityLimit) return r;
  }
  {
    std::lock_guard<std::mutex> lk(s->m);
    f.t[kTCollect] = now_us();
    f.state = Frame::kFree;
  }
  s->cv.notify_all();
  return r;
}

int cairo_stream_payload_bits(cairo_stream* s, int ticket, uint64_t* nbits) {
  if (!s || ticket < 0 || !nbits) return kInvalidArg;
  Frame& f = s->at(ticket);
  bool pending;
  {
    std::lock_guard<std::mutex> lk(s->m);
    if (f.ticket != ticket || f.state == Frame::kFree) return kInvalidResource;
    pending = f.state == Frame::kSubmitted;
  }
  if (pending) {
    const int r = cairo::ctx_flush(s->ctx, ticket);
    if (r) return r;
  }
  std::unique_lock<std::mutex> lk(s->m);
  s->cv.wait(lk, [&] { return f.state == Frame::kDone; });
  *nbits = f.nbits;
  return f.status;
}

int cairo_stream_timeline(cairo_stream* s, int ticket, double* t) {
  if (!s || !t || ticket < 0) return kInvalidArg;
  std::lock_guard<std::mutex> lk(s->m);
  const Frame& f = s->at(ticket);
  if (f.ticket != ticket) return kInvalidResource;
  for (int k = 0; k < kTimes; k++) t[k] = f.t[k];
  return kSuccess;
}

int cairo_stream_destroy(cairo_stream* s) {
  if (!s) return kInvalidArg;
  // finish every submitted frame (their staging slots must be released
  // before the context can be reused), then stop the threads
  int r = cairo::ctx_flush(s->ctx);
  {
    std::unique_lock<std::mutex> lk(s->m);
    s->cv.wait(lk, [&] {
      if (!s->todo.empty() || !s->jobs.empty()) return false;
      for (const Frame& f : s->fr)
        if (f.state == Frame::kSubmitted) return false;
      return true;
    });
    s->stop = true;
  }
  s->cv.notify_all();
  cairo::ctx_wake(s->ctx);
  s->completer.join();
  for (auto& w : s->workers) w.join();
  delete s;
  return r;
}

}  // extern "C"
