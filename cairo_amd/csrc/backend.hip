// cairo_amd/csrc/backend.hip -- device context and frame orchestration.
//
// One context = one encoder's device state in HBM (DESIGN.md "Data layout"):
//   ring          R contiguous plane sets (reconstruction slots, frame n -> n % R)
//   staging slots (64 for pipelined callers, 2 for the synchronous drop-in
//     encoder/decoder), one per frame in flight, each with its own
//     source planes (convert output), output_cache planes (coefficients),
//     block table, inter-search records, granules, RGB staging and pinned
//     host buffers for the table + coefficients
//   sync          batch flags (zeroed per launch)
// Frames are submitted into a batch (up to batch_max, cairo_default_batch)
// that is launched when full or when a caller waits on one of its frames:
//   memset(sync) -> convert (all frames) -> engine (inter search, row coding,
//   deblock, pipelined across the frames)
// and on the copy stream, after the engine: D2H of each frame's table and
// coefficients into its pinned staging (the host entropy stage reads those
// while the GPU runs the next batch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/cairo_amd.h"
#include "ctx_internal.h"
#include "kernels.h"
#include "precode.h"

using namespace cairo;

namespace {

// staging slots (frames in flight): three 32-frame batches, so that the host
// entropy of one batch overlaps the GPU work of the next two
constexpr int kDefaultStages = 96;
constexpr int kMaxStages = 256;
constexpr int kLaunchSlots = 64;    // per-launch host records (frame views, timing events), reused round-robin
constexpr int kTimed = 3;        // timed kernels: convert, (inter: fused), engine
// Frames per launch by default, from measured sweeps (DESIGN.md §4.2,
// tools/sweep_bench.sh).  With the pools shared between consecutive launches
// (k_engine next_task) a batch's tail no longer idles half the workers, so
// larger batches pay: 32 up to about 1080p (1080p: 2981 at 12, 3460 at 24,
// 3551 at 32 Mpix/s); at 4K 28 was best in round 3 (4443-4454 vs 4235 at
// 32); on the round-4 engine larger launches pay there: 32 over 28 (5838 vs
// 5808 Mpix/s, three alternating rounds, profiles/r04/batch_ab_4k.txt), and
// with the cap raised to 48: 32 / 36 / 40 / 44 -> 5820 / 5828 / 5856 / 5868
// (two rounds, profiles/r04/batch_cap_4k.txt).  But two 40-frame launches
// in flight leave only 16 of the default 96 staging slots to the host entropy
// pipeline: end to end fell to 82 % of the hot path (profiles/r04/
// bench_4k_batch40.json), so the default stays at 32 everywhere.
inline int default_batch(size_t mbs) {
  (void)mbs;
  return 32;
}
constexpr int kSyncAreas = 3;    // launch b uses area b % 3; launch b+1 reads it too
// The output_cache slots are allocated in chunks of at most this size, each
// exported with its own IPC handle (cairo_peer): an IPC import of one
// fine-grained allocation of 2 GiB or more never returned.
constexpr size_t kCoefChunkBytes = size_t(1) << 30;
// Reconstruction slots of a member of a group over several devices or
// processes: every member keeps the same layout, N * S slots (S = ceil(R / N)),
// frame m in slot (m % N) * S + (m / N) % S -- its producer's own block, a
// mirror block on every other member -- for any N <= kMaxGroup.
constexpr int kMirrorSlots = kMaxGroup > kMaxRing ? kMaxGroup : kMaxRing;
constexpr int kSuccess = 0, kInvalidArg = 1, kOutOfMemory = 3, kHardwareFail = 5,  // evx_status (base.h:150-172)
              kInvalidResource = 8;

struct Stage {
  uint8_t* table = nullptr;  // pinned, mapped (k_feed_copy writes it in feed mode)
  int16_t* coef = nullptr;   // pinned, 1.5 * wa * ha
  int32_t* err = nullptr;    // pinned, mapped: the context's TimeoutInfo words after the frame
  uint8_t* table_dev = nullptr;  // device addresses of table / err
  int32_t* err_dev = nullptr;
  hipEvent_t d2h_done = nullptr;
  // The launch that converts this slot's staged host RGB: a later frame's
  // upload into the same staging buffer waits for it (rgb_read).
  hipEvent_t rgb_read = nullptr;
  bool rgb_pending = false;
  int ticket = -1;
  bool busy = false;      // submitted, not yet released
  bool launched = false;  // its batch has been launched
  uint32_t index = 0, type = 0, quality = 0;
};

struct TimedBatch {
  hipEvent_t ev[kTimed + 1] = {};
  int frames = 0;
  bool pending = false;
};

// Length of the union of [start, end) intervals (ms): the time the engine
// was running at all, with the two in-flight launches overlapping.
double union_length(std::vector<std::pair<double, double>>& iv) {
  std::sort(iv.begin(), iv.end());
  double total = 0, s = 0, e = -1e300;
  for (const auto& p : iv) {
    if (p.first > e) {
      if (e > s) total += e - s;
      s = p.first;
      e = p.second;
    } else if (p.second > e) {
      e = p.second;
    }
  }
  if (e > s) total += e - s;
  return total;
}

}  // namespace

struct cairo_ctx {
  int device = 0;
  uint32_t w = 0, h = 0, wa = 0, ha = 0, wmb = 0, hmb = 0, ring = 0;
  size_t plane_elems = 0, mbs = 0, nref = 1;
  hipStream_t ks = nullptr, cs = nullptr;
  hipStream_t ks2 = nullptr;         // launches alternate between ks and ks2 (consecutive batches overlap)
  // Host RGB uploads (rgb_on_device = 0), issued at submit on a stream of
  // their own so that they overlap the launches in flight; a launch waits for
  // the last one (the stream is in order).  Made on first use; a group member
  // keeps uploading on its launch stream (its queue budget, join_group).
  hipStream_t us = nullptr;
  hipEvent_t up_last = nullptr;
  bool up_pending = false;  // an upload the next launch has not waited for
  hipEvent_t engine_done = nullptr;  // last launched batch finished (copy stream waits on it)
  hipEvent_t batch_end[kSyncAreas] = {};  // end of the launch that used sync area k (every task done)
  hipEvent_t batch_ready[kSyncAreas] = {};  // its frames converted, views and sync area set up
  hipEvent_t pre_done[kSyncAreas] = {};  // its precode's feeds written (the host copy follows on cs)
  bool host_uploads = false;  // host-RGB frames were submitted (the copy stream carries their uploads)
  // the last launch, whose remaining tasks the next launch's workers take first
  const FrameArgs* prev_fa = nullptr;
  const int32_t* prev_order[2] = {};
  const int32_t* prev_seg[2] = {};
  int32_t* prev_sync = nullptr;
  int prev_total = 0, prev_area = 0, prev_decode = 0;
  int order_slope = kOrderSlope;  // of the task order tables (3N + 2 in an N-member group)
  long long batches = 0;             // launches so far
  // per-slot device buffers
  int16_t* src = nullptr;
  int16_t* coef[CAIRO_MAX_COEF_CHUNKS] = {};  // output_cache: slot s in chunk s / coef_per, at s % coef_per
  int coef_chunks = 0, coef_per = 0;
  BlockDesc *table = nullptr, *idesc = nullptr;
  uint64_t* gran = nullptr;
  uint8_t* rgb = nullptr;
  int16_t* ring_buf = nullptr;
  int ring_slots = 0;  // R; kMirrorSlots once allocated for a group over devices / processes
  uint64_t* progress = nullptr;  // [stages][hmb] tagged deblock progress of each slot's frame
  bool fresh = true;             // no frame since create / reset: the next has no predecessor
  long since_fresh = 0;          // frames since create / reset (frame_links)
  // Frame-interleaved group (cairo_ctx_join_group): member grank of gsize
  // encodes the stream's frames n = grank (mod gsize), reading the others'
  // reconstructions, output_cache and progress words in place.
  struct Peer {
    int16_t* ring = nullptr;
    int16_t* coef[CAIRO_MAX_COEF_CHUNKS] = {};
    int coef_chunks = 0, coef_per = 1;
    uint64_t* progress = nullptr;
    int stages = 0;
    bool imported = false;  // opened from another process's IPC handles
  };
  int gsize = 1, grank = 0, gbase = 0;  // gbase: ticket of the group's frame grank
  Peer gp[kMaxGroup];
  int16_t* zero = nullptr;  // a zero plane set: references before the stream start
  bool fine_grained = false;  // ring / coef / progress allocated fine-grained (cross-device sharing)
  // Outputs for the host entropy stage (cairo_ctx_set_outputs): the
  // coefficient planes (D2H per frame) and/or the GPU precode's feed bits
  // (precode.hip), written straight into mapped pinned host memory.
  int outputs = CAIRO_OUT_COEF;
  size_t feed_words = 0;          // per staging slot
  uint32_t* feed_dev = nullptr;   // [stages][feed_words]
  uint32_t* feed_hdr = nullptr;   // [stages][kFeedHdrWords]
  uint32_t* feed_scratch = nullptr;  // [stages][feed_scratch_words(mbs)]
  uint32_t* feed_host = nullptr;  // mapped pinned [stages][kFeedHdrWords + feed_words]
  hipStream_t fs = nullptr;       // synchronous coefficient fetches (a frame whose feed overflowed)
  // (The precode runs on the launch's stream, between its kernel and the
  // launch two ahead: on a stream of its own its kernels took the slots the
  // next launch's workers need, -2 to -5 % at 4K)
  bool sys = false;           // a member is another process or device: system-scope hand-offs
  int32_t *sync = nullptr;
  int32_t* sticky = nullptr;  // TimeoutInfo words (kernels.h), cleared only by zero_state
  int inject = 0;             // test hook (cairo_ctx_set_debug 16): EngineArgs::inject
  int32_t* order = nullptr;  // [kMaxBatch][kMaxBatch * hmb]: pool task order per batch size
  FrameArgs* fdesc_host = nullptr;  // pinned [kLaunchSlots][kMaxBatch]: per-frame views per launch
  FrameArgs* fdesc_host_dev = nullptr;  // its device-visible address (read by the convert kernel)
  FrameArgs* fdesc = nullptr;       // device copy
  int fdesc_next = 0;
  // the H2D copy of each fdesc_host slot: a slot is rewritten only after its
  // previous copy ran (more than kLaunchSlots launches may be queued, e.g.
  // batch 1 with 96 staging slots, and the copy waits behind earlier launches)
  hipEvent_t fdesc_done[kLaunchSlots] = {};
  bool fdesc_used[kLaunchSlots] = {};
  int32_t* trace_host = nullptr;  // diagnostic live trace (mapped), opt-in via set_debug(4)
  int32_t* trace_dev = nullptr;
  size_t sync_words = 0;
  int stages = kDefaultStages;
  std::vector<Stage> st;  // [stages]
  int next_ticket = 0;
  uint32_t epoch = 0;
  int batch_max = 16;
  FrameDesc pend[kMaxBatch];
  int npend = 0;
  int last_slot = -1;  // slot of the last launched frame
  uint32_t last_epoch = 0;  // and its epoch (the tag of its inter records)
  int wg_rows = 0;
  int wg_helpers = 0;  // helpers of the launch's 2 * wg_rows workgroups (0: half)
  int max_rows = 0;  // row coders (= helpers) per launch that stay co-resident with the other in-flight launch
  bool profiling = false;
  TimedBatch tb[kLaunchSlots];
  int tb_next = 0;
  double acc_ms[kTimed] = {0, 0, 0};
  int acc_frames = 0;
  hipEvent_t t_base = nullptr;  // profiling epoch: engine intervals are measured from it
  std::vector<std::pair<double, double>> busy;  // engine [start, end) per launch, ms after t_base
  int16_t* predeblock = nullptr;  // debug: pre-deblock reconstruction of the last frame (opt-in)
  uint64_t* stamps = nullptr;     // diagnostic phase stamps (opt-in)
  uint64_t* acct = nullptr;       // diagnostic time accounting (opt-in; CAIRO_ACCT builds fill it)
  // Thread safety (the frame pipeline of pipeline.cpp calls in from its
  // completion and entropy threads): every public entry point holds mu;
  // HIP event waits on a frame's outputs run outside it.  launched_cv is
  // signalled when a batch launches.
  std::mutex mu;
  std::condition_variable launched_cv;
  std::mutex tmu;                             // guards timeout (written by threads waiting outside mu)
  int32_t timeout[TimeoutInfo::kWords] = {};  // the last reported TimeoutInfo words
};

namespace {

int fail(hipError_t e, const char* what) {
  if (e == hipSuccess) return kSuccess;
  fprintf(stderr, "[cairo_amd] %s: %s\n", what, hipGetErrorString(e));
  return kHardwareFail;
}
#define CK(x)                                   \
  do {                                          \
    int _r = fail((x), #x);                     \
    if (_r != kSuccess) return _r;              \
  } while (0)

PlaneSet planes_at(int16_t* base, const cairo_ctx* c) {
  return ring_slot(base, 0, (int)c->wa, (int)c->ha, 0);
}
PlaneSet slot_planes(int16_t* base, const cairo_ctx* c, int slot) {
  return ring_slot(base, c->plane_elems, (int)c->wa, (int)c->ha, slot);
}
// Staging slot s's output_cache (chunked allocation).
int16_t* coef_base(const cairo_ctx* c, int slot) {
  return c->coef[slot / c->coef_per] + (size_t)(slot % c->coef_per) * c->plane_elems;
}
PlaneSet coef_planes(const cairo_ctx* c, int slot) { return planes_at(coef_base(c, slot), c); }
PlaneSet peer_coef_planes(const cairo_ctx::Peer& p, const cairo_ctx* c, int slot) {
  return planes_at(p.coef[slot / p.coef_per] + (size_t)(slot % p.coef_per) * c->plane_elems, c);
}
// Allocate the output_cache: one allocation for a context nobody imports;
// fine-grained chunks of at most kCoefChunkBytes, each exported with its own
// IPC handle, for cross-device sharing (cairo_ctx_peer_info).  On failure
// nothing stays allocated.
hipError_t alloc_coef(const cairo_ctx* c, bool fine, int16_t* out[CAIRO_MAX_COEF_CHUNKS], int* chunks, int* per) {
  const size_t slot_bytes = c->plane_elems * 2;
  if (fine && slot_bytes > kCoefChunkBytes) {
    fprintf(stderr, "[cairo_amd] peer_info: one output_cache slot (%zu bytes) exceeds the %zu-byte IPC export limit\n",
            slot_bytes, kCoefChunkBytes);
    return hipErrorInvalidValue;
  }
  const int p = fine ? (int)std::min<size_t>((size_t)c->stages, kCoefChunkBytes / slot_bytes) : c->stages;
  const int n = (c->stages + p - 1) / p;
  if (n > CAIRO_MAX_COEF_CHUNKS) {
    fprintf(stderr, "[cairo_amd] peer_info: %d output_cache chunks needed, at most %d\n", n, CAIRO_MAX_COEF_CHUNKS);
    return hipErrorInvalidValue;
  }
  for (int k = 0; k < CAIRO_MAX_COEF_CHUNKS; k++) out[k] = nullptr;
  for (int k = 0; k < n; k++) {
    const size_t bytes = slot_bytes * (size_t)std::min(p, c->stages - k * p);
    const hipError_t e = fine ? hipExtMallocWithFlags((void**)&out[k], bytes, hipDeviceMallocFinegrained)
                              : hipMalloc((void**)&out[k], bytes);
    if (e != hipSuccess) {
      for (int j = 0; j <= k; j++)
        if (out[j]) (void)hipFree(out[j]);
      for (int j = 0; j < CAIRO_MAX_COEF_CHUNKS; j++) out[j] = nullptr;
      return e;
    }
  }
  *chunks = n;
  *per = p;
  return hipSuccess;
}

size_t stamp_words(const cairo_ctx* c) {
  // frames, engine entry/exit, then 3 stamps per inter task
  return kMaxBatch * stamp_frame_words((int)c->wmb, (int)c->hmb) + 2 +
         (size_t)kMaxBatch * c->hmb * ((c->wmb + 3) / 4) * kIStamps;
}

EngineArgs engine_args(const cairo_ctx* c) {
  EngineArgs e;
  memset(&e, 0, sizeof(e));
  e.wa = (int)c->wa, e.ha = (int)c->ha, e.w = (int)c->w, e.h = (int)c->h;
  e.wmb = (int)c->wmb, e.hmb = (int)c->hmb, e.ring = (int)c->ring;
  e.src_base = c->src;
  e.plane_elems = c->plane_elems;
  e.table_base = c->table;
  e.idesc_base = c->idesc;
  e.gran_base = c->gran;
  e.sync = c->sync;
  e.sticky = c->sticky;
  e.inject = c->inject;
  e.stamps = c->stamps;
  e.acct = c->acct;
  e.trace = c->trace_dev;
  return e;
}

// Close the group's imported peer mappings and forget the group.
void leave_group(cairo_ctx* c) {
  for (int i = 0; i < c->gsize; i++) {
    cairo_ctx::Peer& p = c->gp[i];
    if (p.imported) {
      for (void* q : {(void*)p.ring, (void*)p.progress})
        if (q) (void)hipIpcCloseMemHandle(q);
      for (int k = 0; k < p.coef_chunks; k++)
        if (p.coef[k]) (void)hipIpcCloseMemHandle(p.coef[k]);
    }
    p = cairo_ctx::Peer();
  }
  if (c->zero) (void)hipFree(c->zero);
  c->zero = nullptr;
  c->gsize = 1;
  c->grank = 0;
  c->sys = false;
}

// (frame, row) task order of the engine pools for every batch size, by
// row + slope * frame (kOrderSlope for one context; a group of N members
// needs 3N + 2: kernels.h kOrderSlope).
std::vector<int32_t> task_order(int hmb, int slope) {
  const int per = kMaxBatch * hmb;
  std::vector<int32_t> ord((size_t)kMaxBatch * per, 0);
  for (int nf = 1; nf <= kMaxBatch; nf++) {
    int32_t* o = &ord[(size_t)(nf - 1) * per];
    int n = 0;
    for (int d = 0; d < hmb + slope * nf; d++)
      for (int f = 0; f < nf; f++) {
        const int r = d - slope * f;
        if (r >= 0 && r < hmb) o[n++] = (f << 16) | r;
      }
  }
  return ord;
}

// The device block of task orders (OrderBlock): for every batch size the
// plain order (one queue per pool) and the labelled one (task_order stably
// partitioned by task_label: one queue per label and pool), then each one's
// label segments.
struct OrderBlock {
  static size_t order_at(int hmb, int banded, int nf) { return ((size_t)banded * kMaxBatch + nf - 1) * kMaxBatch * hmb; }
  static size_t seg_at(int hmb, int banded, int nf) {
    return (size_t)2 * kMaxBatch * kMaxBatch * hmb + ((size_t)banded * kMaxBatch + nf - 1) * (kLabels + 1);
  }
  static size_t words(int hmb) { return seg_at(hmb, 2, 1); }
};

std::vector<int32_t> order_block(int hmb, int slope) {
  const std::vector<int32_t> ord = task_order(hmb, slope);
  std::vector<int32_t> blk(OrderBlock::words(hmb), 0);
  for (int nf = 1; nf <= kMaxBatch; nf++) {
    const int32_t* o = &ord[(size_t)(nf - 1) * kMaxBatch * hmb];
    const int total = nf * hmb;
    std::copy(o, o + total, &blk[OrderBlock::order_at(hmb, 0, nf)]);
    int32_t* seg = &blk[OrderBlock::seg_at(hmb, 0, nf)];
    for (int l = 1; l <= kLabels; l++) seg[l] = total;
    int32_t* ob = &blk[OrderBlock::order_at(hmb, 1, nf)];
    int32_t* sb = &blk[OrderBlock::seg_at(hmb, 1, nf)];
    int n = 0;
    for (int l = 0; l < kLabels; l++) {
      sb[l] = n;
      for (int i = 0; i < total; i++)
        if (task_label(o[i] >> 16, o[i] & 0xFFFF, hmb) == l) ob[n++] = o[i];
    }
    sb[kLabels] = n;
  }
  return blk;
}

// Whether a launch's pool uses per-label (XCD-banded) queues: frames of at
// least kBandMinRows macroblock rows, both pools splitting evenly over the
// labels, and the pool enabled in kBandPools.  flush() and cairo_task_queues
// share it, so the tests check the layout the engine runs.
bool banded_pool(int hmb, int n_helpers, int n_rows, int pool) {
  return hmb >= kBandMinRows && n_helpers % kLabels == 0 && n_rows % kLabels == 0 && ((kBandPools >> pool) & 1);
}

int upload_orders(cairo_ctx* c, int slope) {
  c->order_slope = slope;
  const std::vector<int32_t> blk = order_block((int)c->hmb, slope);
  CK(hipMemcpy(c->order, blk.data(), blk.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  c->prev_total = 0;  // the previous launch's queue used the other order
  return kSuccess;
}

void free_ctx(cairo_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->ks) (void)hipStreamSynchronize(c->ks);
  if (c->ks2) (void)hipStreamSynchronize(c->ks2);
  if (c->cs) (void)hipStreamSynchronize(c->cs);
  for (auto& s : c->st) {
    if (s.table) (void)hipHostFree(s.table);
    if (s.coef) (void)hipHostFree(s.coef);
    if (s.err) (void)hipHostFree(s.err);
    if (s.d2h_done) (void)hipEventDestroy(s.d2h_done);
    if (s.rgb_read) (void)hipEventDestroy(s.rgb_read);
  }
  for (auto& t : c->tb)
    for (auto& e : t.ev)
      if (e) (void)hipEventDestroy(e);
  if (c->engine_done) (void)hipEventDestroy(c->engine_done);
  if (c->t_base) (void)hipEventDestroy(c->t_base);
  for (auto& ev : c->batch_end)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : c->batch_ready)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : c->pre_done)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : c->fdesc_done)
    if (ev) (void)hipEventDestroy(ev);
  if (c->fdesc_host) (void)hipHostFree(c->fdesc_host);
  if (c->feed_host) (void)hipHostFree(c->feed_host);
  if (c->fs) (void)hipStreamDestroy(c->fs);
  if (c->trace_host) (void)hipHostFree(c->trace_host);
  leave_group(c);
  for (int16_t* q : c->coef)
    if (q) (void)hipFree(q);
  for (void* p : {(void*)c->fdesc, (void*)c->order, (void*)c->src, (void*)c->table, (void*)c->idesc, (void*)c->progress, (void*)c->feed_dev, (void*)c->feed_hdr, (void*)c->feed_scratch,
                  (void*)c->gran, (void*)c->rgb, (void*)c->ring_buf, (void*)c->sync, (void*)c->sticky,
                  (void*)c->predeblock, (void*)c->stamps, (void*)c->acct})
    (void)hipFree(p);
  if (c->us) (void)hipStreamSynchronize(c->us);
  if (c->up_last) (void)hipEventDestroy(c->up_last);
  if (c->us) (void)hipStreamDestroy(c->us);
  if (c->ks) (void)hipStreamDestroy(c->ks);
  if (c->ks2) (void)hipStreamDestroy(c->ks2);
  if (c->cs) (void)hipStreamDestroy(c->cs);
  delete c;
}

// Fresh-encoder state (every stream idle): zero planes, tables and granules,
// the launch sync areas and the sticky timeout word, so a context that once
// reported a timed-out wait is usable again after cairo_ctx_reset.
int zero_state(cairo_ctx* c) {
  const size_t S = (size_t)c->stages;
  CK(hipMemsetAsync(c->src, 0, c->plane_elems * 2 * S, c->ks));
  for (int k = 0; k < c->coef_chunks; k++)
    CK(hipMemsetAsync(c->coef[k], 0, c->plane_elems * 2 * (size_t)std::min(c->coef_per, c->stages - k * c->coef_per),
                      c->ks));
  CK(hipMemsetAsync(c->ring_buf, 0, c->plane_elems * 2 * c->ring_slots, c->ks));
  CK(hipMemsetAsync(c->table, 0, c->mbs * sizeof(BlockDesc) * S, c->ks));
  // inter records: a frame whose search was cut short by a timed-out wait
  // still reads in-frame motion vectors
  CK(hipMemsetAsync(c->idesc, 0, c->nref * c->mbs * sizeof(BlockDesc) * S, c->ks));
  // granule tags start at 0; the n-th submission after a reset publishes tag n
  CK(hipMemsetAsync(c->gran, 0, c->mbs * kGranuleStride * sizeof(uint64_t) * S, c->ks));
  CK(hipMemsetAsync(c->sync, 0, c->sync_words * sizeof(int32_t) * kSyncAreas, c->ks));
  CK(hipMemsetAsync(c->progress, 0, (size_t)c->hmb * sizeof(uint64_t) * S, c->ks));
  CK(hipMemsetAsync(c->sticky, 0, TimeoutInfo::kWords * sizeof(int32_t), c->ks));
  CK(hipStreamSynchronize(c->ks));
  {
    std::lock_guard<std::mutex> lk(c->tmu);
    memset(c->timeout, 0, sizeof(c->timeout));
  }
  c->epoch = 0;
  c->last_slot = -1;
  c->batches = 0;
  c->prev_total = 0;  // its sync areas are zero now
  c->fresh = true;  // the first frame after a reset depends on no earlier frame
  c->since_fresh = 0;
  // tickets restart at 0 (every stage is idle here): a group member's k-th
  // frame after a (re)join is its ticket k, which its peers assume when they
  // locate its output_cache and progress words (frame_links)
  c->next_ticket = 0;
  for (auto& s : c->st) {
    memset(s.err, 0, TimeoutInfo::kWords * sizeof(int32_t));
    s.ticket = -1;
  }
  return kSuccess;
}

int collect_times(cairo_ctx* c, TimedBatch& t) {
  if (!t.pending) return kSuccess;
  CK(hipEventSynchronize(t.ev[kTimed]));
  for (int k = 0; k < kTimed; k++) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t.ev[k], t.ev[k + 1]));
    c->acc_ms[k] += ms;
  }
  float s0 = 0, s1 = 0;  // the engine's interval on the common clock
  CK(hipEventElapsedTime(&s0, c->t_base, t.ev[2]));
  CK(hipEventElapsedTime(&s1, c->t_base, t.ev[3]));
  c->busy.emplace_back((double)s0, (double)s1);
  c->acc_frames += t.frames;
  t.pending = false;
  return kSuccess;
}

// Launch the pending batch.
int flush(cairo_ctx* c) {
  if (c->npend == 0) return kSuccess;
  CK(hipSetDevice(c->device));
  EngineArgs e = engine_args(c);
  e.nframes = c->npend;
  // frame descriptors -> device (a ring of pinned slots: the copy of an earlier
  // launch may still be pending when this one is written)
  const int fslot = c->fdesc_next;
  c->fdesc_next = (c->fdesc_next + 1) % kLaunchSlots;
  if (c->fdesc_used[fslot]) CK(hipEventSynchronize(c->fdesc_done[fslot]));
  FrameArgs* fh = c->fdesc_host + (size_t)fslot * kMaxBatch;
  FrameArgs* fd = c->fdesc + (size_t)fslot * kMaxBatch;
  bool any_inter = false;
  for (int i = 0; i < c->npend; i++) any_inter |= c->pend[i].inter && c->ring > 1;
  e.fa = fd;
  e.decode = c->pend[0].decode;  // a launch never mixes (decode_frame flushes first)
  const int rows = e.nframes * e.hmb;
  (void)any_inter;
  // Launch b alternates streams and sync areas; it follows launch b-1, which
  // may still be running: its frame 0 waits on the deblock progress of b-1's
  // last frame (tagged words in that frame's staging slot).  Residency: a
  // launch takes at most half of the engine's resident
  // workgroup slots (CUs x occupancy, measured at create: 256 x 3 = 768 on a
  // full MI355X), so two launches are always co-resident.  Every row has a
  // coder task and a helper (inter search + deblock) task: two pools.  The
  // pools are shared: launch b's workers take b-1's
  // remaining tasks first (all of them are older), so b-1's tail is not left
  // to b-1's own workers; a batch is complete when its finished-task count
  // says so (k_batch_wait), not when its launch ends.
  const long long b = c->batches++;
  hipStream_t st = (b & 1) ? c->ks2 : c->ks;
  const int area = (int)(b % kSyncAreas);
  e.sync = c->sync + (size_t)area * c->sync_words;
  e.pfa = c->prev_fa;
  for (int k = 0; k < 2; k++) e.porder[k] = c->prev_order[k], e.pseg[k] = c->prev_seg[k];
  e.psync = c->prev_sync;
  e.ptotal = c->prev_decode == e.decode ? c->prev_total : 0;  // a worker runs one kind of task
  e.slope = c->order_slope;
  for (int i = 0; i < c->npend; i++) fh[i] = make_frame_view(e, c->pend[i], i);
  {  // half of the resident slots per launch, split between the pools
    const int total = 2 * (c->wg_rows > 0 ? std::min(c->wg_rows, (c->stamps ? 2 : 1) * c->max_rows) : c->max_rows);
    // default split: even, and 25/48 helpers (200 of 384) on large frames
    // (kernels.h kPrioFrameMBs); multiples of kLabels keep both pools banded
    const bool large = (int)c->wmb * (int)c->hmb > kPrioFrameMBs;
    int nh = c->wg_helpers > 0 ? std::min(c->wg_helpers, total - 1)
                               : (large ? std::max(1, (total * 25 / 48) & ~(kLabels - 1)) : total / 2);
    int nr = total - nh;
    e.n_helpers = std::max(1, std::min(nh, rows));
    e.n_rows = std::max(1, std::min(nr, rows));
  }
  // XCD-banded queues (kernels.h kLabels) on large frames, when both pools
  // split evenly over the labels
  for (int k = 0; k < 2; k++) {
    const int bk = banded_pool((int)c->hmb, e.n_helpers, e.n_rows, k);
    e.nlab[k] = bk ? kLabels : 1;
    e.order[k] = c->order + OrderBlock::order_at((int)c->hmb, bk, e.nframes);
    e.seg[k] = c->order + OrderBlock::seg_at((int)c->hmb, bk, e.nframes);
  }
  // this sync area was last used by launch b-3 (only a launch reads its own
  // area); launch b-2 precedes this one on the same stream
  if (b >= 3) CK(hipStreamWaitEvent(st, c->batch_end[(b - 3) % kSyncAreas], 0));
  TimedBatch* tb = nullptr;
  if (c->profiling) {
    tb = &c->tb[c->tb_next];
    c->tb_next = (c->tb_next + 1) % kLaunchSlots;
    int r = collect_times(c, *tb);  // its events are about to be reused
    if (r) return r;
  }
  if (c->up_pending) {  // the frames' uploads, issued at submit on the upload stream
    CK(hipStreamWaitEvent(st, c->up_last, 0));
    c->up_pending = false;
  }
  for (int i = 0; i < e.nframes; i++) {  // host RGB sources; the decoder's table and coefficients
    const FrameDesc& f = c->pend[i];
    if (f.host_rgb)
      CK(hipMemcpyAsync((void*)f.rgb, f.host_rgb, (size_t)c->w * c->h * 3, hipMemcpyHostToDevice, st));
    if (f.decode) {
      CK(hipMemcpyAsync(c->table + (size_t)f.slot * c->mbs, f.host_table, c->mbs * sizeof(BlockDesc),
                        hipMemcpyHostToDevice, st));
      CK(hipMemcpyAsync(coef_base(c, f.slot), f.host_coef, c->plane_elems * 2, hipMemcpyHostToDevice, st));
    }
  }
  // the frame views and the zeroed sync area are written by the convert
  // kernel below (ConvertArgs), not by runtime copy / fill kernels
  ConvertArgs ca{};
  ca.w = e.w, ca.h = e.h, ca.wa = e.wa, ca.nframes = e.nframes;
  for (int i = 0; i < e.nframes; i++) {
    ca.rgb[i] = fh[i].decode ? nullptr : fh[i].rgb;
    ca.in[i] = fh[i].in;
  }
  static_assert(sizeof(FrameArgs) % sizeof(uint4) == 0, "frame views copied in 16-byte chunks");
  ca.fa_host = (const uint4*)(c->fdesc_host_dev + (size_t)fslot * kMaxBatch);
  ca.fa_dev = (uint4*)fd;
  ca.fa_chunks = (int)(sizeof(FrameArgs) * e.nframes / sizeof(uint4));
  ca.sync = e.sync;
  ca.sync_words = (int)c->sync_words;
  if (c->stamps) {  // engine entry (min) / exit (max) words
    static const uint64_t init[2] = {~0ull, 0};
    CK(hipMemcpyAsync(c->stamps + kMaxBatch * stamp_frame_words((int)c->wmb, (int)c->hmb), init, sizeof(init),
                      hipMemcpyHostToDevice, st));
  }
  if (tb) CK(hipEventRecord(tb->ev[0], st));
  CK(launch_convert_batch(ca, st));
  CK(hipEventRecord(c->fdesc_done[fslot], st));  // fh has been read
  c->fdesc_used[fslot] = true;
  for (int i = 0; i < e.nframes; i++) {  // staged host RGB converted: the buffer may be refilled
    const FrameDesc& f = c->pend[i];
    Stage& s = c->st[f.slot];
    if (!f.decode && f.rgb == c->rgb + (size_t)f.slot * c->w * c->h * 3) {
      CK(hipEventRecord(s.rgb_read, st));
      s.rgb_pending = true;
    }
  }
  CK(hipEventRecord(c->batch_ready[area], st));
  // the previous batch's tasks, which this launch's workers may run, need its
  // frames converted and its views and sync area in place
  if (e.ptotal) CK(hipStreamWaitEvent(st, c->batch_ready[c->prev_area], 0));
  if (tb) CK(hipEventRecord(tb->ev[1], st));
  if (tb) CK(hipEventRecord(tb->ev[2], st));
  CK(launch_engine(e, st));
  // the launch ends when its workers find no task left; its batch is done
  // when every task has finished (the next launch's workers may run the last)
  CK(launch_batch_wait(e.sync, 2 * rows, c->sticky, st));
  c->prev_fa = fd;
  for (int k = 0; k < 2; k++) c->prev_order[k] = e.order[k], c->prev_seg[k] = e.seg[k];
  c->prev_sync = e.sync;
  c->prev_total = rows;
  c->prev_area = area;
  c->prev_decode = e.decode;
  if (tb) {
    CK(hipEventRecord(tb->ev[3], st));
    tb->frames = e.nframes;
    tb->pending = true;
  }
  const int last = c->pend[e.nframes - 1].slot;
  const uint32_t last_epoch = c->pend[e.nframes - 1].epoch;
  if (c->predeblock) CK(launch_unpack_granules(e, e.nframes - 1, planes_at(c->predeblock, c), st));
  hipStream_t ost = st;  // the stream the launch's outputs complete on
  if (c->outputs & CAIRO_OUT_FEED) {  // the entropy precode, straight into mapped host memory
    FeedArgs fa;
    memset(&fa, 0, sizeof(fa));
    fa.nframes = e.nframes;
    fa.fa = fd;
    for (int i = 0; i < e.nframes; i++) {
      fa.slot[i] = c->pend[i].slot;
      fa.host[i] = c->feed_host + (size_t)fa.slot[i] * (kFeedHdrWords + c->feed_words);
    }
    fa.scratch = c->feed_scratch;
    fa.scratch_stride = feed_scratch_words(c->mbs);
    fa.feed = c->feed_dev;
    fa.feed_stride = c->feed_words;
    fa.hdr = c->feed_hdr;
    // each frame's block table and the timeout words go to its mapped pinned
    // stage in the same kernel as the feed: no D2H copy per frame, whose
    // shader blit waits for a workgroup slot of the persistent engine
    for (int i = 0; i < e.nframes; i++) {
      const Stage& s = c->st[fa.slot[i]];
      fa.table_host[i] = c->pend[i].decode ? nullptr : (uint4*)s.table_dev;
      fa.err_host[i] = c->pend[i].decode ? nullptr : s.err_dev;
    }
    fa.table_words = (int)(c->mbs * sizeof(BlockDesc) / sizeof(uint4));
    CK(launch_precode(fa, (int)c->mbs, st));
    // The copy into the mapped host stages is PCIe-bound and no engine
    // launch needs it: on the copy stream, so that the launch two ahead on
    // this stream starts without it (+0.2 %, profiles/r06/ab_4k_feed_copy_aside.txt).
    // Not when the copy stream carries host-RGB uploads (submit): those must
    // not queue behind a feed copy that waits for its launch.
    if (!c->host_uploads) {
      CK(hipEventRecord(c->pre_done[area], st));
      CK(hipStreamWaitEvent(c->cs, c->pre_done[area], 0));
      CK(launch_feed_copy(fa, c->cs));
      ost = c->cs;
    } else {
      CK(launch_feed_copy(fa, st));
    }
  }
  CK(hipEventRecord(c->batch_end[area], ost));
  // the copy stream carries the outputs' copies to the host: the feed copies
  // (k_feed_copy, above) or the host-RGB uploads (submit), and with the
  // coefficient planes their D2H copies (the uploads then go on a stream of
  // their own)
  if ((c->outputs & CAIRO_OUT_COEF) && ost != c->cs) {
    CK(hipStreamWaitEvent(c->cs, c->batch_end[area], 0));
  }
  // outputs for the host entropy stage: with the feed, the precode's last
  // kernel (k_feed_copy) has written each frame's feed, block table and
  // timeout words into its mapped pinned stage; the coefficient planes (and,
  // without the feed, the table and timeout words) go D2H on the copy stream
  for (int i = 0; i < e.nframes; i++) {
    const int slot = c->pend[i].slot;
    Stage& s = c->st[slot];
    if (c->pend[i].decode) {  // the decoder's output is the slot (decode_frame converts it)
      s.launched = true;
      continue;
    }
    if (c->outputs & CAIRO_OUT_COEF) {
      if (!(c->outputs & CAIRO_OUT_FEED)) {
        CK(hipMemcpyAsync(s.table, c->table + (size_t)slot * c->mbs, c->mbs * sizeof(BlockDesc),
                          hipMemcpyDeviceToHost, c->cs));
        CK(hipMemcpyAsync(s.err, c->sticky, TimeoutInfo::kWords * sizeof(int32_t), hipMemcpyDeviceToHost, c->cs));
      }
      CK(hipMemcpyAsync(s.coef, coef_base(c, slot), c->plane_elems * 2, hipMemcpyDeviceToHost, c->cs));
      CK(hipEventRecord(s.d2h_done, c->cs));
    } else {
      CK(hipEventRecord(s.d2h_done, ost));
    }
    s.launched = true;
  }
  c->last_slot = last;
  c->last_epoch = last_epoch;
  c->npend = 0;
  c->launched_cv.notify_all();
  return kSuccess;
}

// The cross-frame views of the frame submitted as ticket t (FrameDesc):
// ring slots by index (common.cpp:192-195), the previous ticket's staging
// slot for the output_cache chain and its deblock progress.
void frame_links(cairo_ctx* c, FrameDesc& f, int t) {
  const int R = (int)c->ring;
  f.sys = c->sys;
  if (c->gsize > 1) {
    // Group member: frame m lives with member m % N as its ticket m / N
    // (staging slot (m / N) % stages, reconstruction slot (m / N) % S with
    // S = ceil(R / N) slots per member, so that a slot is reused only by a
    // frame at least R later; when N * S == R that is frame m + R itself,
    // in place, as in the reference's ring).
    const int N = c->gsize, S = (R + N - 1) / N;
    const long n = f.index;
    const PlaneSet zero = planes_at(c->zero, c);
    // Members on other devices or processes (sys) keep mirrors: every frame
    // read here is local (slot (m % N) * S + (m / N) % S of this member's
    // ring), and this frame's deblock pushes it into the same slot of each
    // member that reads it.  Members on one device read each other's rings.
    const bool mirror = c->sys && c->fine_grained && c->ring_slots >= N * S;
    auto slot_of = [&](long m) { return mirror ? (int)((m % N) * S + (m / N) % S) : (int)((m / N) % S); };
    auto recon_of = [&](long m) {
      if (m < 0) return zero;
      return slot_planes(mirror ? c->ring_buf : c->gp[m % N].ring, c, slot_of(m));
    };
    for (int k = 0; k < kMaxRing; k++) f.recon[k] = k < R ? recon_of(n - k) : zero;
    f.stale = recon_of(n - R);
    f.npush = 0;
    if (mirror) {
      bool seen[kMaxGroup] = {};
      seen[c->grank] = true;
      for (int d = 1; d <= R; d++) {  // the frames n+1..n+R-1 reference it, n+R reads its stale rows
        const int j = (int)((n + d) % N);
        if (seen[j]) continue;
        seen[j] = true;
        f.push[f.npush++] = slot_planes(c->gp[j].ring, c, slot_of(n));
      }
    }
    f.progress = c->progress + (size_t)f.slot * c->hmb;
    f.coef = coef_planes(c, f.slot);
    if (n >= 1) {
      const cairo_ctx::Peer& p = c->gp[(n - 1) % N];
      const int ps = (int)(((n - 1) / N) % p.stages);
      f.coef_prev = peer_coef_planes(p, c, ps);
      f.prev_progress = p.progress + (size_t)ps * c->hmb;
    } else {
      f.coef_prev = zero;
      f.prev_progress = nullptr;
    }
    if (n >= 2) {
      const cairo_ctx::Peer& p = c->gp[(n - 2) % N];
      f.prev2_progress = p.progress + (size_t)(((n - 2) / N) % p.stages) * c->hmb;
    } else {
      f.prev2_progress = nullptr;
    }
    c->fresh = false;
    c->since_fresh++;
    return;
  }
  for (int k = 0; k < kMaxRing; k++)
    f.recon[k] = slot_planes(c->ring_buf, c, k < R ? (int)(((uint32_t)f.index + R - k) % R) : 0);
  f.npush = 0;
  f.stale = f.recon[0];
  const int ps = (t + c->stages - 1) % c->stages;
  f.coef = coef_planes(c, f.slot);
  f.coef_prev = coef_planes(c, ps);
  f.progress = c->progress + (size_t)f.slot * c->hmb;
  f.prev_progress = c->fresh ? nullptr : c->progress + (size_t)ps * c->hmb;
  f.prev2_progress = c->since_fresh < 2 ? nullptr : c->progress + (size_t)((t + 2 * c->stages - 2) % c->stages) * c->hmb;
  c->fresh = false;
  c->since_fresh++;
}

int sync_all(cairo_ctx* c) {
  int r = flush(c);
  if (r) return r;
  CK(hipStreamSynchronize(c->ks));
  CK(hipStreamSynchronize(c->ks2));
  CK(hipStreamSynchronize(c->cs));
  if (c->us) CK(hipStreamSynchronize(c->us));
  return kSuccess;
}

}  // namespace

extern "C" {

int cairo_ctx_create(uint32_t width, uint32_t height, uint32_t ring, int device, cairo_ctx** out) {
  return cairo_ctx_create_ex(width, height, ring, device, kDefaultStages, out);
}

int cairo_ctx_create_ex(uint32_t width, uint32_t height, uint32_t ring, int device, int stages,
                        cairo_ctx** out) {
  // The reference indexes blocks with uint16 (deblock.cpp, serialize.cpp): at
  // most 65535 macroblocks per frame.
  if (!out || width == 0 || height == 0 || (width & 1) || (height & 1) || ring < 1 ||
      ring > (uint32_t)kMaxRing || ((width + 15) / 16) * ((height + 15) / 16) > 65535u || stages < 2 ||
      stages > kMaxStages)
    return kInvalidArg;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
    fprintf(stderr, "[cairo_amd] no HIP device %d available (count %d)\n", device, n);
    return kHardwareFail;
  }
  cairo_ctx* c = new (std::nothrow) cairo_ctx;
  if (!c) return kOutOfMemory;
  c->device = device;
  c->w = width;
  c->h = height;
  c->wa = (width + 15) & ~15u;
  c->ha = (height + 15) & ~15u;
  c->wmb = c->wa / 16;
  c->hmb = c->ha / 16;
  c->ring = ring;
  c->plane_elems = (size_t)c->wa * c->ha * 3 / 2;
  c->mbs = (size_t)c->wmb * c->hmb;
  c->stages = stages;
  c->st.resize((size_t)stages);
  c->batch_max = std::min(default_batch(c->mbs), stages / 2);
  c->nref = ring > 1 ? ring - 1 : 1;
  c->sync_words = (size_t)SyncLayout::words((int)c->hmb, (int)(c->wmb + 3) / 4);
  int r = kSuccess;
#define TRY(x)                         \
  do {                                 \
    r = fail((x), #x);                 \
    if (r != kSuccess) {               \
      free_ctx(c);                     \
      return r;                        \
    }                                  \
  } while (0)
  TRY(hipSetDevice(device));
  {  // engine pools per launch: half of the resident workgroup slots, split
     // between helpers and row coders at submit
    int cus = 0, per_cu = 0;
    TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    TRY(engine_blocks_per_cu(&per_cu));
    c->max_rows = std::max(1, cus * per_cu / 4);
  }
  TRY(hipStreamCreateWithFlags(&c->ks, hipStreamNonBlocking));
  TRY(hipStreamCreateWithFlags(&c->ks2, hipStreamNonBlocking));
  TRY(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
  const size_t S = (size_t)stages;
  TRY(hipMalloc(&c->src, c->plane_elems * 2 * S));
  TRY(alloc_coef(c, false, c->coef, &c->coef_chunks, &c->coef_per));
  TRY(hipMalloc(&c->ring_buf, c->plane_elems * 2 * ring));
  c->ring_slots = (int)ring;
  TRY(hipMalloc(&c->table, c->mbs * sizeof(BlockDesc) * S));
  TRY(hipMalloc(&c->idesc, c->nref * c->mbs * sizeof(BlockDesc) * S));
  TRY(hipMalloc(&c->gran, c->mbs * kGranuleStride * sizeof(uint64_t) * S));
  TRY(hipMalloc(&c->rgb, (size_t)width * height * 3 * S));
  TRY(hipMalloc(&c->sync, c->sync_words * sizeof(int32_t) * kSyncAreas));
  TRY(hipMalloc(&c->progress, (size_t)c->hmb * sizeof(uint64_t) * S));
  TRY(hipMalloc(&c->sticky, TimeoutInfo::kWords * sizeof(int32_t)));
  TRY(hipMemset(c->sticky, 0, TimeoutInfo::kWords * sizeof(int32_t)));
  {  // (frame, row) task order of the engine pools, for every batch size
    TRY(hipHostMalloc(&c->fdesc_host, sizeof(FrameArgs) * kLaunchSlots * kMaxBatch, hipHostMallocMapped));
    TRY(hipHostGetDevicePointer((void**)&c->fdesc_host_dev, c->fdesc_host, 0));
    TRY(hipMalloc(&c->fdesc, sizeof(FrameArgs) * kLaunchSlots * kMaxBatch));
    TRY(hipMalloc(&c->order, OrderBlock::words((int)c->hmb) * sizeof(int32_t)));
    r = upload_orders(c, kOrderSlope);
    if (r != kSuccess) {
      free_ctx(c);
      return r;
    }
  }
  for (auto& s : c->st) {
    TRY(hipHostMalloc(&s.table, c->mbs * sizeof(BlockDesc), hipHostMallocMapped));
    TRY(hipHostMalloc(&s.coef, c->plane_elems * 2, hipHostMallocDefault));
    TRY(hipHostMalloc(&s.err, TimeoutInfo::kWords * sizeof(int32_t), hipHostMallocMapped));
    memset(s.err, 0, TimeoutInfo::kWords * sizeof(int32_t));
    TRY(hipHostGetDevicePointer((void**)&s.table_dev, s.table, 0));
    TRY(hipHostGetDevicePointer((void**)&s.err_dev, s.err, 0));
    TRY(hipEventCreateWithFlags(&s.d2h_done, hipEventDisableTiming));
    TRY(hipEventCreateWithFlags(&s.rgb_read, hipEventDisableTiming));
  }
  for (auto& t : c->tb)
    for (auto& e : t.ev) TRY(hipEventCreate(&e));
  TRY(hipEventCreateWithFlags(&c->engine_done, hipEventDisableTiming));
  TRY(hipEventCreate(&c->t_base));
  for (auto& ev : c->batch_end) TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : c->batch_ready) TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : c->pre_done) TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : c->fdesc_done) TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
#undef TRY
  r = zero_state(c);
  if (r != kSuccess) {
    free_ctx(c);
    return r;
  }
  *out = c;
  return kSuccess;
}

int cairo_ctx_destroy(cairo_ctx* c) {
  if (!c) return kInvalidArg;
  free_ctx(c);
  return kSuccess;
}

int cairo_ctx_reset(cairo_ctx* c) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = sync_all(c);
  if (r) return r;
  for (auto& s : c->st) s.busy = false;
  if (c->gsize > 1) {  // a reset leaves the group (its members reset and rejoin together)
    leave_group(c);
    r = upload_orders(c, kOrderSlope);
    if (r) return r;
  }
  return zero_state(c);
}

int cairo_ctx_stages(const cairo_ctx* c) { return c ? c->stages : 0; }

int cairo_default_batch(uint32_t width, uint32_t height) {
  if (!width || !height) return 0;
  return default_batch((size_t)((width + 15) / 16) * ((height + 15) / 16));
}

int cairo_task_order(int hmb, int frames, int32_t* out, int* slope) {
  if (hmb < 1 || hmb > 0xFFFF || frames < 1 || frames > kMaxBatch || !out) return kInvalidArg;
  const std::vector<int32_t> ord = task_order(hmb, kOrderSlope);
  memcpy(out, &ord[(size_t)(frames - 1) * kMaxBatch * hmb], (size_t)frames * hmb * sizeof(int32_t));
  if (slope) *slope = kOrderSlope;
  return kSuccess;
}

int cairo_task_queues(int hmb, int frames, int n_helpers, int n_rows, int pool, int32_t* order, int32_t* seg,
                      int* nlab) {
  if (hmb < 1 || hmb > 0xFFFF || frames < 1 || frames > kMaxBatch || !order || !seg || n_helpers < 1 || n_rows < 1 ||
      pool < 0 || pool > 1)
    return kInvalidArg;
  const std::vector<int32_t> blk = order_block(hmb, kOrderSlope);
  const int banded = banded_pool(hmb, n_helpers, n_rows, pool);
  memcpy(order, &blk[OrderBlock::order_at(hmb, banded, frames)], (size_t)frames * hmb * sizeof(int32_t));
  memcpy(seg, &blk[OrderBlock::seg_at(hmb, banded, frames)], (kLabels + 1) * sizeof(int32_t));
  if (nlab) *nlab = banded ? kLabels : 1;
  return kSuccess;
}

int cairo_ctx_set_batch(cairo_ctx* c, int frames) {
  if (!c || frames < 1 || frames > kMaxBatch || frames > c->stages / 2) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  int r = flush(c);
  if (r) return r;
  c->batch_max = frames;
  return kSuccess;
}

int cairo_ctx_set_workgroups(cairo_ctx* c, int rows) {
  // more row coders than stay co-resident with the other in-flight launch
  // would leave tasks to workgroups that never get a slot.  With the stamp
  // diagnostics on (set_debug(2), whose caller waits for each batch) one
  // launch may take every slot.
  if (!c || rows < 0 || rows > (c->stamps ? 2 : 1) * c->max_rows) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  c->wg_rows = rows;
  return kSuccess;
}

int cairo_ctx_set_helpers(cairo_ctx* c, int helpers) {
  if (!c || helpers < 0 || helpers >= 2 * (c->stamps ? 2 : 1) * c->max_rows) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  c->wg_helpers = helpers;
  return kSuccess;
}

int cairo_ctx_set_profiling(cairo_ctx* c, int enable) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  if (enable && !c->profiling) {
    int r = flush(c);
    if (r) return r;
    CK(hipEventRecord(c->t_base, c->ks));
  }
  c->profiling = enable != 0;
  return kSuccess;
}

int cairo_ctx_take_timings(cairo_ctx* c, double ms[4], int* frames) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = flush(c);
  if (r) return r;
  for (auto& t : c->tb) {
    r = collect_times(c, t);
    if (r) return r;
  }
  for (int k = 0; k < kTimed; k++) {
    if (ms) ms[k] = c->acc_ms[k];
    c->acc_ms[k] = 0;
  }
  if (ms) ms[kTimed] = union_length(c->busy);
  c->busy.clear();
  if (frames) *frames = c->acc_frames;
  c->acc_frames = 0;
  return kSuccess;
}

int cairo_ctx_busy_intervals(cairo_ctx* c, double* out, int cap, int* n) {
  if (!c || !n || cap < 0 || (cap && !out)) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  // read-only: the launches made so far (a pending partial batch stays pending)
  for (auto& t : c->tb) {
    const int r = collect_times(c, t);
    if (r) return r;
  }
  std::vector<std::pair<double, double>> iv = c->busy;
  std::sort(iv.begin(), iv.end());
  *n = (int)iv.size();
  for (int i = 0; i < cap && i < (int)iv.size(); i++) {
    out[2 * i] = iv[i].first;
    out[2 * i + 1] = iv[i].second;
  }
  return kSuccess;
}

int cairo_ctx_submit(cairo_ctx* c, const uint8_t* rgb, int rgb_on_device, uint32_t index,
                     uint32_t type, uint32_t quality, int* ticket) {
  if (!c || !rgb || !ticket || quality < 1 || quality > 31 || type > 1) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  const int t = c->next_ticket;
  const int slot = t % c->stages;
  Stage& s = c->st[slot];
  if (s.busy) {
    fprintf(stderr, "[cairo_amd] staging slot of ticket %d not released\n", s.ticket);
    return kInvalidResource;
  }
  if (rgb_on_device) {  // the kernels read it: it must be device memory of this context's GPU
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, rgb) != hipSuccess || pa.type != hipMemoryTypeDevice || pa.device != c->device) {
      (void)hipGetLastError();
      fprintf(stderr, "[cairo_amd] submit: rgb_on_device but %p is not device memory of device %d\n", (const void*)rgb,
              c->device);
      return kInvalidArg;
    }
  }
  FrameDesc& f = c->pend[c->npend];
  if (rgb_on_device) {
    f.rgb = rgb;
    f.host_rgb = nullptr;
  } else {  // the caller keeps it valid until wait
    f.rgb = c->rgb + (size_t)slot * c->w * c->h * 3;
    f.host_rgb = rgb;
    if (c->gsize == 1) {
      // Uploaded now, beside the launches in flight.  The staging buffer's
      // previous frame may still wait for its conversion (a caller may release
      // a ticket without waiting for it): the upload waits for the launch that
      // converts it (rgb_read).  With feed outputs only, the copy stream
      // carries nothing else once a context uploads (flush then keeps the feed
      // copies on the launch stream), so the uploads use it: on a stream of
      // their own they ran at 12.3 GB/s instead of 19.1 (bench.py host_rgb,
      // 4K; GPU_MAX_HW_QUEUES is 4 by default: a fifth stream shares a
      // hardware queue with one of the others).  With the coefficient planes' D2H
      // copies queued on the copy stream, they get a stream of their own.
      c->host_uploads = true;
      hipStream_t up = c->cs;
      if (c->outputs & CAIRO_OUT_COEF) {
        if (!c->us) CK(hipStreamCreateWithFlags(&c->us, hipStreamNonBlocking));
        up = c->us;
      }
      if (!c->up_last) CK(hipEventCreateWithFlags(&c->up_last, hipEventDisableTiming));
      if (s.rgb_pending) {
        CK(hipStreamWaitEvent(up, s.rgb_read, 0));
        s.rgb_pending = false;
      }
      CK(hipMemcpyAsync((void*)f.rgb, rgb, (size_t)c->w * c->h * 3, hipMemcpyHostToDevice, up));
      CK(hipEventRecord(c->up_last, up));
      c->up_pending = true;
      f.host_rgb = nullptr;
    }
  }
  if (c->gsize > 1 && (long)index != (long)(t - c->gbase) * c->gsize + c->grank) {
    fprintf(stderr, "[cairo_amd] group member %d of %d: frame %u out of turn\n", c->grank, c->gsize, index);
    return kInvalidArg;
  }
  f.index = (int)index;
  f.inter = type == 1 ? 1 : 0;
  f.quality = (int)quality;
  // granule tag; frames of a stream have consecutive epochs (a group numbers
  // them by stream index)
  f.epoch = c->gsize > 1 ? index + 1 : ++c->epoch;
  f.slot = slot;
  f.member = c->grank;
  f.decode = 0;  // decode_frame never leaves a decode frame pending
  f.host_table = nullptr;
  f.host_coef = nullptr;
  frame_links(c, f, t);
  c->npend++;
  s.busy = true;
  s.launched = false;
  s.ticket = t;
  s.index = index;
  s.type = type;
  s.quality = quality;
  c->next_ticket++;
  *ticket = t;
  if (c->npend >= c->batch_max) return flush(c);
  return kSuccess;
}

static const char* timeout_kind_name(int k) {
  switch (k) {
    case kWaitRecords: return "inter records (row coder)";
    case kWaitGranule: return "granule";
    case kWaitPrevProgress: return "previous frame's deblock progress (row helper)";
    case kWaitRowAbove: return "row above's deblock progress (deblock)";
    case kWaitBatch: return "batch completion";
    case kWaitInjected: return "injected (test hook)";
    case kWaitHostMark: return "marked by the host (test hook)";
    default: return "unknown";
  }
}

// A frame found the context's timeout words set: say on stderr which wait
// gave up first, and keep the words for cairo_ctx_timeout_info.
// w is a copy the host took without ordering between the words (a D2H copy,
// or k_feed_copy's relaxed reads in the mapped stage) while a launch may still
// have been writing the record.  The record's kind is stored last, with a
// system-scope release (report_timeout in kernels.hip), so once a read has
// seen the kind, every word of the record was visible before it: a second
// read of the device words, started now, returns the whole record.
// fs: a stream for that read (nullptr: the context's fetch stream, made under
// mu, which the caller must not hold).
static void report_timeout_host(cairo_ctx* c, const int32_t* seen, uint32_t index, hipStream_t fs = nullptr) {
  int32_t w[TimeoutInfo::kWords];
  memcpy(w, seen, sizeof(w));
  {
    if (!fs) {
      std::lock_guard<std::mutex> lk(c->mu);
      if (!c->fs) (void)hipStreamCreateWithFlags(&c->fs, hipStreamNonBlocking);
      fs = c->fs;
    }
    if (fs && hipMemcpyAsync(w, c->sticky, sizeof(w), hipMemcpyDeviceToHost, fs) == hipSuccess)
      (void)hipStreamSynchronize(fs);
    if (!w[TimeoutInfo::kKind]) memcpy(w, seen, sizeof(w));  // (a reset in between: keep what was seen)
  }
  {
    std::lock_guard<std::mutex> lk(c->tmu);
    memcpy(c->timeout, w, sizeof(c->timeout));
  }
  using T = TimeoutInfo;
  fprintf(stderr,
          "[cairo_amd] an in-kernel wait timed out (reported at frame %u): %s; member %d, frame index %d (epoch %u), "
          "MB row %d, waiting on %d (0x%x) for %d, last seen 0x%08x%08x\n",
          index, timeout_kind_name(w[T::kKind]), w[T::kMember], w[T::kIndex], (uint32_t)w[T::kEpoch], w[T::kRow],
          w[T::kOn], (uint32_t)w[T::kOn], w[T::kNeed], (uint32_t)w[T::kSeenHi], (uint32_t)w[T::kSeenLo]);
}

// Frame outputs once its D2H finished (called without mu held).  poll: wait
// with hipEventQuery + short sleeps instead of hipEventSynchronize -- a
// thread blocked in hipEventSynchronize on the copy stream's event stalls
// another thread enqueueing on that stream (the frame pipeline's completion
// thread vs. the submitting thread: measured 0.43 -> 0.8 ms per 720p frame).
static int frame_result(cairo_ctx* c, Stage& s, cairo_frame_result* out, bool poll = false) {
  CK(hipSetDevice(c->device));
  if (poll) {
    for (;;) {
      const hipError_t q = hipEventQuery(s.d2h_done);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) CK(q);
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  } else {
    CK(hipEventSynchronize(s.d2h_done));
  }
  if (s.err[TimeoutInfo::kKind]) {
    report_timeout_host(c, s.err, s.index);
    return kHardwareFail;
  }
  out->block_table = s.table;
  if (c->outputs & CAIRO_OUT_COEF) {
    out->coef_y = s.coef;
    out->coef_u = s.coef + (size_t)c->wa * c->ha;
    out->coef_v = out->coef_u + (size_t)(c->wa / 2) * (c->ha / 2);
  } else {
    out->coef_y = out->coef_u = out->coef_v = nullptr;
  }
  out->feed = nullptr;
  out->feed_bits = 0;
  out->feed_status = CAIRO_FEED_NONE;
  if (c->outputs & CAIRO_OUT_FEED) {
    const int slot = (int)(&s - c->st.data());
    const volatile uint32_t* h = c->feed_host + (size_t)slot * (kFeedHdrWords + c->feed_words);
    out->feed = (const uint32_t*)h + kFeedHdrWords;
    out->feed_bits = (uint64_t)h[0] | ((uint64_t)h[1] << 32);
    out->feed_status = h[2] ? CAIRO_FEED_OVERFLOW : CAIRO_FEED_VALID;
    if (!h[2] && h[3]) {  // k_feed_write's bounds guard dropped writes: the feed is not the frame's
      fprintf(stderr, "[cairo_amd] frame %u: the precode writer found %u writes outside the frame's feed\n",
              s.index, (uint32_t)h[3]);
      return kHardwareFail;
    }
  }
  out->wa = c->wa;
  out->ha = c->ha;
  out->wmb = c->wmb;
  out->hmb = c->hmb;
  out->index = s.index;
  out->type = s.type;
  out->quality = s.quality;
  return kSuccess;
}

int cairo_ctx_wait(cairo_ctx* c, int ticket, cairo_frame_result* out) {
  if (!c || !out || ticket < 0) return kInvalidArg;
  Stage& s = c->st[ticket % c->stages];
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (!s.busy || s.ticket != ticket) return kInvalidResource;
    CK(hipSetDevice(c->device));
    if (!s.launched) {
      int r = flush(c);
      if (r) return r;
    }
  }
  return frame_result(c, s, out);
}

int cairo_ctx_decode_frame(cairo_ctx* c, const uint8_t* table, const int16_t* coef, uint32_t index,
                           uint8_t* rgb) {
  if (!c || !table || !coef || !rgb) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->gsize > 1) return kInvalidResource;
  CK(hipSetDevice(c->device));
  int r = flush(c);  // encode frames still pending go first, in their own launch
  if (r) return r;
  const int t = c->next_ticket, slot = t % c->stages;
  Stage& s = c->st[slot];
  if (s.busy) {
    fprintf(stderr, "[cairo_amd] staging slot of ticket %d not released\n", s.ticket);
    return kInvalidResource;
  }
  FrameDesc& f = c->pend[0];
  memset(&f, 0, sizeof(f));
  f.index = (int)index;
  f.inter = 1;
  f.quality = 1;
  f.epoch = ++c->epoch;
  f.slot = slot;
  f.decode = 1;
  frame_links(c, f, t);
  f.host_table = reinterpret_cast<const BlockDesc*>(table);
  f.host_coef = coef;
  c->npend = 1;
  s.busy = true;
  s.launched = false;
  s.ticket = t;
  s.index = index;
  s.type = 1;
  s.quality = 0;
  c->next_ticket++;
  const long long b = c->batches;  // the launch flush() is about to make
  r = flush(c);
  if (r == kSuccess) {
    hipStream_t st = (b & 1) ? c->ks2 : c->ks;
    uint8_t* drgb = c->rgb + (size_t)slot * c->w * c->h * 3;
    r = fail(launch_yuv_to_rgb(slot_planes(c->ring_buf, c, (int)(index % c->ring)), (int)c->wa, (int)c->w,
                               (int)c->h, drgb, st), "launch_yuv_to_rgb");
    if (r == kSuccess)
      r = fail(hipMemcpyAsync(s.err, c->sticky, TimeoutInfo::kWords * sizeof(int32_t), hipMemcpyDeviceToHost, st),
               "hipMemcpyAsync");
    if (r == kSuccess)
      r = fail(hipMemcpyAsync(rgb, drgb, (size_t)c->w * c->h * 3, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    if (r == kSuccess) r = fail(hipStreamSynchronize(st), "hipStreamSynchronize");
    if (r == kSuccess && s.err[TimeoutInfo::kKind]) {
      report_timeout_host(c, s.err, index, st);  // (mu held: the launch stream, idle now)
      r = kHardwareFail;
    }
  }
  s.busy = false;
  return r;
}

int cairo_ctx_max_workgroups(const cairo_ctx* c) { return c ? c->max_rows : 0; }

int cairo_ctx_timeout_info(cairo_ctx* c, int32_t* out, int n) {
  if (!c || !out || n < 0 || n > TimeoutInfo::kWords) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->tmu);
  memcpy(out, c->timeout, (size_t)n * sizeof(int32_t));
  return kSuccess;
}

int cairo_ctx_set_outputs(cairo_ctx* c, int outputs) {
  if (!c || outputs < 1 || outputs > (CAIRO_OUT_COEF | CAIRO_OUT_FEED)) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = sync_all(c);  // frames in flight keep the outputs they were launched with
  if (r) return r;
  for (const Stage& s : c->st)
    if (s.busy) return kInvalidResource;
  if ((outputs & CAIRO_OUT_FEED) && !c->feed_host) {
    // all or nothing: a partial allocation would leave feed_dev set with no
    // host buffer for the precode to write into
    const size_t S = (size_t)c->stages;
    const size_t words = feed_words_per_slot(c->mbs);
    uint32_t *dev = nullptr, *hdr = nullptr, *scratch = nullptr, *host = nullptr;
    hipError_t e = hipMalloc(&dev, words * 4 * S);
    if (e == hipSuccess) e = hipMalloc(&hdr, kFeedHdrWords * 4 * S);
    if (e == hipSuccess) e = hipMalloc(&scratch, feed_scratch_words(c->mbs) * 4 * S);
    if (e == hipSuccess) e = hipHostMalloc(&host, (kFeedHdrWords + words) * 4 * S, hipHostMallocMapped);
    if (e != hipSuccess) {
      for (void* q : {(void*)dev, (void*)hdr, (void*)scratch}) (void)hipFree(q);
      if (host) (void)hipHostFree(host);
      return fail(e, "set_outputs: feed buffers");
    }
    c->feed_words = words;
    c->feed_dev = dev, c->feed_hdr = hdr, c->feed_scratch = scratch, c->feed_host = host;
  }
  c->outputs = outputs;
  return kSuccess;
}

int cairo_ctx_fetch_coef(cairo_ctx* c, int ticket, cairo_frame_result* out) {
  if (!c || !out || ticket < 0) return kInvalidArg;
  Stage& s = c->st[ticket % c->stages];
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (!s.busy || s.ticket != ticket || !s.launched) return kInvalidResource;
  }
  CK(hipSetDevice(c->device));
  CK(hipEventSynchronize(s.d2h_done));  // the frame's engine launch has finished
  const int slot = ticket % c->stages;
  if (!(c->outputs & CAIRO_OUT_COEF)) {  // still in the staging slot until its release
    {
      std::lock_guard<std::mutex> lk(c->mu);
      if (!c->fs) CK(hipStreamCreateWithFlags(&c->fs, hipStreamNonBlocking));  // rare: made on first use
    }
    CK(hipMemcpyAsync(s.coef, coef_base(c, slot), c->plane_elems * 2, hipMemcpyDeviceToHost, c->fs));
    CK(hipStreamSynchronize(c->fs));
  }
  out->coef_y = s.coef;
  out->coef_u = s.coef + (size_t)c->wa * c->ha;
  out->coef_v = out->coef_u + (size_t)(c->wa / 2) * (c->ha / 2);
  return kSuccess;
}

int cairo_ctx_flush(cairo_ctx* c) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  return flush(c);
}

int cairo_ctx_peer_info(cairo_ctx* c, int cross_device, cairo_peer* out) {
  if (!c || !out) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->fresh || c->npend || c->gsize > 1) return kInvalidResource;  // before any frame, outside a group
  CK(hipSetDevice(c->device));
  if (cross_device && !c->fine_grained) {
    // Memory another device reads while this one writes it: fine-grained, so
    // that system-scope releases and acquires order it across devices.
    const size_t S = (size_t)c->stages;
    int16_t* ring = nullptr;
    int16_t* coef[CAIRO_MAX_COEF_CHUNKS] = {};
    int chunks = 0, per = 0;
    uint64_t* prog = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&ring, c->plane_elems * 2 * kMirrorSlots, hipDeviceMallocFinegrained);
    if (e == hipSuccess) e = alloc_coef(c, true, coef, &chunks, &per);
    if (e == hipSuccess)
      e = hipExtMallocWithFlags((void**)&prog, (size_t)c->hmb * sizeof(uint64_t) * S, hipDeviceMallocFinegrained);
    if (e != hipSuccess) {
      for (void* q : {(void*)ring, (void*)prog}) (void)hipFree(q);
      for (int16_t* q : coef)
        if (q) (void)hipFree(q);
      return fail(e, "hipExtMallocWithFlags(fine-grained)");
    }
    int r0 = sync_all(c);  // nothing is in flight (fresh), but the zeroing memsets may be
    if (r0) return r0;
    (void)hipFree(c->ring_buf);
    for (int16_t*& q : c->coef) {
      if (q) (void)hipFree(q);
      q = nullptr;
    }
    (void)hipFree(c->progress);
    c->ring_buf = ring, c->progress = prog;
    c->ring_slots = kMirrorSlots;
    for (int k = 0; k < CAIRO_MAX_COEF_CHUNKS; k++) c->coef[k] = coef[k];
    c->coef_chunks = chunks, c->coef_per = per;
    c->fine_grained = true;
    int r = zero_state(c);
    if (r) return r;
  }
  memset(out, 0, sizeof(*out));
  out->width = c->w, out->height = c->h, out->ring = c->ring;
  out->device = c->device;
  out->pid = (int32_t)getpid();
  out->stages = c->stages;
  out->fine_grained = c->fine_grained;
  out->coef_chunks = c->coef_chunks;
  out->coef_chunk_slots = c->coef_per;
  out->ring_addr = (uint64_t)(uintptr_t)c->ring_buf;
  out->progress_addr = (uint64_t)(uintptr_t)c->progress;
  hipIpcMemHandle_t h;
  static_assert(sizeof(h) == sizeof(out->ipc_ring), "IPC handle size");
  CK(hipIpcGetMemHandle(&h, c->ring_buf));
  memcpy(out->ipc_ring, &h, sizeof(h));
  CK(hipIpcGetMemHandle(&h, c->progress));
  memcpy(out->ipc_progress, &h, sizeof(h));
  for (int k = 0; k < c->coef_chunks; k++) {
    out->coef_addr[k] = (uint64_t)(uintptr_t)c->coef[k];
    CK(hipIpcGetMemHandle(&h, c->coef[k]));
    memcpy(out->ipc_coef[k], &h, sizeof(h));
  }
  return kSuccess;
}

int cairo_peer_size(void) { return (int)sizeof(cairo_peer); }

// GPU_MAX_HW_QUEUES as the HIP runtime reads it: once, when it starts.  Read
// here when the library is loaded (before any HIP call of ours); setting it
// later in the process (os.environ after torch started HIP) changes nothing.
static const int g_hw_queues = [] {
  const char* env = getenv("GPU_MAX_HW_QUEUES");
  return env && *env ? atoi(env) : 4;
}();

int cairo_group_check_queues(int local_members, int hw_queues) {
  // Members in one process on one device share that process's hardware
  // queues (GPU_MAX_HW_QUEUES, HIP's default 4).  Each member keeps two launch
  // streams and a copy stream busy; when two members' persistent launches
  // land in one in-order queue, the later cannot start until the earlier
  // ends, which waits on it: a deadlock the bounded in-kernel waits would
  // only report as EVX_ERROR_HARDWAREFAIL after 2 s.  Refuse up front.
  if (local_members < 2) return kSuccess;
  const int have = hw_queues >= 0 ? hw_queues : g_hw_queues;
  const int need = 3 * local_members + 2;
  if (need > 32 || have < need) {
    fprintf(stderr,
            "[cairo_amd] join_group: %d members share this process and device; they need GPU_MAX_HW_QUEUES >= %d "
            "(have %d, at most 32); run one process per member, or set GPU_MAX_HW_QUEUES before the first HIP call\n",
            local_members, need, have);
    return kInvalidArg;
  }
  return kSuccess;
}

int cairo_ctx_join_group(cairo_ctx* c, int size, int rank, const cairo_peer* peers) {
  if (!c || !peers || size < 1 || size > kMaxGroup || rank < 0 || rank >= size) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->fresh || c->npend || c->gsize > 1) return kInvalidResource;
  CK(hipSetDevice(c->device));
  if (size == 1) return kSuccess;
  const pid_t me = getpid();
  bool sys = false;
  int local = 0;  // members in this process on this device, this one included
  for (int i = 0; i < size; i++) {
    const cairo_peer& p = peers[i];
    if (p.width != c->w || p.height != c->h || p.ring != c->ring || p.stages < 2) return kInvalidArg;
    if (i == rank || (p.pid == me && p.device == c->device)) local++;
    if (i == rank) continue;
    if (p.pid != me || p.device != c->device) sys = true;
    if (p.device != c->device || p.pid != me) {
      if (!p.fine_grained || !c->fine_grained) {
        fprintf(stderr, "[cairo_amd] group members on other devices or processes need cairo_ctx_peer_info(..., 1)\n");
        return kInvalidArg;
      }
    }
  }
  if (cairo_group_check_queues(local, -1) != kSuccess) return kInvalidArg;
  for (int i = 0; i < size; i++) {
    cairo_ctx::Peer& q = c->gp[i];
    const cairo_peer& p = peers[i];
    q.stages = p.stages;
    if (i == rank) {
      q.ring = c->ring_buf, q.progress = c->progress;
      for (int k = 0; k < CAIRO_MAX_COEF_CHUNKS; k++) q.coef[k] = c->coef[k];
      q.coef_chunks = c->coef_chunks, q.coef_per = c->coef_per;
      continue;
    }
    if (p.coef_chunks < 1 || p.coef_chunks > CAIRO_MAX_COEF_CHUNKS || p.coef_chunk_slots < 1 ||
        (long)p.coef_chunks * p.coef_chunk_slots < p.stages) {
      c->gsize = i;
      leave_group(c);
      return kInvalidArg;
    }
    q.coef_chunks = p.coef_chunks, q.coef_per = p.coef_chunk_slots;
    if (p.pid == me) {  // same process: the addresses are valid here
      if (p.device != c->device) {
        const hipError_t e = hipDeviceEnablePeerAccess(p.device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          c->gsize = i;
          leave_group(c);
          return fail(e, "hipDeviceEnablePeerAccess");
        }
      }
      q.ring = (int16_t*)(uintptr_t)p.ring_addr;
      q.progress = (uint64_t*)(uintptr_t)p.progress_addr;
      for (int k = 0; k < p.coef_chunks; k++) q.coef[k] = (int16_t*)(uintptr_t)p.coef_addr[k];
    } else {  // another process: open its IPC handles (peer access over xGMI), each allocation < 1 GiB
      q.imported = true;  // leave_group closes whatever is open
      auto open = [&](const uint8_t* bytes, void** dst) {
        hipIpcMemHandle_t h;
        memcpy(&h, bytes, sizeof(h));
        return hipIpcOpenMemHandle(dst, h, hipIpcMemLazyEnablePeerAccess);
      };
      hipError_t e = open(p.ipc_ring, (void**)&q.ring);
      if (e == hipSuccess) e = open(p.ipc_progress, (void**)&q.progress);
      for (int k = 0; e == hipSuccess && k < p.coef_chunks; k++) e = open(p.ipc_coef[k], (void**)&q.coef[k]);
      if (e != hipSuccess) {
        c->gsize = i + 1;
        leave_group(c);
        return fail(e, "hipIpcOpenMemHandle");
      }
    }
  }
  c->gsize = size;
  c->grank = rank;
  c->gbase = c->next_ticket;
  // (CAIRO_GROUP_FORCE_SYS: system-scope hand-offs in one process too, to
  // time their cost on one device)
  c->sys = sys || getenv("CAIRO_GROUP_FORCE_SYS") != nullptr;
  CK(hipMalloc(&c->zero, c->plane_elems * 2));
  CK(hipMemset(c->zero, 0, c->plane_elems * 2));
  // a member's consecutive frames are N stream frames apart
  return upload_orders(c, 3 * size + 2);
}

int cairo_ctx_release(cairo_ctx* c, int ticket) {
  if (!c || ticket < 0) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  Stage& s = c->st[ticket % c->stages];
  if (s.ticket != ticket) return kInvalidResource;
  s.busy = false;
  return kSuccess;
}

int cairo_ctx_sync(cairo_ctx* c) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  return sync_all(c);
}

int cairo_ctx_read_planes(cairo_ctx* c, int which, int16_t* y, int16_t* u, int16_t* v) {
  if (!c || which < 0 || which >= 2 + c->ring_slots) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = sync_all(c);
  if (r) return r;
  if (which < 2 && c->last_slot < 0) return kInvalidResource;
  PlaneSet p = which == 0 ? slot_planes(c->src, c, c->last_slot)
               : which == 1 ? coef_planes(c, c->last_slot)
                            : slot_planes(c->ring_buf, c, which - 2);
  const size_t ly = (size_t)c->wa * c->ha, lc = ly / 4;
  if (y) CK(hipMemcpy(y, p.y, ly * 2, hipMemcpyDeviceToHost));
  if (u) CK(hipMemcpy(u, p.u, lc * 2, hipMemcpyDeviceToHost));
  if (v) CK(hipMemcpy(v, p.v, lc * 2, hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_ctx_read_inter(cairo_ctx* c, uint8_t* descs, int32_t* sads) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = sync_all(c);
  if (r) return r;
  if (c->last_slot < 0) return kInvalidResource;
  const size_t n = c->mbs * (c->ring > 1 ? c->ring - 1 : 0);
  if (!n) return kSuccess;
  const size_t o = (size_t)c->last_slot * c->nref * c->mbs;
  // two tagged granules per record (kernels.h pack_inter_desc); a record
  // whose tag is not the last frame's epoch is stale (an intra or decoded
  // frame has none): refused, not returned as current
  std::vector<uint64_t> g(2 * n);
  CK(hipMemcpy(g.data(), c->idesc + o, n * sizeof(BlockDesc), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < 2 * n; i++)
    if ((uint32_t)(g[i] >> 32) != c->last_epoch) return kInvalidResource;
  for (size_t i = 0; i < n; i++) {
    if (descs) {
      const BlockDesc d = unpack_inter_desc((uint32_t)g[2 * i]);
      memcpy(descs + i * sizeof(BlockDesc), &d, sizeof(d));
    }
    if (sads) sads[i] = (int32_t)(uint32_t)g[2 * i + 1];
  }
  return kSuccess;
}

int cairo_ctx_set_debug(cairo_ctx* c, int flags) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = flush(c);
  if (r) return r;
  if ((flags & 1) && !c->predeblock) CK(hipMalloc(&c->predeblock, c->plane_elems * 2));
  if ((flags & 2) && !c->stamps) CK(hipMalloc(&c->stamps, stamp_words(c) * sizeof(uint64_t)));
  if ((flags & 4) && !c->trace_host) {
    CK(hipHostMalloc(&c->trace_host, 4096 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->trace_host, 0xFF, 4096 * sizeof(int32_t));
    CK(hipHostGetDevicePointer((void**)&c->trace_dev, c->trace_host, 0));
  }
  if (flags & 8) {
    int32_t mark[TimeoutInfo::kWords] = {};  // a complete, claimed record
    mark[TimeoutInfo::kKind] = kWaitHostMark;
    mark[TimeoutInfo::kClaim] = 1;
    CK(hipMemcpy(c->sticky, mark, sizeof(mark), hipMemcpyHostToDevice));
  }
  c->inject = (flags & 16) ? 1 : 0;
  if ((flags & 32) && !c->acct) {
    CK(hipMalloc(&c->acct, kAcctShards * kAcctWords * sizeof(uint64_t)));
    CK(hipMemset(c->acct, 0, kAcctShards * kAcctWords * sizeof(uint64_t)));
  }
  return kSuccess;
}

int cairo_ctx_read_acct(cairo_ctx* c, uint64_t* out, int n, int reset) {
  if (!c || !out || n < 0 || n > kAcctWords) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  memset(out, 0, (size_t)n * sizeof(uint64_t));
  if (!c->acct) return kSuccess;
  CK(hipSetDevice(c->device));
  int r = sync_all(c);
  if (r) return r;
  std::vector<uint64_t> v((size_t)kAcctShards * kAcctWords);
  CK(hipMemcpy(v.data(), c->acct, v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  for (int s = 0; s < kAcctShards; s++)
    for (int k = 0; k < n; k++) out[k] += v[(size_t)s * kAcctWords + k];
  if (reset) CK(hipMemset(c->acct, 0, v.size() * sizeof(uint64_t)));
  return kSuccess;
}

// Diagnostic: the live trace words (no synchronization; readable while the engine runs).
int cairo_ctx_read_trace(cairo_ctx* c, int32_t* out, int n) {
  if (!c || !c->trace_host || !out || n < 0 || n > 4096) return kInvalidArg;
  memcpy(out, (const void*)c->trace_host, n * sizeof(int32_t));
  return kSuccess;
}

int cairo_ctx_read_stamps(cairo_ctx* c, uint64_t* out) {
  if (!c || !c->stamps || !out) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = sync_all(c);
  if (r) return r;
  CK(hipMemcpy(out, c->stamps, stamp_words(c) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_ctx_read_predeblock(cairo_ctx* c, int16_t* y, int16_t* u, int16_t* v) {
  if (!c || !c->predeblock) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = sync_all(c);
  if (r) return r;
  PlaneSet p = planes_at(c->predeblock, c);
  const size_t ly = (size_t)c->wa * c->ha, lc = ly / 4;
  if (y) CK(hipMemcpy(y, p.y, ly * 2, hipMemcpyDeviceToHost));
  if (u) CK(hipMemcpy(u, p.u, lc * 2, hipMemcpyDeviceToHost));
  if (v) CK(hipMemcpy(v, p.v, lc * 2, hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_ctx_read_table(cairo_ctx* c, uint8_t* table) {
  if (!c || !table) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  CK(hipSetDevice(c->device));
  int r = sync_all(c);
  if (r) return r;
  if (c->last_slot < 0) return kInvalidResource;
  CK(hipMemcpy(table, c->table + (size_t)c->last_slot * c->mbs, c->mbs * sizeof(BlockDesc),
               hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_kat_transform(const int16_t* src, const int16_t* pred, const uint8_t* qtype, int count,
                        int16_t* coef, int16_t* recon, int32_t* qvar, int device) {
  if (!src || !pred || !qtype || !coef || !recon || !qvar || count <= 0) return kInvalidArg;
  CK(hipSetDevice(device));
  const size_t n = (size_t)count * 384;
  int16_t *ds = nullptr, *dp = nullptr, *dc = nullptr, *dr = nullptr;
  uint8_t* dq = nullptr;
  int32_t* dv = nullptr;
  int r = kSuccess;
  if ((r = fail(hipMalloc(&ds, n * 2), "malloc")) || (r = fail(hipMalloc(&dp, n * 2), "malloc")) ||
      (r = fail(hipMalloc(&dc, n * 2), "malloc")) || (r = fail(hipMalloc(&dr, n * 2), "malloc")) ||
      (r = fail(hipMalloc(&dq, (size_t)count * 2), "malloc")) ||
      (r = fail(hipMalloc(&dv, (size_t)count * 8), "malloc")))
    goto done;
  if ((r = fail(hipMemcpy(ds, src, n * 2, hipMemcpyHostToDevice), "h2d")) ||
      (r = fail(hipMemcpy(dp, pred, n * 2, hipMemcpyHostToDevice), "h2d")) ||
      (r = fail(hipMemcpy(dq, qtype, (size_t)count * 2, hipMemcpyHostToDevice), "h2d")))
    goto done;
  if ((r = fail(launch_kat_transform(ds, dp, dc, dr, dq, dv, count, nullptr), "kat")) ||
      (r = fail(hipDeviceSynchronize(), "sync")))
    goto done;
  if ((r = fail(hipMemcpy(coef, dc, n * 2, hipMemcpyDeviceToHost), "d2h")) ||
      (r = fail(hipMemcpy(recon, dr, n * 2, hipMemcpyDeviceToHost), "d2h")) ||
      (r = fail(hipMemcpy(qvar, dv, (size_t)count * 8, hipMemcpyDeviceToHost), "d2h")))
    goto done;
done:
  (void)hipFree(ds);
  (void)hipFree(dp);
  (void)hipFree(dc);
  (void)hipFree(dr);
  (void)hipFree(dq);
  (void)hipFree(dv);
  return r;
}

int cairo_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* cairo_version(void) { return "cairo_amd 0.1 (gfx950)"; }
int cairo_api_version(void) { return CAIRO_AMD_API_VERSION; }

}  // extern "C"

namespace cairo {

int ctx_wait_launched(cairo_ctx* c, int ticket, const std::atomic<bool>* stop,
                      cairo_frame_result* out) {
  if (!c || !out || ticket < 0) return kInvalidArg;
  Stage& s = c->st[ticket % c->stages];
  {
    std::unique_lock<std::mutex> lk(c->mu);
    if (!s.busy || s.ticket != ticket) return kInvalidResource;
    c->launched_cv.wait(lk, [&] { return s.launched || (stop && stop->load()); });
    if (!s.launched) return kInvalidResource;
  }
  return frame_result(c, s, out, true);
}

int ctx_flush(cairo_ctx* c, int ticket) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  if (ticket >= 0) {  // only if that frame is still in the pending batch
    const Stage& s = c->st[ticket % c->stages];
    if (!s.busy || s.ticket != ticket || s.launched) return kSuccess;
  }
  CK(hipSetDevice(c->device));
  return flush(c);
}

void ctx_wake(cairo_ctx* c) {
  std::lock_guard<std::mutex> lk(c->mu);
  c->launched_cv.notify_all();
}

int ctx_geometry(cairo_ctx* c, uint32_t* wmb, uint32_t* hmb, uint32_t* ring, int* next_ticket) {
  if (!c) return kInvalidArg;
  std::lock_guard<std::mutex> lk(c->mu);
  *next_ticket = c->next_ticket;
  *wmb = c->wmb;
  *hmb = c->hmb;
  *ring = c->ring;
  return kSuccess;
}

}  // namespace cairo
