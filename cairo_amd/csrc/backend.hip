// cairo_amd/csrc/backend.hip -- device context and frame orchestration.
//
// One context = one encoder's device state in HBM (see DESIGN.md "Data layout"):
//   input_cache   planes (convert output, read by both searches)
//   output_cache  planes (quantized coefficients, persistent across frames)
//   ring          R contiguous plane sets (reconstruction slots)
//   table, inter  block table and per-(MB, ref) inter-search records
//   sync          wavefront progress words, zeroed per frame
// Per frame, on the kernels' stream:
//   [H2D rgb] -> memset(sync) -> K0 convert -> K1 inter -> K2 rows (+ deblock)
// and on the copy stream, after K2: D2H of table + coefficients into a
// pinned staging slot (the host entropy stage reads those while the GPU runs
// the next frames).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <new>

#include "../../include/cairo_amd.h"
#include "kernels.h"

using namespace cairo;

namespace {

constexpr int kStages = 8;
constexpr int kSuccess = 0, kInvalidArg = 1, kOutOfMemory = 3, kHardwareFail = 5,
              kInvalidResource = 8;

constexpr int kTimed = 3;  // timed kernels: convert, inter search, mb rows (+deblock)

struct Stage {
  uint8_t* table = nullptr;  // pinned
  int16_t* coef = nullptr;   // pinned, 1.5 * wa * ha
  int32_t* err = nullptr;    // pinned, 1 word
  hipEvent_t k2_done = nullptr, d2h_done = nullptr;
  hipEvent_t ev[kTimed + 1] = {};  // kernel boundaries of this frame (profiling)
  bool timed = false;     // ev[] recorded, not yet collected
  int ticket = -1;
  bool busy = false;
  uint32_t index = 0, type = 0, quality = 0;
};

}  // namespace

struct cairo_ctx {
  int device = 0;
  uint32_t w = 0, h = 0, wa = 0, ha = 0, wmb = 0, hmb = 0, ring = 0;
  size_t plane_elems = 0;  // Y + U + V of one plane set
  hipStream_t ks = nullptr, cs = nullptr;
  int16_t *in = nullptr, *coef = nullptr, *ring_buf = nullptr;
  BlockDesc *table = nullptr, *inter_desc = nullptr;
  int32_t *inter_sad = nullptr, *sync = nullptr, *sticky = nullptr;
  uint8_t* rgb = nullptr;
  size_t sync_words = 0;
  Stage st[kStages];
  int next_ticket = 0;
  int wg_rows = 0;
  bool profiling = false;
  double acc_ms[kTimed] = {0, 0, 0};
  int acc_frames = 0;
  bool have_inter = false;
  int16_t* predeblock = nullptr;  // debug snapshot of the slot after K2 (opt-in)
  uint64_t* stamps = nullptr;     // diagnostic K2 phase stamps (opt-in)
  uint64_t* granules = nullptr;   // K2 macroblock hand-off granules
  uint32_t epoch = 0;             // granule tag of the last submitted frame
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
  PlaneSet p;
  p.y = base;
  p.u = base + (size_t)c->wa * c->ha;
  p.v = p.u + (size_t)(c->wa / 2) * (c->ha / 2);
  return p;
}

FrameArgs frame_args(const cairo_ctx* c, uint32_t index, uint32_t type, uint32_t quality) {
  FrameArgs a;
  memset(&a, 0, sizeof(a));
  a.wa = (int)c->wa;
  a.ha = (int)c->ha;
  a.w = (int)c->w;
  a.h = (int)c->h;
  a.wmb = (int)c->wmb;
  a.hmb = (int)c->hmb;
  a.ring = (int)c->ring;
  a.index = (int)index;
  a.inter = type == 1 ? 1 : 0;
  a.quality = (int)quality;
  a.rgb = c->rgb;
  a.in = planes_at(c->in, c);
  a.coef = planes_at(c->coef, c);
  a.ring_base = c->ring_buf;
  a.slot_elems = c->plane_elems;
  a.table = c->table;
  a.inter_desc = c->inter_desc;
  a.inter_sad = c->inter_sad;
  a.sync = c->sync;
  a.sticky = c->sticky;
  a.stamps = c->stamps;
  a.granules = c->granules;
  return a;
}

void free_ctx(cairo_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->ks) (void)hipStreamSynchronize(c->ks);
  if (c->cs) (void)hipStreamSynchronize(c->cs);
  for (auto& s : c->st) {
    if (s.table) (void)hipHostFree(s.table);
    if (s.coef) (void)hipHostFree(s.coef);
    if (s.err) (void)hipHostFree(s.err);
    if (s.k2_done) (void)hipEventDestroy(s.k2_done);
    if (s.d2h_done) (void)hipEventDestroy(s.d2h_done);
    for (auto& e : s.ev)
      if (e) (void)hipEventDestroy(e);
  }
  (void)hipFree(c->in);
  (void)hipFree(c->coef);
  (void)hipFree(c->ring_buf);
  (void)hipFree(c->table);
  (void)hipFree(c->inter_desc);
  (void)hipFree(c->inter_sad);
  (void)hipFree(c->sync);
  (void)hipFree(c->sticky);
  (void)hipFree(c->rgb);
  (void)hipFree(c->predeblock);
  (void)hipFree(c->stamps);
  (void)hipFree(c->granules);
  if (c->ks) (void)hipStreamDestroy(c->ks);
  if (c->cs) (void)hipStreamDestroy(c->cs);
  delete c;
}

size_t stamp_words(const cairo_ctx* c) {
  return (size_t)c->wmb * c->hmb * kStampPhases + (size_t)c->hmb * kDbStamps + 2;
}

int zero_state(cairo_ctx* c) {
  CK(hipMemsetAsync(c->in, 0, c->plane_elems * 2, c->ks));
  CK(hipMemsetAsync(c->coef, 0, c->plane_elems * 2, c->ks));
  CK(hipMemsetAsync(c->ring_buf, 0, c->plane_elems * 2 * c->ring, c->ks));
  CK(hipMemsetAsync(c->table, 0, (size_t)c->wmb * c->hmb * sizeof(BlockDesc), c->ks));
  // granule tags start at 0; the n-th submission after a reset publishes tag n.
  CK(hipMemsetAsync(c->granules, 0, (size_t)c->wmb * c->hmb * kGranulesPerMB * sizeof(uint64_t),
                    c->ks));
  CK(hipStreamSynchronize(c->ks));
  c->epoch = 0;
  return kSuccess;
}

}  // namespace

extern "C" {

int cairo_ctx_create(uint32_t width, uint32_t height, uint32_t ring, int device, cairo_ctx** out) {
  // The reference indexes blocks with uint16 (deblock.cpp, serialize.cpp): at
  // most 65535 macroblocks per frame.
  if (!out || width == 0 || height == 0 || (width & 1) || (height & 1) || ring < 1 ||
      ring > (uint32_t)kMaxRing || ((width + 15) / 16) * ((height + 15) / 16) > 65535u)
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
  const size_t mbs = (size_t)c->wmb * c->hmb;
  const size_t nref = ring > 1 ? ring - 1 : 1;
  c->sync_words = (size_t)SyncLayout::words((int)c->hmb);
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
  TRY(hipStreamCreateWithFlags(&c->ks, hipStreamNonBlocking));
  TRY(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
  TRY(hipMalloc(&c->in, c->plane_elems * 2));
  TRY(hipMalloc(&c->coef, c->plane_elems * 2));
  TRY(hipMalloc(&c->ring_buf, c->plane_elems * 2 * ring));
  TRY(hipMalloc(&c->table, mbs * sizeof(BlockDesc)));
  TRY(hipMalloc(&c->inter_desc, nref * mbs * sizeof(BlockDesc)));
  TRY(hipMalloc(&c->inter_sad, nref * mbs * sizeof(int32_t)));
  TRY(hipMalloc(&c->sync, c->sync_words * sizeof(int32_t)));
  TRY(hipMalloc(&c->sticky, sizeof(int32_t)));
  TRY(hipMalloc(&c->granules, mbs * kGranulesPerMB * sizeof(uint64_t)));
  TRY(hipMemset(c->sticky, 0, sizeof(int32_t)));
  TRY(hipMalloc(&c->rgb, (size_t)width * height * 3));
  for (auto& s : c->st) {
    TRY(hipHostMalloc(&s.table, mbs * sizeof(BlockDesc), hipHostMallocDefault));
    TRY(hipHostMalloc(&s.coef, c->plane_elems * 2, hipHostMallocDefault));
    TRY(hipHostMalloc(&s.err, sizeof(int32_t), hipHostMallocDefault));
    TRY(hipEventCreateWithFlags(&s.k2_done, hipEventDisableTiming));
    TRY(hipEventCreateWithFlags(&s.d2h_done, hipEventDisableTiming));
    for (auto& e : s.ev) TRY(hipEventCreate(&e));
  }
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
  CK(hipSetDevice(c->device));
  CK(hipStreamSynchronize(c->cs));
  for (auto& s : c->st) s.busy = false;
  return zero_state(c);
}

int cairo_ctx_stages(const cairo_ctx*) { return kStages; }

int cairo_ctx_set_workgroups(cairo_ctx* c, int rows) {
  if (!c) return kInvalidArg;
  c->wg_rows = rows;
  return kSuccess;
}

int cairo_ctx_set_profiling(cairo_ctx* c, int enable) {
  if (!c) return kInvalidArg;
  c->profiling = enable != 0;
  return kSuccess;
}

static int collect_times(cairo_ctx* c, Stage& s) {
  if (!s.timed) return kSuccess;
  CK(hipEventSynchronize(s.ev[kTimed]));
  for (int k = 0; k < kTimed; k++) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, s.ev[k], s.ev[k + 1]));
    c->acc_ms[k] += ms;
  }
  c->acc_frames++;
  s.timed = false;
  return kSuccess;
}

int cairo_ctx_take_timings(cairo_ctx* c, double ms[3], int* frames) {
  if (!c) return kInvalidArg;
  CK(hipSetDevice(c->device));
  for (auto& s : c->st) {
    int r = collect_times(c, s);
    if (r) return r;
  }
  for (int k = 0; k < kTimed; k++) {
    if (ms) ms[k] = c->acc_ms[k];
    c->acc_ms[k] = 0;
  }
  if (frames) *frames = c->acc_frames;
  c->acc_frames = 0;
  return kSuccess;
}

int cairo_ctx_submit(cairo_ctx* c, const uint8_t* rgb, int rgb_on_device, uint32_t index,
                     uint32_t type, uint32_t quality, int* ticket) {
  if (!c || !rgb || quality < 1 || quality > 31 || type > 1) return kInvalidArg;
  CK(hipSetDevice(c->device));
  const int t = c->next_ticket;
  Stage& s = c->st[t % kStages];
  if (s.busy) {
    fprintf(stderr, "[cairo_amd] staging slot of ticket %d not released\n", s.ticket);
    return kInvalidResource;
  }
  {
    int r = collect_times(c, s);  // this stage's events are about to be reused
    if (r) return r;
  }
  FrameArgs a = frame_args(c, index, type, quality);
  a.epoch = ++c->epoch;
  if (rgb_on_device) {
    a.rgb = rgb;
  } else {
    CK(hipMemcpyAsync(c->rgb, rgb, (size_t)c->w * c->h * 3, hipMemcpyHostToDevice, c->ks));
  }
  // K2 rewrites the coefficient planes and the block table, and the memset
  // below clears the error word: the previous frame's D2H must have finished.
  const Stage& prev = c->st[(t + kStages - 1) % kStages];
  if (prev.ticket >= 0) CK(hipStreamWaitEvent(c->ks, prev.d2h_done, 0));
  CK(hipMemsetAsync(c->sync, 0, c->sync_words * sizeof(int32_t), c->ks));
  const bool prof = c->profiling;
  if (prof) CK(hipEventRecord(s.ev[0], c->ks));
  CK(launch_convert(a, c->ks));
  if (prof) CK(hipEventRecord(s.ev[1], c->ks));
  if (a.inter && c->ring > 1) CK(launch_inter_search(a, c->ks));
  c->have_inter = a.inter && c->ring > 1;
  if (prof) CK(hipEventRecord(s.ev[2], c->ks));
  if (c->stamps) {  // kernel entry (min) / exit (max) words
    const uint64_t init[2] = {~0ull, 0};
    CK(hipMemcpyAsync(c->stamps + stamp_words(c) - 2, init, sizeof(init), hipMemcpyHostToDevice, c->ks));
  }
  CK(launch_mb_rows(a, c->wg_rows, c->ks));  // coding + in-loop deblock
  if (prof) {
    CK(hipEventRecord(s.ev[3], c->ks));
    s.timed = true;
  }
  CK(hipEventRecord(s.k2_done, c->ks));
  if (c->predeblock) CK(launch_unpack_granules(a, planes_at(c->predeblock, c), c->ks));
  // Outputs for the host entropy stage.
  const size_t mbs = (size_t)c->wmb * c->hmb;
  CK(hipStreamWaitEvent(c->cs, s.k2_done, 0));
  CK(hipMemcpyAsync(s.table, c->table, mbs * sizeof(BlockDesc), hipMemcpyDeviceToHost, c->cs));
  CK(hipMemcpyAsync(s.coef, c->coef, c->plane_elems * 2, hipMemcpyDeviceToHost, c->cs));
  CK(hipMemcpyAsync(s.err, c->sticky, sizeof(int32_t), hipMemcpyDeviceToHost, c->cs));
  CK(hipEventRecord(s.d2h_done, c->cs));
  s.busy = true;
  s.ticket = t;
  s.index = index;
  s.type = type;
  s.quality = quality;
  c->next_ticket++;
  *ticket = t;
  return kSuccess;
}

int cairo_ctx_wait(cairo_ctx* c, int ticket, cairo_frame_result* out) {
  if (!c || !out) return kInvalidArg;
  Stage& s = c->st[ticket % kStages];
  if (!s.busy || s.ticket != ticket) return kInvalidResource;
  CK(hipSetDevice(c->device));
  CK(hipEventSynchronize(s.d2h_done));
  if (*s.err) {
    fprintf(stderr, "[cairo_amd] an in-kernel wait timed out (at or before frame %u)\n", s.index);
    return kHardwareFail;
  }
  out->block_table = s.table;
  out->coef_y = s.coef;
  out->coef_u = s.coef + (size_t)c->wa * c->ha;
  out->coef_v = out->coef_u + (size_t)(c->wa / 2) * (c->ha / 2);
  out->wa = c->wa;
  out->ha = c->ha;
  out->wmb = c->wmb;
  out->hmb = c->hmb;
  out->index = s.index;
  out->type = s.type;
  out->quality = s.quality;
  return kSuccess;
}

int cairo_ctx_release(cairo_ctx* c, int ticket) {
  if (!c) return kInvalidArg;
  Stage& s = c->st[ticket % kStages];
  if (s.ticket != ticket) return kInvalidResource;
  s.busy = false;
  return kSuccess;
}

int cairo_ctx_sync(cairo_ctx* c) {
  if (!c) return kInvalidArg;
  CK(hipSetDevice(c->device));
  CK(hipStreamSynchronize(c->ks));
  CK(hipStreamSynchronize(c->cs));
  return kSuccess;
}

int cairo_ctx_read_planes(cairo_ctx* c, int which, int16_t* y, int16_t* u, int16_t* v) {
  if (!c || which < 0 || which >= 2 + (int)c->ring) return kInvalidArg;
  CK(hipSetDevice(c->device));
  CK(hipStreamSynchronize(c->ks));
  CK(hipStreamSynchronize(c->cs));
  int16_t* base = which == 0 ? c->in : which == 1 ? c->coef : c->ring_buf + (size_t)(which - 2) * c->plane_elems;
  PlaneSet p = planes_at(base, c);
  const size_t ly = (size_t)c->wa * c->ha, lc = ly / 4;
  if (y) CK(hipMemcpy(y, p.y, ly * 2, hipMemcpyDeviceToHost));
  if (u) CK(hipMemcpy(u, p.u, lc * 2, hipMemcpyDeviceToHost));
  if (v) CK(hipMemcpy(v, p.v, lc * 2, hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_ctx_read_inter(cairo_ctx* c, uint8_t* descs, int32_t* sads) {
  if (!c) return kInvalidArg;
  CK(hipSetDevice(c->device));
  CK(hipStreamSynchronize(c->ks));
  const size_t n = (size_t)c->wmb * c->hmb * (c->ring > 1 ? c->ring - 1 : 0);
  if (!n) return kSuccess;
  if (descs) CK(hipMemcpy(descs, c->inter_desc, n * sizeof(BlockDesc), hipMemcpyDeviceToHost));
  if (sads) CK(hipMemcpy(sads, c->inter_sad, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_ctx_set_debug(cairo_ctx* c, int flags) {
  if (!c) return kInvalidArg;
  CK(hipSetDevice(c->device));
  if ((flags & 1) && !c->predeblock) CK(hipMalloc(&c->predeblock, c->plane_elems * 2));
  if ((flags & 2) && !c->stamps)
    CK(hipMalloc(&c->stamps, stamp_words(c) * sizeof(uint64_t)));
  return kSuccess;
}

int cairo_ctx_read_stamps(cairo_ctx* c, uint64_t* out) {
  if (!c || !c->stamps || !out) return kInvalidArg;
  CK(hipSetDevice(c->device));
  CK(hipStreamSynchronize(c->ks));
  CK(hipMemcpy(out, c->stamps, stamp_words(c) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_ctx_read_predeblock(cairo_ctx* c, int16_t* y, int16_t* u, int16_t* v) {
  if (!c || !c->predeblock) return kInvalidArg;
  CK(hipSetDevice(c->device));
  CK(hipStreamSynchronize(c->ks));
  PlaneSet p = planes_at(c->predeblock, c);
  const size_t ly = (size_t)c->wa * c->ha, lc = ly / 4;
  if (y) CK(hipMemcpy(y, p.y, ly * 2, hipMemcpyDeviceToHost));
  if (u) CK(hipMemcpy(u, p.u, lc * 2, hipMemcpyDeviceToHost));
  if (v) CK(hipMemcpy(v, p.v, lc * 2, hipMemcpyDeviceToHost));
  return kSuccess;
}

int cairo_ctx_read_table(cairo_ctx* c, uint8_t* table) {
  if (!c || !table) return kInvalidArg;
  CK(hipSetDevice(c->device));
  CK(hipStreamSynchronize(c->ks));
  CK(hipMemcpy(table, c->table, (size_t)c->wmb * c->hmb * sizeof(BlockDesc),
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

}  // extern "C"
