// cairo_amd/csrc/kernels.hip -- the EVX-1 encode hot path on gfx950 (CDNA4).
//
//   k_convert_batch  RGB888 -> planar YUV 4:2:0 int16, every frame of a
//                    launch                                    convert.cpp:95-160
//   k_engine         one persistent launch per batch of frames, pipelined
//                    across frames, two pools of 256-thread workgroups:
//     row helpers    inter search of their MB row (one wave per MB and
//                    reference, LDS window)                    motion.cpp:421-494
//                    + the in-place deblock of the row behind its coder
//                                                              deblock.cpp:201-284
//     row coders     intra search, classify, transform, VAQ, quantize,
//                    reconstruct, left to right                encode.cpp:17-203,
//                                                              decode.cpp:15-144
//   k_yuv_to_rgb     the decoder's output conversion          convert.cpp:162-223
//   k_kat_transform  known-answer entry of the transform chain (tests)
//
// All arithmetic is integer and restates the reference bit for bit (see
// evx_defs.h for the helpers).  Searches evaluate candidates in parallel and
// then replay the reference's sequential, tie-sensitive acceptance in the
// reference's scan order (j outer, i inner) with wave-uniform scalars.
#include "kernels.h"

namespace cairo {

// The per-frame views (FrameArgs) are written by the host before a launch and
// never during it: read them through the constant address space, so that a
// field is fetched once (scalar loads) instead of again after every global
// store, each refetch waiting behind the outstanding hand-off loads.
typedef const __attribute__((address_space(4))) FrameArgs FA;
// Reconstruction buffer k (FrameArgs::recon) of a view, selected with scalar
// branches: a dynamically indexed struct load would go through scratch.
#define RECON_AT(a, k)                                                                   \
  ((k) == 1 ? planes((a).recon[1]) : (k) == 2 ? planes((a).recon[2]) : (k) == 3 ? planes((a).recon[3]) \
                                                                              : planes((a).recon[0]))
// A plane set field of a view, as an ordinary value.
__host__ __device__ inline PlaneSet planes(const __attribute__((address_space(4))) PlaneSet& p) {
  PlaneSet r;
  r.y = p.y;
  r.u = p.u;
  r.v = p.v;
  return r;
}

// ---------------------------------------------------------------------------
// Tables (generated from their definitions; checked against the oracle by the
// parity tests).
// ---------------------------------------------------------------------------

// round(128 cos((2i+1) j pi / 16)), row j = frequency (xftables.h:57-67).
__constant__ int16_t kLut8[64] = {
    128, 128,  128,  128,  128,  128,  128,  128,   //
    126, 106,  71,   25,   -25,  -71,  -106, -126,  //
    118, 49,   -49,  -118, -118, -49,  49,   118,   //
    106, -25,  -126, -71,  71,   126,  25,   -106,  //
    91,  -91,  -91,  91,   91,   -91,  -91,  91,    //
    71,  -126, 25,   106,  -106, -25,  126,  -71,   //
    49,  -118, 118,  -49,  -49,  118,  -118, 49,    //
    25,  -71,  106,  -126, 126,  -106, 71,   -25};
// default_intra_8x8_qm / default_inter_8x8_qm (quantize.cpp:13-35).
__constant__ int16_t kQmIntra[64] = {
    8,  17, 18, 19, 21, 23, 25, 27, 17, 18, 19, 21, 23, 25, 27, 28, 20, 21, 22, 23, 24, 26,
    28, 30, 21, 22, 23, 24, 26, 28, 30, 32, 22, 23, 24, 26, 28, 30, 32, 35, 23, 24, 26, 28,
    30, 32, 35, 38, 25, 26, 28, 30, 32, 35, 38, 41, 27, 28, 30, 32, 35, 38, 41, 45};
__constant__ int16_t kQmInter[64] = {
    16, 17, 18, 19, 20, 21, 22, 23, 17, 18, 19, 20, 21, 22, 23, 24, 18, 19, 20, 21, 22, 23,
    24, 25, 19, 20, 21, 22, 23, 24, 26, 27, 20, 21, 22, 23, 25, 26, 27, 28, 21, 22, 23, 24,
    26, 27, 28, 30, 22, 23, 24, 26, 27, 28, 30, 31, 23, 24, 25, 27, 28, 30, 31, 33};
// alpha_table / beta_table (deblock.cpp:13-27).
__constant__ int16_t kAlpha[32] = {0, 0, 0, 0, 0,  0,  0,  1,  1,  1,  2,  2,  3,  3,  4,  5,
                                   6, 7, 8, 9, 10, 12, 14, 16, 18, 20, 22, 24, 26, 29, 32, 35};
__constant__ int16_t kBeta[32] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 3,
                                  3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 10, 11};

// LDS copies of the tables, loaded once per workgroup (load_tables): a lookup
// with a per-lane index is then an LDS read (lgkmcnt) instead of a global load
// whose vmcnt(0) wait would also drain the outstanding hand-off loads.
// sLut8T (the transpose) makes every transform pass's 8 coefficients one
// 16-byte row read.
__shared__ __attribute__((aligned(16))) int16_t sLut8[64], sLut8T[64];
__shared__ int16_t sQmIntra[64], sQmInter[64], sAlpha[32], sBeta[32];
// Reciprocals for the quantizer's divisions (rdiv_m): the matrices' entries,
// 2 qp and the DC scales for qp = 0..31.
__shared__ uint32_t sMagQmIntra[64], sMagQmInter[64], sMag2qp[32], sMagDcL[32], sMagDcC[32];

// m = ceil(2^32 / d) for 2 <= d: then u / d = mulhi(u, m) exactly for u * d <
// 2^32 (the error term u * (m d - 2^32) / 2^32 stays below 1 / d).
__host__ __device__ inline uint32_t div_magic(uint32_t d) { return 0xFFFFFFFFu / d + 1u; }
// rdiv (rounded_div, half away from zero) by d > 1 with its div_magic m, for
// |n| + d / 2 < 2^32 / d: sign(n) * ((|n| + d/2) / d), which is rdiv's
// truncating division of n -/+ d/2.  One mulhi instead of a division.
__device__ __forceinline__ int32_t rdiv_m(int32_t n, int32_t d, uint32_t m) {
  const uint32_t u = (uint32_t)(n < 0 ? -n : n) + (uint32_t)(d >> 1);
  const int32_t q = (int32_t)__umulhi(u, m);
  return n < 0 ? -q : q;
}

// Whole workgroup; ends with a barrier.
__device__ __forceinline__ void load_tables() {
  const int t = threadIdx.x;
  if (t < 64) {
    sLut8[t] = kLut8[t];
    sLut8T[t] = kLut8[(t & 7) * 8 + (t >> 3)];
    sQmIntra[t] = kQmIntra[t];
    sQmInter[t] = kQmInter[t];
  } else if (t < 96) {
    sAlpha[t - 64] = kAlpha[t - 64];
    sBeta[t - 64] = kBeta[t - 64];
  } else if (t < 128) {
    const int q = t - 96;
    sMag2qp[q] = div_magic(max(2 * q, 2));
    sMagDcL[q] = div_magic(luma_dc_scale(q));
    sMagDcC[q] = div_magic(chroma_dc_scale(q));
  } else if (t < 192) {
    sMagQmIntra[t - 128] = div_magic(kQmIntra[t - 128]);
    sMagQmInter[t - 128] = div_magic(kQmInter[t - 128]);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Wave64 / workgroup helpers
// ---------------------------------------------------------------------------

// Sum / max over the 64 lanes; wave-uniform result.  DPP row rotations reduce
// each 16-lane row, four readlanes combine the rows into a scalar.
__device__ __forceinline__ int wave_sum(int v) {
  v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);  // row_ror:8
  v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v += __builtin_amdgcn_mov_dpp(v, 0x122, 0xF, 0xF, false);  // row_ror:2
  v += __builtin_amdgcn_mov_dpp(v, 0x121, 0xF, 0xF, false);  // row_ror:1
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
         __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ int wave_max(int v) {
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x122, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x121, 0xF, 0xF, false));
  return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Diagnostic live trace (mapped host memory, system scope): word k of this workgroup.
__device__ __forceinline__ void trace(int32_t* t, int k, int v) {
  if (t && threadIdx.x == 0)
    __hip_atomic_store(&t[blockIdx.x * 4 + k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Plane pl (0 Y, 1 U, 2 V) of a plane set.  The three pointers are read as
// values and then selected: selecting between the fields' addresses would keep
// the struct in scratch memory.
__device__ __forceinline__ int16_t* pick(const PlaneSet& p, int pl) {
  int16_t* const y = p.y;
  int16_t* const u = p.u;
  int16_t* const v = p.v;
  return pl == 0 ? y : (pl == 1 ? u : v);
}

// v, opaque to the optimiser: per-lane address math derived from it is
// recomputed where it is used instead of being hoisted out of the macroblock
// loop and kept live across the searches (where it was spilled to scratch,
// and each reload's vmcnt wait also waited for the outstanding hand-off loads).
__device__ __forceinline__ int fresh(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// A value every lane holds identically, moved to an SGPR so that the code
// consuming it is scalar (no exec-mask divergence).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Diagnostic timestamp (100 MHz constant clock) of phase k of macroblock mb.
__device__ __forceinline__ void stamp(FA& a, int mb, int k) {
  if (a.stamps && threadIdx.x == 0)
    a.stamps[(size_t)mb * kStampPhases + k] = __builtin_amdgcn_s_memrealtime();
}

// Time accounting (kernels.h Acct; CAIRO_ACCT=1 builds with cairo_ctx_set_debug
// 32): thread 0 adds 10 ns ticks to its workgroup's shard (posted atomics).
__device__ __forceinline__ uint64_t acct_now() { return CAIRO_ACCT ? __builtin_amdgcn_s_memrealtime() : 0; }
__device__ __forceinline__ void acct_add(uint64_t* acct, int k, uint64_t v) {
  if (CAIRO_ACCT && acct && threadIdx.x == 0)
    __hip_atomic_fetch_add(&acct[(blockIdx.x & (kAcctShards - 1)) * kAcctWords + k], v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Deblock progress words (kernels.h FrameArgs::progress): tag a column count
// with the frame's epoch; relaxed agent-scope 64-bit loads.
__device__ __forceinline__ uint64_t tagged(uint32_t epoch, int cols) {
  return ((uint64_t)epoch << 32) | (uint32_t)cols;
}
__device__ __forceinline__ uint64_t progress_at(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The previous frame's words may live on another device (FrameArgs::sys).
__device__ __forceinline__ uint64_t progress_peer(bool sys, const uint64_t* p) {
  return sys ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
             : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Acquire after a wait (thread 0): agent scope, or system scope when the data
// released by the observed word may come from another device.
__device__ __forceinline__ void acquire_fence(bool sys) {
  if (sys)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// Poll back-off (s_sleep units of 64 clocks) of the progress-word waits and of
// the granule re-polls (sweeps of 0-3 were within noise).
constexpr int kWaitSleep = 2, kGranSleep = 1;

// A bounded wait gave up (~2 s): set the launch's error word, so that every
// other wait ends and every workgroup drains (the host then reports
// EVX_ERROR_HARDWAREFAIL), and -- if no wait of this context gave up before --
// record what this one waited for in the sticky words (kernels.h TimeoutInfo).
// One lane; the cold path of every wait.
__device__ __attribute__((noinline)) void report_timeout(int32_t* err, int32_t* sticky, int kind, uint32_t epoch,
                                                         int index, int row, int member, int need, int on,
                                                         uint64_t seen) {
  __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int32_t none = 0;
  if (!__hip_atomic_compare_exchange_strong(sticky + TimeoutInfo::kClaim, &none, 1, __ATOMIC_RELAXED,
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return;  // an earlier timeout is the one reported
  const int32_t w[8] = {(int32_t)epoch, index, row, member, need, on, (int32_t)(uint32_t)seen, (int32_t)(seen >> 32)};
  for (int k = 0; k < 8; k++) __hip_atomic_store(sticky + 1 + k, w[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the kind last, with a system-scope release: a reader that acquire-loads
  // the kind first (k_feed_copy) sees the whole record; the host's copies,
  // which have no order between the words, only learn from the kind that the
  // record exists and read it again (backend.hip report_timeout_host)
  __hip_atomic_store(sticky + TimeoutInfo::kKind, kind, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void report_timeout(FA& a, int kind, int row, int need, int on, uint64_t seen) {
  report_timeout(a.err, a.sticky, kind, a.epoch, a.index, row, a.member, need, on, seen);
}

// Bounded wait of the row coder for its inter group's records (relaxed
// agent-scope poll + s_sleep); gives up after ~2 s (report_timeout).
__device__ __forceinline__ void wait_records(FA& a, int row, int group) {
  int32_t* word = &a.inter_done[row * a.ng + group];
  int v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (v >= a.nref) return;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < a.nref) {
    if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    __builtin_amdgcn_s_sleep(kWaitSleep);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
      report_timeout(a, kWaitRecords, row, a.nref, group, (uint32_t)v);
      return;
    }
  }
}

// Consumer side of a hand-off: one lane waited; invalidate this CU's L1 and
// let every wave load only after the barrier (MI355X_MICROARCH.md, Valid forms).
__device__ __forceinline__ void acquire_after_wait(bool sys = false) {
  if (threadIdx.x == 0) {
    acquire_fence(sys);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}


// Granule hand-off (kernels.h kGranulesPerMB): one 8-byte sc1 store per
// granule on the producer, sc1 loads on the consumer, the tag is the flag.
// Global address space so the compiler emits global_ (never flat_) accesses.
typedef __attribute__((address_space(1))) uint64_t gbl_u64;
typedef __attribute__((address_space(1))) uint32_t gbl_u32;
__device__ __forceinline__ uint64_t gran_ld(const uint64_t* p) {
  return __hip_atomic_load((const gbl_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gran_st(uint64_t* p, uint64_t v) {
  __hip_atomic_store((gbl_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The record granule p of frame a (tagged inter records, kernels.h
// pack_inter_desc), given a first load g: re-polls until the tag is the
// frame's epoch; bounded (report_timeout: kind records, on = the macroblock).
__device__ __forceinline__ uint32_t rec_settle(FA& a, const uint64_t* p, uint64_t g, int row, int mb) {
  if ((uint32_t)(g >> 32) == a.epoch) return (uint32_t)g;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    __builtin_amdgcn_s_sleep(kWaitSleep);
    g = gran_ld(p);
    if (CAIRO_ACCT && a.acct) {
      const uint64_t act = __ballot(1);
      if ((int)(threadIdx.x & 63) == __ffsll((long long)act) - 1)
        __hip_atomic_fetch_add(&a.acct[(blockIdx.x & (kAcctShards - 1)) * kAcctWords + Acct::kRecPollBytes],
                               8ull * __popcll(act), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if ((uint32_t)(g >> 32) == a.epoch) break;
    if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      report_timeout(a, kWaitRecords, row, (int)a.epoch, mb, g);
      break;
    }
  }
  return (uint32_t)g;
}

// Data of granule p of frame a, given a first load g: re-polls until the tag
// is the frame's epoch.  Bounded like every wait (the error word ends every
// other wait too); row = the waiting task's row, for the timeout record.
__device__ __forceinline__ uint32_t gran_settle(FA& a, const uint64_t* p, uint64_t g, int row) {
  if ((uint32_t)(g >> 32) == a.epoch) return (uint32_t)g;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    __builtin_amdgcn_s_sleep(kGranSleep);
    g = gran_ld(p);
    if (CAIRO_ACCT && a.acct) {  // this wave's re-poll: 8 bytes per active lane
      const uint64_t act = __ballot(1);
      if ((int)(threadIdx.x & 63) == __ffsll((long long)act) - 1)
        __hip_atomic_fetch_add(&a.acct[(blockIdx.x & (kAcctShards - 1)) * kAcctWords + Acct::kGranPollBytes],
                               8ull * __popcll(act), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if ((uint32_t)(g >> 32) == a.epoch) break;
    if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      report_timeout(a, kWaitGranule, row, (int)a.epoch, (int)((p - a.granules) / kGranuleStride), g);
      break;
    }
  }
  return (uint32_t)g;
}

// p, opaque to the optimiser: the frame view's fields are re-read (scalar
// loads that hit the scalar cache) in every macroblock instead of being
// hoisted out of the row loop and kept live in SGPRs, which spill.
__device__ __forceinline__ FA* opaque_view(FA* p) {
  uint64_t v = (uint64_t)p;
  asm volatile("" : "+s"(v));
  return (FA*)v;
}

// Dequeue the next task index for this workgroup (uniform result).
__device__ __forceinline__ int dequeue(int32_t* ticket, int* lds_slot) {
  __syncthreads();
  if (threadIdx.x == 0)
    *lds_slot = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return *lds_slot;
}

// ---------------------------------------------------------------------------
// K0: RGB888 -> YUV 4:2:0 int16 (convert.cpp:11-14, 30-73, 95-160)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_convert_batch(ConvertArgs e) {
  if ((int)blockIdx.z == e.nframes) {
    // the launch's frame views (mapped host memory -> device) and zeroed sync
    // area, spread over the slice's blocks
    const int nb = gridDim.x * gridDim.y, t = (blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
    for (int k = t; k < e.fa_chunks; k += nb * 256) e.fa_dev[k] = e.fa_host[k];
    for (int k = t; k < e.sync_words; k += nb * 256) e.sync[k] = 0;
    return;
  }
  const uint8_t* rgb = e.rgb[blockIdx.z];
  const int qx = blockIdx.x * 256 + threadIdx.x;  // quad column
  const int qy = blockIdx.y;                      // quad row
  if (qx >= (e.w >> 1) || !rgb) return;
  const PlaneSet in = e.in[blockIdx.z];
  int su = 0, sv = 0;
#pragma unroll
  for (int dy = 0; dy < 2; dy++) {
    const uint8_t* p = rgb + ((size_t)(2 * qy + dy) * e.w + 2 * qx) * 3;
    int16_t* y = in.y + (size_t)(2 * qy + dy) * e.wa + 2 * qx;
#pragma unroll
    for (int dx = 0; dx < 2; dx++) {
      int r = p[3 * dx], g = p[3 * dx + 1], b = p[3 * dx + 2];
      y[dx] = (int16_t)(((77 * r + 150 * g + 29 * b + 128) >> 8) + 16);
      su = (int16_t)(su + (((-43 * r - 85 * g + 128 * b + 128) / 256) + 128));
      sv = (int16_t)(sv + (((128 * r - 107 * g - 21 * b + 128) / 256) + 128));
    }
  }
  in.u[(size_t)qy * (e.wa >> 1) + qx] = (int16_t)((su + 2) >> 2);
  in.v[(size_t)qy * (e.wa >> 1) + qx] = (int16_t)((sv + 2) >> 2);
}

hipError_t launch_convert_batch(const ConvertArgs& e, hipStream_t s) {
  dim3 grid((e.w / 2 + 255) / 256, e.h / 2, e.nframes + 1);
  hipLaunchKernelGGL(k_convert_batch, grid, dim3(256), 0, s, e);
  return hipGetLastError();
}

// Biased 16-bit storage (v ^ 0x8000): unsigned order equals signed order.
__device__ __forceinline__ int unbias(int16_t b) { return (int)(int16_t)(b ^ (int16_t)0x8000); }

// Sum / max over one 16-lane DPP row (a candidate's group); all 16 lanes get it.
__device__ __forceinline__ int row16_sum(int v) {
  v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x122, 0xF, 0xF, false);
  v += __builtin_amdgcn_mov_dpp(v, 0x121, 0xF, 0xF, false);
  return v;
}
__device__ __forceinline__ int row16_max(int v) {
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x122, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x121, 0xF, 0xF, false));
  return v;
}

// A 16-lane group evaluates one candidate: lane i owns luma row i (16 px) and
// 4 pixels of U and V (row i>>1, columns (i&1)*4..+3).  Source pixels as
// biased u16 pairs.
struct SrcRow {
  uint32_t y[8], u[2], v[2];
};
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ int src_px(const uint32_t* p, int k) {  // unbiased pixel k
  return unbias((int16_t)(p[k >> 1] >> (16 * (k & 1))));
}

// |src - cand| over biased pairs: SAD (v_sad_u16) and the two one-sided
// saturated differences, whose packed maxima give the MAD.
__device__ __forceinline__ void pk_diff(uint32_t a, uint32_t b, uint32_t& sad, u16x2& m1, u16x2& m2) {
  sad = __builtin_amdgcn_sad_u16(a, b, sad);
  m1 = __builtin_elementwise_max(m1, __builtin_elementwise_sub_sat(as_u16x2(a), as_u16x2(b)));
  m2 = __builtin_elementwise_max(m2, __builtin_elementwise_sub_sat(as_u16x2(b), as_u16x2(a)));
}

// The acceptance rules (evaluate_motion_candidate / _subpel_, motion.cpp:111-223)
// use a candidate's MAD only through "mad < thr" and, in copy mode (the best's
// MAD below thr), "mad < best mad" / "==": every MAD at or above thr acts the
// same.  MAD >= max |dY| >= SAD / 256, so a candidate whose luma SAD exceeds
// 256 * (thr - 1) has MAD >= thr: its exact MAD is never needed, and kMadFar
// stands for it.  A wave computes the MADs of its candidates only when one of
// them could be below thr (the search's copy-mode tests, the state's MAD and
// the block type see the same outcomes).
constexpr int kMadFar = 65535;
__device__ __forceinline__ bool mad_needed(int sad, int thr) { return sad <= 256 * (thr - 1); }

// ---------------------------------------------------------------------------
// Inter-search window in LDS, shared by the 4 waves of a workgroup that search
// 4 horizontally adjacent macroblocks: 80 luma rows x 128 columns (origin 32 px
// left of / above the first macroblock) and 40 x 64 per chroma plane, covering
// every candidate the searches can reach.
// ---------------------------------------------------------------------------

// Luma pitch: 136 elements (68 dwords): window rows stay 16-byte aligned for
// the 16-byte LDS-DMA (dma_window) and hold a 128-column row plus a pad.
constexpr int kWinL = 80, kWinLW = 128, kWinLP = 136;  // luma rows, width, pitch (elements)
constexpr int kWinC = 40, kWinCP = 72;  // chroma rows, pitch (64 columns)

struct alignas(16) Window {
  int16_t y[kWinL * kWinLP];
  int16_t u[kWinC * kWinCP];
  int16_t v[kWinC * kWinCP];
};

// Eight int16 as biased u16 (v ^ 0x8000: unsigned order = signed order, so
// the candidate rows can use packed u16 SAD / saturating-difference ops).
__device__ __forceinline__ uint4 bias4(uint4 v) {
  v.x ^= 0x80008000u, v.y ^= 0x80008000u, v.z ^= 0x80008000u, v.w ^= 0x80008000u;
  return v;
}

// Attribution builds (tools/attr_traffic.sh, tools/attr_valu.sh; never a
// product build).  Traffic: bit 0 skips the search-window loads (the windows
// hold stale LDS), bit 2 the row coder's inter-prediction loads (constant
// predictions); the searches and codes then run on wrong data -- same task
// shapes, wrong results -- so the drop in fabric reads against the default
// build is what those loads cost.  Instructions: bit 8 skips the helpers'
// integer and sub-pel steps (zero-MV records), bit 16 the row coders' intra
// search (stages and sub-pel), bit 32 the deblock filters, bit 64 the row
// coders' transform chain (DCT, quantize, dequantize, IDCT); the drop in
// SQ_INSTS_VALU is what those phases issue (the decisions change too, so the
// other phases' counts move a little).  Refused unless the build says it is a
// tools build.
#ifndef CAIRO_ATTR_SKIP
#define CAIRO_ATTR_SKIP 0
#endif
#if CAIRO_ATTR_SKIP && !defined(CAIRO_TOOLS_BUILD)
#error "CAIRO_ATTR_SKIP produces wrong output: tools builds only (define CAIRO_TOOLS_BUILD)"
#endif

// Stage the in-frame part of window rows [r0, r1) x columns [c0, c1) (luma;
// columns multiples of 16; chroma rows [r0/2, r1/2), columns halved) with
// origin (ox, oy) (luma pixels, multiples of 16) from plane set p by LDS-DMA
// (global_load_lds: no VGPR destination, so every load of the window is in
// flight at once -- one fabric round trip), 16 bytes per lane: the window's
// rows are numbered as 16-byte chunks over the PADDED pitch (17 per luma row,
// 9 per chroma row), so one wave instruction fills 64 consecutive chunks
// (~3.8 luma rows) and the lanes that land in a row's pad, outside [c0, c1)
// or outside the frame are masked off (an LDS-DMA writes wave-uniform base +
// lane x 16).  All 256 threads participate; the values land raw (bias_window
// follows).
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void dma_window(Window& w, const PlaneSet& p, int wa, int ha, int ox, int oy, int r0,
                                           int r1, int c0, int c1) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (CAIRO_ATTR_SKIP & 1) return;
  constexpr int kLC = kWinLP / 8, kCC = kWinCP / 8;
  static_assert(kWinLP % 8 == 0 && kWinCP % 8 == 0, "16-byte chunked pitches");
  const int k0 = r0 * kLC, k1 = r1 * kLC;
  for (int kb = k0 + 64 * wave; kb < k1; kb += 256) {
    const int k = kb + lane, r = k / kLC, cc = k - r * kLC, c = cc << 3;
    const int gy = oy + r, gx = ox + c;
    if (k < k1 && cc < (kWinLW >> 3) && c >= c0 && c < c1 && gy >= 0 && gy < ha && gx >= 0 && gx < wa)
      __builtin_amdgcn_global_load_lds((const void*)&p.y[(size_t)gy * wa + gx], (lds_void*)&w.y[kb << 3], 16, 0, 0);
  }
  const int cr0 = r0 >> 1, cr1 = r1 >> 1, ck0 = cr0 * kCC, ck1 = cr1 * kCC;
  const int ni = (ck1 - ck0 + 63) >> 6;  // instructions per chroma plane
  const int cw = wa >> 1, ch = ha >> 1, cox = ox >> 1, coy = oy >> 1;
  for (int i = wave; i < 2 * ni; i += 4) {
    const int pl = i >= ni, kb = ck0 + ((i - (pl ? ni : 0)) << 6);
    const int k = kb + lane, r = k / kCC, cc = k - r * kCC, c = cc << 3;
    const int gy = coy + r, gx = cox + c;
    if (k < ck1 && cc < 8 && 2 * c >= c0 && 2 * c < c1 && gy >= 0 && gy < ch && gx >= 0 && gx < cw)
      __builtin_amdgcn_global_load_lds((const void*)&pick(p, 1 + pl)[(size_t)gy * cw + gx],
                                       (lds_void*)&(pl ? w.v : w.u)[kb << 3], 16, 0, 0);
  }
}
// Bias window rows [r0, r1) x columns [c0, c1) in LDS (v ^ 0x8000), in
// 16-byte chunks: luma 16 lanes per row (8 columns each), chroma 8 lanes per
// row.  All 256 threads; after every wave's DMA has landed (vmcnt, barrier).
__device__ __forceinline__ void bias_window(Window& w, int r0, int r1, int c0, int c1) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  {
    const int k0 = c0 >> 3, k1 = c1 >> 3;  // luma chunks of the staged columns
    const int rr = lane >> 4, kk = lane & 15;
    if (kk >= k0 && kk < k1)
      for (int r = r0 + 4 * wave + rr; r < r1; r += 16) {
        uint4* q = (uint4*)&w.y[r * kWinLP + 8 * kk];
        *q = bias4(*q);
      }
    const int cr0 = r0 >> 1, cr1 = r1 >> 1, ck0 = c0 >> 4, ck1 = c1 >> 4;
    const int crr = lane >> 3, ckk = lane & 7;
    if (ckk >= ck0 && ckk < ck1)
      for (int k = 8 * wave + crr; k < 2 * (cr1 - cr0); k += 32) {
        const int pl = k >= cr1 - cr0, r = cr0 + k - (pl ? cr1 - cr0 : 0);
        uint4* q = (uint4*)&(pl ? w.v : w.u)[r * kWinCP + 8 * ckk];
        *q = bias4(*q);
      }
  }
}
__device__ __forceinline__ void load_window_dma(Window& w, const PlaneSet& p, int wa, int ha, int ox, int oy, int r0,
                                                int r1, int c0, int c1) {
  dma_window(w, p, wa, ha, ox, oy, r0, r1, c0, c1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
  __syncthreads();                                    // ... every wave's
  bias_window(w, r0, r1, c0, c1);
}

__device__ __forceinline__ void acct_window(uint64_t* acct, int r0, int r1, int c0, int c1) {
  acct_add(acct, Acct::kWinBytes, (uint64_t)(r1 - r0) * (c1 - c0) * 3);  // luma + 2 quarter chroma planes, int16
  acct_add(acct, Acct::kWinStages, 1);
}
__device__ __forceinline__ void stage_window(Window& w, const PlaneSet& p, int wa, int ha, int ox, int oy, int r0,
                                             int r1, int c0, int c1) {
  load_window_dma(w, p, wa, ha, ox, oy, r0, r1, c0, c1);
}

// Per-lane slice of a macroblock: luma row l>>2, columns (l&3)*4..+3, and the
// chroma pixel (l>>3, l&7) of U and V.
struct Px6 {
  int y0, y1, y2, y3, u, v;
};

// This lane's slice of the window at (wx, wy), as raw biased values (v + 0x8000).
__device__ __forceinline__ Px6 px_from_window_b(const Window& w, int wx, int wy) {
  int l = lane_id();
  const uint16_t* py = (const uint16_t*)&w.y[(wy + (l >> 2)) * kWinLP + wx + (l & 3) * 4];
  int cwx = wx >> 1, cwy = wy >> 1;
  Px6 r;
  r.y0 = py[0];
  r.y1 = py[1];
  r.y2 = py[2];
  r.y3 = py[3];
  r.u = ((const uint16_t*)w.u)[(cwy + (l >> 3)) * kWinCP + cwx + (l & 7)];
  r.v = ((const uint16_t*)w.v)[(cwy + (l >> 3)) * kWinCP + cwx + (l & 7)];
  return r;
}

__device__ __forceinline__ Px6 px_from_planes(const PlaneSet& p, int wa, int x, int y) {
  int l = lane_id();
  const int16_t* py = &p.y[(size_t)(y + (l >> 2)) * wa + x + (l & 3) * 4];
  int cw = wa >> 1;
  Px6 r;
  r.y0 = py[0];
  r.y1 = py[1];
  r.y2 = py[2];
  r.y3 = py[3];
  r.u = p.u[(size_t)((y >> 1) + (l >> 3)) * cw + (x >> 1) + (l & 7)];
  r.v = p.v[(size_t)((y >> 1) + (l >> 3)) * cw + (x >> 1) + (l & 7)];
  return r;
}

// lerp_macroblock_half / _quarter (macroblock.h:203-241), per pixel.
__device__ __forceinline__ int lerp_px(int a, int b, int quarter) {
  return quarter ? (int16_t)(round_out(3 * a + b, 2) / 4) : (int16_t)(round_out(a + b, 1) / 2);
}
// The same on biased values (v + 0x8000, in [0, 65535]), biased result, for
// v_sad_u16 and the packed u16 ops.  round_out(n, h) / 2h truncates toward
// zero, which is (n + h - (n < 0)) >> s with an arithmetic shift (h =
// 2^(s-1), n = a+b or 3a+b); on the biased sum t = a'+b' = n + 0x10000 (or
// 3a'+b' = n + 0x20000) that is (t + h - (n < 0)) >> s, logical, and n < 0 is
// bit 16 (bit 17) of t clear.  The reference's int16 cast never truncates
// here: |(3a+b)/4|, |(a+b)/2| <= 0x7FFF.  4 instructions instead of 8, and no
// unbiasing of the window values.
__device__ __forceinline__ uint32_t lerp_half_bb(uint32_t a, uint32_t b) {
  const uint32_t t = a + b;  // [0, 0x1FFFE]
  return (t + ((t >> 16) & 1)) >> 1;
}
__device__ __forceinline__ uint32_t lerp_quarter_bb3(uint32_t a3, uint32_t b) {  // a3 = 3a'
  const uint32_t t = a3 + b;  // [0, 0x3FFFC]
  return (t + 1 + ((t >> 17) & 1)) >> 2;
}
__device__ __forceinline__ uint32_t lerp_quarter_bb(uint32_t a, uint32_t b) { return lerp_quarter_bb3(3 * a, b); }
__device__ __forceinline__ uint32_t absdiff_b(uint32_t x, uint32_t y) {  // biased values
  return __builtin_amdgcn_sad_u16(x, y, 0);
}

// One candidate row of the inter search: a 16-lane group evaluates the
// candidate at window position (wx, wy); lane i owns luma row i (16 px) and
// 4 pixels of U and V (row i>>1, columns (i&1)*4..+3).  Window values and the
// source rows are biased u16 pairs; unaligned columns are realigned with
// v_alignbyte_b32.  Returns the candidate's SAD (luma) and MAD (luma + chroma)
// in every lane of the group (compute_block_sad / _mad, analysis.h:42-125).
__device__ __forceinline__ void inter_cand_row(const Window& w, int wx, int wy, int i, const SrcRow& s, int thr,
                                               int& sad, int& mad) {
  const int sh = (wx & 1) * 2;
  const uint32_t* row = (const uint32_t*)&w.y[(wy + i) * kWinLP] + (wx >> 1);
  uint32_t d[9];
#pragma unroll
  for (int k = 0; k < 9; k++) d[k] = row[k];
  uint32_t sm = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) sm = __builtin_amdgcn_sad_u16(s.y[k], __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh), sm);
  sad = row16_sum((int)sm);
  mad = kMadFar;
  if (__ballot(mad_needed(sad, thr))) {  // (wave-uniform) some candidate of the wave may have MAD < thr
    u16x2 m1 = {0, 0}, m2 = {0, 0};
    uint32_t dummy = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) pk_diff(s.y[k], __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh), dummy, m1, m2);
    const int cr = (wy >> 1) + (i >> 1), cc = (wx >> 1) + (i & 1) * 4, shc = (cc & 1) * 2;
    const uint32_t* ru = (const uint32_t*)&w.u[cr * kWinCP] + (cc >> 1);
    const uint32_t* rv = (const uint32_t*)&w.v[cr * kWinCP] + (cc >> 1);
    const uint32_t u0 = ru[0], u1 = ru[1], u2 = ru[2], v0 = rv[0], v1 = rv[1], v2 = rv[2];
    pk_diff(s.u[0], __builtin_amdgcn_alignbyte(u1, u0, shc), dummy, m1, m2);
    pk_diff(s.u[1], __builtin_amdgcn_alignbyte(u2, u1, shc), dummy, m1, m2);
    pk_diff(s.v[0], __builtin_amdgcn_alignbyte(v1, v0, shc), dummy, m1, m2);
    pk_diff(s.v[1], __builtin_amdgcn_alignbyte(v2, v1, shc), dummy, m1, m2);
    const u16x2 m = __builtin_elementwise_max(m1, m2);
    mad = row16_max(max((int)m.x, (int)m.y));
  }
}

// Biased source rows of macroblock (px, py) for lane group slot i (SrcRow layout).
__device__ __forceinline__ SrcRow load_src_rows(const PlaneSet& in, int wa, int px, int py, int i) {
  SrcRow s;
  const uint4* ry = (const uint4*)(in.y + (size_t)(py + i) * wa + px);
  const uint4 r0 = ry[0], r1 = ry[1];
  s.y[0] = r0.x, s.y[1] = r0.y, s.y[2] = r0.z, s.y[3] = r0.w;
  s.y[4] = r1.x, s.y[5] = r1.y, s.y[6] = r1.z, s.y[7] = r1.w;
  const size_t co = (size_t)((py >> 1) + (i >> 1)) * (wa >> 1) + (px >> 1) + (i & 1) * 4;
  const uint2 u2 = *(const uint2*)(in.u + co), v2 = *(const uint2*)(in.v + co);
  s.u[0] = u2.x, s.u[1] = u2.y, s.v[0] = v2.x, s.v[1] = v2.y;
#pragma unroll
  for (int k = 0; k < 8; k++) s.y[k] ^= 0x80008000u;
#pragma unroll
  for (int k = 0; k < 2; k++) s.u[k] ^= 0x80008000u, s.v[k] ^= 0x80008000u;
  return s;
}

// Wave-uniform SAD (luma) and MAD (luma + chroma) between src and cand
// (compute_block_sad / compute_block_mad, analysis.h:42-55, 103-125).
__device__ __forceinline__ void sad_mad(const Px6& s, const Px6& c, int& sad, int& mad) {
  int d0 = abs(s.y0 - c.y0), d1 = abs(s.y1 - c.y1), d2 = abs(s.y2 - c.y2), d3 = abs(s.y3 - c.y3);
  int du = abs(s.u - c.u), dv = abs(s.v - c.v);
  sad = wave_sum(d0 + d1 + d2 + d3);
  mad = wave_max(max(max(max(d0, d1), max(d2, d3)), max(du, dv)));
}

// Running selection of a search (evx_motion_selection, motion.cpp:43-55).
struct Sel {
  int bx, by, sad, mad, ssd, sp_idx, sp_amt, sp_en;
};

// evaluate_motion_candidate acceptance (motion.cpp:111-149).
__device__ __forceinline__ void accept_int(Sel& s, int cx, int cy, int sad, int mad, int px, int py,
                                           int thr) {
  int ssd = (cx - px) * (cx - px) + (cy - py) * (cy - py);
  bool acc = (s.mad < thr) ? (mad < s.mad || (mad == s.mad && ssd < s.ssd))
                           : (sad < s.sad || (sad == s.sad && ssd < s.ssd && sad < kSadGate) ||
                              mad < thr);
  if (acc) {
    s.bx = cx;
    s.by = cy;
    s.sad = sad;
    s.ssd = ssd;
    s.mad = mad;
  }
}
// evaluate_subpel_motion_candidate acceptance (motion.cpp:151-223).
__device__ __forceinline__ void accept_sub(Sel& s, int idx, int quarter, int sad, int mad,
                                           int thr) {
  bool acc = (s.mad < thr) ? (mad < s.mad) : ((sad < s.sad && sad < kSadGate) || mad < thr);
  if (acc) {
    s.sp_en = 1;
    s.sp_amt = quarter;
    s.sp_idx = idx;
    s.sad = sad;
    s.mad = mad;
  }
}


// ---------------------------------------------------------------------------
// Parallel replay of the reference's sequential candidate acceptance.
//
// Lanes 0..15 of a wave hold candidates in scan order (index c = lane).  The
// fold of evaluate_motion_candidate (motion.cpp:111-149) over a step is:
//  * copy mode (best_mad < thr): keep the lexicographic minimum of
//    (mad, ssd), earlier wins exact ties;
//  * otherwise the first candidate with mad < thr is taken unconditionally and
//    switches to copy mode; without one, the minimum of (sad, ssd gated by
//    sad < 8192), earlier wins ties.
// evaluate_subpel_motion_candidate (motion.cpp:151-223) is the same with keys
// (mad) and (sad, only if sad < 8192).  Keys carry the index, so every key is
// unique and min() picks exactly the candidate the sequential loop ends on.
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t row0_min(uint32_t v) {  // min over lanes 0..15
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x122, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xF, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
}

__device__ __forceinline__ uint32_t key_copy(int mad, int ssd, int idx) {
  return ((uint32_t)min(mad, 65535) << 16) | ((uint32_t)min(ssd, 4095) << 4) | (uint32_t)idx;
}
__device__ __forceinline__ uint32_t key_sad(int sad, int ssd, int idx) {
  if (sad < kSadGate)
    return ((uint32_t)sad << 18) | ((uint32_t)min(ssd, 16383) << 4) | (uint32_t)idx;
  return 0x80000000u | ((uint32_t)min(sad, (1 << 27) - 1) << 4) | (uint32_t)idx;
}

// Integer step: this lane's candidate (valid, cx, cy, sad, mad); c = lane & 15.
__device__ __forceinline__ void select_int(Sel& s, bool valid, int cx, int cy, int sad, int mad,
                                           int px, int py, int thr, int lane) {
  const int c = lane & 15;
  const bool live = lane < 16 && valid;
  const int ssd = (cx - px) * (cx - px) + (cy - py) * (cy - py);
  const uint32_t fm = (uint32_t)__ballot(live && mad < thr);
  int w = -1;  // winning candidate, -1 = keep the state
  if (s.mad < thr || fm) {
    const int f = s.mad < thr ? -1 : (int)__builtin_ctz(fm);
    const uint32_t k = row0_min(live && c >= f ? key_copy(mad, ssd, c + 1) : 0xFFFFFFFFu);
    if (f >= 0) w = (int)(k & 15) - 1;  // candidate f is always in the running
    else if (k < key_copy(s.mad, s.ssd, 0)) w = (int)(k & 15) - 1;
  } else {
    const uint32_t k = row0_min(live ? key_sad(sad, ssd, c + 1) : 0xFFFFFFFFu);
    if (k < key_sad(s.sad, s.ssd, 0)) w = (int)(k & 15) - 1;
  }
  if (w >= 0) {
    s.bx = __builtin_amdgcn_readlane(cx, w);
    s.by = __builtin_amdgcn_readlane(cy, w);
    s.sad = __builtin_amdgcn_readlane(sad, w);
    s.ssd = __builtin_amdgcn_readlane(ssd, w);
    s.mad = __builtin_amdgcn_readlane(mad, w);
  }
}

// Sub-pel step: candidate c = 2*n + q (neighbour n, q = quarter).
__device__ __forceinline__ void select_sub(Sel& s, bool valid, int sad, int mad, int thr, int lane) {
  const int c = lane & 15;
  const bool live = lane < 16 && valid;
  const uint32_t fm = (uint32_t)__ballot(live && mad < thr);
  int w = -1;
  if (s.mad < thr || fm) {
    const int f = s.mad < thr ? -1 : (int)__builtin_ctz(fm);
    const uint32_t k = row0_min(live && c >= f ? (((uint32_t)min(mad, 65535) << 5) | (uint32_t)(c + 1))
                                               : 0xFFFFFFFFu);
    if (f >= 0) w = (int)(k & 31) - 1;
    else if (k < ((uint32_t)min(s.mad, 65535) << 5)) w = (int)(k & 31) - 1;
  } else {
    const uint32_t k =
        row0_min(live && sad < kSadGate ? (((uint32_t)sad << 5) | (uint32_t)(c + 1)) : 0xFFFFFFFFu);
    if (k < ((uint32_t)min(s.sad, 1 << 26) << 5)) w = (int)(k & 31) - 1;
  }
  if (w >= 0) {
    const int n = w >> 1, k9 = n < 4 ? n : n + 1;
    s.sp_en = 1;
    s.sp_amt = w & 1;
    s.sp_idx = frac_index(k9 % 3 - 1, k9 / 3 - 1);
    s.sad = __builtin_amdgcn_readlane(sad, w);
    s.mad = __builtin_amdgcn_readlane(mad, w);
  }
}

__device__ __forceinline__ bool in_frame(int x, int y, int wa, int ha) {
  return x >= 0 && x <= wa - kMB && y >= 0 && y <= ha - kMB;
}

__device__ __forceinline__ BlockDesc make_desc(const Sel& s, int px, int py, int thr, bool intra,
                                               int target) {
  BlockDesc d;
  uint32_t t = intra ? kIntra : 0u;
  if (s.bx != px || s.by != py || s.sp_en) t |= kMotion;
  if (s.mad < thr) t |= kCopy;
  d.block_type = t;
  d.prediction_target = (uint8_t)target;
  d.pad = 0;
  d.motion_x = (int16_t)(s.bx - px);
  d.motion_y = (int16_t)(s.by - py);
  d.sp_pred = (uint8_t)s.sp_en;
  d.sp_amount = (uint8_t)s.sp_amt;
  d.sp_index = (uint8_t)s.sp_idx;
  d.q_index = 0;
  d.variance = 0;
  return d;
}

// ---------------------------------------------------------------------------
// Inter search task (calculate_inter_prediction, motion.cpp:421-494): one
// workgroup searches macroblocks 4g..4g+3 of row r against reference offset
// `off`, one wave per macroblock, in the shared window.
// ---------------------------------------------------------------------------

// The window is staged in three parts, each when the previous frame is final
// over it.  The previous frame's deblock progress word of MB row k counts
// columns whose pixel rows 16k-3 .. 16k+12 are final (rows 16k+13..15 change
// again with row k+1's top edge, kernels.hip deblock_chunk).
//  * Level 1, window rows [0, 77) x columns [0, 112): frame rows py-32..py+44,
//    columns 64g-32..64g+79.  Needs progress of row r+2 at 64g+80.  It holds
//    every candidate with a vertical offset up to +29 (the first three steps
//    16 + 8 + 4 and more) whose columns stay inside.
//  * Level 2c, columns [112, 128) of those rows: progress of row r+2 at
//    64g+96 (one macroblock later), when a step of the right-hand macroblock
//    could reach it.
//  * Level 2r, window rows [77, 80): progress of row r+3 at 64g+96, only for a
//    vertical offset beyond +29.
// So a frame follows its predecessor at MB row r+2, 5-6 macroblocks ahead.
constexpr int kLvl1Rows = 77, kLvl1Cols = 112;

// Thread 0's value v, broadcast to the workgroup (two barriers).
__device__ __forceinline__ int wg_broadcast(volatile int* slot, int v) {
  if (threadIdx.x == 0) *slot = v;
  __syncthreads();
  const int r = *slot;
  __syncthreads();
  return r;
}

// The row's deblock (defined below), advanced while a helper waits.
struct DbLds;
struct DbState;
__device__ __forceinline__ bool deblock_chunk_ready(FA& a, int r, const DbState& st);
__device__ __forceinline__ void deblock_chunk(FA& a, int r, DbLds& D, DbState& st, bool known_ready = false);
__device__ __forceinline__ bool deblock_pending(FA& a, const DbState& st);

// Helper wait (whole workgroup): until the deblock progress of frame
// index-back (back = 1: the previous frame, 2: the one before) of MB row rr
// reaches need, running this row's ready deblock chunks meanwhile (kDeblock);
// then acquire what the progress word released.  Bounded like every wait (the
// error word ends it).
template <bool kDeblock = true>
__device__ __forceinline__ void helper_wait(FA& a, int back, int r, int rr, int need, DbLds& D, DbState& st,
                                            int* flag) {
  volatile int* vflag = flag;
  const uint64_t* pp = back == 1 ? a.prev_progress : a.prev2_progress;
  uint64_t t0 = 0;
  const uint64_t ta = acct_now();
  uint64_t tdb = 0;  // accounting: time in deblock chunks run here
  for (;;) {
    int d = 0;
    if (threadIdx.x == 0) {
      // the progress poll and the deblock readiness loads in flight together
      const uint64_t pv = pp ? progress_peer(a.sys, pp + rr) : ~0ull;
      const bool dbr = kDeblock && deblock_pending(a, st) && deblock_chunk_ready(a, r, st);
      if (a.inject && r == min(1, a.hmb - 1)) {  // test hook: this wait "times out" at once
        report_timeout(a, kWaitInjected, r, need, rr | (back << 16), pv);
        d = 1;
      } else if (pv >= tagged(a.epoch - back, need)) {
        d = 1;
      } else if (dbr) {
        d = 2;
      } else {  // nothing to do: back off
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (!t0) t0 = now;
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          d = 1;
        } else if (now - t0 > 200000000ull) {
          report_timeout(a, kWaitPrevProgress, r, need, rr | (back << 16), pv);
          d = 1;
        }
      }
    }
    d = wg_broadcast(vflag, d);
    if (d == 1) break;
    if (kDeblock && d == 2) {
      const uint64_t tb = acct_now();
      deblock_chunk(a, r, D, st, true);
      tdb += acct_now() - tb;
    }
  }
  if (threadIdx.x == 0) {  // the check used a relaxed load: acquire what it observed
    acquire_fence(a.sys);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  acct_add(a.acct, Acct::kHelperWait, acct_now() - ta - tdb);
}

struct InterLds {
  Window win;
  int need[4];
  int full;  // the whole window is final (staged at once)
  int lvl2[6][4];  // per step (16, 8, 4, 2, 1, sub-pel) and wave: level 2 wanted
  // the group's source macroblocks (raw int16: 16x16 luma, 8x8 U, 8x8 V per
  // wave), loaded once per group; the zero-MV SAD / MAD of the older
  // references, computed together at the group start
  alignas(16) int16_t src[4][384];
  int zsad[kMaxRing][4], zmad[kMaxRing][4];
};

// Wave w's source macroblock (4g + w, r) into L.src[w], row-major: luma
// 16 x 16, then U 8 x 8, then V 8 x 8; lanes 0..47 one 16-byte chunk each (a
// luma half row, a chroma row).  Only this wave reads it back (its LDS
// operations execute in order: no barrier).
__device__ __forceinline__ void group_source(FA& a, int r, int g, InterLds& L) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, x = 4 * g + wave;
  if (x >= a.wmb || lane >= 48) return;
  const PlaneSet in = planes(a.in);
  const int px = x * kMB, py = r * kMB;
  const int16_t* gsrc;
  if (lane < 32) {  // luma row lane >> 1, half lane & 1
    gsrc = in.y + (size_t)(py + (lane >> 1)) * a.wa + px + 8 * (lane & 1);
  } else {  // chroma: 16 chunks, U rows 0..7 then V rows 0..7
    const int k = lane - 32;
    gsrc = pick(in, 1 + (k >> 3)) + (size_t)((py >> 1) + (k & 7)) * (a.wa >> 1) + (px >> 1);
  }
  *(uint4*)&L.src[wave][8 * lane] = *(const uint4*)gsrc;
}

// Macroblock (x, r)'s source into dst (group_source's layout) by ONE LDS-DMA
// wave instruction of wave 0, lanes 0..47 (16 bytes each; an LDS-DMA writes
// dst + lane x 16).  The source planes do not change during a launch.  Lands
// behind wave 0's next vmcnt wait; readable by every wave after the barrier
// that follows it.
__device__ __forceinline__ void src_dma(FA& a, int x, int r, int16_t* dst) {
  const int lane = threadIdx.x;
  if (lane >= 48) return;
  const PlaneSet in = planes(a.in);
  const int px = x * kMB, py = r * kMB;
  const int16_t* gsrc = lane < 32 ? in.y + (size_t)(py + (lane >> 1)) * a.wa + px + 8 * (lane & 1)
                                  : pick(in, 1 + ((lane - 32) >> 3)) +
                                        (size_t)((py >> 1) + (lane & 7)) * (a.wa >> 1) + (px >> 1);
  __builtin_amdgcn_global_load_lds((const void*)gsrc, (lds_void*)dst, 16, 0, 0);
}

// This lane's Px6 slice (px_from_planes layout) and its SrcRow (load_src_rows
// layout, biased) of wave w's source macroblock, from L.src.
__device__ __forceinline__ Px6 src_px_lds(const InterLds& L, int wave) {
  const int l = threadIdx.x & 63;
  const int16_t* m = L.src[wave];
  Px6 p;
  const int16_t* y = &m[(l >> 2) * 16 + (l & 3) * 4];
  p.y0 = y[0], p.y1 = y[1], p.y2 = y[2], p.y3 = y[3];
  p.u = m[256 + (l >> 3) * 8 + (l & 7)];
  p.v = m[320 + (l >> 3) * 8 + (l & 7)];
  return p;
}
__device__ __forceinline__ SrcRow src_rows_lds(const InterLds& L, int wave, int i) {
  const uint32_t* m = (const uint32_t*)L.src[wave];
  SrcRow s;
#pragma unroll
  for (int k = 0; k < 8; k++) s.y[k] = m[i * 8 + k] ^ 0x80008000u;
  const int co = (i >> 1) * 4 + (i & 1) * 2;  // dwords: row i>>1 of 8 px = 4 dwords, half i&1
  s.u[0] = m[128 + co] ^ 0x80008000u, s.u[1] = m[128 + co + 1] ^ 0x80008000u;
  s.v[0] = m[160 + co] ^ 0x80008000u, s.v[1] = m[160 + co + 1] ^ 0x80008000u;
  return s;
}

// The zero-MV SAD / MAD of references 2..nref for the group (all loads of a
// wave issued together), into L.zsad / L.zmad.  After the wait for frame
// index-2's level-1 window (which covers the zero-MV block).
__device__ __forceinline__ void zero_mv_older(FA& a, int r, int g, InterLds& L) {
  const int wave = threadIdx.x >> 6, x = 4 * g + wave;
  acct_add(a.acct, Acct::kZeroMvBytes, 768ull * (a.nref - 1) * (uint64_t)min(4, a.wmb - 4 * g));
  if (x >= a.wmb) return;
  const int px = x * kMB, py = r * kMB;
  const Px6 src = src_px_lds(L, wave);
  Px6 ref[kMaxRing - 1];
#pragma unroll
  for (int off = 2; off < kMaxRing; off++)
    if (off <= a.nref) ref[off - 1] = px_from_planes(RECON_AT(a, off), a.wa, px, py);
#pragma unroll
  for (int off = 2; off < kMaxRing; off++) {
    if (off > a.nref) break;
    int sad, mad;
    sad_mad(src, ref[off - 1], sad, mad);
    if ((threadIdx.x & 63) == 0) L.zsad[off][wave] = sad, L.zmad[off][wave] = mad;
  }
}

// Need of the group's level-1 / level-2 windows: (MB row whose deblock
// progress counts, luma columns).
__device__ __forceinline__ int inter_need_cols(FA& a, int g, int level) {
  return min(64 * g + (level == 1 ? 80 : 96), a.wa);
}

// Reference offset `off` of group g of row r: the tagged records of the
// group's macroblocks are stored and left in flight (the coder polls them).
__device__ __forceinline__ void inter_task(FA& a0, int r, int g, int off, InterLds& L, DbLds& D, DbState& st,
                                           int* flag, uint64_t* is) {
  FA& a = *opaque_view(&a0);
  const int wave = uni(threadIdx.x >> 6);  // scalar: the acceptance replay runs on SGPRs
  const int x = 4 * g + wave;
  const bool valid = x < a.wmb;
  const int px = x * kMB, py = r * kMB, mb = r * a.wmb + x;
  const int mbs = a.wmb * a.hmb;
  const int thr = (a.quality >> 2) + 1;
  const PlaneSet ref = RECON_AT(a, off);
  Sel s;
  Px6 src;
  s.bx = px;
  s.by = py;
  s.ssd = INT32_MAX;
  s.sp_idx = s.sp_amt = s.sp_en = 0;
  s.sad = s.mad = 0;
  SrcRow srow;  // biased source rows of this lane's group slot (integer steps)
  const int ox = 4 * g * kMB - 32, oy = py - 32;  // window origin
  if (valid) {  // the source from the group's LDS copy
    src = src_px_lds(L, wave);
    srow = src_rows_lds(L, wave, threadIdx.x & 15);
    if (off >= 2) {  // zero-MV computed at the group start
      s.sad = L.zsad[off][wave], s.mad = L.zmad[off][wave];
    } else {  // zero-MV candidate straight from the planes
      sad_mad(src, px_from_planes(ref, a.wa, px, py), s.sad, s.mad);
    }
  }
  const bool need = valid && s.mad >= thr && !(CAIRO_ATTR_SKIP & 8);
  if ((threadIdx.x & 63) == 0) L.need[wave] = need;
  if (threadIdx.x == 0) {
    // Is the reference already final over the whole window (level 2 too)?
    // Always, in practice, for the older references (frame index-2 runs far
    // ahead): then the window is staged in one go and the steps skip the
    // per-step level-2 decisions and their barriers.
    const int back = off == 1 ? 1 : 2;
    const uint64_t* pp = back == 1 ? a.prev_progress : a.prev2_progress;
    const uint64_t want = tagged(a.epoch - back, inter_need_cols(a, g, 2));
    // both words loaded before either is tested (one round trip)
    const uint64_t w3 = pp ? progress_peer(a.sys, pp + min(r + 3, a.hmb - 1)) : 0;
    const uint64_t w2 = pp ? progress_peer(a.sys, pp + min(r + 2, a.hmb - 1)) : 0;
    const int full = !pp || ((w3 >= want) & (w2 >= want));
    if (full && pp) {  // acquire what the progress words released (the loads below follow the barrier)
      acquire_fence(a.sys);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    L.full = full;
  }
  __syncthreads();
  if (is && off == 1) is[3] = __builtin_amdgcn_s_memrealtime();
  acct_add(a.acct, Acct::kInterTasks, 1);
  acct_add(a.acct, Acct::kZeroMvBytes, (off == 1 ? 768ull : 0ull) * (uint64_t)min(4, a.wmb - 4 * g));
  if (L.need[0] | L.need[1] | L.need[2] | L.need[3]) {
    const bool full = L.full != 0;  // workgroup-uniform
    acct_add(a.acct, Acct::kSearchedTasks, 1);
    acct_window(a.acct, 0, full ? kWinL : kLvl1Rows, 0, full ? kWinLW : kLvl1Cols);
    stage_window(L.win, ref, a.wa, a.ha, ox, oy, 0, full ? kWinL : kLvl1Rows, 0, full ? kWinLW : kLvl1Cols);
    __syncthreads();
    if (is && off == 1) is[4] = __builtin_amdgcn_s_memrealtime();
    bool lvl2c = full, lvl2r = full;  // workgroup-uniform
    bool lvl2_open = true;  // workgroup-uniform: some wave's search may still leave level 1
    // steps 16, 8, 4, 2, 1, then the sub-pel step (reach 1 around the best)
    for (int si = 0; si < 6; si++) {
      const int step = si < 5 ? kRadius >> si : 1;
      if (!lvl2r && lvl2_open) {
        // this wave's candidates of the step reach window rows by+step-oy+15
        // and columns bx+step-ox+15 at most; those of every remaining step
        // (reach rem = step + step/2 + ... + 1 + the sub-pel 1) no further
        // than by+rem-oy+15: once no wave can leave level 1 any more, the
        // waves run their remaining steps without workgroup barriers
        const int rem = si < 5 ? 2 * step : 1;
        const int want = need ? (s.by + step - oy > kLvl1Rows - kMB) * 2 + (!lvl2c && s.bx + step - ox > kLvl1Cols - kMB)
                              : 0;
        const int may = need && (s.by + rem - oy > kLvl1Rows - kMB || (!lvl2c && s.bx + rem - ox > kLvl1Cols - kMB));
        if ((threadIdx.x & 63) == 0) L.lvl2[si][wave] = want | (may << 2);
        __syncthreads();
        const int m4 = L.lvl2[si][0] | L.lvl2[si][1] | L.lvl2[si][2] | L.lvl2[si][3];
        const int m = m4 & 3;
        lvl2_open = (m4 >> 2) != 0;
        if (m) {
          if (is) is[5] = __builtin_amdgcn_s_memrealtime();
          // (no deblock meanwhile: rare, and its inputs' registers would spill
          // the search state live here)
          helper_wait<false>(a, off == 1 ? 1 : 2, r, min(r + ((m & 2) ? 3 : 2), a.hmb - 1), inter_need_cols(a, g, 2),
                             D, st, flag);
          if (m & 2) stage_window(L.win, ref, a.wa, a.ha, ox, oy, kLvl1Rows, kWinL, 0, kWinLW);
          if (!lvl2c) stage_window(L.win, ref, a.wa, a.ha, ox, oy, 0, kLvl1Rows, kLvl1Cols, kWinLW);
          if (m & 2) acct_window(a.acct, kLvl1Rows, kWinL, 0, kWinLW);
          if (!lvl2c) acct_window(a.acct, 0, kLvl1Rows, kLvl1Cols, kWinLW);
          __syncthreads();
          if (is) is[6] = __builtin_amdgcn_s_memrealtime(), is[7] += (m & 2) ? 0x10000 : 1;
          lvl2c = true;
          lvl2r = (m & 2) != 0;
        }
      }
      if (is && off == 1 && (si == 1 || si == 5)) is[si == 1 ? 8 : 9] = __builtin_amdgcn_s_memrealtime();
      if (!need) continue;
      // The 9 (or 16) candidates of a step are independent: evaluate them all
      // first (their wave reductions overlap), then replay the sequential
      // acceptance in scan order (j-outer, i-inner, motion.cpp:225-275) on
      // the wave-uniform results.  An out-of-frame candidate is evaluated at
      // the current best and not offered.
      if (si < 5) {
        // The 3x3's centre (candidate 4 in scan order) is the current best:
        // its SAD and MAD are the state's (same position, same source), so only
        // the 8 others are evaluated, in 2 passes of four 16-lane groups:
        // pass p, group g -> candidate 4p + g, skipping 4.  Lane c < 9 then
        // collects candidate c (ds_bpermute from its group's first lane; the
        // centre from the state) and select_int replays the sequential
        // acceptance on lanes 0..15 (the centre can still win there when an
        // earlier candidate of the step was taken first).
        const int bx = s.bx, by = s.by;
        const int lane = threadIdx.x & 63, gi = lane & 15, grp = lane >> 4;
        const int my_pass = gi < 4 ? 0 : 1, my_grp = gi < 4 ? gi : gi - 5;  // where candidate gi is evaluated
        int sadv = s.sad, madv = s.mad;  // lane 4: the centre
#pragma unroll
        for (int pass = 0; pass < 2; pass++) {
          const int c = 4 * pass + grp + (pass > 0);  // 0..3, then 5..8
          const int cx = bx + (c % 3 - 1) * step, cy = by + (c / 3 - 1) * step;
          const bool ok = in_frame(cx, cy, a.wa, a.ha);
          int sad, mad;
          inter_cand_row(L.win, (ok ? cx : bx) - ox, (ok ? cy : by) - oy, gi, srow, thr, sad, mad);
          const int from = (16 * (my_grp & 3)) << 2;
          const int vs = __builtin_amdgcn_ds_bpermute(from, sad), vm = __builtin_amdgcn_ds_bpermute(from, mad);
          if (my_pass == pass && gi != 4) sadv = vs, madv = vm;
        }
        {
          const int cx = bx + (gi % 3 - 1) * step, cy = by + (gi / 3 - 1) * step;
          select_int(s, gi < 9 && in_frame(cx, cy, a.wa, a.ha), cx, cy, sadv, madv, px, py, thr, lane);
        }
      } else {
        // Sub-pel: half then quarter lerp toward each of the 8 neighbours.
        // lerps and differences on the window's biased values (lerp_half_bb):
        // the source biased once, 3 * best once
        const Px6 best = px_from_window_b(L.win, s.bx - ox, s.by - oy);
        s.sp_idx = s.sp_amt = s.sp_en = 0;
        const int bx = s.bx, by = s.by;
        const uint32_t sb0 = src.y0 + 0x8000, sb1 = src.y1 + 0x8000, sb2 = src.y2 + 0x8000, sb3 = src.y3 + 0x8000,
                       sbu = src.u + 0x8000, sbv = src.v + 0x8000;
        const uint32_t b30 = 3 * best.y0, b31 = 3 * best.y1, b32 = 3 * best.y2, b33 = 3 * best.y3, b3u = 3 * best.u,
                       b3v = 3 * best.v;
        // accepted in the order they are evaluated (neighbour-major, half
        // then quarter), each as soon as its sums exist: no array of 16
        // results stays live (it pushed the engine into scratch spills).
        // accept_sub (motion.cpp:151-223) needs the MAD only through
        // "mad < limit" (copy mode: the best MAD, else thr), which is "no
        // lane's maximum reaches limit": one ballot instead of a wave-wide
        // max; the exact MAD (and, in copy mode, the SAD) is reduced only for
        // an accepted candidate.
#pragma unroll
        for (int n = 0; n < 8; n++) {
          const int k9 = n < 4 ? n : n + 1, i = k9 % 3 - 1, j = k9 / 3 - 1, tx = bx + i, ty = by + j;
          const bool ok = in_frame(tx, ty, a.wa, a.ha);
          if (!ok) continue;  // (wave-uniform) out of frame: not offered
          const Px6 nb = px_from_window_b(L.win, tx - ox, ty - oy);
          const int idx = frac_index(i, j);
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const uint32_t d0 = absdiff_b(sb0, q ? lerp_quarter_bb3(b30, nb.y0) : lerp_half_bb(best.y0, nb.y0)),
                           d1 = absdiff_b(sb1, q ? lerp_quarter_bb3(b31, nb.y1) : lerp_half_bb(best.y1, nb.y1)),
                           d2 = absdiff_b(sb2, q ? lerp_quarter_bb3(b32, nb.y2) : lerp_half_bb(best.y2, nb.y2)),
                           d3 = absdiff_b(sb3, q ? lerp_quarter_bb3(b33, nb.y3) : lerp_half_bb(best.y3, nb.y3)),
                           du = absdiff_b(sbu, q ? lerp_quarter_bb3(b3u, nb.u) : lerp_half_bb(best.u, nb.u)),
                           dv = absdiff_b(sbv, q ? lerp_quarter_bb3(b3v, nb.v) : lerp_half_bb(best.v, nb.v));
            const int lsum = (int)(d0 + d1 + d2 + d3);
            const int lmax = (int)max(max(max(d0, d1), d2), max(max(d3, du), dv));
            const bool copy = s.mad < thr;
            const bool mad_lt = __ballot(lmax >= (copy ? s.mad : thr)) == 0;
            int sad = 0;
            bool acc;
            if (copy) {
              acc = mad_lt;
            } else {
              sad = wave_sum(lsum);
              acc = (sad < s.sad && sad < kSadGate) || mad_lt;
            }
            if (acc) {
              s.sp_en = 1;
              s.sp_amt = q;
              s.sp_idx = idx;
              s.sad = copy ? wave_sum(lsum) : sad;
              s.mad = wave_max(lmax);
            }
          }
        }
      }
    }
  }
  if (is && off == 1) is[10] = __builtin_amdgcn_s_memrealtime();
  if (valid && (threadIdx.x & 63) == 0) {
    // two tagged granules (kernels.h pack_inter_desc): the coder polls them,
    // so nothing waits for these stores
    const BlockDesc d = make_desc(s, px, py, thr, false, off);
    uint64_t* rec = (uint64_t*)&a.inter_desc[(off - 1) * mbs + mb];
    const uint64_t tag = (uint64_t)a.epoch << 32;
    gran_st(rec, tag | pack_inter_desc(d));
    gran_st(rec + 1, tag | (uint32_t)s.sad);
  }
  // the next task rewrites the window: every wave is done reading it (its
  // LDS reads returned); the records' stores stay in flight (each one waits
  // about 3.5 us for its write-through acknowledgement)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------
// Transform / quantization on a macroblock held block-major in LDS:
// element (b, r, c) at b*64 + r*8 + c; b = 0..3 luma quadrants TL TR BL BR,
// 4 = U, 5 = V (transform.cpp:264-594, quantize.cpp:79-379).
// ---------------------------------------------------------------------------

constexpr int kMBElems = 384;
typedef short int8v __attribute__((ext_vector_type(8)));

// Pixel coordinates of element e of the macroblock whose luma origin is (x, y):
// plane 0/1/2 and (px, py) inside that plane.
__device__ __forceinline__ void elem_coords(int e, int x, int y, int& plane, int& ex, int& ey) {
  int b = e >> 6, r = (e >> 3) & 7, c = e & 7;
  if (b < 4) {
    plane = 0;
    ex = x + (b & 1) * 8 + c;
    ey = y + (b >> 1) * 8 + r;
  } else {
    plane = b - 3;
    ex = (x >> 1) + c;
    ey = (y >> 1) + r;
  }
}

// One 8x8 block per wave, one element per lane (lane = r*8 + c).  LDS scratch
// a/b (64 int16 each) carry the passes; the wave's LDS operations execute in
// order, so no workgroup barrier is needed.

__device__ __forceinline__ int8v load_row8(const int16_t* p) {  // 8 int16, 16-B aligned
  return *(const int8v*)p;
}

// transform_8x8 (transform.cpp:264-301): rows, int16 scratch, then columns.
// x = this lane's residual (r, c); returns its coefficient (r, c).
__device__ __forceinline__ int fdct_lane(int16_t* sa, int16_t* sb, int lane, int16_t x) {
  const int r8 = lane >> 3, c8 = lane & 7;
  sa[lane] = x;
  __builtin_amdgcn_wave_barrier();
  {
    const int8v row = load_row8(&sa[r8 * 8]), lut = load_row8(&sLut8[c8 * 8]);
    int t = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) t += row[k] * lut[k];
    t = c8 == 0 ? (t * 45) / 128 : t / 2;
    sb[c8 * 8 + r8] = (int16_t)rdiv(t, 128);  // transposed
  }
  __builtin_amdgcn_wave_barrier();
  const int8v col = load_row8(&sb[c8 * 8]), lut = load_row8(&sLut8[r8 * 8]);  // column c8 of the row pass
  int t = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) t += col[k] * lut[k];
  t = r8 == 0 ? (t * 45) / 128 : t / 2;
  return (int16_t)rdiv(t, 128);
}

// inverse_transform_8x8 (transform.cpp:330-366): columns then rows, per-term
// truncation.  d = this lane's dequantized coefficient (r, c); returns the
// inverse-transformed sample (r, c) before the prediction is added.
__device__ __forceinline__ int idct_lane(int16_t* sa, int16_t* sb, int lane, int16_t d) {
  const int r8 = lane >> 3, c8 = lane & 7;
  sa[c8 * 8 + r8] = d;  // transposed: row c8 of sa = column c8
  __builtin_amdgcn_wave_barrier();
  {
    const int8v col = load_row8(&sa[c8 * 8]), lut = load_row8(&sLut8T[r8 * 8]);  // lut[k] = sLut8[k * 8 + r8]
    int t = ((col[0] * lut[0]) * 45) / 128;
#pragma unroll
    for (int k = 1; k < 8; k++) t += (col[k] * lut[k]) / 2;
    sb[r8 * 8 + c8] = (int16_t)rdiv(t, 128);
  }
  __builtin_amdgcn_wave_barrier();
  const int8v row = load_row8(&sb[r8 * 8]), lut = load_row8(&sLut8T[c8 * 8]);
  int t = ((row[0] * lut[0]) * 45) / 128;
#pragma unroll
  for (int k = 1; k < 8; k++) t += (row[k] * lut[k]) / 2;
  return rdiv(t, 128);
}

// VAQ over the 16x16 luma coefficients (analysis.h:176-198, quantize.cpp:60-77):
// wave w holds luma quadrant w; the first coefficient of quadrant 0 is skipped;
// wrapping int32 arithmetic.  Contains one workgroup barrier; returns
// (qp, variance2) uniform across the workgroup.
__device__ __forceinline__ int vaq_mb(int32_t* red, int wave, int lane, int coef, int quality,
                                      int32_t* var_out) {
  const bool use = !(wave == 0 && lane == 0) && coef != 0;
  const int ws = wave_sum(use ? coef : 0), wq = wave_sum(use ? coef * coef : 0),
            wc = wave_sum(use ? 1 : 0);
  if (lane == 0) red[wave] = ws, red[4 + wave] = wq, red[8 + wave] = wc;
  __syncthreads();
  const uint32_t S = (uint32_t)red[0] + (uint32_t)red[1] + (uint32_t)red[2] + (uint32_t)red[3];
  const uint32_t Q = (uint32_t)red[4] + (uint32_t)red[5] + (uint32_t)red[6] + (uint32_t)red[7];
  const int32_t C = red[8] + red[9] + red[10] + red[11];
  const int32_t v2 = C > 0 ? (int32_t)(Q - (uint32_t)rdiv((int32_t)(S * S), C)) : 0;
  *var_out = v2;
  return (int)vaq_from_variance((uint32_t)quality, v2);
}

// quantize_macroblock (quantize.cpp:357-367): element-wise.
// The divisions by reciprocal (rdiv_m; qp is 1..31, |c| < 2^15, the
// divisors at most 62: every quotient exact).
__device__ __forceinline__ int16_t quant_elem(int e, int32_t c, int qp, bool intra_path) {
  int b = e >> 6, k = e & 63;
  if (intra_path) {
    if (k == 0)
      return (int16_t)(b < 4 ? rdiv_m(c, luma_dc_scale(qp), sMagDcL[qp]) : rdiv_m(c, chroma_dc_scale(qp), sMagDcC[qp]));
    return (int16_t)rdiv_m(rdiv_m(c * kQScale, sQmIntra[k], sMagQmIntra[k]), qp << 1, sMag2qp[qp]);
  }
  int16_t qf = (int16_t)rdiv_m(c * kQScale, sQmInter[k], sMagQmInter[k]);
  return (int16_t)rdiv_m(qf - sign16(qf) * qp, qp << 1, sMag2qp[qp]);
}
// inverse_quantize_macroblock (quantize.cpp:369-379): element-wise.
__device__ __forceinline__ int16_t dequant_elem(int e, int32_t v, int qp, bool intra_path) {
  int b = e >> 6, k = e & 63;
  if (intra_path) {
    if (k == 0) return (int16_t)(v * (b < 4 ? luma_dc_scale(qp) : chroma_dc_scale(qp)));
    return (int16_t)((2 * v * sQmIntra[k] * qp) / kQScale);
  }
  return (int16_t)(((2 * v) * sQmInter[k] * qp) / kQScale);
}

// ---------------------------------------------------------------------------
// Deblocking (deblock.cpp:201-284), fused into the row workers of K2.  The
// reference filters in place in raster order: per 8-row band, for each 8-px
// unit x the horizontal edge H(x) (top of the band) then the vertical edge V(x)
// (left of the unit).  H(x) touches only columns x..x+7 (rows y-3..y+2) and
// V(x) columns x-3..x+2, so within a band every H is independent of every V
// but its own and its left neighbour's: all H edges of a band, then all V
// edges, is the raster result.  Band b+1's H edges read rows that band b's V
// edges wrote, so bands run in order.  MB row r owns luma bands 2r, 2r+1 and
// chroma band r; it is filtered by the workgroup that coded it, after row r-1
// is fully filtered, while later rows keep coding: they read the current
// frame only through granules (pre-deblock values), and their stale row below
// has not been touched yet.
// ---------------------------------------------------------------------------

// deblock_filter_values on 8 samples v[0..7] = p3 p2 p1 p0 q0 q1 q2 q3, in registers.
__device__ __forceinline__ void dfilter_reg(int* v, int qp, int strength, bool luma) {
  const int p3 = v[0], p2 = v[1], p1 = v[2], p0 = v[3], q0 = v[4], q1 = v[5], q2 = v[6], q3 = v[7];
  const int16_t dpq = (int16_t)iabs(p0 - q0), dp = (int16_t)iabs(p1 - p0), dq = (int16_t)iabs(q1 - q0);
  if ((CAIRO_ATTR_SKIP & 32) || strength == 0 || dpq >= sAlpha[qp] || dp >= sBeta[qp] || dq >= sBeta[qp]) return;
  if (strength == 2) {
    v[3] = (int16_t)rdiv(p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1, 8);
    v[2] = (int16_t)rdiv(p2 + p1 + p0 + q0, 4);
    v[4] = (int16_t)rdiv(p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2, 8);
    v[5] = (int16_t)rdiv(p0 + q0 + q1 + q2, 4);
    if (luma) {
      v[1] = (int16_t)rdiv(2 * p3 + 3 * p2 + p1 + p0 + q0, 8);
      v[6] = (int16_t)rdiv(2 * q3 + 3 * q2 + q1 + q0 + p0, 8);
    }
  } else {
    v[3] = (int16_t)rdiv(((q0 + p0) * 4) + p1 - q1, 8);
    v[4] = (int16_t)rdiv(((q0 + p0) * 4) + q1 - p1, 8);
    if (luma) {
      v[2] = (int16_t)rdiv((p2 * 4) + (p0 * 2) + (q0 * 2), 8);
      v[5] = (int16_t)rdiv((q2 * 4) + (q0 * 2) + (p0 * 2), 8);
    }
  }
}

// Edge strength and qp (compute_deblock_strength / compute_average_qp,
// deblock.cpp:49-79) from the LDS row cache: entry = copy << 8 | q_index.
__device__ __forceinline__ int edge_strength_q(int l, int r, int& qp) {
  const bool cl = l >> 8, cr = r >> 8;
  const int ql = l & 0xFF, qr = r & 0xFF;
  qp = (!cl && !cr) ? ((ql + qr) >> 1) : (!cl ? ql : (!cr ? qr : 0));
  return (cl && cr) ? 0 : ((cl != cr) ? 1 : 2);
}

// Column-granular deblock of MB row r (whole workgroup), trailing the row
// coder one chunk of 2^db_shift luma columns (whole macroblocks) at a time
// (FrameArgs::db_shift, make_frame_view): each chunk costs
// a granule round trip, a write-through drain and a few barriers, latencies
// that a wider chunk amortizes (16 / 32 / 64 / 80 / 96 columns:
// 4784 / 4940 / 5040 / 4986 / 4968 Mpix/s at 4K).  Inputs: row r's
// pre-deblock pixels and block info from its granules; the 4 pixel rows above
// (row r-1's final output, sc1) once row r-1's progress word passes the chunk.
// All filtering happens in a circular LDS tile (luma rows 16r-4..16r+15 x 128
// columns, chroma rows 8r-4..8r+7 x 64).  Per chunk [c0, c1):
//   band A (luma band 2r, chroma band r): H edges of [c0, c1), then V edges
//     of the units in [c0, c1);
//   band B (luma band 2r+1): its H edge at column x reads band A rows that
//     band A's V edges at units <= x+8 rewrite, so H runs up to c1-8 and its
//     V edges (which read H's columns u-4..u+3) up to unit c1-16;
// then every column no later edge touches (< c1-12) is written out with sc1
// stores and published as the row's progress.  Row r needs row r-1 one
// chunk ahead; a chunk runs only once its inputs are present (the helper
// interleaves it with the inter search), so a wide chunk delays the row's
// progress but never stalls the helper.
// The chunk width is per frame (FrameArgs::db_shift, make_frame_view), by
// frame width.
constexpr int kDbChunk = 64;  // the widest chunk: luma columns (tile width, info table, arrays)
constexpr int kDbMBs = kDbChunk / 16;
__device__ __forceinline__ int db_chunks(const FA& a) { return (a.wa + (1 << a.db_shift) - 1) >> a.db_shift; }
constexpr int kDbLW = 128, kDbLP = 130;  // luma tile columns (circular), pitch
constexpr int kDbCW = 64, kDbCP = 66;    // chroma

struct DbLds {
  int16_t y[20 * kDbLP];      // rows 16r-4 .. 16r+15
  int16_t u[12 * kDbCP];      // rows 8r-4 .. 8r+7
  int16_t v[12 * kDbCP];
  int16_t info[2][8];         // (copy << 8 | q_index) of MB rows r-1 (0), r (1), column & 7
};

__device__ __forceinline__ int16_t* db_px(DbLds& D, int pl, int row, int col) {
  if (pl == 0) return &D.y[row * kDbLP + (col & (kDbLW - 1))];
  return &(pl == 1 ? D.u : D.v)[row * kDbCP + (col & (kDbCW - 1))];
}

// One 8-sample line through an edge, filtered in the tile.  Horizontal edge
// (vertical line): samples at (row0 + k, col); vertical edge: (row0, col0 + k).
__device__ __forceinline__ void db_line(DbLds& D, int pl, bool vert_line, int row0, int col0, int lq,
                                        int rq) {
  int qp;
  const int st = edge_strength_q(lq, rq, qp);
  if (!st) return;
  int v[8], w[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    v[k] = w[k] = *db_px(D, pl, vert_line ? row0 + k : row0, vert_line ? col0 : col0 + k);
  dfilter_reg(w, qp, st, pl == 0);
#pragma unroll
  for (int k = 1; k < 7; k++)
    if (w[k] != v[k]) *db_px(D, pl, vert_line ? row0 + k : row0, vert_line ? col0 : col0 + k) = (int16_t)w[k];
}

__device__ __forceinline__ const uint64_t* gran_mb(FA& a, int mbx, int mby) {
  return a.granules + (size_t)(mby * a.wmb + mbx) * kGranuleStride;
}

// Deblock progress of one MB row: next chunk, columns written, band B's next
// H column and next V unit.
struct DbState {
  int k, w0, hb0, vb0;
  uint64_t busy = 0;  // diagnostic: time in deblock_chunk (thread 0, 10 ns ticks; only with stamps)
};

// Are chunk st.k's inputs present (row r-1's progress, this row's granules)?
// Evaluated by thread 0 only.
__device__ __forceinline__ bool deblock_pending(FA& a, const DbState& st) {
  return st.k < db_chunks(a);
}

__device__ __forceinline__ bool deblock_chunk_ready(FA& a, int r, const DbState& st) {
  const int c1 = min((st.k + 1) << a.db_shift, a.wa);
  // Row r-1's progress and the info granule of the chunk's last macroblock
  // (stored last; the row is coded left to right), both loads issued before
  // either is tested: one fabric round trip, not two.
  const uint64_t p = r > 0 ? progress_at(&a.progress[r - 1]) : ~0ull;
  const uint64_t g = gran_ld(gran_mb(a, (c1 - 1) >> 4, r) + kGranulesPerMB);
  return (p >= tagged(a.epoch, c1)) & ((uint32_t)(g >> 32) == a.epoch);
}

// Deblock chunk st.k of MB row r (whole workgroup; waits for its inputs, or
// known_ready: deblock_chunk_ready said so).
__device__ __forceinline__ void deblock_chunk(FA& a0, int r, DbLds& D, DbState& st, bool known_ready) {
  FA& a = *opaque_view(&a0);
  const int tid = threadIdx.x;
  const uint64_t tb = a.stamps && tid == 0 ? __builtin_amdgcn_s_memrealtime() : 0;
  const uint64_t ta = acct_now();
  const PlaneSet cs = planes(a.recon[0]);
  const int cw = a.wa >> 1;
  const int y0 = 16 * r - 4, c0y = 8 * r - 4;  // tile origins (pixel rows)
  const int nch = db_chunks(a);
  uint64_t* prog = a.progress;
  const uint64_t above = tagged(a.epoch, 0);
  int& w0 = st.w0;
  int& hb0 = st.hb0;
  int& vb0 = st.vb0;
  {
    const int k = st.k;
    const int c0 = k << a.db_shift, c1 = min(c0 + (1 << a.db_shift), a.wa);
    const bool last = k == nch - 1;
    // ---- inputs of chunk k: waves 0-2 the granules of its macroblocks;
    //      wave 3 polls row r-1's progress (rows above final through column
    //      c1), then loads the block info and those 4 rows ----
    const int hb1 = last ? a.wa : c1 - 8, vb1 = last ? a.wa : c1 - 8;
    {
      const int m0 = c0 >> 4, nmb = (c1 - c0 + 15) >> 4;  // 1 to kDbMBs macroblocks
      if (tid < kGranulesPerMB) {
        uint64_t g[kDbMBs];
#pragma unroll
        for (int q = 0; q < kDbMBs; q++)  // all loads issued before the first settles
          if (q < nmb) g[q] = gran_ld(gran_mb(a, m0 + q, r) + tid);
#pragma unroll
        for (int q = 0; q < kDbMBs; q++) {
          if (q >= nmb) break;
          const int m = m0 + q;
          const uint32_t d = gran_settle(a, gran_mb(a, m, r) + tid, g[q], r);
          int pl, row, col;
          if (tid < 128) {
            pl = 0, row = 4 + (tid >> 3), col = m * 16 + 2 * (tid & 7);
          } else {
            const int u = tid - 128;
            pl = 1 + (u >> 5), row = 4 + ((u & 31) >> 2), col = m * 8 + 2 * (u & 3);
          }
          int16_t* p = db_px(D, pl, row, col);
          p[0] = (int16_t)(d & 0xFFFF);
          p[1] = (int16_t)(d >> 16);
        }
      } else {  // wave 3 (uniform loop: every lane reads the same word)
        if (r > 0 && !known_ready && uni((int)(progress_at(&prog[r - 1]) < (above | (uint32_t)c1)))) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (uni((int)(progress_at(&prog[r - 1]) < (above | (uint32_t)c1)))) {
            if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
              if (tid == kGranulesPerMB)
                report_timeout(a, kWaitRowAbove, r, c1, r - 1, progress_at(&prog[r - 1]));
              break;
            }
          }
        }
        const int t3 = tid - kGranulesPerMB;  // 0..63
        if (t3 < 2 * nmb) {  // block info of rows r-1 (0) and r (1), per macroblock
          const int row = r - 1 + (t3 & 1), m = m0 + (t3 >> 1);
          int e = 0;
          if (row >= 0) {
            const uint64_t* gp = gran_mb(a, m, row) + kGranulesPerMB;
            e = (int)gran_settle(a, gp, gran_ld(gp), r);
          }
          D.info[t3 & 1][m & 7] = (int16_t)e;
        } else if (r > 0) {  // 4 final rows above: luma 4 x (c1-c0)/2 dwords, chroma 2 x 4 x (c1-c0)/4 (sc1)
          const int nlw = (c1 - c0) >> 1, ncw = (c1 - c0) >> 2;
          // index space: a whole chunk's dwords per row (luma 2^(s-1), chroma
          // 2^(s-2)), so that row and column are shifts
          const int s1 = a.db_shift - 1, s2 = a.db_shift - 2, nall = 8 << s1;
          // every load of this lane issued before the first LDS store: one
          // fabric round trip, not one per load (nall <= 256 dwords over >= 56
          // lanes: at most kAbove each)
          constexpr int kAbove = (8 << (6 - 1)) / (64 - 2 * kDbMBs) + 1;
          uint32_t v[kAbove];
          int16_t* dst[kAbove];
          for (int i0 = t3 - 2 * nmb; i0 < nall; i0 += kAbove * (64 - 2 * nmb)) {  // one pass when batched
#pragma unroll
          for (int u = 0; u < kAbove; u++) {
            const int i = i0 + u * (64 - 2 * nmb);
            dst[u] = nullptr;
            if (i >= nall) continue;
            int pl, row, col;
            const int16_t* g;
            if (i < (4 << s1)) {
              const int d = i & ((1 << s1) - 1);
              if (d >= nlw) continue;
              pl = 0, row = i >> s1, col = c0 + 2 * d;
              g = cs.y + (size_t)(y0 + row) * a.wa + col;
            } else {
              const int j = i - (4 << s1), pj = j >> (s2 + 2), jj = j & ((4 << s2) - 1), d = jj & ((1 << s2) - 1);
              if (d >= ncw) continue;
              pl = 1 + pj, row = jj >> s2, col = (c0 >> 1) + 2 * d;
              g = pick(cs, 1 + pj) + (size_t)(c0y + row) * cw + col;
            }
            v[u] = __hip_atomic_load((const __attribute__((address_space(1))) uint32_t*)g, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            dst[u] = db_px(D, pl, row, col);
          }
#pragma unroll
          for (int u = 0; u < kAbove; u++)
            if (dst[u]) {
              dst[u][0] = (int16_t)(v[u] & 0xFFFF);
              dst[u][1] = (int16_t)(v[u] >> 16);
            }
          }
        }
      }
    }
    __syncthreads();
    const uint64_t td1 = acct_now();
    // ---- the filters, in four dependent phases (band A H edges, band A V
    //      edges, band B H, band B V); the lines of one phase are disjoint.
    //      All in wave 0, whose LDS accesses execute in order (no workgroup
    //      barrier between the phases; spreading a 64-column chunk's phases
    //      over the four waves with barriers was 0.3 % slower at 4K,
    //      profiles/r04/ab_4k_s.txt, ab_4k_t.txt) ----
    {
      constexpr int nthr = 64;
      const bool part = tid < nthr;
      const int ls = a.db_shift, kL = 1 << ls, kC = kL >> 1;  // luma / chroma columns of a whole chunk
      // band A H edges of [c0, c1): luma kL columns, then chroma 2 x kC
      for (int i = tid; part && r > 0 && i < kL + 2 * kC; i += nthr) {
        if (i < kL) {
          const int col = c0 + i;
          if (col < c1) db_line(D, 0, true, 0, col, D.info[0][(col >> 4) & 7], D.info[1][(col >> 4) & 7]);
        } else {
          const int j = i - kL, pl = 1 + (j >> (ls - 1)), col = (c0 >> 1) + (j & (kC - 1));
          if (col < (c1 >> 1))
            db_line(D, pl, true, 0, col, D.info[0][(col >> 3) & 7], D.info[1][(col >> 3) & 7]);
        }
      }
      __builtin_amdgcn_wave_barrier();
      // band A V edges of the luma units c0, c0+8, ... and the chroma units c0/2, c0/2+8, ...
      for (int i = tid; part && i < kL + 2 * kC; i += nthr) {
        if (i < kL) {
          const int x = c0 + 8 * (i >> 3), row = 4 + (i & 7);
          if (x > 0 && x < c1)
            db_line(D, 0, false, row, x - 4, D.info[1][((x - 1) >> 4) & 7], D.info[1][(x >> 4) & 7]);
        } else {
          const int j = i - kL, pl = 1 + (j >> (ls - 1)), x = (c0 >> 1) + 8 * ((j & (kC - 1)) >> 3), row = 4 + (j & 7);
          if (x > 0 && x < (c1 >> 1))
            db_line(D, pl, false, row, x - 4, D.info[1][((x - 1) >> 3) & 7], D.info[1][(x >> 3) & 7]);
        }
      }
      __builtin_amdgcn_wave_barrier();
      // band B H edges of [hb0, hb1), then V edges of units [vb0, vb1)
      for (int col = hb0 + tid; part && col < hb1; col += nthr)
        db_line(D, 0, true, 8, col, D.info[1][(col >> 4) & 7], D.info[1][(col >> 4) & 7]);
      __builtin_amdgcn_wave_barrier();
      for (int i = tid; part && i < 8 * ((vb1 - vb0 + 7) >> 3); i += nthr) {
        const int x = vb0 + 8 * (i >> 3), row = 12 + (i & 7);
        if (x < vb1) db_line(D, 0, false, row, x - 4, D.info[1][((x - 1) >> 4) & 7], D.info[1][(x >> 4) & 7]);
      }
    }
    __syncthreads();
    const uint64_t td2 = acct_now();
    acct_add(a.acct, Acct::kDbInputs, td1 - ta);
    acct_add(a.acct, Acct::kDbFilter, td2 - td1);
    hb0 = max(hb0, hb1);
    vb0 = max(vb0, vb1);
    const int w1 = last ? a.wa : max(w0, c1 - 12);
    // ---- write out columns [w0, w1): luma rows 16r-3..16r+15, chroma 8r-3..8r+7 ----
    if (w1 > w0) {
      const int rl0 = r > 0 ? 1 : 4, rc0 = r > 0 ? 1 : 4;  // first tile row written
      const int nl = (w1 - w0) >> 1, nc = (w1 - w0) >> 2;
      const int nrl = 20 - rl0, nrc = 12 - rc0;
      // index space: per row, sl = 1 or 2 bands of 32 dwords (luma; chroma 16),
      // so that row, band and column are shifts and masks
      const int sl = nl > 32 ? 1 : 0, sc = nc > 16 ? 1 : 0;
      const int NL = nrl << (5 + sl), NC = nrc << (4 + sc);
      for (int i = tid; i < NL + 2 * NC; i += 256) {
        int pl, row, col;
        int16_t* g;
        if (i < NL) {
          const int d = i & ((32 << sl) - 1);
          if (d >= nl) continue;
          pl = 0, row = rl0 + (i >> (5 + sl)), col = w0 + 2 * d;
          g = cs.y + (size_t)(y0 + row) * a.wa + col;
        } else {
          const int j = i - NL, pj = j >= NC, jj = j - (pj ? NC : 0), d = jj & ((16 << sc) - 1);
          if (d >= nc) continue;
          pl = 1 + pj, row = rc0 + (jj >> (4 + sc)), col = (w0 >> 1) + 2 * d;
          g = pick(cs, 1 + pj) + (size_t)(c0y + row) * cw + col;
        }
        const int16_t* p = db_px(D, pl, row, col);
        const uint32_t d = (uint32_t)(uint16_t)p[0] | ((uint32_t)(uint16_t)p[1] << 16);
        __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)g, d, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        const size_t off = (size_t)(g - pick(cs, pl));
        for (int q = 0; q < a.npush; q++)  // the readers' mirrors (uniform loop)
          __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)(pick(planes(a.push[q]), pl) + off), d,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (a.sys) {  // the next frame may read this row from another device
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
          __hip_atomic_store(&prog[r], above | (uint32_t)w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
          __hip_atomic_store(&prog[r], above | (uint32_t)w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (a.stamps && tid == 0 && k < kDbStamps)
        a.stamps[(size_t)a.wmb * a.hmb * kStampPhases + (size_t)r * kDbStamps + k] = __builtin_amdgcn_s_memrealtime();
      w0 = w1;
    }
    acct_add(a.acct, Acct::kDbWrite, acct_now() - td2);
  }
  st.k++;
  if (tb) st.busy += __builtin_amdgcn_s_memrealtime() - tb;
  acct_add(a.acct, Acct::kHelperDeblock, acct_now() - ta);
  acct_add(a.acct, Acct::kHelperChunks, 1);
}

// ---------------------------------------------------------------------------
// K2: the macroblock wavefront.  One workgroup owns one macroblock row at a
// time (dequeued in order) and walks it left to right.  MB (bx, by) starts
// when row by-1 has finished MB bx+2, i.e. the schedule t = bx + 3*by that
// reproduces the raster order's reads of in-progress (rows above, left) and
// stale (row below, frame n-R) reconstruction bit for bit.
//
// The current slot around the row lives in a circular LDS window: MB rows
// by-3..by+1 (80 pixel rows) by 128 columns addressed with absolute x & 127.
// A step brings in only the new column (rows by-3..by-1 at bx+2) and one stale
// macroblock (row by+1 at bx-1); the row's own reconstruction is written
// straight into the window.  Finished macroblocks are handed to the rows
// below as tagged granules (no flag, no fence: MI355X_MICROARCH.md R2), and
// "row by-1 finished bx+2" is simply "granules of (bx+2, by-1) carry this
// frame's tag".
// ---------------------------------------------------------------------------

// Window storage: values are biased (v ^ 0x8000) so that unsigned 16-bit
// order equals signed order (reconstructions are unclamped int16, SURVEY.md
// Appendix A.4), which lets the candidate search use packed u16 instructions.
// Columns are circular (x & 127, chroma x & 63); the first 16 (4) columns are
// repeated after the last so that a row read never wraps.  Luma pitch
// (elements): 128 + 16-column tail + pad.  Only 2- and 4-byte accesses touch
// this window, so the pitch is free: an odd number of dwords (150 elements =
// 75) puts the 16 rows of a candidate's lane group on 16 distinct banks of
// either parity, so the wave's other groups (offsets of a search step) do not
// all land on the same 16 even banks (148 = 74 dwords).
constexpr int kCwLP = 150;
static_assert(kCwLP % 2 == 0 && kCwLP >= 144, "coder window rows: dword pairs, 128 + 16-column tail");
constexpr int kCwCP = 74;   // chroma pitch: 64 + 4-column tail + pad
constexpr int kLumaTail = 16, kChromaTail = 4;

struct alignas(16) RowWindow {
  int16_t y[80 * kCwLP];
  int16_t u[40 * kCwCP];
  int16_t v[40 * kCwCP];
};

// The row coder's source macroblocks go through LDS: wave 0 stages
// macroblock bx+1's source (src_dma) at bx's start, with the fresh granule
// load (an LDS-DMA in flight makes the compiler drain vmcnt at the next
// barrier or global-load use: hipcc, ROCm 7.2), so neither the source rows at
// a macroblock's start nor the residual's source elements after its search
// cost a fabric round trip.
constexpr int kWaitVm0 = 0x0F70;  // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15) (gfx9 encoding)

// A macroblock's end waits only for its coefficient stores (which its info
// granule releases to the deblock and, through its progress, to the next
// frame's copy macroblocks), not for the pixel-granule and table stores
// issued after them: vmcnt retires in order, so wave w waits until no more
// than the stores it issued after its last coefficient store are
// outstanding.  Those are, in program order (compiler barriers keep it):
// one pixel-granule store per 8x8 block the wave owns (blocks w and w+4:
// two for waves 0 and 1, one for waves 2 and 3), then, on wave 0, the
// 16-byte block-table store.
constexpr int kBlocksOfWave[4] = {2, 2, 1, 1};
// s_waitcnt vmcnt(N) (N < 16: gfx9 encoding, expcnt and lgkmcnt left free),
// also a compiler barrier.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 16, "vmcnt immediate");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
  asm volatile("" ::: "memory");
}
constexpr int kStoresAfterCoef[4] = {kBlocksOfWave[0] + 1, kBlocksOfWave[1], kBlocksOfWave[2], kBlocksOfWave[3]};
static_assert(kStoresAfterCoef[0] == 3 && kStoresAfterCoef[1] == 2 && kStoresAfterCoef[2] == 1 &&
                  kStoresAfterCoef[3] == 1,
              "the s_waitcnt immediates in code_row");


struct alignas(16) RowLds {
  RowWindow win;
  alignas(16) int16_t src[2][384];  // source macroblocks bx, bx+1 (by bx & 1), group_source layout
  int16_t bufA[kMBElems], bufB[kMBElems];  // per-block transform scratch, block-major
  int32_t cand[2][16][2];                  // double-buffered candidate (sad, mad)
  int32_t red[12];
};

// Pixel pair (int16 lo = column col, hi = col+1; col even) of plane pl at
// window row `row`.
__device__ __forceinline__ void win_put2(RowWindow& w, int pl, int row, int col, uint32_t pair) {
  const uint32_t b = pair ^ 0x80008000u;
  if (pl == 0) {
    const int c = col & 127;
    *(uint32_t*)&w.y[row * kCwLP + c] = b;
    if (c < kLumaTail) *(uint32_t*)&w.y[row * kCwLP + 128 + c] = b;
  } else {
    int16_t* t = pl == 1 ? w.u : w.v;
    const int c = col & 63;
    *(uint32_t*)&t[row * kCwCP + c] = b;
    if (c < kChromaTail) *(uint32_t*)&t[row * kCwCP + 64 + c] = b;
  }
}
__device__ __forceinline__ void win_put1(RowWindow& w, int pl, int row, int col, int v) {
  const int16_t b = (int16_t)(v ^ 0x8000);
  if (pl == 0) {
    const int c = col & 127;
    w.y[row * kCwLP + c] = b;
    if (c < kLumaTail) w.y[row * kCwLP + 128 + c] = b;
  } else {
    int16_t* t = pl == 1 ? w.u : w.v;
    const int c = col & 63;
    t[row * kCwCP + c] = b;
    if (c < kChromaTail) t[row * kCwCP + 64 + c] = b;
  }
}

// Dword k (0..191) of macroblock (mbx, mby): its address in plane set p (same
// order as the granules, kernels.h), and its store into the window.
__device__ __forceinline__ const int16_t* win_src(const PlaneSet& p, int wa, int mbx, int mby, int k) {
  if (k < 128) return p.y + (size_t)(mby * 16 + (k >> 3)) * wa + mbx * 16 + 2 * (k & 7);
  const int u = k - 128, pl = u >> 5, r = (u & 31) >> 2, d = u & 3;
  return pick(p, 1 + pl) + (size_t)(mby * 8 + r) * (wa >> 1) + mbx * 8 + 2 * d;
}
__device__ __forceinline__ void win_put_k(RowWindow& w, int oy, int mbx, int mby, int k, uint32_t pair) {
  k = fresh(k);
  if (k < 128) {
    win_put2(w, 0, mby * 16 + (k >> 3) - oy, mbx * 16 + 2 * (k & 7), pair);
  } else {
    const int u = k - 128, pl = u >> 5, r = (u & 31) >> 2, d = u & 3;
    win_put2(w, 1 + pl, mby * 8 + r - (oy >> 1), mbx * 8 + 2 * d, pair);
  }
}

__device__ __forceinline__ void cand_row(const RowWindow& w, int oy, int cx, int cy, int i,
                                         const SrcRow& s, int thr, int& sad, int& mad) {
  const int c = cx & 127, sh = (c & 1) * 2;
  const uint32_t* row = (const uint32_t*)&w.y[(cy + i - oy) * kCwLP] + (c >> 1);
  uint32_t d[9];
#pragma unroll
  for (int k = 0; k < 9; k++) d[k] = row[k];
  uint32_t sm = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) sm = __builtin_amdgcn_sad_u16(s.y[k], __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh), sm);
  sad = row16_sum((int)sm);
  mad = kMadFar;
  if (__ballot(mad_needed(sad, thr))) {  // (wave-uniform) some candidate of the wave may have MAD < thr
    u16x2 m1 = {0, 0}, m2 = {0, 0};
    uint32_t dummy = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) pk_diff(s.y[k], __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh), dummy, m1, m2);
    const int cr = (cy >> 1) + (i >> 1) - (oy >> 1), cc = ((cx >> 1) + (i & 1) * 4) & 63, shc = (cc & 1) * 2;
    const uint32_t* ru = (const uint32_t*)&w.u[cr * kCwCP] + (cc >> 1);
    const uint32_t* rv = (const uint32_t*)&w.v[cr * kCwCP] + (cc >> 1);
    const uint32_t u0 = ru[0], u1 = ru[1], u2 = ru[2], v0 = rv[0], v1 = rv[1], v2 = rv[2];
    pk_diff(s.u[0], __builtin_amdgcn_alignbyte(u1, u0, shc), dummy, m1, m2);
    pk_diff(s.u[1], __builtin_amdgcn_alignbyte(u2, u1, shc), dummy, m1, m2);
    pk_diff(s.v[0], __builtin_amdgcn_alignbyte(v1, v0, shc), dummy, m1, m2);
    pk_diff(s.v[1], __builtin_amdgcn_alignbyte(v2, v1, shc), dummy, m1, m2);
    const u16x2 m = __builtin_elementwise_max(m1, m2);
    mad = row16_max(max((int)m.x, (int)m.y));
  }
}

// lerp_px on both halves of two biased u16 pairs; the result as a biased pair.
// On the biased halves directly (lerp_half_bb).
__device__ __forceinline__ uint32_t lerp_pair(uint32_t pa, uint32_t pb, int q) {
  const uint32_t a0 = pa & 0xFFFFu, b0 = pb & 0xFFFFu, a1 = pa >> 16, b1 = pb >> 16;
  const uint32_t l0 = q ? lerp_quarter_bb(a0, b0) : lerp_half_bb(a0, b0);
  const uint32_t l1 = q ? lerp_quarter_bb(a1, b1) : lerp_half_bb(a1, b1);
  return l0 | (l1 << 16);
}

// Sub-pel candidate: lerp of the best block (bx, by) toward neighbour (tx, ty),
// read like cand_row (aligned dwords of the circular window and its
// duplicated tail, realigned by v_alignbyte_b32); the lerped pairs are
// re-biased so that SAD and MAD use the same packed u16 ops.
__device__ __forceinline__ void subpel_row(const RowWindow& w, int oy, int bx, int by, int tx,
                                           int ty, int q, int i, const SrcRow& s, int thr, int& sad,
                                           int& mad) {
  uint32_t sm = 0;
  uint32_t l[8];  // the lerped luma pairs (biased)
  {
    const int ca = bx & 127, cb = tx & 127, sha = (ca & 1) * 2, shb = (cb & 1) * 2;
    const uint32_t* ra = (const uint32_t*)&w.y[(by + i - oy) * kCwLP] + (ca >> 1);
    const uint32_t* rb = (const uint32_t*)&w.y[(ty + i - oy) * kCwLP] + (cb >> 1);
    uint32_t da[9], db[9];
#pragma unroll
    for (int k = 0; k < 9; k++) da[k] = ra[k], db[k] = rb[k];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      l[k] = lerp_pair(__builtin_amdgcn_alignbyte(da[k + 1], da[k], sha),
                       __builtin_amdgcn_alignbyte(db[k + 1], db[k], shb), q);
      sm = __builtin_amdgcn_sad_u16(s.y[k], l[k], sm);
    }
  }
  sad = row16_sum((int)sm);
  mad = kMadFar;
  if (!__ballot(mad_needed(sad, thr))) return;  // (wave-uniform) kMadFar above
  u16x2 m1 = {0, 0}, m2 = {0, 0};
  {
    uint32_t dummy = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) pk_diff(s.y[k], l[k], dummy, m1, m2);
  }
  {
    const int ra = (by >> 1) + (i >> 1) - (oy >> 1), rb = (ty >> 1) + (i >> 1) - (oy >> 1);
    const int xa = ((bx >> 1) + (i & 1) * 4) & 63, xb = ((tx >> 1) + (i & 1) * 4) & 63;
    const int sha = (xa & 1) * 2, shb = (xb & 1) * 2;
    uint32_t dummy = 0;
#pragma unroll
    for (int pl = 0; pl < 2; pl++) {
      const int16_t* t = pl ? w.v : w.u;
      const uint32_t* pa = (const uint32_t*)&t[ra * kCwCP] + (xa >> 1);
      const uint32_t* pb = (const uint32_t*)&t[rb * kCwCP] + (xb >> 1);
      const uint32_t a0 = pa[0], a1 = pa[1], a2 = pa[2], b0 = pb[0], b1 = pb[1], b2 = pb[2];
      const uint32_t* sp = pl ? s.v : s.u;
      pk_diff(sp[0], lerp_pair(__builtin_amdgcn_alignbyte(a1, a0, sha), __builtin_amdgcn_alignbyte(b1, b0, shb), q),
              dummy, m1, m2);
      pk_diff(sp[1], lerp_pair(__builtin_amdgcn_alignbyte(a2, a1, sha), __builtin_amdgcn_alignbyte(b2, b1, shb), q),
              dummy, m1, m2);
    }
  }
  const u16x2 m = __builtin_elementwise_max(m1, m2);
  mad = row16_max(max((int)m.x, (int)m.y));
}

__device__ __forceinline__ bool intra_valid(int cx, int cy, int px, int py, int wa, int ha) {
  if (cy > py - kMB && cx > px - kMB) return false;  // not yet coded (motion.cpp:239-243)
  return in_frame(cx, cy, wa, ha);
}

// Pixel (ex, ey) of plane pl (0 Y, 1 U, 2 V) from the window.
__device__ __forceinline__ int win_px(const RowWindow& w, int oy, int pl, int ex, int ey) {
  if (pl == 0) return unbias(w.y[(ey - oy) * kCwLP + (ex & 127)]);
  const int16_t* t = pl == 1 ? w.u : w.v;
  return unbias(t[(ey - (oy >> 1)) * kCwCP + (ex & 63)]);
}

__device__ __forceinline__ const int16_t* plane_of(const PlaneSet& p, int pl) {
  return pick(p, pl);
}

// Sample of element e (block-major) of the block at (mx, my) of plane set p.
__device__ __forceinline__ int pred_at(const PlaneSet& p, int wa, int e, int mx, int my) {
  if (CAIRO_ATTR_SKIP & 4) return 128;
  int pl, ex, ey;
  elem_coords(e, mx, my, pl, ex, ey);
  const int pitch = pl == 0 ? wa : (wa >> 1);
  return plane_of(p, pl)[(size_t)ey * pitch + ex];
}
// Prediction sample of element e (block-major) of the block at (mx, my) of
// plane set p, lerped toward (mx+dx, my+dy) when sp (macroblock.h:203-259).
__device__ __forceinline__ int pred_global(const PlaneSet& p, int wa, int e, int mx, int my, bool sp,
                                           int dx, int dy, int amount) {
  const int v = pred_at(p, wa, e, mx, my);
  return sp ? lerp_px(v, pred_at(p, wa, e, mx + dx, my + dy), amount) : v;
}

// A block descriptor from its four words (all lanes hold the same), fields in
// SGPRs; q_index and variance cleared as in uni_desc.  One 16-byte load per
// descriptor instead of a load (and a wait) per field.
__device__ __forceinline__ BlockDesc uni_desc_words(uint4 w) {
  BlockDesc d;
  d.block_type = (uint32_t)uni((int)w.x);
  const uint32_t w1 = (uint32_t)uni((int)w.y), w2 = (uint32_t)uni((int)w.z), w3 = (uint32_t)uni((int)w.w);
  d.prediction_target = (uint8_t)w1;
  d.pad = 0;
  d.motion_x = (int16_t)(w1 >> 16);
  d.motion_y = (int16_t)w2;
  d.sp_pred = (uint8_t)(w2 >> 16);
  d.sp_amount = (uint8_t)(w2 >> 24);
  d.sp_index = (uint8_t)w3;
  d.q_index = 0;
  d.variance = 0;
  return d;
}

__device__ __forceinline__ BlockDesc uni_desc(const BlockDesc& d) {
  BlockDesc u;
  u.block_type = (uint32_t)uni((int)d.block_type);
  u.prediction_target = (uint8_t)uni(d.prediction_target);
  u.pad = 0;
  u.motion_x = (int16_t)uni(d.motion_x);
  u.motion_y = (int16_t)uni(d.motion_y);
  u.sp_pred = (uint8_t)uni(d.sp_pred);
  u.sp_amount = (uint8_t)uni(d.sp_amount);
  u.sp_index = (uint8_t)uni(d.sp_index);
  u.q_index = 0;
  u.variance = 0;
  return u;
}

__device__ __forceinline__ uint64_t* gran_at(FA& a, int mbx, int mby, int k) {
  return a.granules + (size_t)(mby * a.wmb + mbx) * kGranuleStride + k;
}

// Store lane pairs (lane, lane^1) of an 8x8 block's int16 values as dwords
// with write-through (sc1) stores: the next frame reads them back (output_cache
// carry of copy macroblocks) on another CU.  e = element (block-major).
__device__ __forceinline__ void coef_store_pair(FA& a, int e, int px, int py, int value) {
  const int nb = __builtin_amdgcn_mov_dpp(value, 0xB1, 0xF, 0xF, false);  // lane ^ 1
  if (!(threadIdx.x & 1)) {
    int pl, ex, ey;
    elem_coords(fresh(e), px, py, pl, ex, ey);
    int16_t* cp = pick(planes(a.coef), pl);
    __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)(cp + (size_t)ey * (pl ? a.wa >> 1 : a.wa) + ex),
                       ((uint32_t)value & 0xFFFFu) | ((uint32_t)nb << 16), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Code MB row `by` of frame a (intra search, classify, transform, VAQ,
// quantize, reconstruct), left to right; whole workgroup.
// kDecode: the decoder's reconstruction (decode_slice, decode.cpp:146-170) from
// the given block table and coefficients, without the searches.
template <bool kDecode>
__device__ __forceinline__ void code_row(FA& a0, int by, RowLds& L, int* flag, int32_t* tr) {
  FA& a = a0;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int grp = tid >> 4, gi = tid & 15;
  const int thr = (a.quality >> 2) + 1;
  const PlaneSet cs = planes(a.stale);  // the stale rows below (frame index-R)
  const uint32_t tag = a.epoch;
  const int cw = a.wa >> 1;
  const int nblk = wave < 2 ? 2 : 1;  // wave w owns 8x8 blocks w and w+4
  const int mbs = a.wmb * a.hmb;
  {
    const int py = by * kMB, oy = py - 48;
    if (!kDecode) {  // macroblock 0's source; later ones are staged a macroblock ahead
      src_dma(a, 0, by, L.src[0]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int bx = 0; bx < a0.wmb; bx++) {
      FA* ap = opaque_view(&a0);
      const int px = bx * kMB, mb = by * ap->wmb + bx;
      trace(tr, 1, bx);
      trace(tr, 2, (int)ap->epoch * 1000 + by);
      stamp(*ap, mb, 0);
      if (ap->stamps && tid == 0) ap->stamps[(size_t)mb * kStampPhases + 10] = __builtin_amdgcn_s_memtime();
      // The row above's fresh column block (bx+2, by-1): its first granule
      // load is issued before the group-start wait below, so that a granule
      // already there costs no round trip after it (the tag is the flag: a
      // 64-bit load needs no acquire).
      // macroblock bx+1's source into LDS, in flight with the fresh granule
      // load below, whose wait covers it (the buffer was last read in bx-1)
      if (!kDecode && bx + 1 < ap->wmb) src_dma(*ap, bx + 1, by, L.src[(bx + 1) & 1]);
      const bool fresh_col = by > 0 && bx != 0 && bx + 2 < ap->wmb && tid < kGranulesPerMB;
      const uint64_t* fresh_gp = fresh_col ? gran_at(*ap, bx + 2, by - 1, tid) : nullptr;
      const uint64_t fresh_g = fresh_col ? gran_ld(fresh_gp) : 0;
      // At a group start the coder needs the group's inter records, and every
      // cross-frame dependency they carry (the stale rows, references and
      // previous output_cache), only for the classification: the intra search
      // reads nothing but the LDS window.  So it runs first (early), while the
      // records may still be on their way; the acquire, when the records are
      // already in, completes behind it (it issues no vector-memory access).
      const bool gstart = (bx & 3) == 0;
      const bool early = !kDecode && gstart;  // workgroup-uniform
      // The macroblock's inter records (2 * nref tagged granules; every lane
      // of a wave the same addresses): inside a group they are normally in
      // already, so their loads go out here, in flight with the fresh
      // granule's, instead of a round trip of their own after it (settled by
      // tag in load_inter).  At a group start, after the search.
      const int nref = ap->inter ? ap->ring - 1 : 0;
      uint64_t rg[kMaxRing - 1][2];
      auto issue_records = [&]() {
#pragma unroll
        for (int o = 0; o < kMaxRing - 1; o++) {
          if (o >= nref) break;
          const uint64_t* r = (const uint64_t*)&ap->inter_desc[o * mbs + mb];
          rg[o][0] = gran_ld(r);
          rg[o][1] = gran_ld(r + 1);
        }
      };
      if (!early) issue_records();
#ifdef CAIRO_ACCT_STORE_TAIL
      {  // diagnostic (tools builds): how long the previous macroblock's stores still take here
        const uint64_t ts = acct_now();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acct_add(ap->acct, Acct::kCoderStoreTail, acct_now() - ts);
      }
#endif
      uint64_t tacc = acct_now();
      // thread 0: one poll of the group's record count, issued with the fresh
      // granule load and tested after the window update (which waits for it anyway)
      // With tagged records (inter frames) the group is ready once its first
      // macroblock's record of reference 1 -- the helper's last search, after
      // its wait for the previous frame -- carries this frame's tag; otherwise
      // (intra and decoded frames: the helper's carrier) once inter_done says so.
      const bool by_tag = ap->inter;  // workgroup-uniform
      const uint64_t* grec = (const uint64_t*)&ap->inter_desc[mb];  // reference 1, this MB
      uint64_t rd0 = 0;
      if (early && tid == 0)
        rd0 = by_tag ? gran_ld(grec)
                     : (uint64_t)__hip_atomic_load(&ap->inter_done[by * ap->ng + (bx >> 2)], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      bool ready0 = false;  // thread 0: the records were in before the search
      if (gstart && !early) {  // inter records of MBs bx..bx+3, and every cross-frame dependency they carry
        if (tid == 0) {
          if (by_tag) rec_settle(*ap, grec, gran_ld(grec), by, mb);
          else wait_records(*ap, by, bx >> 2);
        }
        acquire_after_wait(ap->sys);  // the stale rows, references and previous output_cache
        acct_add(ap->acct, Acct::kCoderGroupWait, acct_now() - tacc);
      }
      tacc = acct_now();

      // ---- window.  Reconstruction of the rows above arrives as granules
      //      (this frame's data, polled by tag); the stale row below is the
      //      previous launch's slot.  Immediate: the fresh column block
      //      (bx+2, by-1), or at bx == 0 the first three columns.  Prefetched
      //      for MB bx+1 and committed at the end of this macroblock: column
      //      bx+3 of rows by-3, by-2 (final once row by-1 passed bx+2) and the
      //      stale block (bx, by+1), read before row by+1 may rewrite it ----
      if (by > 0) {
        if (bx == 0) {
          int lx[9], ly[9], n = 0;
          for (int r = max(by - 3, 0); r <= by - 1; r++)
            for (int c = 0; c <= 2 && c < ap->wmb; c++) lx[n] = c, ly[n++] = r;
          for (int k = tid; k < n * kGranulesPerMB; k += 256) {
            const int i = k / kGranulesPerMB, kk = k - i * kGranulesPerMB;
            const uint64_t* gp = gran_at(*ap, lx[i], ly[i], kk);
            win_put_k(L.win, oy, lx[i], ly[i], kk, gran_settle(*ap, gp, gran_ld(gp), by));
          }
        } else if (fresh_col) {
          win_put_k(L.win, oy, bx + 2, by - 1, tid,
                    gran_settle(*ap, fresh_gp, fresh_g, by));
        }
      }
      acct_add(ap->acct, Acct::kCoderWindow, acct_now() - tacc);
      // the source DMA has landed (free where the granule wait above covered
      // it): a wait the compiler sees, so it knows no LDS-DMA is in flight and
      // the barrier before the search does not drain the loads issued below
      const uint64_t tv0 = acct_now();
      if (!kDecode) __builtin_amdgcn_s_waitcnt(kWaitVm0);
      acct_add(ap->acct, Acct::kCoderVm0, acct_now() - tv0);
      if (early && tid == 0) {
        ready0 = by_tag ? (uint32_t)(rd0 >> 32) == ap->epoch : (int)rd0 >= ap->nref;
        if (ready0) acquire_fence(ap->sys);  // completes during the search; waited for after it
      }
      // source rows of this lane's group slot
      SrcRow s;  // biased u16 pairs (the encoder's source; unused when decoding)
      if (!kDecode) {
        // staged in LDS during macroblock bx-1 (landed behind its final drain
        // and barrier; at bx == 0 behind the row start's)
        const uint32_t* m = (const uint32_t*)L.src[bx & 1];
#pragma unroll
        for (int k = 0; k < 8; k++) s.y[k] = m[gi * 8 + k] ^ 0x80008000u;
        const int co = (gi >> 1) * 4 + (gi & 1) * 2;
        s.u[0] = m[128 + co] ^ 0x80008000u, s.u[1] = m[128 + co + 1] ^ 0x80008000u;
        s.v[0] = m[160 + co] ^ 0x80008000u, s.v[1] = m[160 + co + 1] ^ 0x80008000u;
      }
      const bool pf3 = by >= 3 && bx + 3 < ap->wmb, pf2 = by >= 2 && bx + 3 < ap->wmb;
      const bool pfs = by + 1 < ap->hmb && bx + 1 < ap->wmb;
      uint64_t pg3 = 0, pg2 = 0;
      uint32_t pst = 0;
      if (tid < kGranulesPerMB) {
        if (pf3) pg3 = gran_ld(gran_at(*ap, bx + 3, by - 3, tid));
        if (pf2) pg2 = gran_ld(gran_at(*ap, bx + 3, by - 2, tid));
        if (pfs && !early) pst = *(const uint32_t*)win_src(cs, ap->wa, bx, by + 1, tid);  // (early: after the wait)
      }

      // ---- inter predictions, prefetched (the K1 records are final) ----
      // the prediction of the best inter record: the classification below
      // is a lexicographic minimum of (not copy, sad) over [intra, ref 1..],
      // the earlier winning ties, so the only inter record that can win is
      // the minimum over the references alone -- known from the records,
      // before the search.  Its block (and a sub-pel winner's neighbour)
      // loads overlap the search.
      BlockDesc ib;  // set by reference 1 (o == 0) before it is compared
      int ib_sad = 0;
      int ipa[2] = {0, 0}, ipb[2] = {0, 0};
      auto load_inter = [&]() {  // the records (issue_records), then the predictions
#pragma unroll
        for (int o = 0; o < kMaxRing - 1; o++) {
          if (o >= nref) break;
          const uint64_t* r = (const uint64_t*)&ap->inter_desc[o * mbs + mb];
          const BlockDesc rd = unpack_inter_desc((uint32_t)uni((int)rec_settle(*ap, r, rg[o][0], by, mb)));
          const int rs = uni((int)rec_settle(*ap, r + 1, rg[o][1], by, mb));
          if (o == 0) {
            ib = rd, ib_sad = rs;
          } else {
            const bool ci = (rd.block_type & kCopy) != 0, cb = (ib.block_type & kCopy) != 0;
            if (ci != cb ? ci : rs < ib_sad) ib = rd, ib_sad = rs;
          }
        }
        if (nref == 0) return;
        const BlockDesc& d = ib;
        const PlaneSet rp = RECON_AT(*ap, d.prediction_target);
        const bool mot = (d.block_type & kMotion) != 0, sp = mot && d.sp_pred;
        const int mx = px + (mot ? d.motion_x : 0), my = py + (mot ? d.motion_y : 0);
        int dx = 0, dy = 0;
        if (sp) frac_dir(d.sp_index, &dx, &dy);
        _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {
          ipa[bi] = pred_at(rp, ap->wa, (wave + 4 * bi) * 64 + lane, mx, my);
          if (sp) ipb[bi] = pred_at(rp, ap->wa, (wave + 4 * bi) * 64 + lane, mx + dx, my + dy);
        }
      };
      const uint64_t tr0 = acct_now();
      if (!early) load_inter();
      stamp(*ap, mb, 1);
      const uint64_t tr1 = acct_now();
      __syncthreads();
      stamp(*ap, mb, 2);
      tacc = acct_now();
      acct_add(ap->acct, Acct::kCoderRecords, tr1 - tr0);
      acct_add(ap->acct, Acct::kCoderPreBarrier, tacc - tr1);

      BlockDesc d;
      bool from_inter = false;  // an inter record won / an inter type is decoded (prediction in wpv)
      int wpv[2] = {0, 0};
      if (!kDecode) {
        // ---- intra search (calculate_intra_prediction, motion.cpp:354-419) ----
        Sel sel;
        {
          int sm = 0;
  #pragma unroll
          for (int k = 0; k < 16; k++) sm += abs(src_px(s.y, k));
          sel.sad = uni(row16_sum(sm));  // compute_block_sad(src): every group holds the total
        }
        sel.bx = px;
        sel.by = py;
        sel.mad = INT32_MAX;
        sel.ssd = INT32_MAX;
        sel.sp_idx = sel.sp_amt = sel.sp_en = 0;
        int buf = 0;
        uint64_t t_ev = 0, t_ba = 0, t_se = 0;  // (CAIRO_ACCT builds: the stages' phases)
  #pragma unroll 1
        for (int stage = 0; stage < ((CAIRO_ATTR_SKIP & 16) ? 0 : 5); stage++) {
          const int step = stage == 0 ? kRadius : (kRadius >> stage);
          const int jlo = stage == 0 ? -2 * kRadius : -step;
          const int bx0 = sel.bx, by0 = sel.by;
          const uint64_t ts0 = acct_now();
          if (grp < 9) {  // group g < 9 evaluates candidate g; groups 9..15 idle (7/16 of the work saved)
            const int c = min(grp, 8);
            const int cx = bx0 - step + (c % 3) * step, cy = by0 + jlo + (c / 3) * step;
            const bool ok = intra_valid(cx, cy, px, py, ap->wa, ap->ha);
            int sad, mad;
            cand_row(L.win, oy, cx, ok ? cy : py - 48, gi, s, thr, sad, mad);
            if (gi == 0 && grp < 9) {
              L.cand[buf][grp][0] = ok ? sad : -1;
              L.cand[buf][grp][1] = mad;
            }
          }
          const uint64_t ts1 = acct_now();
          __syncthreads();
          const uint64_t ts2 = acct_now();
          {
            const int c = lane & 15;
            const int vs = L.cand[buf][c][0], vm = L.cand[buf][c][1];
            const int cx = bx0 - step + (c % 3) * step, cy = by0 + jlo + (c / 3) * step;
            select_int(sel, c < 9 && vs >= 0, cx, cy, vs, vm, px, py, thr, lane);
          }
          buf ^= 1;
          if (CAIRO_ACCT) {
            const uint64_t ts3 = uni((int)sel.bx) == -99999 ? 0 : acct_now();  // after the replay's result
            t_ev += ts1 - ts0, t_ba += ts2 - ts1, t_se += ts3 - ts2;
          }
        }
        acct_add(ap->acct, Acct::kSrchEval, t_ev);
        acct_add(ap->acct, Acct::kSrchBarrier, t_ba);
        acct_add(ap->acct, Acct::kSrchSelect, t_se);
        stamp(*ap, mb, 3);
        if (!(CAIRO_ATTR_SKIP & 16)) {  // sub-pel (perform_intra_subpixel_motion_search, motion.cpp:277-317)
          const int bx0 = sel.bx, by0 = sel.by;
          // candidate c = 2 nn + q; q is wave-uniform (waves 0 and 2 the half
          // steps, 1 and 3 the quarter steps), so a wave runs one lerp, not both
          const int q = (grp >> 2) & 1, nn = (grp & 3) | ((grp >> 3) << 2), c = 2 * nn + q;
          const int k9 = nn < 4 ? nn : nn + 1;  // skip the centre of the 3x3
          const int tx = bx0 + k9 % 3 - 1, ty = by0 + k9 / 3 - 1;
          const bool ok = intra_valid(tx, ty, px, py, ap->wa, ap->ha);
          int sad, mad;
          const uint64_t ts0 = acct_now();
          subpel_row(L.win, oy, bx0, ok ? by0 : py - 48, tx, ok ? ty : py - 48, uni(q), gi, s, thr, sad, mad);
          if (gi == 0) {
            L.cand[buf][c][0] = ok ? sad : -1;
            L.cand[buf][c][1] = mad;
          }
          const uint64_t ts1 = acct_now();
          __syncthreads();
          const uint64_t ts2 = acct_now();
          const int vs = L.cand[buf][lane & 15][0], vm = L.cand[buf][lane & 15][1];
          sel.sp_idx = sel.sp_amt = sel.sp_en = 0;
          select_sub(sel, vs >= 0, vs, vm, thr, lane);
          if (CAIRO_ACCT) {
            const uint64_t ts3 = uni((int)sel.sp_idx) == -99999 ? 0 : acct_now();
            acct_add(ap->acct, Acct::kSubEval, ts1 - ts0);
            acct_add(ap->acct, Acct::kSubBarrier, ts2 - ts1);
            acct_add(ap->acct, Acct::kSubSelect, ts3 - ts2);
          }
        }
        stamp(*ap, mb, 4);
        acct_add(ap->acct, Acct::kCoderSearch, acct_now() - tacc);
        if (early) {  // the group's records (and the cross-frame dependencies), then this MB's
          tacc = acct_now();
          if (tid == 0) {
            if (!ready0) {
              if (by_tag) rec_settle(*ap, grec, gran_ld(grec), by, mb);
              else wait_records(*ap, by, bx >> 2);
              acquire_fence(ap->sys);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the acquire has completed
          }
          __syncthreads();
          acct_add(ap->acct, Acct::kCoderGroupWait, acct_now() - tacc);
          tacc = acct_now();
          if (tid < kGranulesPerMB && pfs) pst = *(const uint32_t*)win_src(cs, ap->wa, bx, by + 1, tid);
          issue_records();
          load_inter();
          acct_add(ap->acct, Acct::kCoderInter, acct_now() - tacc);
        }
        d = make_desc(sel, px, py, thr, true, 0);
        int best_sad = sel.sad;

        // ---- classify_block (encode.cpp:17-67) ----
        if (nref > 0) {
          const bool ci = (ib.block_type & kCopy) != 0, cb = (d.block_type & kCopy) != 0;
          if (ci != cb ? ci : ib_sad < best_sad) {
            d = ib;
            best_sad = ib_sad;
            from_inter = true;
            const bool sp = (d.block_type & kMotion) && d.sp_pred;
            _Pragma("unroll") for (int bi = 0; bi < 2; bi++) {
              // pinned here: the lerp would otherwise be hoisted above the
              // search, waiting for the loads there
              asm volatile("" : "+v"(ipa[bi]), "+v"(ipb[bi]));
              wpv[bi] = sp ? lerp_px(ipa[bi], ipb[bi], d.sp_amount) : ipa[bi];
            }
          }
        }
      } else {
        // ---- decoder (decode_slice, decode.cpp:146-170): the block desc is
        //      given; an inter type predicts from its reference slot ----
        const uint4 tw = *(const uint4*)&ap->table[mb];
        d = uni_desc_words(tw);
        d.q_index = (uint8_t)(uni((int)tw.w) >> 8);  // uni_desc leaves it to the quantizer
        if (!(d.block_type & kIntra)) {
          from_inter = true;
          const PlaneSet rp = RECON_AT(*ap, d.prediction_target);
          const bool mot = (d.block_type & kMotion) != 0, sp = mot && d.sp_pred;
          int dx = 0, dy = 0;
          if (sp) frac_dir(d.sp_index, &dx, &dy);
          _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk)
            wpv[bi] = pred_global(rp, ap->wa, (wave + 4 * bi) * 64 + lane, px + (mot ? d.motion_x : 0),
                                  py + (mot ? d.motion_y : 0), sp, dx, dy, d.sp_amount);
        }
      }
      ap = opaque_view(ap);  // after the searches: the view's fields re-read, not live across them
      stamp(*ap, mb, 5);
      const uint64_t tx5 = acct_now();
      // this lane's source elements for the residual, loaded after the
      // searches: live across them, they pushed the engine into scratch
      // spills
      int svp[2] = {0, 0};
      if (!kDecode) {
        _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {
          int pl, ex, ey;
          elem_coords((wave + 4 * bi) * 64 + lane, 0, 0, pl, ex, ey);
          svp[bi] = L.src[bx & 1][pl == 0 ? ey * 16 + ex : 256 + (pl - 1) * 64 + ey * 8 + ex];
        }
      }

      // ---- per-wave 8x8 blocks (encode_block encode.cpp:69-163,
      //      decode_block decode.cpp:15-144) ----
      const uint32_t type = d.block_type;
      const bool has_pred = type != kIntra;
      const bool intra_path = (type & kIntra) && !(type & kMotion);
      int pv[2] = {0, 0}, cf[2] = {0, 0};
      if (from_inter) {
        pv[0] = wpv[0];
        pv[1] = wpv[1];
      } else if (has_pred) {  // intra motion: prediction from the window
        const int mx = px + d.motion_x, my = py + d.motion_y;
        const bool sp = d.sp_pred;
        int dx = 0, dy = 0;
        if (sp) frac_dir(d.sp_index, &dx, &dy);
        _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {
          const int e = (wave + 4 * bi) * 64 + lane;
          int pl, ex, ey;
          elem_coords(e, mx, my, pl, ex, ey);
          int v = win_px(L.win, oy, pl, ex, ey);
          if (sp) {
            int nx, ny;
            elem_coords(e, mx + dx, my + dy, pl, nx, ny);
            v = lerp_px(v, win_px(L.win, oy, pl, nx, ny), d.sp_amount);
          }
          pv[bi] = v;
        }
      }
      if (!(type & kCopy) && !kDecode) {
        _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {  // residual (int16) -> forward transform
          const int b = wave + 4 * bi, e = b * 64 + lane;
          int pl, ex, ey;
          elem_coords(e, px, py, pl, ex, ey);
          const int sv = svp[bi];
          const int16_t res = has_pred ? (int16_t)(sv - pv[bi]) : (int16_t)sv;
          // a zero block transforms to zero (transform.cpp:264-301: every term
          // and every rounded_div of 0 is 0): no LDS passes (wave-uniform)
          cf[bi] = (CAIRO_ATTR_SKIP & 64) ? res
                   : (__ballot(res != 0) ? fdct_lane(&L.bufA[b * 64], &L.bufB[b * 64], lane, res) : 0);
        }
      }
      stamp(*ap, mb, 6);
      // The prefetched window blocks for MB bx+1 (loaded before the search),
      // into the window before this macroblock's first store: settled after
      // the stores, their wait (vmcnt retires in order) also waited for the
      // stores' write-through acknowledgements.  This macroblock no longer
      // reads the cells they land in: block bx+3 is beyond its search's reach
      // (px+47), and the stale block (bx, by+1) lies where its candidates are
      // not yet coded.
      if (tid < kGranulesPerMB) {
        if (pf3)
          win_put_k(L.win, oy, bx + 3, by - 3, tid,
                    gran_settle(*ap, gran_at(*ap, bx + 3, by - 3, tid), pg3, by));
        if (pf2)
          win_put_k(L.win, oy, bx + 3, by - 2, tid,
                    gran_settle(*ap, gran_at(*ap, bx + 3, by - 2, tid), pg2, by));
        if (pfs) win_put_k(L.win, oy, bx, by + 1, tid, pst);
      }
      if (!(type & kCopy)) {
        int qp;
        if (!kDecode) {
          int32_t v2;
          qp = vaq_mb(L.red, wave, lane, cf[0], ap->quality, &v2);
          d.q_index = (uint8_t)qp;
          d.variance = (int16_t)v2;
        } else {
          qp = d.q_index;
        }
        _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {
          const int b = wave + 4 * bi, e = b * 64 + lane;
          int16_t qv;
          if (!kDecode) {
            qv = (CAIRO_ATTR_SKIP & 64) ? (int16_t)cf[bi] : quant_elem(e, cf[bi], qp, intra_path);
            coef_store_pair(*ap, e, px, py, qv);
          } else {  // the decoded coefficients (the decoder's input_cache)
            int pl, ex, ey;
            elem_coords(e, px, py, pl, ex, ey);
            qv = plane_of(planes(ap->coef), pl)[(size_t)ey * (pl ? cw : ap->wa) + ex];
          }
          // a block whose coefficients all quantized to zero inverse-transforms
          // to zero (transform.cpp:330-366, per-term truncations of 0): its
          // reconstruction is the prediction, without the LDS passes
          const int t = (CAIRO_ATTR_SKIP & 64) ? qv
                        : (__ballot(qv != 0) ? idct_lane(&L.bufA[b * 64], &L.bufB[b * 64], lane,
                                                         dequant_elem(e, qv, qp, intra_path))
                                             : 0);
          pv[bi] = (int16_t)(has_pred ? t + pv[bi] : t);  // reconstruction (unclamped)
        }
      } else {  // copy: output_cache keeps this macroblock's previous coefficients
        d.q_index = 0;
        d.variance = 0;
        if (!kDecode) {
          int cp[2] = {0, 0};  // both loads issued before the first store (which may alias them)
          _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {
            const int e = (wave + 4 * bi) * 64 + lane;
            int pl, ex, ey;
            elem_coords(e, px, py, pl, ex, ey);
            cp[bi] = pick(planes(ap->coef_prev), pl)[(size_t)ey * (pl ? cw : ap->wa) + ex];
          }
          _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk)
            coef_store_pair(*ap, (wave + 4 * bi) * 64 + lane, px, py, cp[bi]);
        }
      }
      stamp(*ap, mb, 7);
      const uint64_t tx7 = acct_now();
      asm volatile("" ::: "memory");  // program order: the coefficient stores, then (kStoresAfterCoef) ...
      // publish first (the next row's coder waits for exactly these): pixel
      // pairs (lane, lane^1) of each 8x8 block as granules.  No drain before
      // them: the coefficient stores only have to be visible to whoever
      // observes the info granule below (the deblock, and through its
      // progress the next frame's copy macroblocks), which is stored after
      // the drain.
      _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {
        const int b = wave + 4 * bi;
        const int nb = __builtin_amdgcn_mov_dpp(pv[bi], 0xB1, 0xF, 0xF, false);  // lane ^ 1
        if (!(lane & 1)) {
          const int r = lane >> 3, c2 = (lane & 7) >> 1;
          const int k = b < 4 ? (((b >> 1) * 8 + r) * 8 + (b & 1) * 4 + c2) : (128 + (b - 4) * 32 + r * 4 + c2);
          gran_st(gran_at(*ap, bx, by, k),
                  ((uint64_t)tag << 32) | ((uint32_t)pv[bi] & 0xFFFFu) | ((uint32_t)nb << 16));
        }
      }
      stamp(*ap, mb, 8);
      // reconstruction -> the window (the slot is written by the deblock,
      // from the granules)
      _Pragma("unroll") for (int bi = 0; bi < 2; bi++) if (bi < nblk) {
        const int b = wave + 4 * bi, e = b * 64 + lane;
        int pl, ex, ey;
        elem_coords(e, px, py, pl, ex, ey);
        win_put1(L.win, pl, pl == 0 ? ey - oy : ey - (oy >> 1), ex, pv[bi]);
      }
      asm volatile("" ::: "memory");  // ... the pixel-granule stores, then the table store
      if (tid == 0 && !kDecode) *(uint4*)&ap->table[mb] = __builtin_bit_cast(uint4, d);  // one 16-byte store
      // every wave's coefficient stores drained, then the block info for the
      // deblock (its edge strengths); thread 0's drain covers only wave 0, so
      // the other waves drain before the barrier of the next macroblock --
      // the deblock reads their coefficients only through this granule, hence
      // the barrier: info after all four waves drained
      const uint64_t tx8 = acct_now();
      if (!kDecode) {
        // only the coefficient stores (kStoresAfterCoef): the pixel-granule
        // and table stores after them need no drain (tag-polled; read after
        // the launch).  More vector-memory operations after them (granule
        // re-polls, stamps) only make the wait longer.
        if (wave == 0) wait_vmcnt<kStoresAfterCoef[0]>();
        else if (wave == 1) wait_vmcnt<kStoresAfterCoef[1]>();
        else if (wave == 2) wait_vmcnt<kStoresAfterCoef[2]>();
        else wait_vmcnt<kStoresAfterCoef[3]>();
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (tid == 0)
        gran_st(gran_at(*ap, bx, by, kGranulesPerMB),
                ((uint64_t)tag << 32) | ((d.block_type & kCopy) ? 0x100u : 0u) | d.q_index);
      stamp(*ap, mb, 9);
      if (CAIRO_ACCT) {
        const uint64_t tx9 = acct_now();
        acct_add(ap->acct, Acct::kCoderXform, tx7 - tx5);
        acct_add(ap->acct, Acct::kCoderPublish, tx8 - tx7);
        acct_add(ap->acct, Acct::kCoderDrain, tx9 - tx8);
      }
      if (ap->stamps && tid == 0) ap->stamps[(size_t)mb * kStampPhases + 11] = __builtin_amdgcn_s_memtime();
    }
  }
}



struct HelperLds {
  InterLds inter;
  DbLds db;  // (unused with the coder-side deblock)
};

struct EngineLds {
  union {
    RowLds row;
    HelperLds helper;
  } u;
  int slot;
  int flag;  // helper decisions broadcast from thread 0 (kept out of the union)
};

// Row helper (j, r): the inter search of MB row r, group by group as the
// previous frame becomes final over each group's search window (the row
// coder waits for exactly these), and the deblock of row r, chunk by chunk as
// the coder's granules arrive (advanced whenever the inter search is waiting
// or done).  Never blocks on its own row coder while an inter group is due.
__device__ __forceinline__ void row_helper(FA& a0, int r, HelperLds& L, int* flag, int32_t* tr) {
  FA& a = a0;
  const int tid = threadIdx.x;
  const int nch = db_chunks(a);
  volatile int* vflag = flag;
  DbState st{0, 0, 0, 8};
  for (int g = 0; g < a0.ng; g++) {
    FA& a = *opaque_view(&a0);
    trace(tr, 1, g);
    trace(tr, 2, (int)a.epoch * 1000 + r);
    uint64_t* is = a.istamps && tid == 0 ? a.istamps + (size_t)(r * a.ng + g) * kIStamps : nullptr;
    if (is) is[0] = __builtin_amdgcn_s_memrealtime(), is[3] = is[4] = is[5] = is[6] = is[7] = is[8] = is[9] = is[10] = 0;
    // The older references (offsets 2..R-1) first: frame index-2 is final
    // over the group's level-1 window long before the previous frame is (its
    // progress word, tagged epoch-2, also covers frame index-3: that frame's
    // row r+2 waited for index-3's row r+4 over a wider window), so these
    // searches fill what used to be the wait for the previous frame.
    if (a.inter) group_source(a, r, g, L.inter);
    if (a.inter && a.nref >= 2) {
      helper_wait(a, 2, r, min(r + 2, a.hmb - 1), inter_need_cols(a, g, 1), L.db, st, flag);
      const uint64_t ts = acct_now();
      zero_mv_older(a, r, g, L.inter);
      for (int off = 2; off <= a.nref; off++) inter_task(a, r, g, off, L.inter, L.db, st, flag, is);
      acct_add(a.acct, Acct::kHelperSearch, acct_now() - ts);
    }
    // level 1 of the group's window in the previous frame; deblock meanwhile
    // (leaving the chunks to the catch-up after the group's records instead
    // measured neutral in round 4; catch-ups between the older references'
    // searches too, in round 5)
    helper_wait(a, 1, r, min(r + 2, a.hmb - 1), inter_need_cols(a, g, 1), L.db, st, flag);
    if (is) is[1] = __builtin_amdgcn_s_memrealtime();
    trace(tr, 3, 50);
    if (a.inter) {
      const uint64_t ts = acct_now();
      inter_task(a, r, g, 1, L.inter, L.db, st, flag, is);
      acct_add(a.acct, Acct::kHelperSearch, acct_now() - ts);
    } else if (tid == 0) {  // intra frame: carry the dependency only
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&a.inter_done[r * a.ng + g], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (is) is[2] = __builtin_amdgcn_s_memrealtime();
    int caught = 0;
    const uint64_t tc = acct_now();
    uint64_t tcdb = 0;
    for (;;) {  // catch the deblock up with what has arrived
      int d = 0;
      if (tid == 0) d = st.k < nch && deblock_chunk_ready(a, r, st);
      if (!wg_broadcast(vflag, d)) break;
      const uint64_t tb = acct_now();
      deblock_chunk(a, r, L.db, st, true);
      tcdb += acct_now() - tb;
      caught++;
    }
    acct_add(a.acct, Acct::kHelperCatchup, acct_now() - tc - tcdb);
    if (is) is[11] = ((uint64_t)caught << 32) | (uint32_t)(__builtin_amdgcn_s_memrealtime() - is[2]);
  }
  trace(tr, 1, 1000);
  // The rest of the row trails its coder: one lane polls each chunk's
  // readiness (row r-1's progress and the chunk's last info granule, with
  // back-off) while the other waves sit at the barrier, instead of every
  // lane of the chunk's loads re-polling its own granule.
  while (st.k < nch) {
    trace(tr, 3, 60000 + st.k);
    int d = 0;
    if (tid == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (!(d = deblock_chunk_ready(a, r, st))) {
        if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
            __builtin_amdgcn_s_memrealtime() - t0 > 100000000ull)
          break;  // deblock_chunk's own bounded waits report it
        __builtin_amdgcn_s_sleep(kWaitSleep);
      }
    }
    deblock_chunk(a, r, L.db, st, wg_broadcast(vflag, d) != 0);
  }
  trace(tr, 3, 100000);
  if (a.stamps && tid == 0) {  // the row's deblock times, in per-row stamp slots no chunk uses at these widths
    uint64_t* ds = a.stamps + (size_t)a.wmb * a.hmb * kStampPhases + (size_t)r * kDbStamps;
    ds[kDbStamps - 1] = st.busy;
  }
}

// ---------------------------------------------------------------------------
// The engine: one persistent launch encodes a batch of consecutive frames,
// pipelined across frames.  Two worker pools (helpers and row coders,
// spread over the block indices: is_helper) dequeue (frame, row) tasks in their e.order (by row + slope * frame):
//   helper (j, r): inter search of row r, group g (MBs 4g..4g+3) once the
//           previous frame is final on MB rows r-2..r+2 over the group's
//           search window [64g-32, 64g+96) (this also covers every older
//           frame, transitively); and the deblock of row r behind its coder;
//   rows   (j, r): code MB row r; before MBs 4g..4g+3 it waits for group g's
//           inter records (and thereby every cross-frame dependency: the
//           frames still reading this slot's old content are done with it
//           there, the stale rows below are final); rows above arrive as
//           granules.
// Every wait targets an earlier frame, or an earlier row, or the same row's
// other worker, which never waits back (a helper only polls its coder's
// granules, without blocking, while an inter group is due).  Each pool
// dequeues in order, so the oldest unfinished task always progresses: no
// deadlock with every workgroup resident.
// ---------------------------------------------------------------------------

constexpr int kPrioLevel = 2;        // (1 and 3 measured the same)

// Pool of workgroup b out of n, nh of them helpers: spread evenly over the
// block indices (so over every XCD, which take blocks round-robin), and a
// launch that is only partly resident (a shared or partitioned GPU) still
// has workers of both pools.
__device__ __forceinline__ bool is_helper(int b, int nh, int n) {
  return ((b + 1) * nh) / n > (b * nh) / n;
}

// The next task of a pool.  Each label has a queue in the task order (row +
// e.slope * frame) in this launch and one in the previous launch's (whose
// frames come first, so its frame j is this launch's frame j - pframes); a
// label's head is the earlier of the two, so the previous batch's tail
// interleaves with this batch's first rows as the order says and the two
// co-resident launches share their pools.  A worker takes its own label's
// head unless another label's head is more than kSteal keys earlier (or its
// own queues are exhausted): then it takes that one.  Every task a worker
// takes is thus no later than its own label's head, so the oldest unfinished
// task always has a free worker: its label's workers hold only
// finished tasks.  Returns the task's index in its order (prev: the previous
// launch's), or -1 when every queue is exhausted.
constexpr int kSteal = 2;
__device__ __forceinline__ int next_task(const EngineArgs& e, int pool, int lab, EngineLds& L, bool& prev) {
  const int ptotal = e.ptotal;
  if (threadIdx.x < 64) {  // wave 0; lane l < nlab looks after label l
    const int l = threadIdx.x, nlab = e.nlab[pool];
    const bool act = l < nlab;
    const int pframes = ptotal / e.hmb;
    const int tk = (pool ? SyncLayout::kTicketRows : SyncLayout::kTicketHelpers) + (act ? l : 0);
    const int32_t* __restrict__ order = e.order[pool];
    const int32_t* __restrict__ porder = e.porder[pool];
    int b0 = 0, n0 = 0, pb0 = 0, pn0 = 0;
    if (act) {
      b0 = e.seg[pool][l], n0 = e.seg[pool][l + 1] - b0;
      if (ptotal) pb0 = e.pseg[pool][l], pn0 = e.pseg[pool][l + 1] - pb0;
    }
    constexpr int kNone = 0x7FFFFFFF;
    int res = -1, q = 0;
    for (;;) {
      int key = kNone;
      bool usep = false;
      if (act) {
        const int tp = pn0 ? __hip_atomic_load(e.psync + tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        const int tb = __hip_atomic_load(e.sync + tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int kp = kNone, kb = kNone;
        if (tp < pn0) {
          const int op = porder[pb0 + tp];
          kp = (op & 0xFFFF) + e.slope * (op >> 16);
        }
        if (tb < n0) {
          const int ob = order[b0 + tb];
          kb = (ob & 0xFFFF) + e.slope * (pframes + (ob >> 16));
        }
        usep = kp <= kb && kp != kNone;
        key = min(kp, kb);
      }
      int mn = key;
      for (int o = 1; o < kLabels; o <<= 1) mn = min(mn, __shfl_xor(mn, o));
      mn = __shfl(mn, 0);
      if (mn == kNone) break;  // every queue exhausted
      const int own = __shfl(key, lab);
      const int z = (own != kNone && own - mn <= kSteal) ? lab : __ffsll(__ballot(act && key == mn)) - 1;
      int ok = 0;
      if (l == z) {
        const int tt = __hip_atomic_fetch_add((usep ? e.psync : e.sync) + tk, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        if (tt < (usep ? pn0 : n0)) ok = 1, res = tt + (usep ? pb0 : b0), q = usep;
      }
      if (__shfl(ok, z)) {  // else taken meanwhile: look again
        res = __shfl(res, z), q = __shfl(q, z);
        break;
      }
    }
    if (l == 0) {
      L.slot = res;
      L.flag = q;
    }
  }
  __syncthreads();
  const int t = uni(L.slot);
  prev = uni(L.flag) != 0;
  __syncthreads();
  return t;
}

// This workgroup's label and pool.  With per-label queues (e.nlab ==
// kLabels) the block indices split into kLabels classes (b % kLabels), each
// with its share of both pools; the launch's workers agree on one offset
// (the first to arrive proposes XCC_ID - b, i.e. the offset that makes a
// label an XCD when blocks are dealt round-robin) so labels stay a
// partition of the classes whatever the placement.
__device__ __forceinline__ int worker_label(const EngineArgs& e, int b, bool& helper, EngineLds& L) {
  const int n = e.n_helpers + e.n_rows;
  if (e.nlab[0] == 1 && e.nlab[1] == 1) {
    helper = is_helper(b, e.n_helpers, n);
    return 0;
  }
  helper = is_helper(b / kLabels, e.n_helpers / kLabels, n / kLabels);
  if (e.nlab[helper ? 0 : 1] == 1) return 0;
  if (threadIdx.x == 0) {
    const int xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & (kLabels - 1);  // HW_REG_XCC_ID[3:0]
    int want = ((xcc - b) & (kLabels - 1)) + 1, seen = 0;
    if (!__hip_atomic_compare_exchange_strong(e.sync + SyncLayout::kLabelOff, &seen, want, __ATOMIC_RELAXED,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      want = seen;
    L.slot = (b + want - 1) & (kLabels - 1);
  }
  __syncthreads();
  const int lab = uni(L.slot);
  __syncthreads();
  return lab;
}

// A finished task counts toward its batch's completion (k_batch_wait) once
// all its stores are visible.
__device__ __forceinline__ void task_done(int32_t* sync) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(sync + SyncLayout::kDone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <bool kDecode>
__global__ __launch_bounds__(256, 3) void k_engine(EngineArgs e) {
  __shared__ EngineLds L;
  load_tables();
  const int b = blockIdx.x, hmb = e.hmb;
  uint64_t* ks = e.stamps ? e.stamps + (size_t)kMaxBatch * stamp_frame_words(e.wmb, hmb) : nullptr;
  if (ks && threadIdx.x == 0)
    __hip_atomic_fetch_min(&ks[0], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool helper;
  const int lab = worker_label(e, b, helper, L);
  if (helper) {
    // The helpers' inter records gate every row coder at its group starts:
    // on large frames they win the SIMD issue arbitration against the coders'
    // waves (A/B: 1080p +3 %, 4K +3 %; 720p -1 %, so not there).
    if (e.wmb * e.hmb > kPrioFrameMBs) __builtin_amdgcn_s_setprio(kPrioLevel);
    for (;;) {
      bool prev;
      const uint64_t tq = acct_now();
      const int t = next_task(e, 0, lab, L, prev);
      acct_add(e.acct, Acct::kHelperDequeue, acct_now() - tq);
      if (t < 0) break;
      trace(e.trace, 0, 1000000 + t);
      const int32_t o = (prev ? e.porder : e.order)[0][t];
      const uint64_t tt = acct_now();
      row_helper(((FA*)(prev ? e.pfa : e.fa))[uni(o >> 16)], o & 0xFFFF, L.u.helper, &L.flag, e.trace);
      task_done(prev ? e.psync : e.sync);
      acct_add(e.acct, Acct::kHelperTotal, acct_now() - tt);
      acct_add(e.acct, Acct::kHelperTasks, 1);
      trace(e.trace, 0, 2000000 + t);
    }
  } else {
    for (;;) {
      bool prev;
      const uint64_t tq = acct_now();
      const int t = next_task(e, 1, lab, L, prev);
      acct_add(e.acct, Acct::kCoderDequeue, acct_now() - tq);
      if (t < 0) break;
      trace(e.trace, 0, 3000000 + t);
      const int32_t o = (prev ? e.porder : e.order)[1][t];
      const uint64_t tt = acct_now();
      code_row<kDecode>(((FA*)(prev ? e.pfa : e.fa))[uni(o >> 16)], o & 0xFFFF, L.u.row, &L.flag, e.trace);
      task_done(prev ? e.psync : e.sync);
      acct_add(e.acct, Acct::kCoderTotal, acct_now() - tt);
      acct_add(e.acct, Acct::kCoderTasks, 1);
      acct_add(e.acct, Acct::kCoderMBs, (uint64_t)e.wmb);
      trace(e.trace, 0, 4000000 + t);
    }
  }
  if (ks && threadIdx.x == 0)
    __hip_atomic_fetch_max(&ks[1], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(192) void k_unpack_granules(EngineArgs e, int j, PlaneSet dst) {
  FA& a = ((FA*)e.fa)[j];
  const int mb = blockIdx.x, k = threadIdx.x;
  const int mbx = mb % a.wmb, mby = mb / a.wmb;
  const uint32_t v = (uint32_t)a.granules[(size_t)mb * kGranuleStride + k];
  int16_t* p;
  if (k < 128) {
    p = dst.y + (size_t)(mby * 16 + (k >> 3)) * a.wa + mbx * 16 + 2 * (k & 7);
  } else {
    const int u = k - 128, pl = u >> 5, r = (u & 31) >> 2, d = u & 3;
    p = (pl ? dst.v : dst.u) + (size_t)(mby * 8 + r) * (a.wa >> 1) + mbx * 8 + 2 * d;
  }
  p[0] = (int16_t)(v & 0xFFFF);
  p[1] = (int16_t)(v >> 16);
}

hipError_t launch_unpack_granules(const EngineArgs& e, int j, PlaneSet dst, hipStream_t s) {
  hipLaunchKernelGGL(k_unpack_granules, dim3(e.wmb * e.hmb), dim3(kGranulesPerMB), 0, s, e, j, dst);
  return hipGetLastError();
}

FrameArgs make_frame_view(const EngineArgs& e, const FrameDesc& f, int j) {
  FrameArgs a{};
  a.wa = e.wa, a.ha = e.ha, a.w = e.w, a.h = e.h, a.wmb = e.wmb, a.hmb = e.hmb, a.ring = e.ring;
  a.index = f.index;
  a.decode = f.decode;
  a.inter = f.inter && e.ring > 1 && !f.decode;  // a decoded frame's helpers only carry dependencies
  a.quality = f.quality;
  a.epoch = f.epoch;
  a.in = ring_slot(e.src_base, e.plane_elems, e.wa, e.ha, f.slot);
  a.coef = f.coef;
  a.coef_prev = f.coef_prev;
  for (int k = 0; k < kMaxRing; k++) a.recon[k] = f.recon[k];
  a.stale = f.stale;
  const size_t mbs = (size_t)e.wmb * e.hmb, nref = e.ring > 1 ? e.ring - 1 : 1;
  a.table = e.table_base + (size_t)f.slot * mbs;
  a.inter_desc = e.idesc_base + (size_t)f.slot * nref * mbs;
  a.granules = e.gran_base + (size_t)f.slot * mbs * kGranuleStride;
  a.err = e.sync + SyncLayout::kErr;
  a.sticky = e.sticky;
  a.member = f.member;
  a.inject = e.inject;
  a.ng = (e.wmb + 3) >> 2;
  a.nref = a.inter ? e.ring - 1 : 1;
  a.inter_done = e.sync + SyncLayout::inter_done(e.hmb, a.ng, j);
  a.progress = f.progress;
  a.prev_progress = f.prev_progress;
  a.prev2_progress = f.prev2_progress;
  a.npush = f.npush;
  for (int k = 0; k < kMaxPush; k++) a.push[k] = f.push[k];
  a.sys = f.sys;
  // deblock chunk width: a wider chunk amortizes the chunk's fixed latencies
  // (granule round trip, drain, barriers) over more columns but publishes the
  // row's progress later, which the next frame's searches wait for; narrow
  // frames feel the latter more (A/B, Mpix/s, chunk 16 / 32 / 64: 720p
  // 3859-3870 / 3384-3435 / 2893-2916, 1080p 4549 / 4660 / 4133, 4K 4784 /
  // 4940 / 5040)
  a.db_shift = e.wmb >= 200 ? 6 : e.wmb >= 100 ? 5 : 4;
  a.stamps = e.stamps ? e.stamps + (size_t)j * stamp_frame_words(e.wmb, e.hmb) : nullptr;
  a.acct = e.acct;
  {
    const int ng = (e.wmb + 3) / 4;
    a.istamps = e.stamps ? e.stamps + (size_t)kMaxBatch * stamp_frame_words(e.wmb, e.hmb) + 2 +
                               (size_t)j * e.hmb * ng * kIStamps
                         : nullptr;
  }
  a.rgb = f.rgb;
  return a;
}

hipError_t engine_blocks_per_cu(int* n) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, reinterpret_cast<const void*>(&k_engine<false>), 256, 0);
}

// One wave: thread 0 polls the batch's finished-task count.
__global__ __launch_bounds__(64) void k_batch_wait(int32_t* sync, int tasks, int32_t* sticky) {
  if (threadIdx.x) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(sync + SyncLayout::kDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < tasks) {
    __builtin_amdgcn_s_sleep(8);
    if (__hip_atomic_load(sync + SyncLayout::kErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {  // 4 s
      report_timeout(sync + SyncLayout::kErr, sticky, kWaitBatch, 0, -1, -1, -1, tasks, 0,
                     (uint32_t)__hip_atomic_load(sync + SyncLayout::kDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

hipError_t launch_batch_wait(int32_t* sync, int tasks, int32_t* sticky, hipStream_t s) {
  hipLaunchKernelGGL(k_batch_wait, dim3(1), dim3(64), 0, s, sync, tasks, sticky);
  return hipGetLastError();
}

hipError_t launch_engine(const EngineArgs& e, hipStream_t s) {
  if (e.decode)
    hipLaunchKernelGGL(k_engine<true>, dim3(e.n_helpers + e.n_rows), dim3(256), 0, s, e);
  else
    hipLaunchKernelGGL(k_engine<false>, dim3(e.n_helpers + e.n_rows), dim3(256), 0, s, e);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// convert_image YUV -> RGB (convert.cpp:16-19, 75-93, 162-223): one thread per
// horizontal pixel pair; saturate narrows to int16 before clipping
// (math.h:218-221).  The crop is min(W, Wa) x min(H, Ha) = W x H.
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint8_t sat8(int32_t v) {
  const int16_t s = (int16_t)v;
  return (uint8_t)(s < 0 ? 0 : (s > 255 ? 255 : s));
}

__global__ __launch_bounds__(256) void k_yuv_to_rgb(PlaneSet src, int wa, int w, int h, uint8_t* rgb) {
  const int x2 = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (2 * x2 >= w) return;
  const int u = src.u[(size_t)(y >> 1) * (wa >> 1) + x2] - 128;
  const int v = src.v[(size_t)(y >> 1) * (wa >> 1) + x2] - 128;
  uint8_t* o = rgb + ((size_t)y * w + 2 * x2) * 3;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int yy = src.y[(size_t)y * wa + 2 * x2 + k] - 16;
    o[3 * k] = sat8((256 * yy + 358 * v + 128) >> 8);
    o[3 * k + 1] = sat8((256 * yy - 88 * u - 182 * v + 128) >> 8);
    o[3 * k + 2] = sat8((256 * yy + 452 * u + 128) >> 8);
  }
}

hipError_t launch_yuv_to_rgb(PlaneSet src, int wa, int w, int h, uint8_t* rgb, hipStream_t s) {
  hipLaunchKernelGGL(k_yuv_to_rgb, dim3((w / 2 + 255) / 256, h), dim3(256), 0, s, src, wa, w, h, rgb);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// KAT: transform/quantize/reconstruct chain on independent macroblocks.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_kat_transform(const int16_t* src, const int16_t* pred,
                                                       int16_t* coef, int16_t* recon,
                                                       const uint8_t* qtype, int32_t* qvar) {
  __shared__ alignas(16) int16_t sa[kMBElems], sb[kMBElems];
  __shared__ int32_t red[12];
  load_tables();
  const int m = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t type = qtype[2 * m];
  const int quality = qtype[2 * m + 1];
  const bool has_pred = type != kIntra, intra_path = (type & kIntra) && !(type & kMotion);
  const int nblk = wave < 2 ? 2 : 1;
  int cf[2], pv[2];
  for (int bi = 0; bi < nblk; bi++) {
    const int e = (wave + 4 * bi) * 64 + lane;
    pv[bi] = pred[m * kMBElems + e];
    const int sv = src[m * kMBElems + e];
    cf[bi] = fdct_lane(&sa[e - lane], &sb[e - lane], lane,
                       has_pred ? (int16_t)(sv - pv[bi]) : (int16_t)sv);
  }
  int32_t v2;
  const int qp = vaq_mb(red, wave, lane, cf[0], quality, &v2);
  for (int bi = 0; bi < nblk; bi++) {
    const int e = (wave + 4 * bi) * 64 + lane;
    const int16_t qv = quant_elem(e, cf[bi], qp, intra_path);
    coef[m * kMBElems + e] = qv;
    const int t = idct_lane(&sa[e - lane], &sb[e - lane], lane, dequant_elem(e, qv, qp, intra_path));
    recon[m * kMBElems + e] = (int16_t)(has_pred ? t + pv[bi] : t);
  }
  if (threadIdx.x == 0) {
    qvar[2 * m] = qp;
    qvar[2 * m + 1] = v2;
  }
}

hipError_t launch_kat_transform(const int16_t* src, const int16_t* pred, int16_t* coef,
                                int16_t* recon, const uint8_t* qtype, int32_t* qvar, int count,
                                hipStream_t s) {
  hipLaunchKernelGGL(k_kat_transform, dim3(count), dim3(256), 0, s, src, pred, coef, recon, qtype,
                     qvar);
  return hipGetLastError();
}

}  // namespace cairo
