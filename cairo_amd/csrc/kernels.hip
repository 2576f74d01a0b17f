// cairo_amd/csrc/kernels.hip -- the EVX-1 encode hot path on gfx950 (CDNA4).
//
//   K0 k_convert      RGB888 -> planar YUV 4:2:0 int16        convert.cpp:95-160
//   K1 k_inter_search one wave64 per (macroblock, reference)  motion.cpp:421-494
//   K2 k_mb_rows      row-worker wavefront: intra search, classify, transform,
//                     VAQ, quantize, reconstruct              encode.cpp:17-203,
//                                                             decode.cpp:15-144
//   K3 k_deblock      band-worker wavefront, in place         deblock.cpp:201-284
//
// All arithmetic is integer and restates the reference bit for bit (see
// evx_defs.h for the helpers).  Searches evaluate candidates in parallel and
// then replay the reference's sequential, tie-sensitive acceptance in the
// reference's scan order (j outer, i inner) with wave-uniform scalars.
#include "kernels.h"

namespace cairo {

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

// Bounded wait on a progress word (relaxed agent-scope poll + s_sleep).  On
// timeout (~2 s) the error word is set and the wait gives up, so every
// workgroup still drains and the host reports EVX_ERROR_HARDWAREFAIL.
__device__ __forceinline__ void wait_at_least(int32_t* word, int target, int32_t* err,
                                              int32_t* sticky) {
  if (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sticky, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}

// Consumer side of a hand-off: one lane waited; invalidate this CU's L1 and
// let every wave load only after the barrier (MI355X_MICROARCH.md, Valid forms).
__device__ __forceinline__ void acquire_after_wait() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// Producer side: every storing wave drains, barrier, one lane releases the
// XCD's L2 and stores the progress word.
__device__ __forceinline__ void publish(int32_t* word, int value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Dequeue the next task index for this workgroup (uniform result).
__device__ __forceinline__ int dequeue(int32_t* ticket, int* lds_slot) {
  __syncthreads();
  if (threadIdx.x == 0)
    *lds_slot = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return *lds_slot;
}

// XCD-aware remap: the dispatcher deals workgroups round-robin over the 8
// XCDs; give each XCD a contiguous range of tasks so neighbouring macroblocks
// share one L2 (speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int b, int n) {
  int per = (n + 7) >> 3;
  int xcd = b & 7, k = b >> 3;
  int t = xcd * per + k;
  return t < n ? t : -1;
}

// ---------------------------------------------------------------------------
// K0: RGB888 -> YUV 4:2:0 int16 (convert.cpp:11-14, 30-73, 95-160)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_convert(FrameArgs a) {
  int qx = blockIdx.x * 256 + threadIdx.x;  // quad column
  int qy = blockIdx.y;                      // quad row
  if (qx >= (a.w >> 1)) return;
  int su = 0, sv = 0;
#pragma unroll
  for (int dy = 0; dy < 2; dy++) {
    const uint8_t* p = a.rgb + ((size_t)(2 * qy + dy) * a.w + 2 * qx) * 3;
    int16_t* y = a.in.y + (size_t)(2 * qy + dy) * a.wa + 2 * qx;
#pragma unroll
    for (int dx = 0; dx < 2; dx++) {
      int r = p[3 * dx], g = p[3 * dx + 1], b = p[3 * dx + 2];
      y[dx] = (int16_t)(((77 * r + 150 * g + 29 * b + 128) >> 8) + 16);
      su = (int16_t)(su + (((-43 * r - 85 * g + 128 * b + 128) / 256) + 128));
      sv = (int16_t)(sv + (((128 * r - 107 * g - 21 * b + 128) / 256) + 128));
    }
  }
  a.in.u[(size_t)qy * (a.wa >> 1) + qx] = (int16_t)((su + 2) >> 2);
  a.in.v[(size_t)qy * (a.wa >> 1) + qx] = (int16_t)((sv + 2) >> 2);
}

hipError_t launch_convert(const FrameArgs& a, hipStream_t s) {
  dim3 grid((a.w / 2 + 255) / 256, a.h / 2);
  hipLaunchKernelGGL(k_convert, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Search window in LDS: an 80x80 luma tile and two 40x40 chroma tiles around
// the macroblock, covering every candidate a search can reach.
// ---------------------------------------------------------------------------

constexpr int kWinL = 80, kWinLP = 88;  // luma tile, pitch (elements)
constexpr int kWinC = 40, kWinCP = 48;  // chroma tile, pitch (elements)

struct alignas(16) Window {
  int16_t y[kWinL * kWinLP];
  int16_t u[kWinC * kWinCP];
  int16_t v[kWinC * kWinCP];
};

// Stage the in-frame part of the window with origin (ox, oy) (luma pixels,
// multiples of 16) from plane set p.  All threads of the block participate.
__device__ __forceinline__ void load_window(Window& w, const PlaneSet& p, int wa, int ha, int ox,
                                            int oy, int nthreads) {
  // Luma: 80 rows x 10 chunks of 8 pixels (16 B).
  for (int k = threadIdx.x; k < kWinL * 10; k += nthreads) {
    int r = k / 10, c = (k - r * 10) * 8;
    int gy = oy + r, gx = ox + c;
    if (gy >= 0 && gy < ha && gx >= 0 && gx < wa)
      *(int4*)&w.y[r * kWinLP + c] = *(const int4*)&p.y[(size_t)gy * wa + gx];
  }
  // Chroma: 40 rows x 5 chunks of 8 pixels, per plane.
  int cw = wa >> 1, ch = ha >> 1, cox = ox >> 1, coy = oy >> 1;
  for (int k = threadIdx.x; k < 2 * kWinC * 5; k += nthreads) {
    int pl = k / (kWinC * 5), kk = k - pl * kWinC * 5;
    int r = kk / 5, c = (kk - r * 5) * 8;
    int gy = coy + r, gx = cox + c;
    if (gy >= 0 && gy < ch && gx >= 0 && gx < cw) {
      const int16_t* src = pl ? p.v : p.u;
      int16_t* dst = pl ? w.v : w.u;
      *(int4*)&dst[r * kWinCP + c] = *(const int4*)&src[(size_t)gy * cw + gx];
    }
  }
}

// Per-lane slice of a macroblock: luma row l>>2, columns (l&3)*4..+3, and the
// chroma pixel (l>>3, l&7) of U and V.
struct Px6 {
  int y0, y1, y2, y3, u, v;
};

__device__ __forceinline__ Px6 px_from_window(const Window& w, int wx, int wy) {
  int l = lane_id();
  const int16_t* py = &w.y[(wy + (l >> 2)) * kWinLP + wx + (l & 3) * 4];
  int cwx = wx >> 1, cwy = wy >> 1;  // caller passes window coords with the same parity as frame coords
  Px6 r;
  r.y0 = py[0];
  r.y1 = py[1];
  r.y2 = py[2];
  r.y3 = py[3];
  r.u = w.u[(cwy + (l >> 3)) * kWinCP + cwx + (l & 7)];
  r.v = w.v[(cwy + (l >> 3)) * kWinCP + cwx + (l & 7)];
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
__device__ __forceinline__ Px6 lerp6(const Px6& a, const Px6& b, int q) {
  Px6 r;
  r.y0 = lerp_px(a.y0, b.y0, q);
  r.y1 = lerp_px(a.y1, b.y1, q);
  r.y2 = lerp_px(a.y2, b.y2, q);
  r.y3 = lerp_px(a.y3, b.y3, q);
  r.u = lerp_px(a.u, b.u, q);
  r.v = lerp_px(a.v, b.v, q);
  return r;
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
// K1: inter search, one wave64 per (macroblock, reference offset)
// (calculate_inter_prediction, motion.cpp:421-494)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(64) void k_inter_search(FrameArgs a) {
  __shared__ Window win;
  const int mbs = a.wmb * a.hmb, nref = a.ring - 1;
  const int task = xcd_remap(blockIdx.x, mbs * nref);
  if (task < 0) return;
  const int off = task / mbs + 1, mb = task - (off - 1) * mbs;
  const int px = (mb % a.wmb) * kMB, py = (mb / a.wmb) * kMB;
  const int thr = (a.quality >> 2) + 1;
  const PlaneSet ref = ring_slot(a.ring_base, a.slot_elems, a.wa, a.ha, (a.index + a.ring - off) % a.ring);

  const Px6 src = px_from_planes(a.in, a.wa, px, py);
  Sel s;
  s.bx = px;
  s.by = py;
  s.ssd = INT32_MAX;
  s.sp_idx = s.sp_amt = s.sp_en = 0;
  sad_mad(src, px_from_planes(ref, a.wa, px, py), s.sad, s.mad);

  if (s.mad >= thr) {
    const int ox = px - 32, oy = py - 32;  // window origin
    load_window(win, ref, a.wa, a.ha, ox, oy, 64);
    __syncthreads();
    for (int step = kRadius; step > 0; step >>= 1) {
      const int bx = s.bx, by = s.by;
      for (int j = -step; j <= step; j += step)
        for (int i = -step; i <= step; i += step) {
          const int cx = bx + i, cy = by + j;
          if (!in_frame(cx, cy, a.wa, a.ha)) continue;
          int sad, mad;
          sad_mad(src, px_from_window(win, cx - ox, cy - oy), sad, mad);
          accept_int(s, cx, cy, sad, mad, px, py, thr);
        }
    }
    // Sub-pel: half then quarter lerp toward each of the 8 neighbours.
    const Px6 best = px_from_window(win, s.bx - ox, s.by - oy);
    s.sp_idx = s.sp_amt = s.sp_en = 0;
    const int bx = s.bx, by = s.by;
    for (int j = -1; j <= 1; j++)
      for (int i = -1; i <= 1; i++) {
        if (i == 0 && j == 0) continue;
        const int tx = bx + i, ty = by + j;
        if (!in_frame(tx, ty, a.wa, a.ha)) continue;
        const Px6 nb = px_from_window(win, tx - ox, ty - oy);
        const int idx = frac_index(i, j);
        for (int q = 0; q < 2; q++) {
          int sad, mad;
          sad_mad(src, lerp6(best, nb, q), sad, mad);
          accept_sub(s, idx, q, sad, mad, thr);
        }
      }
  }
  if (threadIdx.x == 0) {
    a.inter_desc[task] = make_desc(s, px, py, thr, false, off);
    a.inter_sad[task] = s.sad;
  }
}

hipError_t launch_inter_search(const FrameArgs& a, hipStream_t s) {
  int n = a.wmb * a.hmb * (a.ring - 1);
  if (n <= 0) return hipSuccess;
  int grid = ((n + 7) / 8) * 8;
  hipLaunchKernelGGL(k_inter_search, dim3(grid), dim3(64), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Transform / quantization on a macroblock held block-major in LDS:
// element (b, r, c) at b*64 + r*8 + c; b = 0..3 luma quadrants TL TR BL BR,
// 4 = U, 5 = V (transform.cpp:264-594, quantize.cpp:79-379).
// ---------------------------------------------------------------------------

constexpr int kMBElems = 384;

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

// Forward row pass (transform_8x8_line_fast along rows) then column pass;
// intermediate stored as int16.  in -> out, scratch tmp.  256 threads.
__device__ void fdct_mb(const int16_t* in, int16_t* tmp, int16_t* out) {
  for (int e = threadIdx.x; e < kMBElems; e += 256) {
    int b = e >> 6, r = (e >> 3) & 7, i = e & 7;
    const int16_t* row = in + b * 64 + r * 8;
    int t = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) t += row[k] * kLut8[i * 8 + k];
    t = i == 0 ? (t * 45) / 128 : t / 2;
    tmp[e] = (int16_t)rdiv(t, 128);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kMBElems; e += 256) {
    int b = e >> 6, i = (e >> 3) & 7, c = e & 7;
    const int16_t* col = tmp + b * 64 + c;
    int t = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) t += col[k * 8] * kLut8[i * 8 + k];
    t = i == 0 ? (t * 45) / 128 : t / 2;
    out[e] = (int16_t)rdiv(t, 128);
  }
  __syncthreads();
}

// Inverse: column pass then row pass (inverse_transform_8x8_line_fast, per-term
// truncation); the row pass adds pred when add != 0 (int16 result, unclamped).
__device__ void idct_mb(const int16_t* in, int16_t* tmp, const int16_t* pred, bool add,
                        int16_t* out) {
  for (int e = threadIdx.x; e < kMBElems; e += 256) {
    int b = e >> 6, i = (e >> 3) & 7, c = e & 7;
    const int16_t* col = in + b * 64 + c;
    int t = ((col[0] * kLut8[i]) * 45) / 128;
#pragma unroll
    for (int k = 1; k < 8; k++) t += (col[k * 8] * kLut8[k * 8 + i]) / 2;
    tmp[e] = (int16_t)rdiv(t, 128);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kMBElems; e += 256) {
    int b = e >> 6, r = (e >> 3) & 7, i = e & 7;
    const int16_t* row = tmp + b * 64 + r * 8;
    int t = ((row[0] * kLut8[i]) * 45) / 128;
#pragma unroll
    for (int k = 1; k < 8; k++) t += (row[k] * kLut8[k * 8 + i]) / 2;
    t = rdiv(t, 128);
    out[e] = (int16_t)(add ? t + pred[e] : t);
  }
  __syncthreads();
}

// variance2 of the 16x16 luma coefficients (analysis.h:176-198): skip only the
// first coefficient of the top-left quadrant; wrapping int32 arithmetic.
// Threads 0..255 hold one luma coefficient each.  Returns a uniform value.
__device__ int32_t variance2_mb(const int16_t* coef, int32_t* red /* LDS, 12 words */) {
  int e = threadIdx.x;  // < 256: luma
  int32_t t = coef[e];
  bool use = e != 0 && t != 0;
  uint32_t sum = use ? (uint32_t)t : 0u, sq = use ? (uint32_t)(t * t) : 0u;
  int cnt = use ? 1 : 0;
  int ws = wave_sum((int)sum), wq = wave_sum((int)sq), wc = wave_sum(cnt);
  int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    red[w] = ws;
    red[4 + w] = wq;
    red[8 + w] = wc;
  }
  __syncthreads();
  uint32_t S = (uint32_t)red[0] + (uint32_t)red[1] + (uint32_t)red[2] + (uint32_t)red[3];
  uint32_t Q = (uint32_t)red[4] + (uint32_t)red[5] + (uint32_t)red[6] + (uint32_t)red[7];
  int32_t C = red[8] + red[9] + red[10] + red[11];
  __syncthreads();
  if (C <= 0) return 0;
  int32_t sq2 = (int32_t)(S * S);
  return (int32_t)(Q - (uint32_t)rdiv(sq2, C));
}

// quantize_macroblock (quantize.cpp:357-367): element-wise.
__device__ __forceinline__ int16_t quant_elem(int e, int32_t c, int qp, bool intra_path) {
  int b = e >> 6, k = e & 63;
  if (intra_path) {
    if (k == 0) return (int16_t)rdiv(c, b < 4 ? luma_dc_scale(qp) : chroma_dc_scale(qp));
    return (int16_t)rdiv(rdiv(c * kQScale, kQmIntra[k]), qp << 1);
  }
  int16_t qf = (int16_t)rdiv(c * kQScale, kQmInter[k]);
  return (int16_t)rdiv(qf - sign16(qf) * qp, qp << 1);
}
// inverse_quantize_macroblock (quantize.cpp:369-379): element-wise.
__device__ __forceinline__ int16_t dequant_elem(int e, int32_t v, int qp, bool intra_path) {
  int b = e >> 6, k = e & 63;
  if (intra_path) {
    if (k == 0) return (int16_t)(v * (b < 4 ? luma_dc_scale(qp) : chroma_dc_scale(qp)));
    return (int16_t)((2 * v * kQmIntra[k] * qp) / kQScale);
  }
  return (int16_t)(((2 * v) * kQmInter[k] * qp) / kQScale);
}

// Shared per-macroblock encode/reconstruct chain (encode_block + decode_block
// for the non-copy types): residual -> fdct -> VAQ -> quantize -> dequantize ->
// idct (+pred).  src/pred/res/tmp/coef/rec are LDS arrays of 384.
// Returns q_index; variance via *var.
__device__ uint32_t code_mb(const int16_t* src, const int16_t* pred, uint32_t type, int quality,
                            int16_t* res, int16_t* tmp, int16_t* coef, int16_t* qc,
                            int16_t* rec, int32_t* red, int32_t* var) {
  const bool has_pred = type != kIntra;  // INTRA_DEFAULT transforms the source
  for (int e = threadIdx.x; e < kMBElems; e += 256)
    res[e] = has_pred ? (int16_t)(src[e] - pred[e]) : src[e];
  __syncthreads();
  fdct_mb(res, tmp, coef);
  int32_t v2 = variance2_mb(coef, red);
  uint32_t qp = vaq_from_variance((uint32_t)quality, v2);
  *var = v2;
  const bool intra_path = (type & kIntra) && !(type & kMotion);
  for (int e = threadIdx.x; e < kMBElems; e += 256) {
    int16_t q = quant_elem(e, coef[e], (int)qp, intra_path);
    qc[e] = q;
    res[e] = dequant_elem(e, q, (int)qp, intra_path);
  }
  __syncthreads();
  idct_mb(res, tmp, pred, has_pred, rec);
  return qp;
}

// ---------------------------------------------------------------------------
// K2: the macroblock wavefront.  One workgroup owns one macroblock row at a
// time (dequeued in order) and walks it left to right.  MB (bx, by) starts
// when row by-1 has finished MB bx+2, i.e. the schedule t = bx + 3*by that
// reproduces the raster order's reads of in-progress (rows above, left) and
// stale (row below, frame n-R) reconstruction bit for bit.
// ---------------------------------------------------------------------------

struct alignas(16) MbLds {
  Window win;
  int16_t src[kMBElems], pred[kMBElems], res[kMBElems], tmp[kMBElems], coef[kMBElems],
      qc[kMBElems], rec[kMBElems];
  int32_t cand[2][16][2];  // double-buffered candidate (sad, mad)
  int32_t red[12];
  int slot;
};

// Evaluate candidate c of a 3x3 step (j outer, i inner) for the intra search.
__device__ __forceinline__ bool intra_valid(int cx, int cy, int px, int py, int wa, int ha) {
  if (cy > py - kMB && cx > px - kMB) return false;  // not yet coded (motion.cpp:239-243)
  return in_frame(cx, cy, wa, ha);
}

__global__ __launch_bounds__(256) void k_mb_rows(FrameArgs a) {
  __shared__ MbLds L;
  const int wave = threadIdx.x >> 6;
  const int thr = (a.quality >> 2) + 1;
  const int cur = a.index % a.ring;
  const PlaneSet cs = ring_slot(a.ring_base, a.slot_elems, a.wa, a.ha, cur);
  int32_t* err = a.sync + SyncLayout::kErr;
  int32_t* done = a.sync + SyncLayout::kRowDone;

  for (;;) {
    const int by = dequeue(a.sync + SyncLayout::kRowTicket, &L.slot);
    if (by >= a.hmb) break;
    const int py = by * kMB;
    for (int bx = 0; bx < a.wmb; bx++) {
      const int px = bx * kMB, mb = by * a.wmb + bx;
      if (by > 0) {
        if (threadIdx.x == 0) wait_at_least(&done[by - 1], min(bx + 3, a.wmb), err, a.sticky);
        acquire_after_wait();
      }
      // Stage the current slot around the MB: x in [px-32, px+48), y in [py-48, py+32).
      const int ox = px - 32, oy = py - 48;
      load_window(L.win, cs, a.wa, a.ha, ox, oy, 256);
      for (int e = threadIdx.x; e < kMBElems; e += 256) {
        int pl, ex, ey;
        elem_coords(e, px, py, pl, ex, ey);
        const int16_t* p = pl == 0 ? a.in.y : (pl == 1 ? a.in.u : a.in.v);
        L.src[e] = p[(size_t)ey * (pl ? a.wa >> 1 : a.wa) + ex];
      }
      __syncthreads();

      // ---- intra search (calculate_intra_prediction, motion.cpp:354-419) ----
      const Px6 src6 = px_from_planes(a.in, a.wa, px, py);
      Sel s;
      s.bx = px;
      s.by = py;
      s.sad = wave_sum(abs(src6.y0) + abs(src6.y1) + abs(src6.y2) + abs(src6.y3));
      s.mad = INT32_MAX;
      s.ssd = INT32_MAX;
      s.sp_idx = s.sp_amt = s.sp_en = 0;
      int buf = 0;
      for (int stage = 0; stage < 5; stage++) {
        const int step = stage == 0 ? kRadius : (kRadius >> stage);
        const int bx0 = s.bx, by0 = s.by;
        // candidate c: j = jlo + (c/3)*step, i = -step + (c%3)*step
        const int jlo = stage == 0 ? -2 * kRadius : -step;
        for (int c = wave; c < 9; c += 4) {
          const int cx = bx0 - step + (c % 3) * step, cy = by0 + jlo + (c / 3) * step;
          int sad = -1, mad = -1;
          if (intra_valid(cx, cy, px, py, a.wa, a.ha))
            sad_mad(src6, px_from_window(L.win, cx - ox, cy - oy), sad, mad);
          if (lane_id() == 0) {
            L.cand[buf][c][0] = sad;
            L.cand[buf][c][1] = mad;
          }
        }
        __syncthreads();
        for (int c = 0; c < 9; c++) {
          const int sad = L.cand[buf][c][0];
          if (sad < 0) continue;
          const int cx = bx0 - step + (c % 3) * step, cy = by0 + jlo + (c / 3) * step;
          accept_int(s, cx, cy, sad, L.cand[buf][c][1], px, py, thr);
        }
        buf ^= 1;
      }
      {  // sub-pel (perform_intra_subpixel_motion_search, motion.cpp:277-317)
        const int bx0 = s.bx, by0 = s.by;
        const Px6 best = px_from_window(L.win, bx0 - ox, by0 - oy);
        for (int n = wave; n < 8; n += 4) {
          const int k = n < 4 ? n : n + 1;  // skip the centre of the 3x3
          const int i = k % 3 - 1, j = k / 3 - 1;
          const int tx = bx0 + i, ty = by0 + j;
          const bool ok = intra_valid(tx, ty, px, py, a.wa, a.ha);
          Px6 nb;
          if (ok) nb = px_from_window(L.win, tx - ox, ty - oy);
          for (int q = 0; q < 2; q++) {
            int sad = -1, mad = -1;
            if (ok) sad_mad(src6, lerp6(best, nb, q), sad, mad);
            if (lane_id() == 0) {
              L.cand[buf][2 * n + q][0] = sad;
              L.cand[buf][2 * n + q][1] = mad;
            }
          }
        }
        __syncthreads();
        s.sp_idx = s.sp_amt = s.sp_en = 0;
        for (int n = 0; n < 8; n++) {
          const int k = n < 4 ? n : n + 1;
          const int idx = frac_index(k % 3 - 1, k / 3 - 1);
          for (int q = 0; q < 2; q++) {
            const int sad = L.cand[buf][2 * n + q][0];
            if (sad < 0) continue;
            accept_sub(s, idx, q, sad, L.cand[buf][2 * n + q][1], thr);
          }
        }
      }
      BlockDesc d = make_desc(s, px, py, thr, true, 0);
      int best_sad = s.sad;

      // ---- classify_block (encode.cpp:17-67) ----
      if (a.inter) {
        const int mbs = a.wmb * a.hmb;
        for (int off = 1; off < a.ring; off++) {
          const BlockDesc in = a.inter_desc[(off - 1) * mbs + mb];
          const int isad = a.inter_sad[(off - 1) * mbs + mb];
          const bool ci = (in.block_type & kCopy) != 0, cb = (d.block_type & kCopy) != 0;
          if (ci != cb) {
            if (ci) {
              d = in;
              best_sad = isad;
            }
          } else if (isad < best_sad) {
            d = in;
            best_sad = isad;
          }
        }
      }

      // ---- prediction block (encode.cpp:80-141, decode.cpp:29-128) ----
      const uint32_t type = d.block_type;
      const bool intra = (type & kIntra) != 0;
      const PlaneSet pp =
          intra ? cs
                : ring_slot(a.ring_base, a.slot_elems, a.wa, a.ha,
                            (a.index + a.ring - d.prediction_target) % a.ring);
      if (type != kIntra) {
        const int mx = px + ((type & kMotion) ? d.motion_x : 0);
        const int my = py + ((type & kMotion) ? d.motion_y : 0);
        int dx = 0, dy = 0;
        const bool sp = (type & kMotion) && d.sp_pred;
        if (sp) frac_dir(d.sp_index, &dx, &dy);
        for (int e = threadIdx.x; e < kMBElems; e += 256) {
          int pl, ex, ey, nx, ny;
          elem_coords(e, mx, my, pl, ex, ey);
          int v;
          if (intra) {
            // from the staged window (identical bytes to the current slot)
            const int16_t* t = pl == 0 ? L.win.y : (pl == 1 ? L.win.u : L.win.v);
            const int pitch = pl == 0 ? kWinLP : kWinCP;
            const int wx = pl == 0 ? ox : (ox >> 1), wy = pl == 0 ? oy : (oy >> 1);
            v = t[(ey - wy) * pitch + ex - wx];
            if (sp) {
              elem_coords(e, mx + dx, my + dy, pl, nx, ny);
              v = lerp_px(v, t[(ny - wy) * pitch + nx - wx], d.sp_amount);
            }
          } else {
            const int16_t* t = pl == 0 ? pp.y : (pl == 1 ? pp.u : pp.v);
            const int pitch = pl == 0 ? a.wa : (a.wa >> 1);
            v = t[(size_t)ey * pitch + ex];
            if (sp) {
              elem_coords(e, mx + dx, my + dy, pl, nx, ny);
              v = lerp_px(v, t[(size_t)ny * pitch + nx], d.sp_amount);
            }
          }
          L.pred[e] = (int16_t)v;
        }
        __syncthreads();
      }

      // ---- encode_block + decode_block ----
      if (type & kCopy) {
        for (int e = threadIdx.x; e < kMBElems; e += 256) L.rec[e] = L.pred[e];
        d.q_index = 0;
        d.variance = 0;
      } else {
        int32_t v2;
        uint32_t qp = code_mb(L.src, L.pred, type, a.quality, L.res, L.tmp, L.coef, L.qc, L.rec,
                              L.red, &v2);
        d.q_index = (uint8_t)qp;
        d.variance = (int16_t)v2;
        for (int e = threadIdx.x; e < kMBElems; e += 256) {
          int pl, ex, ey;
          elem_coords(e, px, py, pl, ex, ey);
          int16_t* p = pl == 0 ? a.coef.y : (pl == 1 ? a.coef.u : a.coef.v);
          p[(size_t)ey * (pl ? a.wa >> 1 : a.wa) + ex] = L.qc[e];
        }
      }
      for (int e = threadIdx.x; e < kMBElems; e += 256) {
        int pl, ex, ey;
        elem_coords(e, px, py, pl, ex, ey);
        int16_t* p = pl == 0 ? cs.y : (pl == 1 ? cs.u : cs.v);
        p[(size_t)ey * (pl ? a.wa >> 1 : a.wa) + ex] = L.rec[e];
      }
      if (threadIdx.x == 0) a.table[mb] = d;
      publish(&done[by], bx + 1);
    }
  }
}

hipError_t launch_mb_rows(const FrameArgs& a, int workgroups, hipStream_t s) {
  int g = workgroups > 0 ? workgroups : a.hmb;
  if (g > a.hmb) g = a.hmb;
  hipLaunchKernelGGL(k_mb_rows, dim3(g), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K3: deblocking (deblock.cpp:201-284).  One workgroup owns one 8-row band of
// one plane at a time and walks it in chunks of 32 edge units; within a chunk
// all horizontal edges run, then all vertical edges (equivalent to the raster
// interleaving: V(x) only reads H(x-1), H(x)).  Band y's chunk [c, c+32)
// starts when band y-1 has finished unit c+32 (t = x + 2y schedule).
// ---------------------------------------------------------------------------

constexpr int kDbChunk = 32;

// deblock_filter_values (deblock.cpp:81-129) on one line through an edge.
__device__ __forceinline__ void dfilter(int16_t* p, int step, int qp, int strength, bool luma) {
  const int p3 = p[-4 * step], p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
  const int q0 = p[0], q1 = p[step], q2 = p[2 * step], q3 = p[3 * step];
  const int16_t dpq = (int16_t)iabs(p0 - q0), dp = (int16_t)iabs(p1 - p0),
                dq = (int16_t)iabs(q1 - q0);
  if (dpq >= kAlpha[qp] || dp >= kBeta[qp] || dq >= kBeta[qp]) return;
  if (strength == 2) {
    p[-step] = (int16_t)rdiv(p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1, 8);
    p[-2 * step] = (int16_t)rdiv(p2 + p1 + p0 + q0, 4);
    p[0] = (int16_t)rdiv(p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2, 8);
    p[step] = (int16_t)rdiv(p0 + q0 + q1 + q2, 4);
    if (luma) {
      p[-3 * step] = (int16_t)rdiv(2 * p3 + 3 * p2 + p1 + p0 + q0, 8);
      p[2 * step] = (int16_t)rdiv(2 * q3 + 3 * q2 + q1 + q0 + p0, 8);
    }
  } else {
    p[-step] = (int16_t)rdiv(((q0 + p0) * 4) + p1 - q1, 8);
    p[0] = (int16_t)rdiv(((q0 + p0) * 4) + q1 - p1, 8);
    if (luma) {
      p[-2 * step] = (int16_t)rdiv((p2 * 4) + (p0 * 2) + (q0 * 2), 8);
      p[step] = (int16_t)rdiv((q2 * 4) + (q0 * 2) + (p0 * 2), 8);
    }
  }
}

// compute_average_qp / compute_deblock_strength (deblock.cpp:49-79).
__device__ __forceinline__ int edge_strength(const BlockDesc& l, const BlockDesc& r, int& qp) {
  const bool cl = (l.block_type & kCopy) != 0, cr = (r.block_type & kCopy) != 0;
  qp = (!cl && !cr) ? ((l.q_index + r.q_index) >> 1) : (!cl ? l.q_index : (!cr ? r.q_index : 0));
  return (cl && cr) ? 0 : ((cl != cr) ? 1 : 2);
}

__global__ __launch_bounds__(256) void k_deblock(FrameArgs a) {
  __shared__ int slot;
  const int plane = blockIdx.y;
  const bool luma = plane == 0;
  const int mbsz = luma ? 16 : 8;
  const int width = luma ? a.wa : (a.wa >> 1), height = luma ? a.ha : (a.ha >> 1);
  const PlaneSet cs = ring_slot(a.ring_base, a.slot_elems, a.wa, a.ha, a.index % a.ring);
  int16_t* img = plane == 0 ? cs.y : (plane == 1 ? cs.u : cs.v);
  const int nx = width / 8, nbands = height / 8;
  const int wib = width / mbsz;
  int32_t* err = a.sync + SyncLayout::kErr;
  int32_t* prog = a.sync + SyncLayout::db_base(a.hmb, plane);
  for (;;) {
    const int band = dequeue(a.sync + SyncLayout::kDbTicket + plane, &slot);
    if (band >= nbands) break;
    const int j = band * 8;
    for (int c = 0; c < nx; c += kDbChunk) {
      const int cend = min(c + kDbChunk, nx);
      if (band > 0) {
        if (threadIdx.x == 0) wait_at_least(&prog[band - 1], min(cend + 1, nx), err, a.sticky);
        acquire_after_wait();
        // horizontal edges H(x, j), x in [c, cend): column filters
        const int x = c + (threadIdx.x >> 3);
        if (x < cend) {
          const int col = x * 8 + (threadIdx.x & 7);
          const uint32_t li = (uint32_t)((x * 8) / mbsz + ((j - 1) / mbsz) * wib);
          const uint32_t ri = (uint32_t)((x * 8) / mbsz + (j / mbsz) * wib);
          int qp;
          const int st = edge_strength(a.table[(uint16_t)li], a.table[(uint16_t)ri], qp);
          if (st) dfilter(img + (size_t)j * width + col, width, qp, st, luma);
        }
        __syncthreads();
      }
      // vertical edges V(x, j), x in [max(c,1), cend): row filters
      {
        const int x = c + (threadIdx.x >> 3);
        if (x >= 1 && x < cend) {
          const int row = j + (threadIdx.x & 7);
          const uint32_t li = (uint32_t)((x * 8 - 1) / mbsz + (j / mbsz) * wib);
          const uint32_t ri = (uint32_t)((x * 8) / mbsz + (j / mbsz) * wib);
          int qp;
          const int st = edge_strength(a.table[(uint16_t)li], a.table[(uint16_t)ri], qp);
          if (st) dfilter(img + (size_t)row * width + x * 8, 1, qp, st, luma);
        }
      }
      publish(&prog[band], cend);
    }
  }
}

hipError_t launch_deblock(const FrameArgs& a, int workgroups, hipStream_t s) {
  int g = workgroups > 0 ? workgroups : (a.ha / 8);
  if (g > a.ha / 8) g = a.ha / 8;
  hipLaunchKernelGGL(k_deblock, dim3(g, 3), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// KAT: transform/quantize/reconstruct chain on independent macroblocks.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_kat_transform(const int16_t* src, const int16_t* pred,
                                                       int16_t* coef, int16_t* recon,
                                                       const uint8_t* qtype, int32_t* qvar) {
  __shared__ int16_t s_src[kMBElems], s_pred[kMBElems], res[kMBElems], tmp[kMBElems],
      cf[kMBElems], qc[kMBElems], rec[kMBElems];
  __shared__ int32_t red[12];
  const int m = blockIdx.x;
  for (int e = threadIdx.x; e < kMBElems; e += 256) {
    s_src[e] = src[m * kMBElems + e];
    s_pred[e] = pred[m * kMBElems + e];
  }
  __syncthreads();
  int32_t v2;
  uint32_t q = code_mb(s_src, s_pred, qtype[2 * m], qtype[2 * m + 1], res, tmp, cf, qc, rec, red,
                       &v2);
  for (int e = threadIdx.x; e < kMBElems; e += 256) {
    coef[m * kMBElems + e] = qc[e];
    recon[m * kMBElems + e] = rec[e];
  }
  if (threadIdx.x == 0) {
    qvar[2 * m] = (int32_t)q;
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
