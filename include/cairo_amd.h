/*
 * include/cairo_amd.h -- C ABI of libcairo_amd.so, the MI355X-native EVX-1
 * encode path.  Plain pointers and sizes only.
 *
 * Two layers:
 *
 *  1. The encode-path backend ("cairo_ctx_*").  It replaces the hot stages
 *     inside engine_encode_frame (reference encode.cpp:205-232): convert_image
 *     (convert.cpp:95-160), encode_slice (encode.cpp:165-203, with
 *     motion.cpp / transform.cpp / quantize.cpp / decode.cpp:15-144) and
 *     deblock_image_filter (deblock.cpp:277-284, fused into the row kernel).  Its outputs are exactly what
 *     the host entropy stage serialize_slice (serialize.cpp:319-340) consumes:
 *     the block table (evx_block_desc[], common.h:78-95, 16 B each) and the
 *     persistent quantized-coefficient planes (output_cache, common.h:108).
 *
 *  2. C wrappers of the drop-in C++ API (include/evx1.h), for FFI callers
 *     (ctypes): evx_encoder_* mirror evx1_encoder (reference evx1.h:66-94) and
 *     create_encoder / destroy_encoder (evx1.cpp:8-63); cairo_serialize_slice
 *     exposes the host entropy stage on its own.
 *
 * Status codes are evx_status values (reference base.h:150-172); a HIP
 * failure or a timed-out in-kernel wait maps to EVX_ERROR_HARDWAREFAIL (5).
 */
#ifndef CAIRO_AMD_H
#define CAIRO_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CAIRO_API __attribute__((visibility("default")))

/* Version of this C ABI.  It is bumped whenever an exported entry point
 * changes its signature or meaning; a caller built against one header checks
 * cairo_api_version() == CAIRO_AMD_API_VERSION at start-up.
 *   1  round 3: cairo_task_queues(hmb, frames, pool, ...)
 *   2  round 4: cairo_task_queues gains n_helpers and n_rows,
 *      cairo_group_check_queues gains hw_queues
 *   3  round 5: cairo_ctx_read_inter refuses stale (untagged) records */
#define CAIRO_AMD_API_VERSION 3
CAIRO_API int cairo_api_version(void);

typedef struct cairo_ctx cairo_ctx;

/* Outputs a context hands to the host entropy stage (cairo_ctx_set_outputs). */
#define CAIRO_OUT_COEF 1 /* the output_cache planes (default)                   */
#define CAIRO_OUT_FEED 2 /* the GPU entropy precode: the exact feed bits the    */
                         /* reference's coder consumes    */
#define CAIRO_FEED_NONE 0
#define CAIRO_FEED_VALID 1
#define CAIRO_FEED_OVERFLOW 2 /* a coefficient section exceeds the reference's   */
                              /* 32 Mbit feed stream: code it from the planes */

/* Host-visible outputs of one frame; valid until cairo_ctx_release(ticket). */
typedef struct cairo_frame_result {
  const uint8_t *block_table; /* wmb*hmb evx_block_desc (16 B, pack(2) layout) */
  const int16_t *coef_y;      /* output_cache Y, wa x ha, pitch wa (NULL      */
  const int16_t *coef_u;      /*   without CAIRO_OUT_COEF: cairo_ctx_fetch_coef) */
  const int16_t *coef_v;      /* output_cache V                               */
  uint32_t wa, ha, wmb, hmb;
  uint32_t index, type, quality;
  const uint32_t *feed;       /* CAIRO_OUT_FEED: feed bits, LSB-first words   */
  uint64_t feed_bits;
  int32_t feed_status;        /* CAIRO_FEED_*                                 */
} cairo_frame_result;

/* Context = one encoder's device state: R ring slots, input and output_cache
 * planes, block table, inter-search records, staging.  width/height are the
 * nominal frame size (aligned up to 16 internally, evx1enc.cpp:79-80); ring is
 * R = EVX_REFERENCE_FRAME_COUNT (1..4); device is the HIP ordinal. */
CAIRO_API int cairo_ctx_create(uint32_t width, uint32_t height, uint32_t ring, int device,
                               cairo_ctx **out);
/* The same with an explicit number of staging slots (frames in flight,
 * 2..256; cairo_ctx_create uses 96: three 32-frame launches, so that the
 * host entropy of one overlaps the GPU work of the next two).  A synchronous
 * caller (one frame in flight, as evx1_encoder::encode) needs 2: about
 * 0.35 GB of HBM for a 4K R = 4 context instead of 12 GB.  Frames per launch
 * are at most stages / 2. */
CAIRO_API int cairo_ctx_create_ex(uint32_t width, uint32_t height, uint32_t ring, int device,
                                  int stages, cairo_ctx **out);
CAIRO_API int cairo_ctx_destroy(cairo_ctx *ctx);
/* Zero every plane (fresh-encoder state, common.cpp:79-150) and clear a
 * reported in-kernel timeout, so the context is usable again. */
CAIRO_API int cairo_ctx_reset(cairo_ctx *ctx);

/* Submit frame (index, type 0=intra/1=inter, quality).  rgb is RGB888 with
 * pitch 3*width, in host memory (rgb_on_device = 0) or device memory of this
 * context's GPU (1; must stay valid until the frame's wait).  Frames are
 * encoded in batches of up to cairo_ctx_set_batch frames, pipelined on the GPU
 * in one launch; a batch launches when full or when a frame of it is waited
 * on.  Returns a ticket. */
CAIRO_API int cairo_ctx_submit(cairo_ctx *ctx, const uint8_t *rgb, int rgb_on_device,
                               uint32_t index, uint32_t type, uint32_t quality, int *ticket);
/* Wait until the frame's block table and coefficients are host-visible. */
CAIRO_API int cairo_ctx_wait(cairo_ctx *ctx, int ticket, cairo_frame_result *out);
/* The decoder's hot path (decode_slice + deblock + convert_image,
 * decode.cpp:146-198): reconstruct frame `index` from its block table
 * (wmb*hmb 16-B descs) and coefficient planes (y | u | v contiguous, the
 * decoder's input_cache) into ring slot index % R, deblock it, and write it as
 * RGB888 (width*height*3, pitch 3*width) to host memory rgb.  Synchronous.
 * The descs must be valid (motion inside the frame; see decoder.cpp). */
CAIRO_API int cairo_ctx_decode_frame(cairo_ctx *ctx, const uint8_t *block_table, const int16_t *coef,
                                     uint32_t index, uint8_t *rgb);
/* Hand the ticket's staging buffers back (required before ticket+stages). */
CAIRO_API int cairo_ctx_release(cairo_ctx *ctx, int ticket);
/* Launch any pending frames and block until all GPU work is finished. */
CAIRO_API int cairo_ctx_sync(cairo_ctx *ctx);
/* Staging slots = frames that may be in flight (submitted, not released). */
CAIRO_API int cairo_ctx_stages(const cairo_ctx *ctx);
/* Frames per engine launch, 1..min(32, stages/2) (default 32 for frames of up to
 * 16000 macroblocks, 28 above). */
CAIRO_API int cairo_ctx_set_batch(cairo_ctx *ctx, int frames);
/* The default frames per launch for a frame size (no device needed; 0 for an
 * empty size). */
CAIRO_API int cairo_default_batch(uint32_t width, uint32_t height);
/* The engine's (frame, row) task order for a launch of `frames` frames of hmb
 * macroblock rows: frames * hmb words (frame << 16 | row), sorted by row +
 * slope * frame; *slope receives the slope.  A launch's workers also take the
 * previous launch's tasks, merged by the same key with that launch's frames
 * first (no device needed; for tests of the deadlock-freedom argument). */
CAIRO_API int cairo_task_order(int hmb, int frames, int32_t *out, int *slope);
/* The queues of one pool (0 row helpers, 1 row coders) of a launch of one
 * context with n_helpers + n_rows workers (kernels.h kLabels): the same tasks
 * as cairo_task_order, stably partitioned by label, label l's queue being
 * order[seg[l] .. seg[l+1]) (seg: 9 words).  *nlab receives 8 where the engine
 * bands that pool (frames of at least 100 macroblock rows, both worker counts
 * multiples of 8: one queue per XCD), else 1 (seg = {0, total, ...}) -- the
 * predicate the launch itself applies.  No device needed. */
CAIRO_API int cairo_task_queues(int hmb, int frames, int n_helpers, int n_rows, int pool, int32_t *order,
                                int32_t *seg, int *nlab);

/* Introspection (synchronous; of the last submitted frame).  which: 0 input,
 * 1 output_cache, 2+k ring slot k. */
CAIRO_API int cairo_ctx_read_planes(cairo_ctx *ctx, int which, int16_t *y, int16_t *u,
                                    int16_t *v);
/* Inter-search records of the last frame: (ring-1)*mbs descs and SADs. */
CAIRO_API int cairo_ctx_read_inter(cairo_ctx *ctx, uint8_t *descs, int32_t *sads);
CAIRO_API int cairo_ctx_read_table(cairo_ctx *ctx, uint8_t *table);
/* Debug: flags & 1 snapshots the reconstruction before the deblock of every
 * frame (cairo_ctx_read_predeblock returns the last snapshot); flags & 2
 * records per-macroblock phase timestamps of the wavefront kernel (12 x u64
 * per MB, 100 MHz clock; cairo_ctx_read_stamps). */
CAIRO_API int cairo_ctx_set_debug(cairo_ctx *ctx, int flags);
CAIRO_API int cairo_ctx_read_stamps(cairo_ctx *ctx, uint64_t *out);
/* Debug: flags & 4 keeps a live per-workgroup state trace of the engine in
 * mapped host memory; read it (n int32 words) without synchronizing.
 * flags & 8 (test hook) marks the device's sticky timeout word as if an
 * in-kernel wait had timed out: every later frame reports
 * EVX_ERROR_HARDWAREFAIL until cairo_ctx_reset. */
CAIRO_API int cairo_ctx_read_trace(cairo_ctx *ctx, int32_t *out, int n);
/* flags & 16 (test hook) makes the row helpers of MB row min(1, hmb-1) of
 * every frame launched from now on record a timeout of their first progress
 * wait through the device's own reporting path (CAIRO_WAIT_INJECTED), without
 * waiting; setting flags without 16 clears it. */

/* The in-kernel wait that timed out first, as the last frame that reported
 * EVX_ERROR_HARDWAREFAIL saw it (zeros: none since create / reset).  Up to 16
 * int32 words: kind (CAIRO_WAIT_*), the waiting frame's epoch, its stream
 * index, its MB row, the group member (0 alone), what it needed (columns, a
 * count or a tag), what it waited on (CAIRO_WAIT_RECORDS: inter group;
 * _GRANULE: macroblock index; _PREV_PROGRESS / _INJECTED: row | back << 16;
 * _ROW_ABOVE: row), and the last value it saw (low, high word). */
#define CAIRO_WAIT_RECORDS 1
#define CAIRO_WAIT_GRANULE 2
#define CAIRO_WAIT_PREV_PROGRESS 3
#define CAIRO_WAIT_ROW_ABOVE 4
#define CAIRO_WAIT_BATCH 5
#define CAIRO_WAIT_INJECTED 6
#define CAIRO_WAIT_HOST_MARK 9
CAIRO_API int cairo_ctx_timeout_info(cairo_ctx *ctx, int32_t *out, int n);
/* Debug: flags & 32 turns on the engine's time accounting, which a library
 * built with CAIRO_ACCT=1 (tools/build_variant.sh) fills: per role and phase,
 * the 10 ns ticks summed over every task since the last reset, then bytes
 * requested by the window staging and the polls (24 words, kernels.h Acct;
 * zeros from a regular build).  Synchronous; reset = 1 zeroes
 * the counters after reading them. */
CAIRO_API int cairo_ctx_read_acct(cairo_ctx *ctx, uint64_t *out, int n, int reset);
CAIRO_API int cairo_ctx_read_predeblock(cairo_ctx *ctx, int16_t *y, int16_t *u, int16_t *v);

/* Per-kernel timing (HIP events on the kernels' stream), opt-in. */
CAIRO_API int cairo_ctx_set_profiling(cairo_ctx *ctx, int enable);
/* Accumulated ms per kernel since the last call: [convert, 0 (inter search
 * runs inside the engine), engine (inter search + row coding + in-loop
 * deblock) summed over launches, engine busy time = the length of the union
 * of the launches' intervals (two launches run at once, so the sum counts
 * overlapped time twice)], and the number of frames they cover; resets the
 * accumulators.  Enabling profiling starts the common clock of the busy
 * intervals. */
CAIRO_API int cairo_ctx_take_timings(cairo_ctx *ctx, double ms[4], int *frames);
/* The engine launches' [start, end) intervals (ms on the profiling clock,
 * pairs, sorted by start) collected since the last cairo_ctx_take_timings,
 * without resetting them: the busy-time union can be recomputed from them.
 * *n receives the count; at most cap pairs are written. */
CAIRO_API int cairo_ctx_busy_intervals(cairo_ctx *ctx, double *out, int cap, int *n);
/* Row-coder workgroups of the engine per launch (0 = automatic: a quarter of
 * the device's resident engine workgroups, 192 on a full MI355X; larger
 * values are rejected, since every launch must stay co-resident with the
 * one before it). */
CAIRO_API int cairo_ctx_set_workgroups(cairo_ctx *ctx, int mb_rows);

/* ---- frame-interleaved groups (multi-GPU single stream) ----
 * N contexts (one per GPU and process, or several on one device) encode ONE
 * stream: member k encodes the frames n = k (mod N), in order, reading the
 * other members' reconstructions (references, the stale rows of frame n-R),
 * output_cache (copy macroblocks) and deblock progress in place -- over xGMI
 * when they live on other GPUs.  The hand-off is a per-row progress word; no
 * collective and no copy is on the data path.  Output is the single-context
 * stream, bit for bit.
 *
 * Protocol: create every member (same width, height, ring), call
 * cairo_ctx_peer_info on each (cross_device = 1 if any member is another
 * process or device: the shared buffers are then re-allocated fine-grained),
 * exchange the records (any transport: they are plain bytes), then
 * cairo_ctx_join_group on each with all N records in rank order, before any
 * frame.  Submit frame n to member n % N with index n; before waiting on a
 * frame, every member must have launched (cairo_ctx_flush) its frames that
 * precede it in the stream -- a member's in-kernel wait on another's
 * unlaunched frame times out after 2 s (EVX_ERROR_HARDWAREFAIL).  Members on
 * one device share its workgroup slots: give each cairo_ctx_max_workgroups /
 * (members on the device) row coders (cairo_ctx_set_workgroups).
 * cairo_ctx_reset leaves the group. */
#define CAIRO_MAX_COEF_CHUNKS 16
typedef struct cairo_peer {
  uint32_t width, height, ring;
  int32_t device, pid, stages, fine_grained;
  int32_t coef_chunks;      /* the output_cache slots live in this many allocations */
  int32_t coef_chunk_slots; /* staging slots per chunk: slot s is in chunk s / coef_chunk_slots */
  int32_t reserved;
  uint64_t ring_addr, progress_addr;             /* device addresses in the owner's process */
  uint64_t coef_addr[CAIRO_MAX_COEF_CHUNKS];
  uint8_t ipc_ring[64], ipc_progress[64];        /* hipIpcMemHandle_t of each allocation */
  uint8_t ipc_coef[CAIRO_MAX_COEF_CHUNKS][64];
} cairo_peer;
/* A member's output_cache (2 bytes x 1.5 x Wa x Ha per staging slot) is
 * allocated in chunks of at most 1 GiB, each exported with its own IPC handle:
 * an IPC import of a single fine-grained allocation of 2 GiB or more never
 * returned on the test boxes (a 4K member with 96 slots has 2.4 GB of it). */
/* sizeof(cairo_peer), for bindings that exchange the records as bytes. */
CAIRO_API int cairo_peer_size(void);
CAIRO_API int cairo_ctx_peer_info(cairo_ctx *ctx, int cross_device, cairo_peer *out);
CAIRO_API int cairo_ctx_join_group(cairo_ctx *ctx, int size, int rank, const cairo_peer *peers);
/* Whether local_members group members may share one process and device:
 * they need GPU_MAX_HW_QUEUES >= 3 * local_members + 2 (at most 32), or two
 * members' persistent launches can land in one in-order hardware queue and
 * deadlock.  hw_queues < 0: the process's GPU_MAX_HW_QUEUES as read when the
 * library was loaded (the HIP runtime reads it once, when it starts: set it
 * before the process starts; 4 when unset).  0 = fine (always for fewer than
 * 2), else EVX_ERROR_INVALID_ARGS with a message on stderr.
 * cairo_ctx_join_group applies it with hw_queues = -1; no device needed. */
CAIRO_API int cairo_group_check_queues(int local_members, int hw_queues);
/* Launch the pending (partial) batch now. */
CAIRO_API int cairo_ctx_flush(cairo_ctx *ctx);
/* Choose the outputs (CAIRO_OUT_COEF and/or CAIRO_OUT_FEED) for frames
 * submitted from now on; no frame may be in flight. */
CAIRO_API int cairo_ctx_set_outputs(cairo_ctx *ctx, int outputs);
/* The coefficient planes of a waited, unreleased frame (a D2H copy from its
 * staging slot when the context does not copy them already). */
CAIRO_API int cairo_ctx_fetch_coef(cairo_ctx *ctx, int ticket, cairo_frame_result *out);
/* Of a launch's 2 * workgroups workers, how many are row helpers (inter
 * search + deblock) rather than row coders (0: half). */
CAIRO_API int cairo_ctx_set_helpers(cairo_ctx *ctx, int helpers);
/* Upper bound of cairo_ctx_set_workgroups on this device. */
CAIRO_API int cairo_ctx_max_workgroups(const cairo_ctx *ctx);

/* Known-answer check of the device transform chain: count macroblocks of 384
 * int16 (block-major: Y TL,TR,BL,BR, U, V; 64 each).  qtype[2m] = block type,
 * qtype[2m+1] = frame quality.  Host buffers in and out. */
CAIRO_API int cairo_kat_transform(const int16_t *src, const int16_t *pred, const uint8_t *qtype,
                                  int count, int16_t *coef, int16_t *recon, int32_t *qvar,
                                  int device);

/* ---- host entropy stage (serialize_slice, serialize.cpp:319-340) ---------
 * Appends the ABAC payload of one frame to out (LSB-first bit order) at bit
 * *bit_pos, advancing it.  coef planes have pitch wa (luma) / wa/2 (chroma). */
CAIRO_API int cairo_serialize_slice(const uint8_t *block_table, uint32_t wmb, uint32_t hmb,
                                    uint32_t ring, const int16_t *coef_y, const int16_t *coef_u,
                                    const int16_t *coef_v, uint8_t *out, uint32_t out_bytes,
                                    uint32_t *bit_pos);

/* The same payload from a frame's GPU-precoded feed (cairo_frame_result.feed
 * with CAIRO_FEED_VALID): only the arithmetic coder runs. */
CAIRO_API int cairo_serialize_feed(const uint32_t *feed, uint64_t feed_bits, uint8_t *out,
                                   uint32_t out_bytes, uint32_t *bit_pos);
/* The host precode alone (serialize.cpp:10-286, stream.cpp:550-581,
 * golomb.cpp:8-91, with the 32 Mbit per-section drop rule): the feed bits the
 * arithmetic coder consumes, LSB-first in 32-bit words -- what the GPU precode
 * writes for a CAIRO_FEED_VALID frame.  *feed_bits receives the bit count;
 * EVX_ERROR_CAPACITY_LIMIT (7) if feed_words cannot hold them. */
CAIRO_API int cairo_precode_slice(const uint8_t *block_table, uint32_t wmb, uint32_t hmb, uint32_t ring,
                                  const int16_t *coef_y, const int16_t *coef_u, const int16_t *coef_v,
                                  uint32_t *feed, uint64_t feed_words, uint64_t *feed_bits);

/* ---- host entropy decode (unserialize_slice, unserialize.cpp:321-342) ----
 * Decodes the ABAC payload of one frame starting at bit *read_index of data
 * (LSB-first, up to write_index) into the block table (wmb*hmb 16-B descs) and
 * the coefficient planes, which persist across frames: fields a block does not
 * carry keep their previous values, as in the reference decoder's context.
 * Advances *read_index.  EVX_ERROR_INVALID_RESOURCE (8) on a corrupt payload. */
CAIRO_API int cairo_unserialize_slice(const uint8_t *data, uint32_t *read_index, uint32_t write_index,
                                      uint32_t wmb, uint32_t hmb, uint32_t ring, uint8_t *block_table,
                                      int16_t *coef_y, int16_t *coef_u, int16_t *coef_v);

/* ---- frame pipeline ---------------------------------
 * GPU hot path + host entropy for a stream of frames: the caller submits
 * frames, a completion thread picks up each frame's outputs, a pool of entropy
 * workers runs serialize_slice on them in parallel (frames are
 * entropy-independent: the ABAC model restarts per slice, serialize.cpp:323),
 * and collect appends a frame's payload bits.  Appending the frame descriptors
 * and payloads in ticket order yields the reference stream (evx1enc.cpp:119-168).
 * The stream drives ctx exclusively while it exists (no direct cairo_ctx_submit
 * / wait / release); destroy it before the context.  A host RGB source must
 * stay valid until its frame is collected. */
typedef struct cairo_stream cairo_stream;
/* threads: entropy workers (0 = hardware threads - 1, at most 15). */
CAIRO_API int cairo_stream_create(cairo_ctx *ctx, int threads, cairo_stream **out);
/* Blocks while the frame's staging slot (ticket - stages) is still being
 * entropy-coded; EVX_ERROR_INVALID_RESOURCE (8) if ticket - 2*stages has not
 * been collected. */
CAIRO_API int cairo_stream_submit(cairo_stream *s, const uint8_t *rgb, int rgb_on_device,
                                  uint32_t index, uint32_t type, uint32_t quality, int *ticket);
/* Wait for the frame's payload and append it at bit *bit_pos of out
 * (out_bytes capacity, LSB-first; out == NULL only advances *bit_pos).  If it
 * does not fit, returns EVX_ERROR_CAPACITY_LIMIT (7) and keeps the payload:
 * collect again with a larger buffer. */
CAIRO_API int cairo_stream_collect(cairo_stream *s, int ticket, uint8_t *out, uint64_t out_bytes,
                                   uint64_t *bit_pos);
/* Wait for the frame's payload and return its size in bits (not collected). */
CAIRO_API int cairo_stream_payload_bits(cairo_stream *s, int ticket, uint64_t *nbits);
/* Diagnostic timeline of a collected frame (valid until ticket + 2*stages is
 * submitted): t[5] = submitted, outputs on the host, entropy start, entropy
 * end, collected; microseconds of a monotonic clock. */
CAIRO_API int cairo_stream_timeline(cairo_stream *s, int ticket, double *t);
/* Finish all submitted frames and stop the threads. */
CAIRO_API int cairo_stream_destroy(cairo_stream *s);
/* Append n bits of src at bit *pos of dst (cap_bits), bit_stream semantics. */
CAIRO_API int cairo_bits_append(uint8_t *dst, uint64_t cap_bits, uint64_t *pos, const uint8_t *src,
                                uint64_t n);

/* ---- drop-in encoder, C view of evx1_encoder (evx1.h:66-94) ------------- */
CAIRO_API int evx_encoder_create(void **enc);
CAIRO_API int evx_encoder_destroy(void *enc);
CAIRO_API int evx_encoder_clear(void *enc);
CAIRO_API int evx_encoder_insert_intra(void *enc);
CAIRO_API int evx_encoder_set_quality(void *enc, uint8_t quality);
/* Encode one RGB888 frame, appending to the bit stream bs (evx_bitstream_*). */
CAIRO_API int evx_encoder_encode(void *enc, const void *rgb, uint32_t width, uint32_t height,
                                 void *bs);
/* Debug view of the last encoded frame (EVX_PEEK_STATE, evx1.h): RGB888 of
 * the nominal frame size into rgb (evx1enc.cpp:170-305). */
CAIRO_API int evx_encoder_peek(void *enc, int state, void *rgb);
CAIRO_API int evx_encoder_set_ring(void *enc, uint32_t ring); /* before first encode */
CAIRO_API int evx_encoder_set_device(void *enc, int device);  /* before first encode */

/* ---- drop-in decoder, C view of evx1_decoder (evx1.h:97-112) ------------
 * decode() reads [header +] one frame record from bs (its read index onward),
 * writes the frame as RGB888 (width*height*3 from the stream header) to rgb,
 * and empties bs, as the reference does (evx1dec.cpp:90-124). */
CAIRO_API int evx_decoder_create(void **dec);
CAIRO_API int evx_decoder_destroy(void *dec);
CAIRO_API int evx_decoder_clear(void *dec);
CAIRO_API int evx_decoder_decode(void *dec, void *bs, void *rgb);
CAIRO_API int evx_decoder_set_device(void *dec, int device); /* before first decode */

/* bit_stream (reference bitstream.h:43-92) */
CAIRO_API void *evx_bitstream_create(uint32_t size_in_bits);
CAIRO_API void evx_bitstream_destroy(void *bs);
CAIRO_API const uint8_t *evx_bitstream_data(void *bs);
CAIRO_API uint32_t evx_bitstream_occupancy(void *bs); /* bits */
CAIRO_API void evx_bitstream_empty(void *bs);
/* Append count bits of data (LSB-first) -- bit_stream::write_bits. */
CAIRO_API int evx_bitstream_write_bits(void *bs, const void *data, uint32_t count);

/* band4 synthetic content generator; RGB888, pitch 3*w. */
CAIRO_API void cairo_make_band4(uint8_t *rgb, uint32_t w, uint32_t h, uint32_t t, uint32_t seed);

/* Library/device information. */
CAIRO_API const char *cairo_version(void);
CAIRO_API int cairo_device_count(void);

#ifdef __cplusplus
}
#endif
#endif
