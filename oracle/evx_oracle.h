/*
 * oracle/evx_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the hinike/cairo (EVX-1) encoder, used as the
 * parity checker for the MI355X implementation in cairo_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline -- never as the product
 * path.  The product (libcairo_amd.so) neither links nor loads it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference checkout, /root/reference in the build container).
 *
 * Pinning: the reference cannot be built in this image without a stand-in for
 * an Apple/Windows SDK header (base.h:42-65 #errors on Linux), so the
 * restatement is pinned against the reference outputs recorded in
 * SURVEY.md §8(c) (stream sizes, per-frame bit counts and FNV-1a-64 stream
 * hashes of six CIF configurations) -- see tests/golden/ and DESIGN.md.
 */
#ifndef EVX_ORACLE_H
#define EVX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_encoder orc_encoder;

/* Encoder lifecycle (evx1.cpp:8-63, evx1enc.cpp:13-64). ring = ring size R
 * (EVX_REFERENCE_FRAME_COUNT, config.h:39), runtime here. */
orc_encoder *orc_create(int ring);
void orc_destroy(orc_encoder *enc);
void orc_clear(orc_encoder *enc);
void orc_insert_intra(orc_encoder *enc);
void orc_set_quality(orc_encoder *enc, int quality);

/* evx1_encoder_impl::encode (evx1enc.cpp:92-156).  Appends the frame to
 * out (LSB-first bit order) starting at bit *bit_pos, advancing it.
 * Returns 0 (EVX_SUCCESS) or an evx_status code. */
int orc_encode(orc_encoder *enc, const uint8_t *rgb, int width, int height,
               uint8_t *out, uint32_t out_capacity_bytes, uint32_t *bit_pos);

/* Introspection for parity tests.  which: 0 = input_cache, 1 = output_cache,
 * 2 + k = ring slot k.  plane: 0 Y, 1 U, 2 V.  Pitch = plane width. */
const int16_t *orc_plane(const orc_encoder *enc, int which, int plane);
/* Pre-deblock reconstruction of the last encoded frame (snapshot). */
const int16_t *orc_predeblock_plane(const orc_encoder *enc, int plane);
const uint8_t *orc_block_table(const orc_encoder *enc); /* 16 B per MB */
/* Inter search records of the last frame: [(offset-1) * mbs + mb] x 16 B
 * block desc, and the returned SAD per record. */
const uint8_t *orc_inter_descs(const orc_encoder *enc);
const int32_t *orc_inter_sads(const orc_encoder *enc);
int orc_dims(const orc_encoder *enc, int *wa, int *ha, int *ring, int *index);
uint32_t orc_frame_index(const orc_encoder *enc);

/* Stand-alone kernels for known-answer tests (no encoder state). */
void orc_convert_rgb(const uint8_t *rgb, int w, int h, int16_t *y, int16_t *u,
                     int16_t *v, int wa, int ha);
void orc_transform_8x8(const int16_t *src, int sp, int16_t *dst, int dp);
void orc_sub_transform_8x8(const int16_t *src, int sp, const int16_t *sub,
                           int bp, int16_t *dst, int dp);
void orc_inverse_transform_8x8(const int16_t *src, int sp, int16_t *dst, int dp);
void orc_inverse_transform_add_8x8(const int16_t *src, int sp, const int16_t *add,
                                   int ap, int16_t *dst, int dp);
int32_t orc_variance2(const int16_t *luma16x16, int stride);
uint8_t orc_vaq(uint8_t quality, const int16_t *luma16x16, int stride);
/* type = block type, blocks = 6 contiguous 8x8 (Y0 Y1 Y2 Y3 U V order of the
 * 16x16 macroblock quadrants: TL TR BL BR). */
void orc_quantize_mb(uint8_t qp, int type, const int16_t *src16, const int16_t *su,
                     const int16_t *sv, int16_t *dst16, int16_t *du, int16_t *dv);
void orc_dequantize_mb(uint8_t qp, int type, const int16_t *src16, const int16_t *su,
                       const int16_t *sv, int16_t *dst16, int16_t *du, int16_t *dv);
/* Deblock a full plane set in place (deblock.cpp:201-284). */
void orc_deblock(const uint8_t *block_table, int16_t *y, int16_t *u, int16_t *v,
                 int wa, int ha);

/* band4 synthetic content, RGB888 tightly packed. */
void orc_make_frame(uint8_t *rgb, int w, int h, uint32_t t, uint32_t seed);
/* Work counters since the last reset (process-wide): calls of the SAD, MAD,
 * zero-SAD and lerp macroblock helpers (256, 384, 256 and 384 pixel
 * operations each), for the algorithmic op count of SURVEY.md §8(d). */
void orc_op_counts(uint64_t out[4], int reset);
/* FNV-1a-64 over bytes, continuing from h. */
uint64_t orc_fnv1a64(uint64_t h, const uint8_t *data, uint64_t n);
/* the arithmetic coder alone over a raw LSB-first feed (one slice + flush) */
uint32_t orc_abac_feed(const uint32_t *words, uint64_t nbits, uint8_t *out, uint32_t cap_bits, int *err);

#ifdef __cplusplus
}
#endif
#endif
