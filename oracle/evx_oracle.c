/*
 * oracle/evx_oracle.c -- TEST INFRASTRUCTURE ONLY (see evx_oracle.h).
 *
 * A deliberately plain, slow, bit-serial restatement of the EVX-1 encoder of
 * hinike/cairo.  Structure follows the reference call tree so every step can
 * be audited against it; citations are file:line in the reference checkout.
 * Integer semantics are restated exactly: int16 narrowing on stores, C
 * truncating division, evx_round_out, rounded_div with its sign-bit test,
 * wrapping int32 where the reference can overflow (variance2).
 */
#include "evx_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define MBS 16                       /* EVX_MACROBLOCK_SIZE, macroblock.h:56 */
#define SAD_GATE 8192                /* EVX_MOTION_SAD_THRESHOLD, motion.cpp:19 */
#define SEARCH_RADIUS 16             /* EVX_MOTION_SEARCH_RADIUS, motion.cpp:24 */
#define QSCALE 16                    /* EVX_QUANTIZER_SCALE_FACTOR, quantize.cpp:9 */
#define FEED_CAPACITY_BITS (32u * 1024u * 1024u) /* common.cpp:147 */
#define PERIODIC_INTRA 3600          /* config.h:41 */
#define DEFAULT_QUALITY 8            /* config.h:40 */

enum { T_INTRA = 1, T_MOTION = 2, T_COPY = 4 };          /* types.h:68-87 */

/* ------------------------------------------------------------------ */
/* integer helpers (math.h)                                            */
/* ------------------------------------------------------------------ */

/* math.h:69-113: LUT log2 over bytes, composed for u16 / u32. */
static uint8_t lut_log2_u8(uint8_t v) {
    uint8_t r = 0;
    while (v >>= 1) r++;
    return r;
}
static uint8_t lut_log2_u16(uint16_t v) {
    return v <= 0xFF ? lut_log2_u8((uint8_t)v) : (uint8_t)(8 + lut_log2_u8((uint8_t)(v >> 8)));
}
static uint8_t lut_log2_u32(uint32_t v) {
    return v <= 0xFFFF ? lut_log2_u16((uint16_t)v)
                       : (uint8_t)(16 + lut_log2_u16((uint16_t)(v >> 16)));
}

/* math.h:149-161 abs: MIN maps to MAX. */
static int32_t iabs32(int32_t v) {
    if (v == INT32_MIN) return INT32_MAX;
    return v < 0 ? -v : v;
}
/* math.h:128-133 sign(int16). */
static int16_t sign16(int16_t v) { return (int16_t)((v > 0) - (v < 0)); }
/* math.h:209-212 clip_range(int16). */
static int16_t clip16(int16_t v, int16_t lo, int16_t hi) { return v < lo ? lo : (v > hi ? hi : v); }
/* math.h:60 evx_round_out. */
static int32_t round_out(int32_t n, int32_t a) { return n < 0 ? n - a : n + a; }
/* math.h:224-232 rounded_div: half away from zero, sign test on bit 31,
 * restated with wrapping add/sub. */
static int32_t rdiv(int32_t n, int32_t d) {
    if (((uint32_t)n ^ (uint32_t)d) & 0x80000000u)
        return (int32_t)((uint32_t)n - (uint32_t)(d / 2)) / d;
    return (int32_t)((uint32_t)n + (uint32_t)(d / 2)) / d;
}

/* ------------------------------------------------------------------ */
/* planes and macroblock views (image.cpp, imageset.cpp, macroblock.h) */
/* ------------------------------------------------------------------ */

typedef struct {
    int16_t *y, *u, *v;
    int w, h; /* luma dims; chroma w/2 x h/2; pitch == width (image.cpp:55-68) */
} planes;

static int planes_alloc(planes *p, int w, int h) {
    p->w = w;
    p->h = h;
    p->y = (int16_t *)calloc((size_t)w * h, 2);
    p->u = (int16_t *)calloc((size_t)(w / 2) * (h / 2), 2);
    p->v = (int16_t *)calloc((size_t)(w / 2) * (h / 2), 2);
    return p->y && p->u && p->v;
}
static void planes_free(planes *p) {
    free(p->y);
    free(p->u);
    free(p->v);
    memset(p, 0, sizeof(*p));
}

typedef struct {
    int16_t *y, *u, *v;
    int stride; /* luma stride in elements; chroma uses stride >> 1 */
} mbv;

/* create_macroblock, macroblock.h:82-88 (chroma at (x>>1, y>>1)). */
static mbv mb_at(const planes *p, int x, int y) {
    mbv m;
    m.y = p->y + (size_t)y * p->w + x;
    m.u = p->u + (size_t)(y >> 1) * (p->w >> 1) + (x >> 1);
    m.v = p->v + (size_t)(y >> 1) * (p->w >> 1) + (x >> 1);
    m.stride = p->w;
    return m;
}

typedef struct {
    int16_t y[256], u[64], v[64];
} scratch_mb;

static mbv mb_scratch(scratch_mb *s) {
    mbv m;
    m.y = s->y;
    m.u = s->u;
    m.v = s->v;
    m.stride = 16;
    return m;
}

#define CS(m) ((m).stride >> 1)

/* copy_macroblock, macroblock.h:157-169 */
static void mb_copy(mbv s, mbv d) {
    for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) d.y[j * d.stride + i] = s.y[j * s.stride + i];
    for (int j = 0; j < 8; j++)
        for (int i = 0; i < 8; i++) {
            d.u[j * CS(d) + i] = s.u[j * CS(s) + i];
            d.v[j * CS(d) + i] = s.v[j * CS(s) + i];
        }
}

/* Work counters (test infrastructure): macroblock-sized metric and lerp
 * evaluations, for the algorithmic pixel-op count of SURVEY.md §8(d). */
static uint64_t g_ops[4]; /* blk_sad, blk_mad, blk_sad0, mb_lerp calls */

/* lerp_macroblock_half / _quarter, macroblock.h:203-241 */
static void mb_lerp(mbv a, mbv b, mbv d, int quarter) {
    g_ops[3]++;
    for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) {
            int32_t t;
            if (quarter) {
                t = 3 * a.y[j * a.stride + i] + b.y[j * b.stride + i];
                d.y[j * d.stride + i] = (int16_t)(round_out(t, 2) / 4);
            } else {
                t = a.y[j * a.stride + i] + b.y[j * b.stride + i];
                d.y[j * d.stride + i] = (int16_t)(round_out(t, 1) / 2);
            }
        }
    for (int j = 0; j < 8; j++)
        for (int i = 0; i < 8; i++) {
            int32_t tu, tv;
            if (quarter) {
                tu = 3 * a.u[j * CS(a) + i] + b.u[j * CS(b) + i];
                tv = 3 * a.v[j * CS(a) + i] + b.v[j * CS(b) + i];
                d.u[j * CS(d) + i] = (int16_t)(round_out(tu, 2) / 4);
                d.v[j * CS(d) + i] = (int16_t)(round_out(tv, 2) / 4);
            } else {
                tu = a.u[j * CS(a) + i] + b.u[j * CS(b) + i];
                tv = a.v[j * CS(a) + i] + b.v[j * CS(b) + i];
                d.u[j * CS(d) + i] = (int16_t)(round_out(tu, 1) / 2);
                d.v[j * CS(d) + i] = (int16_t)(round_out(tv, 1) / 2);
            }
        }
}

/* ------------------------------------------------------------------ */
/* block metrics (analysis.h)                                          */
/* ------------------------------------------------------------------ */

/* compute_block_sad(left, right), analysis.h:42-55 */
static int32_t blk_sad(mbv a, mbv b) {
    int32_t s = 0;
    g_ops[0]++;
    for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) s += iabs32(a.y[j * a.stride + i] - b.y[j * b.stride + i]);
    return s;
}
/* compute_block_sad(delta), analysis.h:57-68 */
static int32_t blk_sad0(mbv a) {
    int32_t s = 0;
    g_ops[2]++;
    for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) s += iabs32(a.y[j * a.stride + i]);
    return s;
}
/* compute_block_mad, analysis.h:103-125 (luma then chroma) */
static int32_t blk_mad(mbv a, mbv b) {
    int32_t m = 0;
    g_ops[1]++;
    for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) {
            int32_t t = iabs32(a.y[j * a.stride + i] - b.y[j * b.stride + i]);
            if (t > m) m = t;
        }
    for (int j = 0; j < 8; j++)
        for (int i = 0; i < 8; i++) {
            int32_t tu = iabs32(a.u[j * CS(a) + i] - b.u[j * CS(b) + i]);
            int32_t tv = iabs32(a.v[j * CS(a) + i] - b.v[j * CS(b) + i]);
            if (tu > m) m = tu;
            if (tv > m) m = tv;
        }
    return m;
}
/* compute_block_variance2, analysis.h:176-198.  int32 arithmetic of the
 * reference restated with explicit wrap-around. */
static int32_t variance2(const int16_t *y, int stride) {
    uint32_t sum = 0, sumsq = 0;
    int32_t count = 0;
    for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) {
            if (i == 0 && j == 0) continue;
            int32_t t = y[j * stride + i];
            if (t) {
                sum += (uint32_t)t;
                sumsq += (uint32_t)(t * t);
                count++;
            }
        }
    if (count <= 0) return 0;
    int32_t s = (int32_t)sum;
    int32_t sq = (int32_t)((uint32_t)s * (uint32_t)s);
    return (int32_t)(sumsq - (uint32_t)rdiv(sq, count));
}
int32_t orc_variance2(const int16_t *y, int stride) { return variance2(y, stride); }

/* ------------------------------------------------------------------ */
/* transform (transform.cpp, xftables.h)                               */
/* ------------------------------------------------------------------ */

/* EVX_TRANSFORM_8x8_TRIG_128_LUT (xftables.h:57-67): round(128 cos((2i+1)j pi/16)),
 * row j = frequency, column i = sample. Generated, not copied. */
static int16_t LUT8[64];
static int lut_ready = 0;
static void init_tables(void) {
    if (lut_ready) return;
    for (int j = 0; j < 8; j++)
        for (int i = 0; i < 8; i++)
            LUT8[j * 8 + i] = (int16_t)lround(128.0 * cos(((2 * i + 1) * j * 3.14159265358979323846) / 16.0));
    lut_ready = 1;
}

/* transform_8x8_line_fast, transform.cpp:264-284 */
static void fline(const int16_t *src, int sp, int16_t *dst, int dp) {
    for (int i = 0; i < 8; i++) {
        int32_t t = 0;
        for (int k = 0; k < 8; k++) t += src[k * sp] * LUT8[i * 8 + k];
        t = i == 0 ? (t * 45) / 128 : t / 2;
        dst[i * dp] = (int16_t)rdiv(t, 128);
    }
}
/* inverse_transform_8x8_line_fast, transform.cpp:330-349 (per-term truncation) */
static void iline(const int16_t *src, int sp, int16_t *dst, int dp) {
    for (int i = 0; i < 8; i++) {
        int32_t t = ((src[0] * LUT8[i]) * 45) / 128;
        for (int k = 1; k < 8; k++) t += (src[k * sp] * LUT8[k * 8 + i]) / 2;
        dst[i * dp] = (int16_t)rdiv(t, 128);
    }
}
/* transform_8x8, transform.cpp:286-301: rows then columns, int16 scratch */
void orc_transform_8x8(const int16_t *src, int sp, int16_t *dst, int dp) {
    int16_t s[64];
    init_tables();
    for (int j = 0; j < 8; j++) fline(src + j * sp, 1, s + j * 8, 1);
    for (int j = 0; j < 8; j++) fline(s + j, 8, dst + j, dp);
}
/* sub_transform_8x8, transform.cpp:435-452 (difference narrowed to int16) */
void orc_sub_transform_8x8(const int16_t *src, int sp, const int16_t *sub, int bp, int16_t *dst,
                           int dp) {
    int16_t d[64], s[64];
    init_tables();
    for (int j = 0; j < 8; j++) {
        for (int i = 0; i < 8; i++) d[j * 8 + i] = (int16_t)(src[j * sp + i] - sub[j * bp + i]);
        fline(d + j * 8, 1, s + j * 8, 1);
    }
    for (int j = 0; j < 8; j++) fline(s + j, 8, dst + j, dp);
}
/* inverse_transform_8x8, transform.cpp:351-366: columns then rows */
void orc_inverse_transform_8x8(const int16_t *src, int sp, int16_t *dst, int dp) {
    int16_t s[64];
    init_tables();
    for (int j = 0; j < 8; j++) iline(src + j, sp, s + j, 8);
    for (int j = 0; j < 8; j++) iline(s + j * 8, 1, dst + j * dp, 1);
}
/* inverse_transform_add_8x8, transform.cpp:396-433 (unclamped int16 result) */
void orc_inverse_transform_add_8x8(const int16_t *src, int sp, const int16_t *add, int ap,
                                   int16_t *dst, int dp) {
    int16_t s[64], r[8];
    init_tables();
    for (int j = 0; j < 8; j++) iline(src + j, sp, s + j, 8);
    for (int j = 0; j < 8; j++) {
        iline(s + j * 8, 1, r, 1);
        for (int i = 0; i < 8; i++) dst[j * dp + i] = (int16_t)(r[i] + add[j * ap + i]);
    }
}

/* 16x16 = four independent 8x8 quadrants (transform.cpp:485-594) and the
 * macroblock wrappers (macroblock.h:265-295). */
static void mb_transform(mbv s, mbv d) {
    for (int q = 0; q < 4; q++) {
        int o = (q >> 1) * 8 * 16 + (q & 1) * 8;
        int os = (q >> 1) * 8 * s.stride + (q & 1) * 8;
        int od = (q >> 1) * 8 * d.stride + (q & 1) * 8;
        (void)o;
        orc_transform_8x8(s.y + os, s.stride, d.y + od, d.stride);
    }
    orc_transform_8x8(s.u, CS(s), d.u, CS(d));
    orc_transform_8x8(s.v, CS(s), d.v, CS(d));
}
static void mb_sub_transform(mbv s, mbv b, mbv d) {
    for (int q = 0; q < 4; q++) {
        int os = (q >> 1) * 8 * s.stride + (q & 1) * 8;
        int ob = (q >> 1) * 8 * b.stride + (q & 1) * 8;
        int od = (q >> 1) * 8 * d.stride + (q & 1) * 8;
        orc_sub_transform_8x8(s.y + os, s.stride, b.y + ob, b.stride, d.y + od, d.stride);
    }
    orc_sub_transform_8x8(s.u, CS(s), b.u, CS(b), d.u, CS(d));
    orc_sub_transform_8x8(s.v, CS(s), b.v, CS(b), d.v, CS(d));
}
static void mb_inverse_transform(mbv s, mbv d) {
    for (int q = 0; q < 4; q++) {
        int os = (q >> 1) * 8 * s.stride + (q & 1) * 8;
        int od = (q >> 1) * 8 * d.stride + (q & 1) * 8;
        orc_inverse_transform_8x8(s.y + os, s.stride, d.y + od, d.stride);
    }
    orc_inverse_transform_8x8(s.u, CS(s), d.u, CS(d));
    orc_inverse_transform_8x8(s.v, CS(s), d.v, CS(d));
}
static void mb_inverse_transform_add(mbv s, mbv a, mbv d) {
    for (int q = 0; q < 4; q++) {
        int os = (q >> 1) * 8 * s.stride + (q & 1) * 8;
        int oa = (q >> 1) * 8 * a.stride + (q & 1) * 8;
        int od = (q >> 1) * 8 * d.stride + (q & 1) * 8;
        orc_inverse_transform_add_8x8(s.y + os, s.stride, a.y + oa, a.stride, d.y + od, d.stride);
    }
    orc_inverse_transform_add_8x8(s.u, CS(s), a.u, CS(a), d.u, CS(d));
    orc_inverse_transform_add_8x8(s.v, CS(s), a.v, CS(a), d.v, CS(d));
}

/* ------------------------------------------------------------------ */
/* quantization (quantize.cpp)                                         */
/* ------------------------------------------------------------------ */

/* default_intra_8x8_qm / default_inter_8x8_qm, quantize.cpp:13-35 */
static const int16_t QM_INTRA[64] = {
    8,  17, 18, 19, 21, 23, 25, 27, 17, 18, 19, 21, 23, 25, 27, 28, 20, 21, 22, 23, 24, 26,
    28, 30, 21, 22, 23, 24, 26, 28, 30, 32, 22, 23, 24, 26, 28, 30, 32, 35, 23, 24, 26, 28,
    30, 32, 35, 38, 25, 26, 28, 30, 32, 35, 38, 41, 27, 28, 30, 32, 35, 38, 41, 45};
static const int16_t QM_INTER[64] = {
    16, 17, 18, 19, 20, 21, 22, 23, 17, 18, 19, 20, 21, 22, 23, 24, 18, 19, 20, 21, 22, 23,
    24, 25, 19, 20, 21, 22, 23, 24, 26, 27, 20, 21, 22, 23, 25, 26, 27, 28, 21, 22, 23, 24,
    26, 27, 28, 30, 22, 23, 24, 26, 27, 28, 30, 31, 23, 24, 25, 27, 28, 30, 31, 33};

/* compute_luma_dc_scale / compute_chroma_dc_scale, quantize.cpp:37-55 */
static int16_t luma_dc_scale(int16_t qp) {
    if (qp < 5) return 8;
    if (qp < 9) return (int16_t)(qp << 1);
    if (qp < 25) return (int16_t)(qp + 8);
    return (int16_t)((qp << 1) - 16);
}
static int16_t chroma_dc_scale(int16_t qp) {
    if (qp < 5) return 8;
    if (qp < 25) return (int16_t)((qp + 13) >> 1);
    return (int16_t)(qp - 6);
}

/* query_block_quantization_parameter, quantize.cpp:60-77 */
static uint8_t vaq(uint8_t quality, const int16_t *y, int stride) {
    uint32_t var = (uint32_t)variance2(y, stride);
    uint8_t idx = (uint8_t)clip16((int16_t)(lut_log2_u32(var) >> 1), 1, 31);
    if (idx > quality) return (uint8_t)clip16((int16_t)(quality + ((idx - quality) >> 1)), 1, 31);
    if (idx < quality) return (uint8_t)clip16((int16_t)(quality - ((quality - idx) >> 1)), 1, 31);
    return quality;
}
uint8_t orc_vaq(uint8_t quality, const int16_t *y, int stride) { return vaq(quality, y, stride); }

/* quantize_{luma,chroma}_intra_block_8x8, quantize.cpp:79-129 */
static void q_intra8(uint8_t qp, const int16_t *s, int sp, int16_t *d, int dp, int chroma) {
    for (int j = 0; j < 8; j++)
        for (int k = 0; k < 8; k++) {
            int16_t v = s[k + j * sp];
            d[k + j * dp] = (int16_t)rdiv(rdiv(v * QSCALE, QM_INTRA[k + j * 8]), qp << 1);
        }
    int16_t dcs = chroma ? chroma_dc_scale(qp) : luma_dc_scale(qp);
    d[0] = (int16_t)rdiv(s[0], dcs);
}
/* quantize_inter_block_8x8, quantize.cpp:146-163 */
static void q_inter8(uint8_t qp, const int16_t *s, int sp, int16_t *d, int dp) {
    for (int j = 0; j < 8; j++)
        for (int k = 0; k < 8; k++) {
            int16_t v = s[k + j * sp];
            int16_t qf = (int16_t)rdiv(v * QSCALE, QM_INTER[k + j * 8]);
            d[k + j * dp] = (int16_t)rdiv(qf - sign16(qf) * qp, qp << 1);
        }
}
/* inverse_quantize_{luma,chroma}_intra_block_8x8, quantize.cpp:182-212 */
static void dq_intra8(uint8_t qp, const int16_t *s, int sp, int16_t *d, int dp, int chroma) {
    for (int j = 0; j < 8; j++)
        for (int k = 0; k < 8; k++) {
            int16_t v = s[k + j * sp];
            d[k + j * dp] = (int16_t)((2 * v * QM_INTRA[k + j * 8] * qp) / QSCALE);
        }
    int16_t dcs = chroma ? chroma_dc_scale(qp) : luma_dc_scale(qp);
    d[0] = (int16_t)(s[0] * dcs);
}
/* inverse_quantize_inter_block_8x8, quantize.cpp:232-243 */
static void dq_inter8(uint8_t qp, const int16_t *s, int sp, int16_t *d, int dp) {
    for (int j = 0; j < 8; j++)
        for (int k = 0; k < 8; k++) {
            int16_t v = s[k + j * sp];
            d[k + j * dp] = (int16_t)(((2 * v) * QM_INTER[k + j * 8] * qp) / QSCALE);
        }
}

static int intra_quant_path(int type) { return (type & T_INTRA) && !(type & T_MOTION); }

/* quantize_macroblock, quantize.cpp:357-367 (+ :256-304) */
static void mb_quantize(uint8_t qp, int type, mbv s, mbv d) {
    for (int q = 0; q < 4; q++) {
        int os = (q >> 1) * 8 * s.stride + (q & 1) * 8;
        int od = (q >> 1) * 8 * d.stride + (q & 1) * 8;
        if (intra_quant_path(type))
            q_intra8(qp, s.y + os, s.stride, d.y + od, d.stride, 0);
        else
            q_inter8(qp, s.y + os, s.stride, d.y + od, d.stride);
    }
    if (intra_quant_path(type)) {
        q_intra8(qp, s.u, CS(s), d.u, CS(d), 1);
        q_intra8(qp, s.v, CS(s), d.v, CS(d), 1);
    } else {
        q_inter8(qp, s.u, CS(s), d.u, CS(d));
        q_inter8(qp, s.v, CS(s), d.v, CS(d));
    }
}
/* inverse_quantize_macroblock, quantize.cpp:369-379 (+ :306-354) */
static void mb_dequantize(uint8_t qp, int type, mbv s, mbv d) {
    for (int q = 0; q < 4; q++) {
        int os = (q >> 1) * 8 * s.stride + (q & 1) * 8;
        int od = (q >> 1) * 8 * d.stride + (q & 1) * 8;
        if (intra_quant_path(type))
            dq_intra8(qp, s.y + os, s.stride, d.y + od, d.stride, 0);
        else
            dq_inter8(qp, s.y + os, s.stride, d.y + od, d.stride);
    }
    if (intra_quant_path(type)) {
        dq_intra8(qp, s.u, CS(s), d.u, CS(d), 1);
        dq_intra8(qp, s.v, CS(s), d.v, CS(d), 1);
    } else {
        dq_inter8(qp, s.u, CS(s), d.u, CS(d));
        dq_inter8(qp, s.v, CS(s), d.v, CS(d));
    }
}

void orc_quantize_mb(uint8_t qp, int type, const int16_t *s16, const int16_t *su, const int16_t *sv,
                     int16_t *d16, int16_t *du, int16_t *dv) {
    mbv s = {(int16_t *)s16, (int16_t *)su, (int16_t *)sv, 16};
    mbv d = {d16, du, dv, 16};
    mb_quantize(qp, type, s, d);
}
void orc_dequantize_mb(uint8_t qp, int type, const int16_t *s16, const int16_t *su,
                       const int16_t *sv, int16_t *d16, int16_t *du, int16_t *dv) {
    mbv s = {(int16_t *)s16, (int16_t *)su, (int16_t *)sv, 16};
    mbv d = {d16, du, dv, 16};
    mb_dequantize(qp, type, s, d);
}

/* ------------------------------------------------------------------ */
/* block descriptor (common.h:78-95, pack(2): 16 bytes)                */
/* ------------------------------------------------------------------ */

typedef struct {
    uint32_t block_type;
    uint8_t prediction_target;
    uint8_t pad;
    int16_t motion_x, motion_y;
    uint8_t sp_pred, sp_amount, sp_index, q_index;
    int16_t variance;
} bdesc;

/* ------------------------------------------------------------------ */
/* colour conversion (convert.cpp:11-14, 30-73, 95-160)               */
/* ------------------------------------------------------------------ */

void orc_convert_rgb(const uint8_t *rgb, int w, int h, int16_t *py, int16_t *pu, int16_t *pv,
                     int wa, int ha) {
    int width = w < wa ? w : wa;
    int height = h < ha ? h : ha;
    for (int y = 0; y < height; y += 2) {
        int16_t *du = pu + (size_t)(y / 2) * (wa / 2);
        int16_t *dv = pv + (size_t)(y / 2) * (wa / 2);
        for (int x = 0; x < width; x += 2) {
            int16_t su = 0, sv = 0;
            for (int dy = 0; dy < 2; dy++)
                for (int dx = 0; dx < 2; dx++) {
                    const uint8_t *p = rgb + ((size_t)(y + dy) * w + (x + dx)) * 3;
                    int16_t r = p[0], g = p[1], b = p[2];
                    py[(size_t)(y + dy) * wa + x + dx] =
                        (int16_t)(((77 * r + 150 * g + 29 * b + 128) >> 8) + 16);
                    su = (int16_t)(su + (((-43 * r - 85 * g + 128 * b + 128) / 256) + 128));
                    sv = (int16_t)(sv + (((128 * r - 107 * g - 21 * b + 128) / 256) + 128));
                }
            du[x / 2] = (int16_t)((su + 2) >> 2);
            dv[x / 2] = (int16_t)((sv + 2) >> 2);
        }
    }
}

/* ------------------------------------------------------------------ */
/* motion search (motion.cpp)                                          */
/* ------------------------------------------------------------------ */

typedef struct {
    int32_t best_x, best_y, best_sad, best_mad, best_ssd;
    int16_t sp_index;
    int sp_amount, sp_enabled;
} msel;

typedef struct {
    const planes *pred;
    int16_t thr; /* mad_skip_threshold */
    int16_t px, py;
    int intra;
} mparams;

/* compute_motion_frac_index_from_direction, motion.cpp:61-85 */
static int16_t frac_index(int i, int j) {
    i++, j++;
    if (j == 0) return (int16_t)i;
    if (j == 1) return i == 0 ? 3 : 4;
    return (int16_t)(i + 5);
}
/* compute_motion_direction_from_frac_index, motion.cpp:87-109 */
static void frac_dir(int idx, int *dx, int *dy) {
    if (idx <= 2) { *dy = -1; *dx = idx - 1; }
    else if (idx == 3) { *dx = -1; *dy = 0; }
    else if (idx == 4) { *dx = 1; *dy = 0; }
    else { *dy = 1; *dx = idx - 6; }
}

/* evaluate_motion_candidate, motion.cpp:111-149 (note && binds tighter than ||) */
static void eval_cand(int32_t cx, int32_t cy, const mparams *pp, mbv src, msel *s) {
    mbv t = mb_at(pp->pred, cx, cy);
    int32_t sad = blk_sad(src, t);
    int32_t ssd = (cx - pp->px) * (cx - pp->px) + (cy - pp->py) * (cy - pp->py);
    int32_t mad = blk_mad(src, t);
    int accept;
    if (s->best_mad < pp->thr)
        accept = mad < s->best_mad || (mad == s->best_mad && ssd < s->best_ssd);
    else
        accept = (sad < s->best_sad || (sad == s->best_sad && ssd < s->best_ssd && sad < SAD_GATE)) ||
                 mad < pp->thr;
    if (accept) {
        s->best_x = cx;
        s->best_y = cy;
        s->best_sad = sad;
        s->best_ssd = ssd;
        s->best_mad = mad;
    }
}

static int out_of_frame(const mparams *pp, int32_t x, int32_t y) {
    return x < 0 || x > pp->pred->w - MBS || y < 0 || y > pp->pred->h - MBS;
}
static int intra_excluded(const mparams *pp, int32_t x, int32_t y) {
    return pp->intra && y > (pp->py - MBS) && x > (pp->px - MBS);
}

/* perform_{intra,inter}_motion_search, motion.cpp:225-275: j-outer, i-inner,
 * base fixed at step start. */
static void grid_search(int left, int top, int right, int bottom, int step, const mparams *pp,
                        mbv src, msel *s) {
    int32_t bx = s->best_x, by = s->best_y;
    for (int j = top; j <= bottom; j += step)
        for (int i = left; i <= right; i += step) {
            int32_t cx = bx + i, cy = by + j;
            if (intra_excluded(pp, cx, cy)) continue;
            if (out_of_frame(pp, cx, cy)) continue;
            eval_cand(cx, cy, pp, src, s);
        }
}

/* evaluate_subpel_motion_candidate, motion.cpp:151-223 */
static void eval_subpel(int32_t tx, int32_t ty, int i, int j, const mparams *pp, mbv src, mbv best,
                        msel *s) {
    scratch_mb cache;
    mbv c = mb_scratch(&cache);
    mbv t = mb_at(pp->pred, tx, ty);
    for (int quarter = 0; quarter < 2; quarter++) {
        mb_lerp(best, t, c, quarter);
        int32_t sad = blk_sad(src, c);
        int32_t mad = blk_mad(src, c);
        int accept;
        if (s->best_mad < pp->thr)
            accept = mad < s->best_mad;
        else
            accept = (sad < s->best_sad && sad < SAD_GATE) || mad < pp->thr;
        if (accept) {
            s->sp_enabled = 1;
            s->sp_amount = quarter;
            s->sp_index = frac_index(i, j);
            s->best_sad = sad;
            s->best_mad = mad;
        }
    }
}

/* perform_{intra,inter}_subpixel_motion_search, motion.cpp:277-352 */
static void subpel_search(const mparams *pp, mbv src, msel *s) {
    mbv best = mb_at(pp->pred, s->best_x, s->best_y);
    s->sp_index = 0;
    s->sp_amount = 0;
    s->sp_enabled = 0;
    for (int j = -1; j <= 1; j++)
        for (int i = -1; i <= 1; i++) {
            int32_t tx = s->best_x + i, ty = s->best_y + j;
            if (i == 0 && j == 0) continue;
            if (intra_excluded(pp, tx, ty)) continue;
            if (out_of_frame(pp, tx, ty)) continue;
            eval_subpel(tx, ty, i, j, pp, src, best, s);
        }
}

static void fill_desc(bdesc *d, const msel *s, const mparams *pp, int intra, int target) {
    /* clear_block_desc (common.cpp:67-73) zeroes 8 bytes; the rest is set
     * below except q_index/variance, which stay stale in the reference and
     * are never read for copy blocks -- zeroed here. */
    memset(d, 0, sizeof(*d));
    int type = intra ? T_INTRA : 0;
    if (s->best_x != pp->px || s->best_y != pp->py || s->sp_enabled) type |= T_MOTION;
    if (s->best_mad < pp->thr) type |= T_COPY;
    d->block_type = (uint32_t)type;
    d->prediction_target = (uint8_t)target;
    d->motion_x = (int16_t)(s->best_x - pp->px);
    d->motion_y = (int16_t)(s->best_y - pp->py);
    d->sp_pred = (uint8_t)s->sp_enabled;
    d->sp_amount = (uint8_t)s->sp_amount;
    d->sp_index = (uint8_t)s->sp_index;
}

/* calculate_intra_prediction, motion.cpp:354-419 */
static int32_t intra_prediction(uint16_t quality, mbv src, int px, int py, const planes *cur,
                                bdesc *out) {
    msel s = {px, py, blk_sad0(src), INT32_MAX, INT32_MAX, 0, 0, 0};
    mparams pp = {cur, (int16_t)((quality >> 2) + 1), (int16_t)px, (int16_t)py, 1};
    grid_search(-SEARCH_RADIUS, -(SEARCH_RADIUS << 1), SEARCH_RADIUS, 0, SEARCH_RADIUS, &pp, src, &s);
    for (int i = SEARCH_RADIUS >> 1; i > 0; i >>= 1) grid_search(-i, -i, i, i, i, &pp, src, &s);
    subpel_search(&pp, src, &s);
    fill_desc(out, &s, &pp, 1, 0);
    return s.best_sad;
}

/* calculate_inter_prediction, motion.cpp:421-494 */
static int32_t inter_prediction(uint16_t quality, mbv src, int px, int py, const planes *ref,
                                int offset, bdesc *out) {
    msel s = {px, py, INT32_MAX, INT32_MAX, INT32_MAX, 0, 0, 0};
    mparams pp = {ref, (int16_t)((quality >> 2) + 1), (int16_t)px, (int16_t)py, 0};
    mbv t = mb_at(ref, px, py);
    s.best_sad = blk_sad(src, t);
    s.best_mad = blk_mad(src, t);
    if (s.best_mad >= pp.thr) {
        for (int i = SEARCH_RADIUS; i > 0; i >>= 1) grid_search(-i, -i, i, i, i, &pp, src, &s);
        subpel_search(&pp, src, &s);
    }
    fill_desc(out, &s, &pp, 0, offset);
    return s.best_sad;
}

/* ------------------------------------------------------------------ */
/* deblocking (deblock.cpp)                                            */
/* ------------------------------------------------------------------ */

/* alpha_table / beta_table, deblock.cpp:13-27 */
static const int16_t ALPHA[32] = {0, 0, 0, 0, 0,  0,  0,  1,  1,  1,  2,  2,  3,  3,  4,  5,
                                  6, 7, 8, 9, 10, 12, 14, 16, 18, 20, 22, 24, 26, 29, 32, 35};
static const int16_t BETA[32] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 3,
                                 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 10, 11};

/* deblock_filter_values, deblock.cpp:81-129 */
static void dfilter(int16_t *p, int step, uint8_t qp, uint8_t strength, int luma) {
    int16_t p3 = p[-4 * step], p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-1 * step];
    int16_t q0 = p[0], q1 = p[step], q2 = p[2 * step], q3 = p[3 * step];
    int16_t d_p0q0 = (int16_t)iabs32(p0 - q0);
    int16_t d_p1p0 = (int16_t)iabs32(p1 - p0);
    int16_t d_q1q0 = (int16_t)iabs32(q1 - q0);
    if (d_p0q0 >= ALPHA[qp] || d_p1p0 >= BETA[qp] || d_q1q0 >= BETA[qp]) return;
    if (strength == 2) {
        p[-1 * step] = (int16_t)rdiv(p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1, 8);
        p[-2 * step] = (int16_t)rdiv(p2 + p1 + p0 + q0, 4);
        p[0] = (int16_t)rdiv(p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2, 8);
        p[step] = (int16_t)rdiv(p0 + q0 + q1 + q2, 4);
        if (luma) {
            p[-3 * step] = (int16_t)rdiv(2 * p3 + 3 * p2 + p1 + p0 + q0, 8);
            p[2 * step] = (int16_t)rdiv(2 * q3 + 3 * q2 + q1 + q0 + p0, 8);
        }
    } else if (strength == 1) {
        p[-1 * step] = (int16_t)rdiv(((q0 + p0) * 4) + p1 - q1, 8);
        p[0] = (int16_t)rdiv(((q0 + p0) * 4) + q1 - p1, 8);
        if (luma) {
            p[-2 * step] = (int16_t)rdiv((p2 * 4) + (p0 * 2) + (q0 * 2), 8);
            p[step] = (int16_t)rdiv((q2 * 4) + (q0 * 2) + (p0 * 2), 8);
        }
    }
}

static const bdesc *tbl(const uint8_t *table, uint32_t idx) {
    return (const bdesc *)(table + 16 * (size_t)idx);
}
/* compute_average_qp / compute_deblock_strength, deblock.cpp:49-79 */
static void edge_params(const bdesc *a, const bdesc *b, uint8_t *qp, uint8_t *strength) {
    int ca = (a->block_type & T_COPY) != 0, cb = (b->block_type & T_COPY) != 0;
    if (!ca && !cb) *qp = (uint8_t)((a->q_index + b->q_index) >> 1);
    else if (!ca) *qp = a->q_index;
    else if (!cb) *qp = b->q_index;
    else *qp = 0;
    *strength = (ca && cb) ? 0 : ((ca ^ cb) ? 1 : 2);
}
/* deblock_macroblock_index (uint16 result), deblock.cpp:44-47 */
static uint16_t dmb_index(uint32_t i, uint32_t j, uint32_t mbsz, uint32_t wib) {
    return (uint16_t)((i / mbsz) + (j / mbsz) * wib);
}

/* deblock_image, deblock.cpp:201-254: in place, raster order */
static void deblock_plane(int mbsz, const uint8_t *table, int luma, int16_t *img, uint32_t width,
                          uint32_t height) {
    int16_t wib = (int16_t)(width / (uint32_t)mbsz);
    uint8_t qp, st;
    for (uint32_t i = 8; i < width; i += 8) {
        edge_params(tbl(table, dmb_index(i - 1, 0, mbsz, wib)), tbl(table, dmb_index(i, 0, mbsz, wib)), &qp, &st);
        if (st)
            for (int r = 0; r < 8; r++) dfilter(img + (size_t)r * width + i, 1, qp, st, luma);
    }
    for (uint32_t j = 8; j < height; j += 8) {
        int16_t *row = img + (size_t)j * width;
        edge_params(tbl(table, dmb_index(0, j - 1, mbsz, wib)), tbl(table, dmb_index(0, j, mbsz, wib)), &qp, &st);
        if (st)
            for (int c = 0; c < 8; c++) dfilter(row + c, (int)width, qp, st, luma);
        for (uint32_t i = 8; i < width; i += 8) {
            edge_params(tbl(table, dmb_index(i, j - 1, mbsz, wib)), tbl(table, dmb_index(i, j, mbsz, wib)), &qp, &st);
            if (st)
                for (int c = 0; c < 8; c++) dfilter(row + i + c, (int)width, qp, st, luma);
            edge_params(tbl(table, dmb_index(i - 1, j, mbsz, wib)), tbl(table, dmb_index(i, j, mbsz, wib)), &qp, &st);
            if (st)
                for (int r = 0; r < 8; r++) dfilter(row + (size_t)r * width + i, 1, qp, st, luma);
        }
    }
}

void orc_deblock(const uint8_t *table, int16_t *y, int16_t *u, int16_t *v, int wa, int ha) {
    deblock_plane(16, table, 1, y, (uint32_t)wa, (uint32_t)ha);
    deblock_plane(8, table, 0, u, (uint32_t)wa / 2, (uint32_t)ha / 2);
    deblock_plane(8, table, 0, v, (uint32_t)wa / 2, (uint32_t)ha / 2);
}

/* ------------------------------------------------------------------ */
/* entropy: bit stream, exp-Golomb, ABAC                               */
/* ------------------------------------------------------------------ */

/* Output bit_stream (bitstream.cpp:181-245): LSB-first, capacity checked. */
typedef struct {
    uint8_t *data;
    uint32_t cap_bits;
    uint32_t w;
    int err;
} obits;

static void put_bit(obits *o, uint32_t b) {
    if (o->w + 1 > o->cap_bits) {
        o->err = 1;
        return;
    }
    uint8_t *p = &o->data[o->w >> 3];
    uint32_t s = o->w & 7;
    *p = (uint8_t)((*p & ~(1u << s)) | ((b & 1u) << s));
    o->w++;
}

/* Adaptive binary arithmetic coder (abac.cpp), precision 16. */
typedef struct {
    uint32_t e3, h0, h1, low, high;
} abac;

static void abac_clear(abac *a) { /* abac.cpp:76-93 */
    a->low = 0;
    a->e3 = 0;
    a->h0 = a->h1 = 1;
    a->high = 0xFFFF;
}
/* encode_symbol + resolve_encode_scaling, abac.cpp:110-135, 178-224 */
static void abac_bit(abac *a, uint32_t bit, obits *o) {
    uint64_t range = a->high - a->low;
    uint32_t mid = a->low + (uint32_t)(range * a->h0 / (a->h0 + a->h1));
    if (bit) {
        a->low = mid + 1;
        a->h1++;
    } else {
        a->high = mid;
        a->h0++;
    }
    for (;;) {
        if ((a->high & 0x8000) == (a->low & 0x8000)) {
            uint32_t msb = (a->high >> 15) & 1;
            a->low -= 0x8000 * msb;
            a->high -= 0x8000 * msb;
            put_bit(o, msb);
            for (uint32_t k = 0; k < a->e3; k++) put_bit(o, !msb);
            a->e3 = 0;
        } else if (a->high <= 0xBFFD && a->low > 0x3FFF) {
            a->high -= 0x4000;
            a->low -= 0x4000;
            a->e3++;
        } else {
            break;
        }
        a->high = ((a->high << 1) & 0xFFFF) | 1;
        a->low = (a->low << 1) & 0xFFFF;
    }
}
/* flush_encoder, abac.cpp:279-310 */
static void abac_flush(abac *a, obits *o) {
    a->e3++;
    uint32_t b = a->low < 0x3FFF ? 0 : 1;
    put_bit(o, b);
    for (uint32_t k = 0; k < a->e3; k++) put_bit(o, !b);
    abac_clear(a);
}

/* The coder alone over a raw feed (LSB-first 32-bit words), one slice:
 * encode_symbol per bit, then flush_encoder (abac.cpp:110-135, 178-224,
 * 279-310).  Test infrastructure: checks the product's closed-form coder on
 * arbitrary bit sequences.  Returns the bits written (0 with *err set if
 * they exceed cap_bits). */
uint32_t orc_abac_feed(const uint32_t *words, uint64_t nbits, uint8_t *out, uint32_t cap_bits, int *err) {
    abac a;
    abac_clear(&a);
    obits o = {out, cap_bits, 0, 0};
    for (uint64_t i = 0; i < nbits; i++) abac_bit(&a, (words[i >> 5] >> (i & 31)) & 1u, &o);
    abac_flush(&a, &o);
    if (err) *err = o.err;
    return o.w;
}

/* The feed stream (common.cpp:147) only bounds how many bits one section may
 * write between empty() calls; every accepted bit is consumed by the coder
 * in order.  Writes that would exceed capacity are dropped whole
 * (bitstream.cpp:206-216), and callers ignore the error (stream.cpp:573-578). */
typedef struct {
    abac *a;
    obits *o;
    uint32_t w; /* write index since the last empty() */
} feed;

static void feed_empty(feed *f) { f->w = 0; }
static void feed_bits(feed *f, uint32_t value, uint32_t count) {
    if (f->w + count > FEED_CAPACITY_BITS) return;
    f->w += count;
    for (uint32_t k = 0; k < count; k++) abac_bit(f->a, (value >> k) & 1u, f->o);
}

/* encode_unsigned_golomb_value (golomb.cpp:8-58) / signed (golomb.cpp:21-84).
 * The EVX_*EXP_GOLOMB tables (egtables.h) equal the generic branch. */
static uint32_t golomb_from(uint32_t value, uint32_t *count) {
    uint32_t bits = (uint32_t)lut_log2_u32(value) + 1, rev = 0;
    for (uint32_t v = value; v; v >>= 1) rev = (rev << 1) | (v & 1);
    *count = 2 * bits - 1;
    return rev << (bits - 1);
}
static void put_ue(feed *f, uint16_t v) {
    uint32_t n;
    uint32_t code = golomb_from((uint32_t)v + 1, &n);
    feed_bits(f, code, n);
}
static void put_se(feed *f, int16_t v) {
    uint32_t n;
    uint32_t value = v == 0 ? 1u : (((uint32_t)iabs32(v) << 1) | (uint32_t)((v >> 15) & 1));
    uint32_t code = golomb_from(value, &n);
    feed_bits(f, code, n);
}

/* EVX_MACROBLOCK_8x8_ZIGZAG, scan.h:60-70 */
static const uint8_t ZIGZAG8[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* entropy_rle_stream_encode_8x8, stream.cpp:550-581 */
static void rle_8x8(feed *f, const int16_t *c) {
    int32_t run;
    for (run = 63; run >= 0; --run)
        if (c[ZIGZAG8[run]]) break;
    run = run + 1;
    put_ue(f, (uint16_t)run);
    for (int32_t k = 0; k < run; k++) put_se(f, c[ZIGZAG8[k]]);
}

/* serialize_block_8x8, serialize.cpp:10-23 */
static void ser_8x8(feed *f, const int16_t *src, uint32_t width, int16_t last_dc) {
    int16_t cache[64];
    for (int j = 0; j < 8; j++) memcpy(cache + j * 8, src + (size_t)j * width, 16);
    cache[0] = (int16_t)(cache[0] - last_dc);
    rle_8x8(f, cache);
}

/* serialize_image_blocks_16x16 / _8x8, serialize.cpp:25-123 */
static void ser_plane(feed *f, const int16_t *img, uint32_t width, uint32_t height, int blk,
                      const uint8_t *table) {
    uint16_t bi = 0;
    feed_empty(f);
    for (uint32_t j = 0; j < height; j += (uint32_t)blk)
        for (uint32_t i = 0; i < width; i += (uint32_t)blk) {
            const bdesc *d = tbl(table, bi++);
            if (d->block_type & T_COPY) continue;
            int16_t last_dc = 0;
            if (i >= (uint32_t)blk)
                last_dc = img[(size_t)j * width + (i - 8)];
            else if (j >= (uint32_t)blk)
                last_dc = img[(size_t)(j - 8) * width + i];
            const int16_t *b = img + (size_t)j * width + i;
            if (blk == 16) {
                ser_8x8(f, b, width, last_dc);
                ser_8x8(f, b + 8, width, b[0]);
                ser_8x8(f, b + 8 * width, width, b[0]);
                ser_8x8(f, b + 8 * width + 8, width, b[8 * width]);
            } else {
                ser_8x8(f, b, width, last_dc);
            }
        }
}

/* serialize_slice, serialize.cpp:319-340 (+ block table :125-317) */
static void serialize_slice(const uint8_t *table, uint16_t count, int ring, const planes *coef,
                            obits *o) {
    abac a;
    feed f = {&a, o, 0};
    abac_clear(&a);
    uint32_t tbits = lut_log2_u8((uint8_t)ring);

    feed_empty(&f); /* serialize_block_types :125-135 */
    for (uint32_t i = 0; i < count; i++) feed_bits(&f, tbl(table, i)->block_type & 7u, 3);

    feed_empty(&f); /* serialize_prediction_targets :137-154 */
    for (uint32_t i = 0; i < count; i++) {
        const bdesc *d = tbl(table, i);
        if (d->block_type & T_INTRA) continue;
        feed_bits(&f, d->prediction_target & ((1u << tbits) - 1u), tbits);
    }

    feed_empty(&f); /* serialize_motion_vectors :156-191 */
    int16_t last = 0;
    for (uint32_t i = 0; i < count; i++) {
        const bdesc *d = tbl(table, i);
        if (!(d->block_type & T_MOTION)) continue;
        put_se(&f, (int16_t)(d->motion_x - last));
        last = d->motion_x;
    }
    last = 0;
    for (uint32_t i = 0; i < count; i++) {
        const bdesc *d = tbl(table, i);
        if (!(d->block_type & T_MOTION)) continue;
        put_se(&f, (int16_t)(d->motion_y - last));
        last = d->motion_y;
    }

    feed_empty(&f); /* serialize_subpixel_motion_params :193-241 */
    for (uint32_t i = 0; i < count; i++) {
        const bdesc *d = tbl(table, i);
        if (d->block_type & T_MOTION) feed_bits(&f, d->sp_pred & 1u, 1);
    }
    for (uint32_t i = 0; i < count; i++) {
        const bdesc *d = tbl(table, i);
        if ((d->block_type & T_MOTION) && d->sp_pred) feed_bits(&f, d->sp_amount & 1u, 1);
    }
    for (uint32_t i = 0; i < count; i++) {
        const bdesc *d = tbl(table, i);
        if ((d->block_type & T_MOTION) && d->sp_pred) feed_bits(&f, d->sp_index & 7u, 3);
    }

    feed_empty(&f); /* serialize_block_quality :243-261 */
    int16_t lq = 0;
    for (uint32_t i = 0; i < count; i++) {
        const bdesc *d = tbl(table, i);
        if (d->block_type & T_COPY) continue;
        put_se(&f, (int16_t)(d->q_index - lq));
        lq = d->q_index;
    }

    /* serialize_macroblocks :125-155 */
    ser_plane(&f, coef->y, (uint32_t)coef->w, (uint32_t)coef->h, 16, table);
    ser_plane(&f, coef->u, (uint32_t)coef->w / 2, (uint32_t)coef->h / 2, 8, table);
    ser_plane(&f, coef->v, (uint32_t)coef->w / 2, (uint32_t)coef->h / 2, 8, table);

    abac_flush(&a, o); /* finish_encode */
}

/* ------------------------------------------------------------------ */
/* frame engine (encode.cpp, decode.cpp)                               */
/* ------------------------------------------------------------------ */

struct orc_encoder {
    int ring, initialized;
    uint32_t type, index;
    uint16_t quality;
    uint16_t width, height;
    int wa, ha, wmb, hmb;
    planes input, output, *slots, predeblock;
    uint8_t *table;
    uint8_t *inter_descs;
    int32_t *inter_sads;
};

static uint32_t slot_of(const orc_encoder *e, int offset) { /* common.cpp:192-195 */
    return (e->index + (uint32_t)e->ring - (uint32_t)offset) % (uint32_t)e->ring;
}

/* classify_block, encode.cpp:17-67 */
static void classify(orc_encoder *e, mbv src, int px, int py, bdesc *out) {
    bdesc best;
    int mb = (py / 16) * e->wmb + px / 16;
    int32_t best_sad = intra_prediction(e->quality, src, px, py, &e->slots[slot_of(e, 0)], &best);
    if (e->type == 1) {
        for (int off = 1; off < e->ring; off++) {
            bdesc in;
            int32_t sad = inter_prediction(e->quality, src, px, py, &e->slots[slot_of(e, off)], off, &in);
            memcpy(e->inter_descs + 16 * ((size_t)(off - 1) * e->wmb * e->hmb + mb), &in, 16);
            e->inter_sads[(size_t)(off - 1) * e->wmb * e->hmb + mb] = sad;
            int ci = (in.block_type & T_COPY) != 0, cb = (best.block_type & T_COPY) != 0;
            if (ci ^ cb) {
                if (ci) {
                    best = in;
                    best_sad = sad;
                }
            } else if (sad < best_sad) {
                best = in;
                best_sad = sad;
            }
        }
    }
    *out = best;
}

/* The prediction block of a motion type (encode.cpp:80-141 / decode.cpp:29-64):
 * the block at the motion vector, or its lerp toward the sub-pel neighbour. */
static mbv motion_pred(const planes *p, const bdesc *d, int px, int py, scratch_mb *cache) {
    mbv beta = mb_at(p, px + d->motion_x, py + d->motion_y);
    if (!d->sp_pred) return beta;
    int dx, dy;
    frac_dir(d->sp_index, &dx, &dy);
    mbv nb = mb_at(p, px + d->motion_x + dx, py + d->motion_y + dy);
    mbv c = mb_scratch(cache);
    mb_lerp(beta, nb, c, d->sp_amount);
    return c;
}

/* encode_block, encode.cpp:69-163 */
static void encode_block(orc_encoder *e, mbv src, int px, int py, bdesc *d, mbv dest) {
    scratch_mb tb_s, mc_s;
    mbv tb = mb_scratch(&tb_s);
    int type = (int)d->block_type;
    if (type & T_COPY) return; /* copy types: nothing (coefficients left stale) */
    if (type == T_INTRA) {
        mb_transform(src, tb);
    } else if (type == (T_INTRA | T_MOTION)) {
        mb_sub_transform(src, motion_pred(&e->slots[slot_of(e, 0)], d, px, py, &mc_s), tb);
    } else if (type == 0) {
        mb_sub_transform(src, mb_at(&e->slots[slot_of(e, d->prediction_target)], px, py), tb);
    } else { /* T_MOTION */
        mb_sub_transform(src, motion_pred(&e->slots[slot_of(e, d->prediction_target)], d, px, py, &mc_s), tb);
    }
    d->q_index = vaq((uint8_t)e->quality, tb.y, tb.stride);
    d->variance = (int16_t)variance2(tb.y, tb.stride);
    mb_quantize(d->q_index, type, tb, dest);
}

/* decode_block, decode.cpp:15-144 (the encoder's in-loop reconstruction) */
static void decode_block(orc_encoder *e, const bdesc *d, mbv coef, int px, int py, mbv dest) {
    scratch_mb tb_s, mc_s;
    mbv tb = mb_scratch(&tb_s);
    int type = (int)d->block_type;
    const planes *p = (type & T_INTRA) ? &e->slots[slot_of(e, 0)] : &e->slots[slot_of(e, d->prediction_target)];
    switch (type) {
    case T_INTRA:
        mb_dequantize(d->q_index, type, coef, tb);
        mb_inverse_transform(tb, dest);
        break;
    case T_INTRA | T_MOTION | T_COPY:
    case T_MOTION | T_COPY:
        mb_copy(motion_pred(p, d, px, py, &mc_s), dest);
        break;
    case T_INTRA | T_MOTION:
    case T_MOTION:
        mb_dequantize(d->q_index, type, coef, tb);
        mb_inverse_transform_add(tb, motion_pred(p, d, px, py, &mc_s), dest);
        break;
    case T_COPY:
        mb_copy(mb_at(p, px, py), dest);
        break;
    case 0:
        mb_dequantize(d->q_index, type, coef, tb);
        mb_inverse_transform_add(tb, mb_at(p, px, py), dest);
        break;
    default:
        break;
    }
}

/* encode_slice, encode.cpp:165-203: raster MB loop */
static void encode_slice(orc_encoder *e) {
    uint32_t bi = 0;
    planes *cur = &e->slots[slot_of(e, 0)];
    for (int j = 0; j < e->ha; j += 16)
        for (int i = 0; i < e->wa; i += 16) {
            bdesc *d = (bdesc *)(e->table + 16 * (size_t)bi++);
            mbv src = mb_at(&e->input, i, j);
            mbv dst = mb_at(&e->output, i, j);
            mbv rec = mb_at(cur, i, j);
            classify(e, src, i, j, d);
            encode_block(e, src, i, j, d, dst);
            decode_block(e, d, dst, i, j, rec);
        }
}

orc_encoder *orc_create(int ring) {
    orc_encoder *e = (orc_encoder *)calloc(1, sizeof(orc_encoder));
    if (!e) return NULL;
    init_tables();
    e->ring = ring;
    e->quality = DEFAULT_QUALITY;
    return e;
}

void orc_clear(orc_encoder *e) { /* evx1enc.cpp:27-40 + clear_frame common.cpp:50-65 */
    if (!e->initialized) return;
    planes_free(&e->input);
    planes_free(&e->output);
    planes_free(&e->predeblock);
    for (int k = 0; k < e->ring; k++) planes_free(&e->slots[k]);
    free(e->slots);
    free(e->table);
    free(e->inter_descs);
    free(e->inter_sads);
    e->slots = NULL;
    e->table = NULL;
    e->inter_descs = NULL;
    e->inter_sads = NULL;
    e->type = 0;
    e->index = 0;
    e->quality = DEFAULT_QUALITY;
    e->initialized = 0;
}

void orc_destroy(orc_encoder *e) {
    if (!e) return;
    orc_clear(e);
    free(e);
}

void orc_insert_intra(orc_encoder *e) { e->type = 0; }
void orc_set_quality(orc_encoder *e, int q) { e->quality = (uint16_t)(q < 1 ? 1 : (q > 31 ? 31 : q)); }

static void append_bytes(obits *o, const uint8_t *b, uint32_t n) {
    for (uint32_t k = 0; k < n; k++)
        for (int s = 0; s < 8; s++) put_bit(o, (b[k] >> s) & 1u);
}

int orc_encode(orc_encoder *e, const uint8_t *rgb, int width, int height, uint8_t *out,
               uint32_t cap_bytes, uint32_t *bit_pos) {
    obits o = {out, cap_bytes * 8u, *bit_pos, 0};
    if (!e->initialized) { /* evx1enc.cpp:66-90, common.cpp:79-150 */
        e->width = (uint16_t)width;
        e->height = (uint16_t)height;
        e->wa = (width + 15) & ~15;
        e->ha = (height + 15) & ~15;
        e->wmb = e->wa / 16;
        e->hmb = e->ha / 16;
        int ok = planes_alloc(&e->input, e->wa, e->ha) && planes_alloc(&e->output, e->wa, e->ha) &&
                 planes_alloc(&e->predeblock, e->wa, e->ha);
        e->slots = (planes *)calloc((size_t)e->ring, sizeof(planes));
        for (int k = 0; k < e->ring && ok; k++) ok = planes_alloc(&e->slots[k], e->wa, e->ha);
        e->table = (uint8_t *)calloc((size_t)e->wmb * e->hmb, 16);
        e->inter_descs = (uint8_t *)calloc((size_t)(e->ring > 1 ? e->ring - 1 : 1) * e->wmb * e->hmb, 16);
        e->inter_sads = (int32_t *)calloc((size_t)(e->ring > 1 ? e->ring - 1 : 1) * e->wmb * e->hmb, 4);
        if (!ok || !e->table || !e->inter_descs || !e->inter_sads) return 10;
        e->initialized = 1;
        /* evx_header (common.h:50-62, pack(2)); byte 7 is an unwritten pad in
         * the reference, written as 0 here. */
        uint8_t h[14] = {'E', 'V', 'X', '1', 14, 0, (uint8_t)e->ring, 0, 47, 2,
                         (uint8_t)(width & 0xFF), (uint8_t)(width >> 8),
                         (uint8_t)(height & 0xFF), (uint8_t)(height >> 8)};
        append_bytes(&o, h, 14);
    }
    if (width != e->width || height != e->height) return 8;
    /* evx_frame {type u32, index u32, quality u16} (common.h:66-72) */
    uint8_t fd[10];
    for (int k = 0; k < 4; k++) fd[k] = (uint8_t)(e->type >> (8 * k));
    for (int k = 0; k < 4; k++) fd[4 + k] = (uint8_t)(e->index >> (8 * k));
    fd[8] = (uint8_t)(e->quality & 0xFF);
    fd[9] = (uint8_t)(e->quality >> 8);
    append_bytes(&o, fd, 10);

    /* engine_encode_frame, encode.cpp:205-232 */
    orc_convert_rgb(rgb, width, height, e->input.y, e->input.u, e->input.v, e->wa, e->ha);
    encode_slice(e);
    planes *cur = &e->slots[slot_of(e, 0)];
    memcpy(e->predeblock.y, cur->y, (size_t)e->wa * e->ha * 2);
    memcpy(e->predeblock.u, cur->u, (size_t)e->wa * e->ha / 2);
    memcpy(e->predeblock.v, cur->v, (size_t)e->wa * e->ha / 2);
    serialize_slice(e->table, (uint16_t)(e->wmb * e->hmb), e->ring, &e->output, &o);
    orc_deblock(e->table, cur->y, cur->u, cur->v, e->wa, e->ha);

    *bit_pos = o.w;
    if (o.err) return 10;
    e->type = 1; /* evx1enc.cpp:138-153 */
    if (((e->index + 1) % PERIODIC_INTRA) == 0) e->type = 0;
    e->index++;
    return 0;
}

const int16_t *orc_plane(const orc_encoder *e, int which, int plane) {
    const planes *p = which == 0 ? &e->input : which == 1 ? &e->output : &e->slots[which - 2];
    return plane == 0 ? p->y : plane == 1 ? p->u : p->v;
}
const int16_t *orc_predeblock_plane(const orc_encoder *e, int plane) {
    return plane == 0 ? e->predeblock.y : plane == 1 ? e->predeblock.u : e->predeblock.v;
}
const uint8_t *orc_block_table(const orc_encoder *e) { return e->table; }
const uint8_t *orc_inter_descs(const orc_encoder *e) { return e->inter_descs; }
const int32_t *orc_inter_sads(const orc_encoder *e) { return e->inter_sads; }
int orc_dims(const orc_encoder *e, int *wa, int *ha, int *ring, int *index) {
    *wa = e->wa;
    *ha = e->ha;
    *ring = e->ring;
    *index = (int)e->index;
    return e->initialized;
}
uint32_t orc_frame_index(const orc_encoder *e) { return e->index; }

/* ------------------------------------------------------------------ */
/* synthetic content and hashing (SURVEY.md §8(c),(d))                 */
/* ------------------------------------------------------------------ */

void orc_make_frame(uint8_t *rgb, int w, int h, uint32_t t, uint32_t seed) {
    uint32_t s = seed * 2654435761u + t * 40503u;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint32_t band = (uint32_t)(y * 4) / (uint32_t)h, r, g, b, n = 0;
            if (band == 0) {
                r = 90, g = 140, b = 200;
            } else if (band == 1) {
                uint32_t bx = (uint32_t)x + 2 * t;
                r = (bx / 2) & 255;
                g = ((bx / 32) & 1) ? 200 : 60;
                b = 100;
            } else if (band == 2) {
                uint32_t bx = (uint32_t)x + 2 * t, by = (uint32_t)y + t;
                r = (bx * 7 + by * 3) & 255;
                g = (((bx >> 3) ^ (by >> 3)) & 1) * 160 + 40;
                b = ((bx * bx + by * by) >> 6) & 255;
            } else {
                uint32_t bx = (uint32_t)x + 3 * t, by = (uint32_t)y + t;
                s = s * 1664525u + 1013904223u;
                n = (s >> 27) & 7;
                r = (bx * 5) & 255;
                g = (by * 3) & 255;
                b = ((bx ^ by) & 63) * 4;
            }
            uint8_t *p = rgb + ((size_t)y * w + x) * 3;
            p[0] = (uint8_t)((r + n) & 255);
            p[1] = (uint8_t)((g + n) & 255);
            p[2] = (uint8_t)((b + n) & 255);
        }
}

uint64_t orc_fnv1a64(uint64_t h, const uint8_t *d, uint64_t n) {
    for (uint64_t k = 0; k < n; k++) {
        h ^= d[k];
        h *= 0x100000001b3ull;
    }
    return h;
}

/* Work counters since the last reset: [blk_sad, blk_mad, blk_sad0, mb_lerp]
 * calls (256, 384, 256 and 384 pixel operations each). */
void orc_op_counts(uint64_t out[4], int reset) {
    for (int k = 0; k < 4; k++) {
        if (out) out[k] = g_ops[k];
        if (reset) g_ops[k] = 0;
    }
}
