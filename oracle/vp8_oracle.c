/*
 * vp8_oracle.c -- TEST INFRASTRUCTURE ONLY (see vp8_oracle.h).
 *
 * Plain-C restatement of the reference hot path, written from RFC 6386 (sections 12, 14, 15)
 * and the reference's observable behaviour.  Each function cites the reference lines it
 * restates.  Straight-line scalar code: clarity over speed.
 */
#include "vp8_oracle.h"

#include <errno.h>
#include <stdio.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#pragma GCC diagnostic ignored "-Wunused-const-variable"
#include "../webp-decoder_amd/host/vp8_tables.inc" /* RFC 6386 14.1 dc/ac_qlookup */

static inline int clampq(int q) { return q < 0 ? 0 : (q > 127 ? 127 : q); }
static inline uint8_t sat8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

/* ---- dequantisation: reference vp8_recon.c:17-76 --------------------------------------- */
typedef struct {
	int y1dc, y1ac, uvdc, uvac, y2dc, y2ac;
} OrDq;

static void or_dequant_setup(const Vp8DecodedFrame* d, OrDq dq[4]) {
	for (int s = 0; s < 4; s++) {
		int q = d->q_index;
		if (d->segmentation_enabled) q = d->segmentation_abs ? d->seg_quant_idx[s] : q + d->seg_quant_idx[s];
		dq[s].y1dc = vp8_dc_qlookup[clampq(q + d->y1_dc_delta_q)];
		dq[s].y1ac = vp8_ac_qlookup[clampq(q)];
		dq[s].uvdc = vp8_dc_qlookup[clampq(q + d->uv_dc_delta_q)];
		if (dq[s].uvdc > 132) dq[s].uvdc = 132;
		dq[s].uvac = vp8_ac_qlookup[clampq(q + d->uv_ac_delta_q)];
		dq[s].y2dc = 2 * vp8_dc_qlookup[clampq(q + d->y2_dc_delta_q)];
		dq[s].y2ac = vp8_ac_qlookup[clampq(q + d->y2_ac_delta_q)] * 155 / 100;
		if (dq[s].y2ac < 8) dq[s].y2ac = 8;
	}
}

/* ---- inverse transforms: RFC 6386 14.3 / 14.4, reference vp8_recon.c:80-148 ------------- */
static void or_iwht(const int16_t in[16], int16_t out[16]) {
	int16_t t[16];
	for (int c = 0; c < 4; c++) {
		int s03 = in[c] + in[12 + c], s12 = in[4 + c] + in[8 + c];
		int d12 = in[4 + c] - in[8 + c], d03 = in[c] - in[12 + c];
		t[c] = (int16_t)(s03 + s12);
		t[4 + c] = (int16_t)(d12 + d03);
		t[8 + c] = (int16_t)(s03 - s12);
		t[12 + c] = (int16_t)(d03 - d12);
	}
	for (int r = 0; r < 4; r++) {
		const int16_t* v = t + 4 * r;
		int s03 = v[0] + v[3], s12 = v[1] + v[2], d12 = v[1] - v[2], d03 = v[0] - v[3];
		out[4 * r + 0] = (int16_t)((s03 + s12 + 3) >> 3);
		out[4 * r + 1] = (int16_t)((d12 + d03 + 3) >> 3);
		out[4 * r + 2] = (int16_t)((s03 - s12 + 3) >> 3);
		out[4 * r + 3] = (int16_t)((d03 - d12 + 3) >> 3);
	}
}

/* x * sqrt(2) * cos(pi/8) and x * sqrt(2) * sin(pi/8) in the RFC's 16.16 fixed point */
static inline int mul_c(int x) { return x + ((x * 20091) >> 16); }
static inline int mul_s(int x) { return (x * 35468) >> 16; }

static void or_idct(const int16_t in[16], int16_t out[16]) {
	int16_t t[16];
	for (int c = 0; c < 4; c++) { /* vertical, truncated to int16 between passes */
		int a = in[c] + in[8 + c], b = in[c] - in[8 + c];
		int cc = mul_s(in[4 + c]) - mul_c(in[12 + c]);
		int dd = mul_c(in[4 + c]) + mul_s(in[12 + c]);
		t[c] = (int16_t)(a + dd);
		t[12 + c] = (int16_t)(a - dd);
		t[4 + c] = (int16_t)(b + cc);
		t[8 + c] = (int16_t)(b - cc);
	}
	for (int r = 0; r < 4; r++) {
		const int16_t* v = t + 4 * r;
		int a = v[0] + v[2], b = v[0] - v[2];
		int cc = mul_s(v[1]) - mul_c(v[3]);
		int dd = mul_c(v[1]) + mul_s(v[3]);
		out[4 * r + 0] = (int16_t)((a + dd + 4) >> 3);
		out[4 * r + 3] = (int16_t)((a - dd + 4) >> 3);
		out[4 * r + 1] = (int16_t)((b + cc + 4) >> 3);
		out[4 * r + 2] = (int16_t)((b - cc + 4) >> 3);
	}
}

/* ---- whole-block predictors: reference vp8_recon.c:152-212, 395-421, 533-560, 605-651 ---- */
/* above[-1] is the corner P; above[0..n-1] the row above; left[0..n-1] the column to the left.
 * Frame-edge fills (RFC 6386 12.2): above row 127, left column 129, corner 127 on the top row
 * and 129 on the left column; DC uses only the edges that exist (128 if neither). */
static void or_pred_block(uint8_t* dst, int stride, int n, int mode, const uint8_t* above, const uint8_t* left,
                          int have_above, int have_left) {
	int log2n = (n == 16) ? 4 : 3;
	for (int r = 0; r < n; r++) {
		for (int c = 0; c < n; c++) {
			int v;
			switch (mode) {
				case 1: v = above[c]; break; /* V */
				case 2: v = left[r]; break;  /* H */
				case 3: v = sat8(left[r] + above[c] - above[-1]); break; /* TM */
				default: { /* DC (also the reference's fallback for out-of-range modes) */
					int sum = 0, cnt = 0;
					if (have_above)
						for (int i = 0; i < n; i++) sum += above[i], cnt++;
					if (have_left)
						for (int i = 0; i < n; i++) sum += left[i], cnt++;
					if (!cnt) v = 128;
					else {
						int sh = log2n + (cnt == 2 * n);
						v = (sum + (1 << (sh - 1))) >> sh;
					}
				}
			}
			dst[r * stride + c] = (uint8_t)v;
		}
	}
}

/* ---- 4x4 sub-block predictors (B_PRED): RFC 6386 12.3, reference vp8_recon.c:214-358 ---- */
/* e[0..12] = L3 L2 L1 L0 P A0 A1 A2 A3 A4 A5 A6 A7 (the RFC's "edge" array). */
static inline int a3(int x, int y, int z) { return (x + 2 * y + z + 2) >> 2; }
static inline int a2(int x, int y) { return (x + y + 1) >> 1; }

static void or_pred_sub(uint8_t b[16], int mode, const uint8_t e[13]) {
	const uint8_t* A = e + 5; /* A[-1] == P == e[4] */
	const uint8_t L[4] = {e[3], e[2], e[1], e[0]};
	for (int r = 0; r < 4; r++) {
		for (int c = 0; c < 4; c++) {
			int v = 128;
			switch (mode) {
				case 0: { /* B_DC */
					int s = 4;
					for (int i = 0; i < 4; i++) s += A[i] + L[i];
					v = s >> 3;
					break;
				}
				case 1: v = sat8(L[r] + A[c] - e[4]); break;      /* B_TM */
				case 2: v = a3(A[c - 1], A[c], A[c + 1]); break;  /* B_VE */
				case 3: /* B_HE: rows smooth P,L0..L3 with L3 repeated */
					v = (r == 3) ? a3(L[2], L[3], L[3]) : a3(r == 0 ? e[4] : L[r - 1], L[r], L[r + 1]);
					break;
				case 4: { /* B_LD: down-left diagonal of A[0..7], A7 repeated */
					int k = r + c;
					v = (k == 6) ? a3(A[6], A[7], A[7]) : a3(A[k], A[k + 1], A[k + 2]);
					break;
				}
				case 5: { /* B_RD: down-right diagonal over the whole edge */
					int k = 3 - r + c;
					v = a3(e[k], e[k + 1], e[k + 2]);
					break;
				}
				default: v = 128; /* modes 6..9 are stated as tables below */
			}
			b[r * 4 + c] = (uint8_t)v;
		}
	}
	/* The remaining modes are small enough to state as explicit tables (RFC 6386 12.3). */
	if (mode == 6) { /* B_VR */
		b[12] = (uint8_t)a3(e[1], e[2], e[3]);
		b[8] = (uint8_t)a3(e[2], e[3], e[4]);
		b[13] = b[4] = (uint8_t)a3(e[3], e[4], e[5]);
		b[9] = b[0] = (uint8_t)a2(e[4], e[5]);
		b[14] = b[5] = (uint8_t)a3(e[4], e[5], e[6]);
		b[10] = b[1] = (uint8_t)a2(e[5], e[6]);
		b[15] = b[6] = (uint8_t)a3(e[5], e[6], e[7]);
		b[11] = b[2] = (uint8_t)a2(e[6], e[7]);
		b[7] = (uint8_t)a3(e[6], e[7], e[8]);
		b[3] = (uint8_t)a2(e[7], e[8]);
	} else if (mode == 7) { /* B_VL */
		b[0] = (uint8_t)a2(A[0], A[1]);
		b[4] = (uint8_t)a3(A[0], A[1], A[2]);
		b[8] = b[1] = (uint8_t)a2(A[1], A[2]);
		b[5] = b[12] = (uint8_t)a3(A[1], A[2], A[3]);
		b[9] = b[2] = (uint8_t)a2(A[2], A[3]);
		b[13] = b[6] = (uint8_t)a3(A[2], A[3], A[4]);
		b[10] = b[3] = (uint8_t)a2(A[3], A[4]);
		b[14] = b[7] = (uint8_t)a3(A[3], A[4], A[5]);
		b[11] = (uint8_t)a3(A[4], A[5], A[6]);
		b[15] = (uint8_t)a3(A[5], A[6], A[7]);
	} else if (mode == 8) { /* B_HD */
		b[12] = (uint8_t)a2(e[0], e[1]);
		b[13] = (uint8_t)a3(e[0], e[1], e[2]);
		b[8] = b[14] = (uint8_t)a2(e[1], e[2]);
		b[9] = b[15] = (uint8_t)a3(e[1], e[2], e[3]);
		b[10] = b[4] = (uint8_t)a2(e[2], e[3]);
		b[11] = b[5] = (uint8_t)a3(e[2], e[3], e[4]);
		b[6] = b[0] = (uint8_t)a2(e[3], e[4]);
		b[7] = b[1] = (uint8_t)a3(e[3], e[4], e[5]);
		b[2] = (uint8_t)a3(e[4], e[5], e[6]);
		b[3] = (uint8_t)a3(e[5], e[6], e[7]);
	} else if (mode == 9) { /* B_HU */
		b[0] = (uint8_t)a2(L[0], L[1]);
		b[1] = (uint8_t)a3(L[0], L[1], L[2]);
		b[2] = b[4] = (uint8_t)a2(L[1], L[2]);
		b[3] = b[5] = (uint8_t)a3(L[1], L[2], L[3]);
		b[6] = b[8] = (uint8_t)a2(L[2], L[3]);
		b[7] = b[9] = (uint8_t)a3(L[2], L[3], L[3]);
		b[10] = b[11] = b[12] = b[13] = b[14] = b[15] = L[3];
	} else if (mode > 9) {
		memset(b, 128, 16);
	}
}

/* ---- macroblock reconstruction: reference vp8_recon.c:423-684 ----------------------------- */
typedef struct {
	uint8_t *y, *u, *v;
	int w, h, cw, ch; /* padded plane sizes (stride = width) */
} OrFrame;

static void or_add_block(uint8_t* dst, int stride, const uint8_t* pred, int pstride, const int16_t res[16]) {
	for (int r = 0; r < 4; r++)
		for (int c = 0; c < 4; c++) dst[r * stride + c] = sat8(pred[r * pstride + c] + res[r * 4 + c]);
}

/* edges of an n-wide block at (x, y) of a plane, with the RFC fills */
static void or_block_edges(const uint8_t* pl, int stride, int x, int y, int n, uint8_t* above /* [-1..n-1] */,
                           uint8_t* left) {
	for (int i = -1; i < n; i++)
		above[i] = (y == 0) ? 127 : (i < 0 ? (x == 0 ? 129 : pl[(y - 1) * stride + x - 1]) : pl[(y - 1) * stride + x + i]);
	for (int i = 0; i < n; i++) left[i] = (x == 0) ? 129 : pl[(y + i) * stride + x - 1];
}

static void or_recon_mb(OrFrame* f, const Vp8DecodedFrame* d, const OrDq* dqs, uint32_t mbr, uint32_t mbc) {
	const uint32_t mb = mbr * d->mb_cols + mbc;
	const OrDq* q = &dqs[d->segmentation_enabled ? (d->segment_id[mb] & 3) : 0];
	const int x = (int)mbc * 16, y = (int)mbr * 16;
	int16_t cf[16], res[16];

	if (d->ymode[mb] == 4) {
		/* B_PRED: 16 sub-blocks in raster order, each predicted from already-reconstructed
		 * pixels.  Edge rules (reference vp8_recon.c:464-504): corner 127 on the frame's top
		 * row, else 129 on its left column; above-right of the rightmost column of sub-blocks
		 * always comes from the row above the MACROBLOCK (x+16..x+19, clamped to the padded
		 * width), 127 on the top MB row. */
		for (int sb = 0; sb < 16; sb++) {
			const int sy = y + (sb >> 2) * 4, sx = x + (sb & 3) * 4;
			uint8_t e[13];
			e[4] = (sy == 0) ? 127 : (sx == 0 ? 129 : f->y[(sy - 1) * f->w + sx - 1]);
			for (int i = 0; i < 8; i++) {
				uint8_t a;
				if (sy == 0) a = 127;
				else if ((sb & 3) == 3 && i >= 4) {
					int col = x + 16 + (i - 4);
					if (col > f->w - 1) col = f->w - 1;
					a = (y == 0) ? 127 : f->y[(y - 1) * f->w + col];
				} else a = f->y[(sy - 1) * f->w + sx + i];
				e[5 + i] = a;
			}
			for (int i = 0; i < 4; i++) e[3 - i] = (sx == 0) ? 129 : f->y[(sy + i) * f->w + sx - 1];
			uint8_t pred[16];
			or_pred_sub(pred, d->bmode[mb * 16 + sb], e);
			const int16_t* c = d->coeff_y + ((size_t)mb * 16 + sb) * 16;
			for (int i = 0; i < 16; i++) cf[i] = (int16_t)(c[i] * (i ? q->y1ac : q->y1dc));
			or_idct(cf, res);
			or_add_block(f->y + sy * f->w + sx, f->w, pred, 4, res);
		}
	} else {
		uint8_t abuf[17], left[16], pred[256];
		or_block_edges(f->y, f->w, x, y, 16, abuf + 1, left);
		or_pred_block(pred, 16, 16, d->ymode[mb], abuf + 1, left, y > 0, x > 0);
		int16_t y2[16], dc[16];
		const int16_t* c2 = d->coeff_y2 + (size_t)mb * 16;
		for (int i = 0; i < 16; i++) y2[i] = (int16_t)(c2[i] * (i ? q->y2ac : q->y2dc));
		or_iwht(y2, dc); /* the 16 luma DCs come from the Y2 block */
		for (int sb = 0; sb < 16; sb++) {
			const int16_t* c = d->coeff_y + ((size_t)mb * 16 + sb) * 16;
			cf[0] = dc[sb];
			for (int i = 1; i < 16; i++) cf[i] = (int16_t)(c[i] * q->y1ac);
			or_idct(cf, res);
			const int oy = (sb >> 2) * 4, ox = (sb & 3) * 4;
			or_add_block(f->y + (y + oy) * f->w + x + ox, f->w, pred + oy * 16 + ox, 16, res);
		}
	}

	const int cx = (int)mbc * 8, cy = (int)mbr * 8;
	for (int p = 0; p < 2; p++) {
		uint8_t* pl = p ? f->v : f->u;
		const int16_t* coef = (p ? d->coeff_v : d->coeff_u) + (size_t)mb * 64;
		uint8_t abuf[9], left[8], pred[64];
		or_block_edges(pl, f->cw, cx, cy, 8, abuf + 1, left);
		or_pred_block(pred, 8, 8, d->uv_mode[mb], abuf + 1, left, cy > 0, cx > 0);
		for (int b = 0; b < 4; b++) {
			for (int i = 0; i < 16; i++) cf[i] = (int16_t)(coef[b * 16 + i] * (i ? q->uvac : q->uvdc));
			or_idct(cf, res);
			const int oy = (b >> 1) * 4, ox = (b & 1) * 4;
			or_add_block(pl + (cy + oy) * f->cw + cx + ox, f->cw, pred + oy * 8 + ox, 8, res);
		}
	}
}

/* ---- loop filter: RFC 6386 15, reference vp8_loopfilter.c ----------------------------------- */
static inline int sclamp(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
static inline int iabs(int v) { return v < 0 ? -v : v; }

/* pixel k positions from the edge (k<0: p side), step = 1 across a vertical edge, stride across
 * a horizontal one.  reference vp8_loopfilter.c:20-104 */
#define PX(k) q0[(k) * step]

static int or_simple_ok(const uint8_t* q0, int step, int limit) {
	return iabs(PX(-1) - PX(0)) * 2 + (iabs(PX(-2) - PX(1)) >> 1) <= limit;
}
static int or_normal_ok(const uint8_t* q0, int step, int E, int I) {
	return or_simple_ok(q0, step, 2 * E + I) && iabs(PX(-4) - PX(-3)) <= I && iabs(PX(-3) - PX(-2)) <= I &&
	       iabs(PX(-2) - PX(-1)) <= I && iabs(PX(3) - PX(2)) <= I && iabs(PX(2) - PX(1)) <= I &&
	       iabs(PX(1) - PX(0)) <= I;
}
static int or_hev(const uint8_t* q0, int step, int T) { return iabs(PX(-2) - PX(-1)) > T || iabs(PX(1) - PX(0)) > T; }

static void or_common_adjust(uint8_t* q0, int step, int outer) {
	int p1 = PX(-2), p0 = PX(-1), q0v = PX(0), q1 = PX(1);
	int a = 3 * (q0v - p0) + (outer ? sclamp(p1 - q1) : 0);
	a = sclamp(a);
	int f1 = sclamp(a + 4) >> 3, f2 = sclamp(a + 3) >> 3;
	PX(0) = sat8(q0v - f1);
	PX(-1) = sat8(p0 + f2);
	if (!outer) {
		int a2v = (f1 + 1) >> 1;
		PX(1) = sat8(q1 - a2v);
		PX(-2) = sat8(p1 + a2v);
	}
}
static void or_mb_adjust(uint8_t* q0, int step) {
	int p2 = PX(-3), p1 = PX(-2), p0 = PX(-1), q0v = PX(0), q1 = PX(1), q2 = PX(2);
	int w = sclamp(sclamp(p1 - q1) + 3 * (q0v - p0));
	int a = (27 * w + 63) >> 7;
	PX(-1) = sat8(p0 + a);
	PX(0) = sat8(q0v - a);
	a = (18 * w + 63) >> 7;
	PX(-2) = sat8(p1 + a);
	PX(1) = sat8(q1 - a);
	a = (9 * w + 63) >> 7;
	PX(-3) = sat8(p2 + a);
	PX(2) = sat8(q2 - a);
}
#undef PX

/* One edge of n positions; `along` walks the edge, `step` crosses it. kind: 0 simple, 1 normal MB
 * edge, 2 normal sub-block edge. */
static void or_edge(uint8_t* q0, int along, int step, int n, int kind, int limit_or_E, int I, int T) {
	for (int i = 0; i < n; i++, q0 += along) {
		if (kind == 0) {
			if (or_simple_ok(q0, step, limit_or_E)) or_common_adjust(q0, step, 1);
		} else if (or_normal_ok(q0, step, limit_or_E, I)) {
			if (kind == 1) {
				if (or_hev(q0, step, T)) or_common_adjust(q0, step, 1);
				else or_mb_adjust(q0, step);
			} else {
				or_common_adjust(q0, step, or_hev(q0, step, T));
			}
		}
	}
}

/* per-MB filter parameters: reference vp8_loopfilter.c:166-199 (frame level or segment level,
 * then ref/mode deltas; note: the reference filters whenever the PER-MB level is non-zero). */
static void or_lf_params(const Vp8DecodedFrame* d, uint32_t mb, int* E, int* I, int* T) {
	int lvl = d->lf_level;
	if (d->segmentation_enabled) {
		int s = d->seg_lf_level[d->segment_id[mb] & 3];
		lvl = d->segmentation_abs ? s : lvl + s;
	}
	lvl = lvl < 0 ? 0 : (lvl > 63 ? 63 : lvl);
	if (d->lf_delta_enabled) {
		lvl += d->lf_ref_delta[0];
		if (d->ymode[mb] == 4) lvl += d->lf_mode_delta[0];
		lvl = lvl < 0 ? 0 : (lvl > 63 ? 63 : lvl);
	}
	int il = lvl;
	if (d->lf_sharpness) {
		il >>= (d->lf_sharpness > 4) ? 2 : 1;
		if (il > 9 - d->lf_sharpness) il = 9 - d->lf_sharpness;
	}
	if (il < 1) il = 1;
	*E = lvl;
	*I = il;
	*T = (lvl >= 40) ? 2 : (lvl >= 15 ? 1 : 0);
}

int oracle_loopfilter(uint8_t* y, uint8_t* u, uint8_t* v, const Vp8DecodedFrame* d) {
	if (!y || !u || !v || !d) {
		errno = EINVAL;
		return -1;
	}
	const int ys = (int)d->mb_cols * 16, cs = (int)d->mb_cols * 8;
	for (uint32_t r = 0; r < d->mb_rows; r++) {
		for (uint32_t c = 0; c < d->mb_cols; c++) {
			const uint32_t mb = r * d->mb_cols + c;
			int E, I, T;
			or_lf_params(d, mb, &E, &I, &T);
			if (E == 0) continue;
			const int inner = (d->has_coeff && d->has_coeff[mb]) || d->ymode[mb] == 4;
			uint8_t* py = y + (size_t)r * 16 * ys + c * 16;
			uint8_t* pu = u + (size_t)r * 8 * cs + c * 8;
			uint8_t* pv = v + (size_t)r * 8 * cs + c * 8;
			if (d->lf_use_simple) { /* luma only, reference vp8_loopfilter.c:228-244 */
				const int mbl = (E + 2) * 2 + I, bl = E * 2 + I;
				if (c) or_edge(py, ys, 1, 16, 0, mbl, 0, 0);
				if (inner)
					for (int k = 4; k < 16; k += 4) or_edge(py + k, ys, 1, 16, 0, bl, 0, 0);
				if (r) or_edge(py, 1, ys, 16, 0, mbl, 0, 0);
				if (inner)
					for (int k = 4; k < 16; k += 4) or_edge(py + k * ys, 1, ys, 16, 0, bl, 0, 0);
			} else { /* normal, reference vp8_loopfilter.c:245-277 */
				if (c) {
					or_edge(py, ys, 1, 16, 1, E + 2, I, T);
					or_edge(pu, cs, 1, 8, 1, E + 2, I, T);
					or_edge(pv, cs, 1, 8, 1, E + 2, I, T);
				}
				if (inner) {
					for (int k = 4; k < 16; k += 4) or_edge(py + k, ys, 1, 16, 2, E, I, T);
					or_edge(pu + 4, cs, 1, 8, 2, E, I, T);
					or_edge(pv + 4, cs, 1, 8, 2, E, I, T);
				}
				if (r) {
					or_edge(py, 1, ys, 16, 1, E + 2, I, T);
					or_edge(pu, 1, cs, 8, 1, E + 2, I, T);
					or_edge(pv, 1, cs, 8, 1, E + 2, I, T);
				}
				if (inner) {
					for (int k = 4; k < 16; k += 4) or_edge(py + k * ys, 1, ys, 16, 2, E, I, T);
					or_edge(pu + 4 * cs, 1, cs, 8, 2, E, I, T);
					or_edge(pv + 4 * cs, 1, cs, 8, 2, E, I, T);
				}
			}
		}
	}
	return 0;
}

int oracle_recon_padded(const Vp8DecodedFrame* d, uint8_t* y, uint8_t* u, uint8_t* v, int filtered) {
	if (!d || !y || !u || !v) {
		errno = EINVAL;
		return -1;
	}
	OrFrame f = {y, u, v, (int)d->mb_cols * 16, (int)d->mb_rows * 16, (int)d->mb_cols * 8, (int)d->mb_rows * 8};
	OrDq dq[4];
	or_dequant_setup(d, dq);
	for (uint32_t r = 0; r < d->mb_rows; r++)
		for (uint32_t c = 0; c < d->mb_cols; c++) or_recon_mb(&f, d, dq, r, c);
	return filtered ? oracle_loopfilter(y, u, v, d) : 0;
}

/* crop: reference vp8_recon.c:693-711 */
int oracle_reconstruct_i420(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, uint8_t* buf, int filtered) {
	if (!kf || !d || !buf || kf->width > d->mb_cols * 16 || kf->height > d->mb_rows * 16) {
		errno = EINVAL;
		return -1;
	}
	const size_t pw = d->mb_cols * 16u, ph = d->mb_rows * 16u;
	uint8_t* pad = (uint8_t*)malloc(pw * ph * 3 / 2);
	if (!pad) {
		errno = ENOMEM;
		return -1;
	}
	uint8_t *py = pad, *pu = pad + pw * ph, *pv = pu + pw * ph / 4;
	if (oracle_recon_padded(d, py, pu, pv, filtered) != 0) {
		free(pad);
		return -1;
	}
	const uint32_t w = kf->width, h = kf->height, cw = (w + 1) / 2, ch = (h + 1) / 2;
	uint8_t* o = buf;
	for (uint32_t r = 0; r < h; r++, o += w) memcpy(o, py + r * pw, w);
	for (uint32_t r = 0; r < ch; r++, o += cw) memcpy(o, pu + r * (pw / 2), cw);
	for (uint32_t r = 0; r < ch; r++, o += cw) memcpy(o, pv + r * (pw / 2), cw);
	free(pad);
	return 0;
}

int oracle_reconstruct(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, Yuv420Image* out, int filtered) {
	if (!kf || !d || !out) {
		errno = EINVAL;
		return -1;
	}
	const uint32_t w = kf->width, h = kf->height, cw = (w + 1) / 2, ch = (h + 1) / 2;
	uint8_t* buf = (uint8_t*)malloc((size_t)w * h + 2 * (size_t)cw * ch);
	if (!buf) {
		errno = ENOMEM;
		return -1;
	}
	if (oracle_reconstruct_i420(kf, d, buf, filtered) != 0) {
		free(buf);
		return -1;
	}
	out->width = w;
	out->height = h;
	out->stride_y = w;
	out->stride_uv = cw;
	out->y = buf;
	out->u = buf + (size_t)w * h;
	out->v = out->u + (size_t)cw * ch;
	return 0;
}

void oracle_image_free(Yuv420Image* img) {
	if (!img) return;
	free(img->y); /* single allocation */
	memset(img, 0, sizeof(*img));
}

/* ---- CPU baseline timing harness ----------------------------------------------------------- */
typedef struct {
	const Vp8KeyFrameHeader* const* kfs;
	const Vp8DecodedFrame* const* frames;
	int nframes, n, filtered;
	int next;
	int err;
	pthread_mutex_t mu;
} OrJob;

static void* or_worker(void* arg) {
	OrJob* j = (OrJob*)arg;
	for (;;) {
		pthread_mutex_lock(&j->mu);
		int i = j->next++;
		pthread_mutex_unlock(&j->mu);
		if (i >= j->n) break;
		Yuv420Image img;
		if (oracle_reconstruct(j->kfs[i % j->nframes], j->frames[i % j->nframes], &img, j->filtered) != 0) j->err = 1;
		else oracle_image_free(&img);
	}
	return NULL;
}

double oracle_time_batch(const Vp8KeyFrameHeader* const* kfs, const Vp8DecodedFrame* const* frames, int nframes, int n,
                         int threads, int filtered) {
	if (!kfs || !frames || nframes <= 0 || n <= 0 || threads <= 0 || threads > 1024) return -1.0;
	OrJob j = {kfs, frames, nframes, n, filtered, 0, 0, PTHREAD_MUTEX_INITIALIZER};
	pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
	if (!th) return -1.0;
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	int started = 0;
	for (int i = 0; i < threads; i++)
		if (pthread_create(&th[i], NULL, or_worker, &j) == 0) started++;
	for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	free(th);
	if (j.err || started == 0) return -1.0;
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ==== m08 / m09: I420 -> RGB24 ("fancy" 4:2:0 upsampling) and the PPM / PNG writers ========
 * Restated per output pixel (the reference walks row pairs and pixel pairs; the values are the
 * same): reference src/m08_yuv2rgb_ppm/yuv2rgb_ppm.c:13-121 (conversion + upsampler),
 * :123-206 (PPM writer); src/m09_png/yuv2rgb_png.c:122-164 (CRC-32, chunks, Adler-32) and
 * :208-364 (PNG writer: filter 0, zlib stored blocks of <= 65535 bytes, one IDAT). */

/* reference yuv2rgb_ppm.c:19-42 (libwebp VP8YuvToRgb, 14-bit fixed point, clip of v >> 6) */
static inline uint8_t or_clip6(int v) { return (uint8_t)(v < 0 ? 0 : (v >> 6 > 255 ? 255 : v >> 6)); }
static void or_yuv_rgb(int y, int u, int v, uint8_t* d) {
	const int yy = (y * 19077) >> 8;
	d[0] = or_clip6(yy + ((v * 26149) >> 8) - 14234);
	d[1] = or_clip6(yy - ((u * 6419) >> 8) - ((v * 13320) >> 8) + 8708);
	d[2] = or_clip6(yy + ((u * 33050) >> 8) - 17685);
}

/* Chroma value of output pixel (x, y) in plane p (stride s, cw x ch samples), reference
 * yuv2rgb_ppm.c:44-121 + row pairing :178-202: row 0 uses chroma row 0 twice; row y >= 1 sits
 * between chroma rows a = (y-1)/2 and b = min(a+1, ch-1), nearer a when y is odd.  Columns:
 * x = 0 and (even width) x = w-1 use one chroma column (3:1 vertical blend); inner pixels pair
 * up as (2k-1, 2k) between columns k-1 and k (9:3:3:1 with libwebp's two-step rounding). */
static int or_chroma(const uint8_t* p, uint32_t s, uint32_t w, uint32_t ch, uint32_t x, uint32_t y) {
	const uint32_t a = y ? (y - 1) >> 1 : 0, b = y ? ((a + 1 < ch) ? a + 1 : ch - 1) : 0;
	const int near_a = (y == 0) || (y & 1);
	const uint8_t* ra = p + (size_t)a * s;
	const uint8_t* rb = p + (size_t)b * s;
	if (x == 0 || ((w & 1) == 0 && x == w - 1)) {
		const uint32_t c = x >> 1;
		const int n = near_a ? ra[c] : rb[c], f = near_a ? rb[c] : ra[c];
		return (3 * n + f + 2) >> 2;
	}
	const uint32_t k = (x + 1) >> 1; /* pair (2k-1, 2k): columns k-1, k */
	const int tl = ra[k - 1], t = ra[k], l = rb[k - 1], u = rb[k];
	const int avg = tl + t + l + u + 8;
	const int d12 = (avg + 2 * (t + l)) >> 3, d03 = (avg + 2 * (tl + u)) >> 3;
	if (near_a) return (x & 1) ? (d12 + tl) >> 1 : (d03 + t) >> 1;
	return (x & 1) ? (d03 + l) >> 1 : (d12 + u) >> 1;
}

void oracle_rgb_row(const Yuv420Image* img, uint32_t y, uint8_t* dst) {
	const uint32_t ch = (img->height + 1u) >> 1;
	for (uint32_t x = 0; x < img->width; x++)
		or_yuv_rgb(img->y[(size_t)y * img->stride_y + x], or_chroma(img->u, img->stride_uv, img->width, ch, x, y),
		           or_chroma(img->v, img->stride_uv, img->width, ch, x, y), dst + 3 * (size_t)x);
}

static int or_ppm_header(uint32_t w, uint32_t h, char* hdr) { return sprintf(hdr, "P6\n%u %u\n255\n", w, h); }

size_t oracle_ppm_size(uint32_t w, uint32_t h) {
	char hdr[64];
	return (size_t)or_ppm_header(w, h, hdr) + (size_t)w * h * 3u;
}

/* reference yuv2rgb_ppm.c:123-206: "P6\n<w> <h>\n255\n" + RGB rows */
long oracle_ppm(const Yuv420Image* img, uint8_t* out, size_t cap) {
	if (!img || !img->y || !img->u || !img->v || img->width == 0 || img->height == 0) return -1;
	char hdr[64];
	const int n = or_ppm_header(img->width, img->height, hdr);
	const size_t total = (size_t)n + (size_t)img->width * img->height * 3u;
	if (cap < total) return -1;
	memcpy(out, hdr, (size_t)n);
	for (uint32_t y = 0; y < img->height; y++) oracle_rgb_row(img, y, out + n + (size_t)y * img->width * 3u);
	return (long)total;
}

/* reference yuv2rgb_png.c:122-133 (bitwise CRC-32, reflected 0xEDB88320) */
static uint32_t or_crc32(uint32_t crc, const uint8_t* p, size_t n) {
	crc = ~crc;
	for (size_t i = 0; i < n; i++) {
		crc ^= p[i];
		for (int k = 0; k < 8; k++) crc = (crc & 1u) ? (0xEDB88320u ^ (crc >> 1)) : (crc >> 1);
	}
	return ~crc;
}
static void or_be32(uint8_t* p, uint32_t v) {
	p[0] = (uint8_t)(v >> 24), p[1] = (uint8_t)(v >> 16), p[2] = (uint8_t)(v >> 8), p[3] = (uint8_t)v;
}

size_t oracle_png_size(uint32_t w, uint32_t h) {
	const uint64_t raw = (uint64_t)h * (1u + 3ull * w);
	const uint64_t blocks = (raw + 65534u) / 65535u;
	return (size_t)(8 + 25 + 12 + (2 + raw + 5 * blocks + 4) + 12);
}

/* reference yuv2rgb_png.c:208-364: signature, IHDR (8-bit RGB), one IDAT holding a zlib stream
 * (0x78 0x01, stored blocks of min(65535, rest) bytes of filter-0 scanlines, Adler-32), IEND */
long oracle_png(const Yuv420Image* img, uint8_t* out, size_t cap) {
	if (!img || !img->y || !img->u || !img->v || img->width == 0 || img->height == 0) return -1;
	const uint32_t w = img->width, h = img->height, sb = 1u + 3u * w;
	const uint64_t raw = (uint64_t)h * sb;
	if (raw > 0x7FFFFFFFu) return -1;
	const size_t total = oracle_png_size(w, h);
	if (cap < total) return -1;
	static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
	uint8_t* o = out;
	memcpy(o, sig, 8), o += 8;
	or_be32(o, 13), memcpy(o + 4, "IHDR", 4);
	or_be32(o + 8, w), or_be32(o + 12, h);
	o[16] = 8, o[17] = 2, o[18] = 0, o[19] = 0, o[20] = 0;
	or_be32(o + 21, or_crc32(0, o + 4, 17)), o += 25;
	const uint64_t blocks = (raw + 65534u) / 65535u, zlen = 2 + raw + 5 * blocks + 4;
	uint8_t* idat = o;
	or_be32(o, (uint32_t)zlen), memcpy(o + 4, "IDAT", 4), o += 8;
	*o++ = 0x78, *o++ = 0x01;
	uint8_t* line = (uint8_t*)malloc(sb);
	if (!line) return -1;
	uint32_t a = 1, b = 0, y = 0, pos = sb; /* pos: next byte of `line` (sb = exhausted) */
	for (uint64_t left = raw; left > 0;) {
		const uint32_t len = left > 65535u ? 65535u : (uint32_t)left;
		*o++ = left <= 65535u ? 1 : 0;
		*o++ = (uint8_t)len, *o++ = (uint8_t)(len >> 8);
		*o++ = (uint8_t)~len, *o++ = (uint8_t)(~len >> 8);
		for (uint32_t i = 0; i < len; i++) {
			if (pos == sb) {
				line[0] = 0;
				oracle_rgb_row(img, y++, line + 1);
				pos = 0;
			}
			const uint8_t c = line[pos++];
			*o++ = c;
			a = (a + c) % 65521u; /* reference yuv2rgb_png.c:150-164 */
			b = (b + a) % 65521u;
		}
		left -= len;
	}
	free(line);
	or_be32(o, (b << 16) | a), o += 4;
	or_be32(o, or_crc32(0, idat + 4, (size_t)(o - idat - 4))), o += 4;
	static const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};
	memcpy(o, iend, 12), o += 12;
	return (long)(o - out);
}
