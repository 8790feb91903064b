/*
 * vp8_synth.c -- seeded synthetic Vp8DecodedFrame generator (build-defined; SURVEY.md §8(c4),
 * §8(d) "second mode").  Used for the benchmark's synthetic batches and for known-answer tests
 * whose expected output hashes were produced by the reference m06/m07 (tests/golden/synth_kat.json).
 *
 * RNG: xorshift64 (x ^= x<<13; x ^= x>>7; x ^= x<<17), state = seed ^ 0x5EED0000DEADBEEF, or
 * 0x5EED if that is 0.  Every draw below consumes exactly the values stated, in the stated
 * order, so the inputs are reproducible bit-for-bit by any implementation of this spec.
 *
 * Profiles:
 *  0  "measured-like" (statistics of libwebp q75 4K / penguin frames): ymode DC .35 V .16 H .10
 *     TM .02 B_PRED .37; uv DC .45 V .30 H .17 TM .08; 4 segments (delta quant -6,0,+6,+12; LF
 *     levels 8,5,23,31 absolute), normal filter, frame level 31, sharpness 0; about 11 % non-zero
 *     coefficients, |c| <= 134, concentrated at low frequencies.
 *  1  stress: all modes uniform, full-range coefficients (|c| <= 2114, the largest token value),
 *     random quantiser / segment / loop-filter parameters (simple or normal, sharpness 0..7,
 *     ref/mode deltas), random Y-DC slots in Y2 macroblocks and random bmode[] in non-B_PRED
 *     macroblocks (both must be ignored), random segment ids even with segmentation off.
 *  2  as 1, plus out-of-range mode values (ymode 5..7, uv_mode 4..7, bmode 10..15), which the
 *     reference treats as DC / DC / 128-fill.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "vp8_front.h"

typedef struct {
	uint64_t s;
} Rng;

static uint64_t rnext(Rng* r) {
	uint64_t x = r->s;
	x ^= x << 13;
	x ^= x >> 7;
	x ^= x << 17;
	r->s = x;
	return x;
}
/* uniform in [0, n) */
static uint32_t runi(Rng* r, uint32_t n) { return (uint32_t)(((rnext(r) >> 32) * (uint64_t)n) >> 32); }
/* pick index from cumulative thresholds out of 1000 */
static int rpick(Rng* r, const int* cum, int n) {
	uint32_t v = runi(r, 1000);
	for (int i = 0; i < n - 1; i++)
		if (v < (uint32_t)cum[i]) return i;
	return n - 1;
}

static const uint8_t k_zz[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};

/* Fill one block with `first`.. coefficients: profile 0 uses a low-frequency-biased sparse
 * pattern, profiles 1/2 a denser full-range one. Returns 1 if any value is non-zero. */
static int synth_block(Rng* r, int16_t* blk, int first, int profile, int busy) {
	int nz = 0;
	if (profile == 0) {
		/* about 45 % of blocks carry coefficients; count 1..6 along the zigzag with gaps */
		if (runi(r, 100) >= (uint32_t)busy) return 0;
		int n = 1 + (int)runi(r, 6);
		int pos = first;
		for (int k = 0; k < n && pos < 16; k++) {
			pos += (int)runi(r, 3); /* gap 0..2 */
			if (pos >= 16) break;
			int mag = 1 + (int)(runi(r, 8) == 0 ? runi(r, 134) : runi(r, 4));
			blk[k_zz[pos]] = (int16_t)(runi(r, 2) ? -mag : mag);
			nz = 1;
			pos++;
		}
	} else {
		if (runi(r, 100) >= 70) return 0;
		for (int pos = first; pos < 16; pos++) {
			if (runi(r, 100) < 40) {
				int mag = 1 + (int)(runi(r, 4) == 0 ? runi(r, 2114) : runi(r, 70));
				blk[k_zz[pos]] = (int16_t)(runi(r, 2) ? -mag : mag);
				nz = 1;
			}
		}
	}
	return nz;
}

int vp8f_synth_frame(uint32_t width, uint32_t height, uint64_t seed, int profile, Vp8KeyFrameHeader* kf,
                     Vp8DecodedFrame* f) {
	if (!kf || !f || width == 0 || height == 0 || width > 16383 || height > 16383 || profile < 0 || profile > 2) {
		errno = EINVAL;
		return -1;
	}
	memset(kf, 0, sizeof(*kf));
	memset(f, 0, sizeof(*f));
	kf->is_key_frame = 1;
	kf->show_frame = 1;
	kf->start_code_ok = 1;
	kf->width = (uint16_t)width;
	kf->height = (uint16_t)height;
	const uint32_t cols = (width + 15) / 16, rows = (height + 15) / 16, total = cols * rows;
	f->mb_cols = f->stats.mb_cols = cols;
	f->mb_rows = f->stats.mb_rows = rows;
	f->mb_total = f->stats.mb_total = total;
	f->segment_id = (uint8_t*)calloc(total, 1);
	f->skip_coeff = (uint8_t*)calloc(total, 1);
	f->has_coeff = (uint8_t*)calloc(total, 1);
	f->ymode = (uint8_t*)calloc(total, 1);
	f->uv_mode = (uint8_t*)calloc(total, 1);
	f->bmode = (uint8_t*)calloc((size_t)total * 16, 1);
	f->coeff_y2 = (int16_t*)calloc((size_t)total * 16, 2);
	f->coeff_y = (int16_t*)calloc((size_t)total * 256, 2);
	f->coeff_u = (int16_t*)calloc((size_t)total * 64, 2);
	f->coeff_v = (int16_t*)calloc((size_t)total * 64, 2);
	if (!f->segment_id || !f->skip_coeff || !f->has_coeff || !f->ymode || !f->uv_mode || !f->bmode || !f->coeff_y2 ||
	    !f->coeff_y || !f->coeff_u || !f->coeff_v) {
		vp8_decoded_frame_free(f);
		errno = ENOMEM;
		return -1;
	}
	Rng rng = {seed ^ 0x5EED0000DEADBEEFull};
	if (rng.s == 0) rng.s = 0x5EED;
	Rng* r = &rng;

	/* frame-level parameters */
	if (profile == 0) {
		f->q_index = 40;
		f->segmentation_enabled = 1;
		f->segmentation_abs = 0;
		static const int8_t sq[4] = {-6, 0, 6, 12};
		static const int8_t sl[4] = {8, 5, 23, 31};
		memcpy(f->seg_quant_idx, sq, 4);
		memcpy(f->seg_lf_level, sl, 4);
		/* absolute LF levels with delta quant would need two modes; the reference keys both on
		 * segmentation_abs, so we express the LF levels as deltas from the frame level 31 */
		for (int i = 0; i < 4; i++) f->seg_lf_level[i] = (int8_t)(sl[i] - 31);
		f->lf_use_simple = 0;
		f->lf_level = 31;
		f->lf_sharpness = 0;
		f->lf_delta_enabled = 0;
	} else {
		f->q_index = (uint8_t)runi(r, 128);
		f->y1_dc_delta_q = (int8_t)((int)runi(r, 31) - 15);
		f->y2_dc_delta_q = (int8_t)((int)runi(r, 31) - 15);
		f->y2_ac_delta_q = (int8_t)((int)runi(r, 31) - 15);
		f->uv_dc_delta_q = (int8_t)((int)runi(r, 31) - 15);
		f->uv_ac_delta_q = (int8_t)((int)runi(r, 31) - 15);
		f->segmentation_enabled = (uint8_t)runi(r, 2);
		f->segmentation_abs = (uint8_t)runi(r, 2);
		for (int i = 0; i < 4; i++) f->seg_quant_idx[i] = (int8_t)((int)runi(r, 255) - 127);
		for (int i = 0; i < 4; i++) f->seg_lf_level[i] = (int8_t)((int)runi(r, 127) - 63);
		f->lf_use_simple = (uint8_t)runi(r, 2);
		f->lf_level = (uint8_t)runi(r, 64);
		f->lf_sharpness = (uint8_t)runi(r, 8);
		f->lf_delta_enabled = (uint8_t)runi(r, 2);
		for (int i = 0; i < 4; i++) f->lf_ref_delta[i] = (int8_t)((int)runi(r, 127) - 63);
		for (int i = 0; i < 4; i++) f->lf_mode_delta[i] = (int8_t)((int)runi(r, 127) - 63);
	}

	static const int ycum[5] = {350, 510, 610, 630, 1000};
	static const int uvcum[4] = {450, 750, 920, 1000};
	for (uint32_t mb = 0; mb < total; mb++) {
		int ym, uvm;
		if (profile == 0) {
			ym = rpick(r, ycum, 5);
			uvm = rpick(r, uvcum, 4);
			f->segment_id[mb] = (uint8_t)runi(r, 4);
		} else {
			ym = (int)runi(r, profile == 2 ? 8 : 5);
			uvm = (int)runi(r, profile == 2 ? 8 : 4);
			f->segment_id[mb] = (uint8_t)runi(r, 4);
		}
		f->ymode[mb] = (uint8_t)ym;
		f->uv_mode[mb] = (uint8_t)uvm;
		uint8_t* bm = f->bmode + (size_t)mb * 16;
		for (int i = 0; i < 16; i++) {
			if (ym == 4 || profile != 0) bm[i] = (uint8_t)runi(r, profile == 2 ? 16 : 10);
			else bm[i] = (uint8_t)(ym == 0 ? 0 : (ym == 1 ? 2 : (ym == 2 ? 3 : 1)));
		}
		const int has_y2 = (ym != 4);
		int any = 0;
		const int busy = (profile == 0) ? 45 : 0;
		if (has_y2) any |= synth_block(r, f->coeff_y2 + (size_t)mb * 16, 0, profile, profile == 0 ? 85 : busy);
		for (int b = 0; b < 16; b++) {
			int16_t* blk = f->coeff_y + ((size_t)mb * 16 + b) * 16;
			any |= synth_block(r, blk, has_y2 ? 1 : 0, profile, busy);
			if (has_y2 && profile != 0) blk[0] = (int16_t)((int)runi(r, 4229) - 2114); /* must be ignored */
		}
		for (int b = 0; b < 4; b++) any |= synth_block(r, f->coeff_u + ((size_t)mb * 4 + b) * 16, 0, profile, busy);
		for (int b = 0; b < 4; b++) any |= synth_block(r, f->coeff_v + ((size_t)mb * 4 + b) * 16, 0, profile, busy);
		f->has_coeff[mb] = (uint8_t)any;
		f->skip_coeff[mb] = (uint8_t)!any;
	}
	return 0;
}
