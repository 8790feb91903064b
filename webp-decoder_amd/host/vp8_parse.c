/*
 * vp8_parse.c -- key-frame header remainder, per-macroblock modes and coefficient tokens
 * (RFC 6386 sections 9, 11, 13), producing the reference's Vp8DecodedFrame.
 *
 * Output semantics follow the reference m05 (src/m05_tokens/vp8_tokens.c) exactly, because the
 * hot path's parity is defined on its output:
 *   - coefficients stored de-zigzagged, natural order (vp8_tokens.c:337);
 *   - skipped MBs and Y2-less MBs get explicit zeros (vp8_tokens.c:445-461, :496-502);
 *   - a block "has coefficients" iff some decoded value is non-zero (vp8_tokens.c:331-339), and
 *     that flag (not the EOB position) drives the neighbour context (vp8_tokens.c:290, :473-474);
 *   - has_coeff[mb] = any block of the MB has a non-zero value (vp8_tokens.c:604);
 *   - non-B_PRED MBs get bmode[] filled with the implied sub-block mode (vp8_tokens.c:913-918);
 *   - only one token partition is supported; more fail with ENOTSUP (vp8_tokens.c:357-360);
 *   - the FNV-1a-64 coefficient hash and Vp8CoeffStats counters (vp8_tokens.c:970-998).
 * All decoder state lives in a per-call context (reentrant, thread-safe).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "vp8_bool.h"
#include "vp8_front.h"

#include "vp8_tables.inc"

/* ---- RFC 6386 constants --------------------------------------------------------------- */

enum { TOK_ZERO = 0, TOK_ONE, TOK_TWO, TOK_THREE, TOK_FOUR, TOK_CAT1, TOK_CAT2, TOK_CAT3, TOK_CAT4,
       TOK_CAT5, TOK_CAT6, TOK_EOB };

/* RFC 6386 13.2 token tree {-EOB, 2, -ZERO, 4, -ONE, 6, 8, 12, -TWO, 10, -THREE, -FOUR, 14, 16,
 * -CAT1, -CAT2, 18, 20, -CAT3, -CAT4, -CAT5, -CAT6}: walked as straight code in read_block */
/* RFC 6386 13.3 band of each scan position, and zigzag scan -> natural index */
static const uint8_t k_band[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};
static const uint8_t k_scan[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
/* RFC 6386 13.2 extra-bit probabilities of DCT_CAT1..6 (0-terminated) and base values */
static const uint8_t k_cat_probs[6][12] = {
    {159, 0}, {165, 145, 0}, {173, 148, 140, 0}, {176, 155, 140, 135, 0}, {180, 157, 141, 134, 130, 0},
    {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0},
};
static const int k_cat_base[6] = {5, 7, 11, 19, 35, 67};

/* RFC 6386 11.2 key-frame luma / chroma mode trees (symbols: DC=0 V=1 H=2 TM=3 B=4) */
static const int8_t k_kf_ymode_tree[8] = {-4, 2, 4, 6, -0, -1, -2, -3};
static const uint8_t k_kf_ymode_prob[4] = {145, 156, 163, 128};
static const int8_t k_uv_mode_tree[6] = {-0, 2, -1, 4, -2, -3};
static const uint8_t k_kf_uv_mode_prob[3] = {142, 114, 183};
/* RFC 6386 11.2 sub-block mode tree (B_DC=0 TM VE HE LD RD VR VL HD HU=9) */
static const int8_t k_bmode_tree[18] = {-0, 2, -1, 4, -2, 6, 8, 12, -3, 10, -5, -6, -4, 14, -7, 16, -8, -9};
/* RFC 6386 9.3 segment id tree */
static const int8_t k_segment_tree[6] = {2, 4, -0, -1, -2, -3};

enum { PLANE_Y_AFTER_Y2 = 0, PLANE_Y2 = 1, PLANE_UV = 2, PLANE_Y_ALONE = 3 };

/* ---- FNV-1a 64 (same constants as the reference's coefficient hash) ---------------------- */

uint64_t vp8f_fnv1a64(const void* data, size_t n, uint64_t h) {
	const uint8_t* p = (const uint8_t*)data;
	for (size_t i = 0; i < n; i++) {
		h ^= p[i];
		h *= 1099511628211ull;
	}
	return h;
}

static inline uint64_t hash_block(uint64_t h, const int16_t* blk) {
	for (int i = 0; i < 16; i++) {
		uint32_t v = (uint32_t)(int32_t)blk[i];
		uint8_t le[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
		h = vp8f_fnv1a64(le, 4, h);
	}
	return h;
}

/* ---- decoder context -------------------------------------------------------------------- */

typedef struct {
	uint8_t probs[4][8][3][11]; /* token probabilities after this frame's updates */
	Vp8Bool tok;                /* token partition (of the current MB row) */
	Vp8Bool parts[8];           /* multi-partition streams: all token partitions */
	unsigned nparts;
	Vp8CoeffStats* st;
	uint64_t hash;
	uint64_t ovr_shift; /* shift count at which the reference-equivalent overread becomes non-zero */
} TokenCtx;

static void note_overread_slow(TokenCtx* t, uint32_t mb, uint32_t plane, uint32_t blk, uint32_t pos, uint32_t stage) {
	Vp8CoeffStats* st = t->st;
	if (st->token_overread_mb_index != 0xFFFFFFFFu) return;
	if (vp8b_ref_overread_bytes(&t->tok) == 0) return;
	st->token_overread_mb_index = mb;
	st->token_overread_plane = plane;
	st->token_overread_block_index = blk;
	st->token_overread_coeff_i = pos;
	st->token_overread_stage = stage;
}
/* (first position at which the partition was over-read: the reference diagnostics, `decoder -info`;
 * read_block checks the shift count against TokenCtx.ovr_shift) */

/* DCT_CAT1..6 magnitude: base + extra bits (RFC 6386 13.2) */
static inline int read_cat(Vp8Bool* b, int cat) {
	const uint8_t* ep = k_cat_probs[cat];
	int extra = 0;
	for (; *ep; ep++) extra = (extra << 1) | vp8b_read_bit(b, *ep);
	return k_cat_base[cat] + extra;
}

/* Decodes one 4x4 block's tokens (RFC 6386 13) into out[] (natural order).  Returns the mask of
 * natural positions holding a non-zero value (the block "has coefficients" iff it is non-zero).
 * The token tree (13.2) is walked as straight code: node 0 (p[0]) EOB?, node 2
 * (p[1]) ZERO?, node 4 (p[2]) ONE?, then TWO/THREE/FOUR (p[3..5]) or the categories (p[6..10]);
 * after a ZERO the next token starts at node 2 (no EOB).  `plane_tag` is only for the overread
 * diagnostics (0=Y 1=Y2 2=U 3=V).
 * The bool decoder state and the statistics live in locals: through the context pointers every
 * statistics store could alias the decoder state, which would then be reloaded and stored around
 * every bool.  `checks` (a constant at each call) adds the reference's overread bookkeeping after
 * every token; read_block runs without it and repeats a block with it only in the one block where
 * the partition's overread first begins. */
static inline __attribute__((always_inline)) uint32_t read_block_impl(TokenCtx* t, Vp8Bool* b, int type, int first, int ctx,
                                                                      int16_t out[16], uint32_t mb, uint32_t plane_tag,
                                                                      uint32_t blk, const int checks) {
	const uint64_t ovr = t->ovr_shift;
	uint32_t eobs = 0, nz = 0, amax = 0;
	uint8_t(*P)[3][11] = t->probs[type];
	memset(out, 0, 16 * sizeof(int16_t));
	uint32_t mask = 0;
	int pos = first;
	const uint8_t* p = P[k_band[pos]][ctx];
	int skip_eob = 0;
#define NOTE_OVR(stage)                                                                   \
	do {                                                                                  \
		if (checks && vp8b_shifts(b) >= ovr) {                                                 \
			t->tok = *b;                                                                  \
			note_overread_slow(t, mb, plane_tag, blk, (uint32_t)pos, (uint32_t)(stage));    \
		}                                                                                 \
	} while (0)
	while (pos < 16) {
		if (!skip_eob) {
			const int more = vp8b_read(b, p[0]);
			if (!more) {
				NOTE_OVR(0);
				eobs++;
				break;
			}
		}
		if (!vp8b_read(b, p[1])) { /* DCT_0 */
			NOTE_OVR(0);
			if (++pos == 16) break;
			p = P[k_band[pos]][0];
			skip_eob = 1;
			continue;
		}
		int mag;
		if (!vp8b_read(b, p[2])) {
			mag = 1;
			NOTE_OVR(0);
		} else {
			if (!vp8b_read(b, p[3])) {
				if (!vp8b_read(b, p[4])) mag = 2;
				else mag = 3 + vp8b_read_bit(b, p[5]);
				NOTE_OVR(0);
			} else {
				int cat;
				if (!vp8b_read(b, p[6])) cat = vp8b_read_bit(b, p[7]);
				else if (!vp8b_read(b, p[8])) cat = 2 + vp8b_read_bit(b, p[9]);
				else cat = 4 + vp8b_read_bit(b, p[10]);
				NOTE_OVR(0);
				mag = read_cat(b, cat);
				NOTE_OVR(1);
			}
		}
		const int sv = vp8b_apply_sign(b, mag);
		NOTE_OVR(2);
		out[k_scan[pos]] = (int16_t)sv;
		mask |= 1u << k_scan[pos];
		nz++;
		if ((uint32_t)mag > amax) amax = (uint32_t)mag;
		if (++pos == 16) break;
		p = P[k_band[pos]][mag == 1 ? 1 : 2];
		skip_eob = 0;
	}
#undef NOTE_OVR
	Vp8CoeffStats* st = t->st;
	st->coeff_eob_tokens += eobs;
	st->coeff_nonzero_total += nz;
	if (amax > st->coeff_abs_max) st->coeff_abs_max = amax;
	return mask;
}

static uint32_t read_block(TokenCtx* t, int type, int first, int ctx, int16_t out[16], uint32_t mb, uint32_t plane_tag,
                           uint32_t blk) {
	const Vp8Bool b0 = t->tok;
	Vp8Bool bs = b0;
	Vp8CoeffStats* st = t->st;
	const uint32_t eob0 = st->coeff_eob_tokens, nz0 = st->coeff_nonzero_total, max0 = st->coeff_abs_max;
	uint32_t mask = read_block_impl(t, &bs, type, first, ctx, out, mb, plane_tag, blk, 0);
	if (vp8b_shifts(&bs) >= t->ovr_shift && st->token_overread_mb_index == 0xFFFFFFFFu) {
		/* the partition's overread begins in this block: decode it again, noting where */
		st->coeff_eob_tokens = eob0, st->coeff_nonzero_total = nz0, st->coeff_abs_max = max0;
		bs = b0;
		mask = read_block_impl(t, &bs, type, first, ctx, out, mb, plane_tag, blk, 1);
	}
	t->tok = bs;
	return mask;
}

/* Where decoded blocks go: the dense Vp8DecodedFrame arrays (the reference's m05 output), or the
 * packed wire format (Vp8gPackedFrame: one non-zero mask per block + the non-zero values). */
typedef struct {
	Vp8gPackedFrame* pk; /* NULL: dense */
	int hash;            /* fold every block into the FNV-1a coefficient hash */
	size_t cap;          /* packed: capacity of pk->values */
	int multi;           /* accept multi-partition token streams (VP8F_MULTI_PARTITION) */
} Sink;

static int sink_values(Sink* s, uint32_t mb, uint32_t bi, const int16_t* blk, uint32_t mask) {
	Vp8gPackedFrame* pk = s->pk;
	pk->masks[(size_t)mb * VP8G_PK_BLOCKS + bi] = (uint16_t)mask;
	if (pk->n_values + 16 > s->cap) {
		size_t nc = s->cap * 2 + 1024;
		int16_t* nv = (int16_t*)realloc(pk->values, nc * sizeof(int16_t));
		if (!nv) {
			errno = ENOMEM;
			return -1;
		}
		pk->values = nv;
		s->cap = nc;
	}
	int16_t* v = pk->values + pk->n_values;
	while (mask) {
		*v++ = blk[__builtin_ctz(mask)];
		mask &= mask - 1u;
	}
	pk->n_values = (uint64_t)(v - pk->values);
	return 0;
}

/* Per-MB token decode over the whole frame (RFC 6386 13, reference vp8_tokens.c:354-622). */
static int read_all_tokens(TokenCtx* t, Vp8DecodedFrame* f, const uint8_t* has_y2, Sink* sk) {
	const uint32_t cols = f->mb_cols;
	uint8_t* above = (uint8_t*)calloc((size_t)cols, 9); /* per MB column: Y[4] U[2] V[2] Y2 */
	if (!above) {
		errno = ENOMEM;
		return -1;
	}
	Vp8CoeffStats* st = t->st;
	const int dense = sk->pk == NULL;
	int16_t tmp[16], y2[16];
	for (uint32_t r = 0; r < f->mb_rows; r++) {
		VP8_TRACE_MARK(2, r); /* token bools of MB row r follow */
		if (t->nparts > 1) { /* RFC 6386 9.5: MB row r reads partition r mod nparts */
			if (r > 0) t->parts[(r - 1) % t->nparts] = t->tok;
			t->tok = t->parts[r % t->nparts];
		}
		uint8_t left[9] = {0};
		for (uint32_t c = 0; c < cols; c++) {
			const uint32_t mb = r * cols + c;
			uint8_t* ab = above + (size_t)c * 9;
			const int skip = f->skip_coeff[mb];
			uint32_t any = 0, y2mask = 0;
			if (!dense) sk->pk->mb_off[mb] = (uint32_t)sk->pk->n_values;
			memset(y2, 0, sizeof(y2));
			if (has_y2[mb]) {
				st->blocks_total_y2++;
				if (!skip) y2mask = read_block(t, PLANE_Y2, 0, left[8] + ab[8], y2, mb, 1, 0);
				if (sk->hash) t->hash = hash_block(t->hash, y2);
				st->blocks_nonzero_y2 += y2mask != 0;
				any |= y2mask;
				left[8] = ab[8] = (uint8_t)(y2mask != 0);
			}
			if (dense) memcpy(f->coeff_y2 + (size_t)mb * 16, y2, sizeof(y2));
			const int ytype = has_y2[mb] ? PLANE_Y_AFTER_Y2 : PLANE_Y_ALONE;
			const int yfirst = has_y2[mb] ? 1 : 0;
			for (int by = 0; by < 4; by++) {
				for (int bx = 0; bx < 4; bx++) {
					const uint32_t bi = (uint32_t)(by * 4 + bx);
					uint32_t m = 0;
					st->blocks_total_y++;
					if (!skip) m = read_block(t, ytype, yfirst, left[by] + ab[bx], tmp, mb, 0, bi);
					else memset(tmp, 0, sizeof(tmp));
					if (sk->hash) t->hash = hash_block(t->hash, tmp);
					if (dense) memcpy(f->coeff_y + ((size_t)mb * 16 + bi) * 16, tmp, sizeof(tmp));
					else if (sink_values(sk, mb, bi, tmp, m) != 0) goto oom;
					st->blocks_nonzero_y += m != 0;
					any |= m;
					left[by] = ab[bx] = (uint8_t)(m != 0);
				}
			}
			for (int pl = 0; pl < 2; pl++) { /* U then V */
				int16_t* base = (pl == 0 ? f->coeff_u : f->coeff_v);
				uint8_t* lc = left + 4 + 2 * pl;
				uint8_t* ac = ab + 4 + 2 * pl;
				for (int by = 0; by < 2; by++) {
					for (int bx = 0; bx < 2; bx++) {
						const uint32_t bi = (uint32_t)(by * 2 + bx);
						uint32_t m = 0;
						if (!skip) m = read_block(t, PLANE_UV, 0, lc[by] + ac[bx], tmp, mb, (uint32_t)(2 + pl), bi);
						else memset(tmp, 0, sizeof(tmp));
						if (sk->hash) t->hash = hash_block(t->hash, tmp);
						if (dense) memcpy(base + ((size_t)mb * 4 + bi) * 16, tmp, sizeof(tmp));
						else if (sink_values(sk, mb, 16u + 4u * (uint32_t)pl + bi, tmp, m) != 0) goto oom;
						if (pl == 0) {
							st->blocks_total_u++;
							st->blocks_nonzero_u += m != 0;
						} else {
							st->blocks_total_v++;
							st->blocks_nonzero_v += m != 0;
						}
						any |= m;
						lc[by] = ac[bx] = (uint8_t)(m != 0);
					}
				}
			}
			/* packed order is Y 0..15, U 0..3, V 0..3, Y2 (decode order has Y2 first) */
			if (!dense && sink_values(sk, mb, 24, y2, y2mask) != 0) goto oom;
			f->has_coeff[mb] = (uint8_t)(any != 0);
		}
	}
	free(above);
	st->token_part_bytes_used = (uint32_t)vp8b_ref_bytes_used(&t->tok);
	st->token_overread_bytes = vp8b_ref_overread_bytes(&t->tok);
	st->token_overread = (uint8_t)(st->token_overread_bytes != 0);
	return 0;
oom:
	free(above);
	errno = ENOMEM;
	return -1;
}

void vp8_decoded_frame_free(Vp8DecodedFrame* f) {
	if (!f) return;
	free(f->segment_id);
	free(f->skip_coeff);
	free(f->has_coeff);
	free(f->ymode);
	free(f->uv_mode);
	free(f->bmode);
	free(f->coeff_y2);
	free(f->coeff_y);
	free(f->coeff_u);
	free(f->coeff_v);
	memset(f, 0, sizeof(*f));
}

static int8_t clamp_s8(int32_t v) { return (int8_t)(v < -128 ? -128 : (v > 127 ? 127 : v)); }

/* optional signed field: flag, then magnitude + sign (RFC 6386 9.3, 9.6) */
static int8_t read_opt_signed(Vp8Bool* b, int nbits) {
	if (!vp8b_read(b, 128)) return 0;
	return clamp_s8(vp8b_signed(b, nbits));
}

/* Frame-level fields of the first partition (RFC 6386 9.3-9.11, 13.4): everything before the
 * first macroblock header.  Leaves h->hb at the first macroblock header. */
typedef struct {
	Vp8Bool hb;
	int seg_map_update;
	uint8_t seg_probs[3];
	int use_skip;
	uint8_t skip_prob;
	unsigned nparts;
	uint8_t probs[4][8][3][11];
} FrameHdr;

static void parse_frame_header(ByteSpan payload, const Vp8KeyFrameHeader* kf, Vp8DecodedFrame* out, FrameHdr* h) {
	Vp8Bool* const hb = &h->hb;
	vp8b_init(hb, payload.data + 10, kf->first_partition_len);
	out->stats.part0_size_bytes = kf->first_partition_len;
	(void)vp8b_read(hb, 128); /* color space */
	(void)vp8b_read(hb, 128); /* clamping type */

	/* RFC 6386 9.3 segmentation */
	h->seg_map_update = 0;
	h->seg_probs[0] = h->seg_probs[1] = h->seg_probs[2] = 255;
	out->segmentation_enabled = (uint8_t)vp8b_read(hb, 128);
	if (out->segmentation_enabled) {
		h->seg_map_update = vp8b_read(hb, 128);
		if (vp8b_read(hb, 128)) { /* update_segment_feature_data */
			out->segmentation_abs = (uint8_t)vp8b_read(hb, 128);
			for (int i = 0; i < 4; i++) out->seg_quant_idx[i] = read_opt_signed(hb, 7);
			for (int i = 0; i < 4; i++) out->seg_lf_level[i] = read_opt_signed(hb, 6);
		}
		if (h->seg_map_update)
			for (int i = 0; i < 3; i++)
				if (vp8b_read(hb, 128)) h->seg_probs[i] = (uint8_t)vp8b_literal(hb, 8);
	}

	/* RFC 6386 9.6 loop filter */
	out->lf_use_simple = (uint8_t)vp8b_read(hb, 128);
	out->lf_level = (uint8_t)vp8b_literal(hb, 6);
	out->lf_sharpness = (uint8_t)vp8b_literal(hb, 3);
	out->lf_delta_enabled = (uint8_t)vp8b_read(hb, 128);
	if (out->lf_delta_enabled && vp8b_read(hb, 128)) {
		for (int i = 0; i < 4; i++) out->lf_ref_delta[i] = read_opt_signed(hb, 6);
		for (int i = 0; i < 4; i++) out->lf_mode_delta[i] = read_opt_signed(hb, 6);
	}

	/* RFC 6386 9.5 token partitions */
	VP8_TRACE_MARK(1, 0); /* the next two partition-0 bools are log2(nparts) */
	h->nparts = 1u << vp8b_literal(hb, 2);

	/* RFC 6386 9.6 quantisation */
	out->q_index = (uint8_t)vp8b_literal(hb, 7);
	out->y1_dc_delta_q = read_opt_signed(hb, 4);
	out->y2_dc_delta_q = read_opt_signed(hb, 4);
	out->y2_ac_delta_q = read_opt_signed(hb, 4);
	out->uv_dc_delta_q = read_opt_signed(hb, 4);
	out->uv_ac_delta_q = read_opt_signed(hb, 4);
	(void)vp8b_read(hb, 128); /* refresh_entropy_probs */

	/* RFC 6386 13.4 token probability updates */
	memcpy(h->probs, vp8_default_coeff_probs, sizeof(h->probs));
	for (int i = 0; i < 4; i++)
		for (int j = 0; j < 8; j++)
			for (int k = 0; k < 3; k++)
				for (int l = 0; l < 11; l++)
					if (vp8b_read(hb, vp8_coeff_update_probs[i][j][k][l])) h->probs[i][j][k][l] = (uint8_t)vp8b_literal(hb, 8);

	h->use_skip = vp8b_read(hb, 128);
	h->skip_prob = h->use_skip ? (uint8_t)vp8b_literal(hb, 8) : 0;

}

static int decode_frame(ByteSpan payload, Vp8DecodedFrame* out, Sink* sk) {
	if (!out) return -1;
	memset(out, 0, sizeof(*out));
	Vp8KeyFrameHeader kf;
	if (vp8_parse_keyframe_header(payload, &kf) != 0) {
		errno = EINVAL;
		return -1;
	}
	if (!kf.is_key_frame) {
		errno = ENOTSUP;
		return -1;
	}
	const uint32_t cols = (kf.width + 15u) >> 4, rows = (kf.height + 15u) >> 4;
	const uint32_t total = cols * rows;
	Vp8CoeffStats* st = &out->stats;
	out->mb_cols = st->mb_cols = cols;
	out->mb_rows = st->mb_rows = rows;
	out->mb_total = st->mb_total = total;
	st->token_overread_mb_index = st->token_overread_plane = st->token_overread_block_index = 0xFFFFFFFFu;
	st->token_overread_coeff_i = st->token_overread_stage = 0xFFFFFFFFu;
	if (cols == 0 || rows == 0 || total > (1u << 20)) {
		errno = EINVAL;
		return -1;
	}

	out->segment_id = (uint8_t*)calloc(total, 1);
	out->skip_coeff = (uint8_t*)calloc(total, 1);
	out->has_coeff = (uint8_t*)calloc(total, 1);
	out->ymode = (uint8_t*)calloc(total, 1);
	out->uv_mode = (uint8_t*)calloc(total, 1);
	out->bmode = (uint8_t*)calloc((size_t)total * 16, 1);
	int coeff_ok;
	if (!sk->pk) {
		out->coeff_y2 = (int16_t*)calloc((size_t)total * 16, sizeof(int16_t));
		out->coeff_y = (int16_t*)calloc((size_t)total * 256, sizeof(int16_t));
		out->coeff_u = (int16_t*)calloc((size_t)total * 64, sizeof(int16_t));
		out->coeff_v = (int16_t*)calloc((size_t)total * 64, sizeof(int16_t));
		coeff_ok = out->coeff_y2 && out->coeff_y && out->coeff_u && out->coeff_v;
	} else {
		/* first guess ~24 values per MB; sink_values() grows it */
		sk->cap = (size_t)total * 24 + 1024;
		sk->pk->masks = (uint16_t*)malloc((size_t)total * VP8G_PK_BLOCKS * sizeof(uint16_t));
		sk->pk->mb_off = (uint32_t*)malloc((size_t)total * sizeof(uint32_t));
		sk->pk->values = (int16_t*)malloc(sk->cap * sizeof(int16_t));
		sk->pk->n_values = 0;
		coeff_ok = sk->pk->masks && sk->pk->mb_off && sk->pk->values;
	}
	uint8_t* has_y2 = (uint8_t*)calloc(total, 1);
	uint8_t* above_b = (uint8_t*)calloc((size_t)cols * 4, 1); /* above sub-block modes, B_DC = 0 */
	TokenCtx* t = (TokenCtx*)calloc(1, sizeof(TokenCtx));
	int rc = -1;
	if (!out->segment_id || !out->skip_coeff || !out->has_coeff || !out->ymode || !out->uv_mode || !out->bmode ||
	    !coeff_ok || !has_y2 || !above_b || !t) {
		errno = ENOMEM;
		goto done;
	}
	if (payload.size < 10u + kf.first_partition_len) {
		errno = EINVAL;
		goto done;
	}

	FrameHdr fh;
	parse_frame_header(payload, &kf, out, &fh);
	Vp8Bool hb = fh.hb;
	const int seg_map_update = fh.seg_map_update, use_skip = fh.use_skip;
	const uint8_t* const seg_probs = fh.seg_probs;
	const uint8_t skip_prob = fh.skip_prob;
	const unsigned nparts = fh.nparts;
	memcpy(t->probs, fh.probs, sizeof(t->probs));

	/* RFC 6386 11 / 19.3 per-macroblock header */
	for (uint32_t r = 0; r < rows; r++) {
		uint8_t left_b[4] = {0, 0, 0, 0};
		for (uint32_t c = 0; c < cols; c++) {
			const uint32_t mb = r * cols + c;
			if (out->segmentation_enabled && seg_map_update)
				out->segment_id[mb] = (uint8_t)vp8b_tree(&hb, k_segment_tree, seg_probs, 0);
			if (use_skip) out->skip_coeff[mb] = (uint8_t)vp8b_read(&hb, skip_prob);
			st->mb_skip_coeff += out->skip_coeff[mb];
			const int ym = vp8b_tree(&hb, k_kf_ymode_tree, k_kf_ymode_prob, 0);
			out->ymode[mb] = (uint8_t)ym;
			st->ymode_counts[ym]++;
			uint8_t* bm = out->bmode + (size_t)mb * 16;
			uint8_t* ab = above_b + (size_t)c * 4;
			if (ym == 4) {
				st->mb_b_pred++;
				for (int i = 0; i < 16; i++) {
					const int y = i >> 2, x = i & 3;
					const uint8_t a = y ? bm[i - 4] : ab[x];
					const uint8_t l = x ? bm[i - 1] : left_b[y];
					bm[i] = (uint8_t)vp8b_tree(&hb, k_bmode_tree, vp8_kf_bmode_prob[a][l], 0);
					st->bmode_counts[bm[i]]++;
				}
				for (int i = 0; i < 4; i++) {
					ab[i] = bm[12 + i];
					left_b[i] = bm[4 * i + 3];
				}
			} else {
				/* implied sub-block context: DC->B_DC, V->B_VE, H->B_HE, TM->B_TM */
				static const uint8_t implied[4] = {0, 2, 3, 1};
				memset(bm, implied[ym], 16);
				memset(ab, implied[ym], 4);
				memset(left_b, implied[ym], 4);
				has_y2[mb] = 1;
			}
			const int uvm = vp8b_tree(&hb, k_uv_mode_tree, k_kf_uv_mode_prob, 0);
			out->uv_mode[mb] = (uint8_t)uvm;
			st->uv_mode_counts[uvm]++;
		}
	}
	st->part0_bytes_used = (uint32_t)vp8b_ref_bytes_used(&hb);
	st->part0_overread_bytes = vp8b_ref_overread_bytes(&hb);
	st->part0_overread = (uint8_t)(st->part0_overread_bytes != 0);

	if (nparts != 1 && !sk->multi) { /* the reference: one token partition (vp8_tokens.c:357-360) */
		errno = ENOTSUP;
		goto done;
	}
	const size_t tok_off = 10u + kf.first_partition_len;
	t->st = st;
	t->hash = 1469598103934665603ull;
	t->nparts = nparts;
	if (nparts == 1) {
		vp8b_init(&t->tok, payload.data + tok_off, payload.size - tok_off);
		st->token_part_size_bytes = (uint32_t)(payload.size - tok_off);
		/* overread iff (shifts >> 3) > size - min(size, 2)  (vp8b_ref_overread_bytes) */
		t->ovr_shift = ((uint64_t)(t->tok.size - vp8b_ref_init_bytes(&t->tok)) + 1u) * 8u;
	} else if (vp8f_partition_table(payload, kf.first_partition_len, nparts, NULL, NULL) != 0) {
		goto done;
	} else {
		/* RFC 6386 9.5: 3-byte little-endian sizes of all but the last partition */
		uint32_t off[8], end[8];
		vp8f_partition_table(payload, kf.first_partition_len, nparts, off, end);
		for (unsigned p = 0; p < nparts; p++) vp8b_init(&t->parts[p], payload.data + off[p], end[p] - off[p]);
		t->tok = t->parts[0];
		st->token_part_size_bytes = (uint32_t)(payload.size - off[0]);
		t->ovr_shift = UINT64_MAX; /* the reference's overread diagnostics are single-partition */
	}
	if (read_all_tokens(t, out, has_y2, sk) != 0) goto done;
	st->coeff_hash_fnv1a64 = sk->hash ? t->hash : 0;
	rc = 0;

done:
	free(has_y2);
	free(above_b);
	free(t);
	if (rc != 0) {
		int e = errno;
		vp8_decoded_frame_free(out);
		if (sk->pk) {
			free(sk->pk->masks);
			free(sk->pk->mb_off);
			free(sk->pk->values);
			sk->pk->masks = NULL, sk->pk->mb_off = NULL, sk->pk->values = NULL, sk->pk->n_values = 0;
		}
		errno = e;
	}
	return rc;
}

int vp8_decode_decoded_frame(ByteSpan payload, Vp8DecodedFrame* out) {
	Sink sk = {NULL, 1, 0, 0};
	return decode_frame(payload, out, &sk);
}

int vp8f_partition_table(ByteSpan payload, uint32_t first_partition_len, unsigned nparts, uint32_t* off, uint32_t* end) {
	size_t o = 10u + (size_t)first_partition_len + 3u * (nparts - 1u);
	if (nparts < 1 || nparts > 8 || o > payload.size) {
		errno = EINVAL;
		return -1;
	}
	const uint8_t* sz = payload.data + 10u + first_partition_len;
	for (unsigned p = 0; p < nparts; p++) {
		const size_t len = p + 1 < nparts ? (size_t)sz[3 * p] | (size_t)sz[3 * p + 1] << 8 | (size_t)sz[3 * p + 2] << 16
		                                  : payload.size - o;
		if (o + len > payload.size) {
			errno = EINVAL;
			return -1;
		}
		if (off) off[p] = (uint32_t)o;
		if (end) end[p] = (uint32_t)(o + len);
		o += len;
	}
	return 0;
}

int vp8f_decode_packed(ByteSpan payload, Vp8gPackedFrame* out, unsigned flags) {
	if (!out) {
		errno = EINVAL;
		return -1;
	}
	memset(out, 0, sizeof(*out));
	Sink sk = {out, (flags & VP8F_PACK_HASH) != 0, 0, (flags & VP8F_MULTI_PARTITION) != 0};
	if (vp8_parse_keyframe_header(payload, &out->kf) != 0) {
		errno = EINVAL;
		return -1;
	}
	return decode_frame(payload, &out->f, &sk);
}

int vp8f_token_header(ByteSpan payload, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* hdr, Vp8gTokFrame* tf, unsigned flags) {
	if (!kf || !hdr || !tf) {
		errno = EINVAL;
		return -1;
	}
	memset(hdr, 0, sizeof(*hdr));
	memset(tf, 0, sizeof(*tf));
	if (vp8_parse_keyframe_header(payload, kf) != 0) {
		errno = EINVAL;
		return -1;
	}
	const uint32_t cols = (kf->width + 15u) >> 4, rows = (kf->height + 15u) >> 4;
	if (cols == 0 || rows == 0 || cols * rows > (1u << 20) || payload.size < 10u + kf->first_partition_len) {
		errno = EINVAL;
		return -1;
	}
	hdr->mb_cols = hdr->stats.mb_cols = cols;
	hdr->mb_rows = hdr->stats.mb_rows = rows;
	hdr->mb_total = hdr->stats.mb_total = cols * rows;
	FrameHdr fh;
	parse_frame_header(payload, kf, hdr, &fh);
	if (fh.nparts != 1 && !(flags & VP8F_MULTI_PARTITION)) { /* the reference: one token partition
	                                                            (vp8_tokens.c:357-360) */
		errno = ENOTSUP;
		return -1;
	}
	if (vp8f_partition_table(payload, kf->first_partition_len, fh.nparts, tf->part_off, tf->part_end) != 0) return -1;
	tf->nparts = fh.nparts;
	tf->mb_cols = cols;
	tf->mb_rows = rows;
	tf->p0_end = 10u + kf->first_partition_len;
	tf->tok_off = tf->part_off[0];
	tf->tok_end = tf->part_end[0];
	tf->b_next = (uint32_t)(fh.hb.next - payload.data);
	tf->b_value = fh.hb.value;
	tf->b_bits = fh.hb.bits;
	tf->b_range = fh.hb.range;
	tf->seg_enabled = hdr->segmentation_enabled;
	tf->seg_map_update = (uint8_t)fh.seg_map_update;
	tf->use_skip = (uint8_t)fh.use_skip;
	tf->skip_prob = fh.skip_prob;
	memcpy(tf->seg_probs, fh.seg_probs, 3);
	for (int i = 0; i < 4; i++)
		for (int j = 0; j < 8; j++)
			for (int k = 0; k < 3; k++) memcpy(tf->coeff_probs[i][j][k], fh.probs[i][j][k], 11);
	return 0;
}

void vp8f_packed_free(Vp8gPackedFrame* p) {
	if (!p) return;
	vp8_decoded_frame_free(&p->f);
	free(p->masks);
	free(p->mb_off);
	free(p->values);
	memset(p, 0, sizeof(*p));
}
