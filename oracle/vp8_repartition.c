/*
 * vp8_repartition.c -- TEST INFRASTRUCTURE (fixture generator for SURVEY §8(f4)); never linked
 * into the product.
 *
 * Re-encodes a single-partition VP8 key frame (.webp, simple lossy) with its coefficient tokens
 * split over 2^log2k token partitions (RFC 6386 9.5: MB row r goes to partition r mod k), so that
 * the multi-partition decode paths can be checked against the original frame's known output.
 * The reference decoder rejects such streams (vp8_tokens.c:357-360, ENOTSUP) and the reference
 * corpus holds none (parity unpinned), hence the generator.
 *
 * How: the host front end is built with VP8_BOOL_TRACE (webp-decoder_amd/host/vp8_bool.h), which
 * reports every decoded (probability, bit) and the MB row of each token bool.  The generator
 * decodes the original frame, then feeds the same decisions to an RFC 6386 7.3 boolean encoder:
 * partition 0 unchanged except the 2-bit log2(nparts) field, the token bools distributed by row.
 * Decoding the result yields exactly the original syntax elements, hence the original pixels.
 * Not thread-safe (one global trace).
 */
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../webp-decoder_amd/host/vp8_bool.h"
#include "../webp-decoder_amd/host/vp8_front.h"

typedef struct {
	uint8_t prob, bit;
	uint32_t row;
} Decision;

typedef struct {
	Decision* v;
	size_t n, cap;
} Trace;

static Trace g_p0, g_tok;
static const uint8_t* g_p0_end;
static size_t g_nparts_at = (size_t)-1;
static uint32_t g_row;
static int g_oom;

static void push(Trace* t, uint32_t prob, int bit, uint32_t row) {
	if (t->n == t->cap) {
		size_t nc = t->cap ? 2 * t->cap : 4096;
		Decision* nv = (Decision*)realloc(t->v, nc * sizeof(Decision));
		if (!nv) {
			g_oom = 1;
			return;
		}
		t->v = nv, t->cap = nc;
	}
	t->v[t->n++] = (Decision){(uint8_t)prob, (uint8_t)bit, row};
}

void vp8_trace_bool(const Vp8Bool* b, uint32_t prob, int bit) {
	if (b->end == g_p0_end) push(&g_p0, prob, bit, 0);
	else push(&g_tok, prob, bit, g_row);
}

void vp8_trace_mark(int what, uint32_t arg) {
	if (what == 1) g_nparts_at = g_p0.n;
	else if (what == 2) g_row = arg;
}

/* ---- RFC 6386 7.3 boolean encoder ---------------------------------------------------------- */
typedef struct {
	uint8_t* buf;
	size_t n, cap;
	uint32_t range, low; /* low: the bottom of the interval, 24 pending bits + carry position */
	int shifts_left;     /* normalisation shifts until the next byte leaves `low` */
	int oom;
} BoolEnc;

static void enc_init(BoolEnc* e) {
	memset(e, 0, sizeof(*e));
	e->range = 255;
	e->shifts_left = 24;
}

static void enc_byte(BoolEnc* e, uint8_t v) {
	if (e->n == e->cap) {
		size_t nc = e->cap ? 2 * e->cap : 4096;
		uint8_t* nb = (uint8_t*)realloc(e->buf, nc);
		if (!nb) {
			e->oom = 1;
			return;
		}
		e->buf = nb, e->cap = nc;
	}
	e->buf[e->n++] = v;
}

/* a carry out of `low` ripples into the bytes already written */
static void enc_carry(BoolEnc* e) {
	size_t i = e->n;
	while (i > 0 && e->buf[i - 1] == 0xFF) e->buf[--i] = 0;
	if (i > 0) e->buf[i - 1]++;
}

static void enc_bool(BoolEnc* e, uint32_t prob, int bit) {
	const uint32_t split = 1u + (((e->range - 1u) * prob) >> 8);
	if (bit) {
		e->low += split;
		e->range -= split;
	} else {
		e->range = split;
	}
	while (e->range < 128u) {
		e->range <<= 1;
		if (e->low & 0x80000000u) enc_carry(e);
		e->low <<= 1;
		if (--e->shifts_left == 0) {
			enc_byte(e, (uint8_t)(e->low >> 24));
			e->low &= 0xFFFFFFu;
			e->shifts_left = 8;
		}
	}
}

static void enc_finish(BoolEnc* e) {
	uint32_t v = e->low;
	int c = e->shifts_left;
	if (v & (1u << (32 - c))) enc_carry(e);
	v <<= c & 7;
	for (c >>= 3; c > 0; c--) v <<= 8;
	for (int i = 0; i < 4; i++, v <<= 8) enc_byte(e, (uint8_t)(v >> 24));
}

static void put_le(uint8_t* p, uint32_t v, int n) {
	for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * i));
}

/* Writes the re-partitioned .webp into out (cap bytes).  Returns its size, or -1 + errno
 * (EINVAL: not a single-partition key frame / log2k out of 0..3; ENOSPC: cap too small). */
long vp8_repartition(const uint8_t* webp, size_t size, int log2k, uint8_t* out, size_t cap) {
	if (!webp || !out || log2k < 0 || log2k > 3) {
		errno = EINVAL;
		return -1;
	}
	WebPContainer c;
	if (webp_parse_simple_lossy((ByteSpan){webp, size}, &c) != 0) return -1;
	const uint8_t* pl = webp + c.vp8_chunk_offset;
	Vp8KeyFrameHeader kf;
	if (vp8_parse_keyframe_header((ByteSpan){pl, c.vp8_chunk_size}, &kf) != 0 || !kf.is_key_frame) {
		errno = EINVAL;
		return -1;
	}
	g_p0.n = g_tok.n = 0;
	g_nparts_at = (size_t)-1;
	g_row = 0;
	g_oom = 0;
	g_p0_end = pl + 10 + kf.first_partition_len;
	Vp8DecodedFrame f;
	const int rc = vp8_decode_decoded_frame((ByteSpan){pl, c.vp8_chunk_size}, &f);
	if (rc != 0) return -1;
	vp8_decoded_frame_free(&f);
	if (g_oom || g_nparts_at + 2 > g_p0.n || g_p0.v[g_nparts_at].bit || g_p0.v[g_nparts_at + 1].bit) {
		errno = EINVAL;
		return -1;
	}
	const uint32_t k = 1u << log2k;
	BoolEnc p0, parts[8];
	enc_init(&p0);
	for (size_t i = 0; i < g_p0.n; i++) {
		int bit = g_p0.v[i].bit;
		if (i == g_nparts_at) bit = (log2k >> 1) & 1; /* log2(nparts), most significant bit first */
		if (i == g_nparts_at + 1) bit = log2k & 1;
		enc_bool(&p0, g_p0.v[i].prob, bit);
	}
	enc_finish(&p0);
	for (uint32_t p = 0; p < k; p++) enc_init(&parts[p]);
	for (size_t i = 0; i < g_tok.n; i++) enc_bool(&parts[g_tok.v[i].row % k], g_tok.v[i].prob, g_tok.v[i].bit);
	size_t payload = 10 + p0.n + 3 * (k - 1);
	int oom = p0.oom;
	for (uint32_t p = 0; p < k; p++) {
		enc_finish(&parts[p]);
		payload += parts[p].n;
		oom |= parts[p].oom;
	}
	long total = -1;
	if (oom || p0.n >= (1u << 19)) {
		errno = oom ? ENOMEM : EINVAL;
	} else if (20 + payload + (payload & 1) > cap) {
		errno = ENOSPC;
	} else {
		uint8_t* o = out;
		memcpy(o, "RIFF", 4);
		put_le(o + 4, (uint32_t)(12 + payload + (payload & 1)), 4);
		memcpy(o + 8, "WEBPVP8 ", 8);
		put_le(o + 16, (uint32_t)payload, 4);
		uint8_t* v = o + 20;
		const uint32_t tag = (uint32_t)pl[0] | (uint32_t)pl[1] << 8 | (uint32_t)pl[2] << 16;
		put_le(v, (tag & 0x1Fu) | (uint32_t)p0.n << 5, 3); /* key frame, version, show, new size */
		memcpy(v + 3, pl + 3, 7);                           /* start code, dimensions, scaling */
		memcpy(v + 10, p0.buf, p0.n);
		uint8_t* q = v + 10 + p0.n;
		for (uint32_t p = 0; p + 1 < k; p++, q += 3) put_le(q, (uint32_t)parts[p].n, 3);
		for (uint32_t p = 0; p < k; p++) {
			memcpy(q, parts[p].buf, parts[p].n);
			q += parts[p].n;
		}
		if (payload & 1) *q = 0;
		total = (long)(20 + payload + (payload & 1));
	}
	free(p0.buf);
	for (uint32_t p = 0; p < k; p++) free(parts[p].buf);
	return total;
}
