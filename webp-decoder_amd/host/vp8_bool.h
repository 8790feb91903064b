/*
 * vp8_bool.h -- RFC 6386 section 7 boolean entropy decoder (host, C11).
 *
 * Formulation: `value` is a window over the partition bits; the arithmetic-coder comparison
 * is done against its top bits, `(value >> bits) >= split`, where `bits` counts the stream
 * bits already loaded below the 8-bit comparison position.  Bytes past the end of the
 * partition read as zero (same as reference bool_decoder.c:5-15).
 *
 * The reference loads 2 bytes at init and then one byte every time 8 normalisation shifts
 * have accumulated (bool_decoder.c:17-39, :59-68).  The total shift count (vp8b_shifts) is what
 * reproduces its diagnostic counters (bytes used / overread bytes, reported by `decoder -info`)
 * without mimicking its byte-by-byte refill schedule.  It is not kept per bool: bits + shifts
 * grows only by 8 per byte loaded, so shifts = 8 * (bytes loaded, padding included) - 8 - bits.
 */
#ifndef VP8_BOOL_H
#define VP8_BOOL_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

typedef struct Vp8Bool Vp8Bool;

/* Test-only trace hooks (oracle/vp8_repartition.c builds the front end with VP8_BOOL_TRACE to
 * record every decoded (probability, bit) and re-encode streams); no-ops in the product. */
#ifdef VP8_BOOL_TRACE
void vp8_trace_bool(const Vp8Bool* b, uint32_t prob, int bit);
void vp8_trace_mark(int what, uint32_t arg);
#define VP8B_TRACE(b, prob, bit) vp8_trace_bool(b, prob, bit)
#define VP8_TRACE_MARK(what, arg) vp8_trace_mark(what, arg)
#else
#define VP8B_TRACE(b, prob, bit) ((void)0)
#define VP8_TRACE_MARK(what, arg) ((void)0)
#endif

struct Vp8Bool {
	const uint8_t* next; /* next unread byte */
	const uint8_t* end;
	uint64_t value;
	int bits;        /* bits below the comparison window */
	uint32_t range;  /* 128..255 between calls */
	const uint8_t* start; /* first byte of the partition */
	uint64_t pad;         /* zero bytes shifted in past the end */
	size_t size;     /* partition size in bytes */
};

static inline void vp8b_fill(Vp8Bool* b) {
	if (b->bits < 0 && b->end - b->next >= 8) {
		/* 7 bytes at once (big-endian): bits -7..-1 -> 49..55, value stays below 2^64 */
		uint64_t w;
		memcpy(&w, b->next, 8);
		b->value = (b->value << 56) | (__builtin_bswap64(w) >> 8);
		b->bits += 56;
		b->next += 7;
		return;
	}
	while (b->bits <= 48) {
		uint64_t byte = 0;
		if (b->next < b->end) byte = *b->next++;
		else b->pad++; /* past the end: shift in zeros (the coder's defined padding) */
		b->value = (b->value << 8) | byte;
		b->bits += 8;
	}
}

static inline void vp8b_init(Vp8Bool* b, const uint8_t* data, size_t size) {
	b->next = data;
	b->end = data + size;
	b->value = 0;
	b->bits = -8;
	b->range = 255;
	b->start = data;
	b->pad = 0;
	b->size = size;
	vp8b_fill(b);
}

static inline int vp8b_read(Vp8Bool* b, uint32_t prob) {
	uint32_t split = 1u + (((b->range - 1u) * prob) >> 8);
	int bit;
	if ((uint32_t)(b->value >> b->bits) >= split) {
		b->value -= (uint64_t)split << b->bits;
		b->range -= split;
		bit = 1;
	} else {
		b->range = split;
		bit = 0;
	}
	/* normalise: range back into [128, 255] */
	int sh = __builtin_clz(b->range) - 24;
	b->range <<= sh;
	b->bits -= sh;
	if (b->bits < 0) vp8b_fill(b);
	VP8B_TRACE(b, prob, bit);
	return bit;
}

/* One bool used as data, not as control (category extra bits, the odd bit of a 3/4 or of a
 * category index): the same update as vp8b_read with selects instead of a branch. */
static inline int vp8b_read_bit(Vp8Bool* b, uint32_t prob) {
	const uint32_t split = 1u + (((b->range - 1u) * prob) >> 8);
	const uint64_t big = (uint64_t)split << b->bits;
	const int bit = b->value >= big;
	const uint64_t m = 0u - (uint64_t)bit;
	b->value -= big & m;
	const uint32_t range = ((b->range - split) & (uint32_t)m) | (split & ~(uint32_t)m);
	const int sh = __builtin_clz(range) - 24;
	b->range = range << sh;
	b->bits -= sh;
	if (b->bits < 0) vp8b_fill(b);
	VP8B_TRACE(b, prob, bit);
	return bit;
}

/* v or -v by one bool at probability 1/2 (a coefficient's sign: as likely one way as the other, so
 * it is applied arithmetically rather than branched on) */
static inline int vp8b_apply_sign(Vp8Bool* b, int v) {
	const uint32_t split = 1u + ((b->range - 1u) >> 1);
	const uint64_t big = (uint64_t)split << b->bits;
	const int neg = b->value >= big;
	const uint64_t m = 0u - (uint64_t)neg;
	b->value -= big & m;
	const uint32_t range = ((b->range - split) & (uint32_t)m) | (split & ~(uint32_t)m);
	const int sh = __builtin_clz(range) - 24;
	b->range = range << sh;
	b->bits -= sh;
	if (b->bits < 0) vp8b_fill(b);
	VP8B_TRACE(b, 128, neg);
	return (v ^ -neg) + neg;
}

static inline uint32_t vp8b_literal(Vp8Bool* b, int n) {
	uint32_t v = 0;
	while (n-- > 0) v = (v << 1) | (uint32_t)vp8b_read(b, 128);
	return v;
}

/* magnitude then sign (RFC 6386 9.3 / 9.6 signed fields) */
static inline int32_t vp8b_signed(Vp8Bool* b, int n) {
	int32_t m = (int32_t)vp8b_literal(b, n);
	if (m == 0) return 0;
	return vp8b_read(b, 128) ? -m : m;
}

/* Tree decode: tree[] holds pairs of (left, right); entries <= 0 are leaves (-symbol). */
static inline int vp8b_tree(Vp8Bool* b, const int8_t* tree, const uint8_t* probs, int node) {
	for (;;) {
		int next = tree[node + vp8b_read(b, probs[node >> 1])];
		if (next <= 0) return -next;
		node = next;
	}
}

/* ---- reference-compatible diagnostics (see header comment) ---- */
/* total normalisation shifts so far (see the header comment) */
static inline uint64_t vp8b_shifts(const Vp8Bool* b) {
	return 8u * ((uint64_t)(b->next - b->start) + b->pad) - 8u - (uint64_t)(int64_t)b->bits;
}
static inline uint64_t vp8b_ref_loads(const Vp8Bool* b) { return vp8b_shifts(b) >> 3; }
static inline size_t vp8b_ref_init_bytes(const Vp8Bool* b) { return b->size < 2 ? b->size : 2; }
static inline uint32_t vp8b_ref_overread_bytes(const Vp8Bool* b) {
	uint64_t avail = b->size - vp8b_ref_init_bytes(b);
	uint64_t loads = vp8b_ref_loads(b);
	return loads > avail ? (uint32_t)(loads - avail) : 0u;
}
static inline size_t vp8b_ref_bytes_used(const Vp8Bool* b) {
	uint64_t used = vp8b_ref_init_bytes(b) + vp8b_ref_loads(b);
	return used > b->size ? b->size : (size_t)used;
}

#endif
