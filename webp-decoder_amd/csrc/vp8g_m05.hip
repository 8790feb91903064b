// vp8g_m05.hip -- m05 on the device: per-macroblock modes and coefficient
// tokens of a batch of key frames, one workgroup per frame.
//
// VP8's arithmetic-coded partitions are serial chains (each bool's range depends on the previous
// one): partition 0 (modes) and one token partition per 1, 2, 4 or 8 (RFC 6386 9.5; the
// reference supports one).  Inside a chain there is no parallelism, so a frame gets one wave per
// chain -- a modes wave and a token wave per partition, coupled through LDS (see "Per-frame
// workgroup" below) -- and the chip is filled with frames.  Every value on a chain is the same in
// all lanes, so the decoder state lives in scalar registers and the bool decoder runs on the
// scalar ALU.  The chains are latency-bound, so nothing on them waits for memory: the probability
// tables and a window of each partition sit in VGPR lanes and are read with v_readlane (see
// "register tables" below).
//
// Semantics are those of the host front end (host/vp8_parse.c, itself pinned to the reference m05:
// src/m05_tokens/vp8_tokens.c:275-352, :354-622, :868-926): de-zigzagged coefficients, explicit
// zeros for skipped / Y2-less blocks (the caller zeroes the coefficient arrays; only non-zero
// values are stored), has_coeff = any non-zero value in the MB, implied sub-block modes for
// non-B_PRED MBs.  The host parses the frame header and the first partition's frame-level fields
// (vp8f_token_header) and hands over the partition-0 bool decoder at the first MB header.  Not
// computed here: the reference's diagnostic statistics (hash, counters, overread position).
#include <errno.h>

#include "vp8g_device.h"

#define VP8_TABLE static constexpr
#include "../host/vp8_tables.inc"
#undef VP8_TABLE

#define VP8G_API extern "C" __attribute__((visibility("default")))
#define DEV __device__ __forceinline__

namespace {

// RFC 6386 13.3: band of each coefficient position and the zigzag scan, 4 bits per position
constexpr uint8_t kBandArr[16] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7};
constexpr uint8_t kScanArr[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr uint64_t pack_nibbles(const uint8_t* a) {
	uint64_t v = 0;
	for (int i = 0; i < 16; i++) v |= (uint64_t)a[i] << (4 * i);
	return v;
}
constexpr uint64_t kBand4 = pack_nibbles(kBandArr), kScan4 = pack_nibbles(kScanArr);
DEV uint32_t nib(uint64_t v, uint32_t i) { return (uint32_t)(v >> (4u * i)) & 15u; }

// RFC 6386 11.5 key-frame sub-block mode probabilities, one 12-byte row (3 dwords) per (above, left)
struct BmodeProbs {
	uint32_t w[100][3];
};
constexpr BmodeProbs make_bmode_probs() {
	BmodeProbs t{};
	for (int a = 0; a < 10; a++)
		for (int l = 0; l < 10; l++)
			for (int k = 0; k < 9; k++) t.w[a * 10 + l][k / 4] |= (uint32_t)vp8_kf_bmode_prob[a][l][k] << (8 * (k % 4));
	return t;
}
__constant__ BmodeProbs kBmodeProbs = make_bmode_probs();

// a row of up to 12 probabilities held as 3 dwords; pb(r, k) with a constant k
struct Row {
	uint32_t w0, w1, w2;
};
DEV uint32_t pb(const Row& r, int k) { return ((k < 4 ? r.w0 : (k < 8 ? r.w1 : r.w2)) >> (8 * (k & 3))) & 255u; }

enum { PLANE_Y_AFTER_Y2 = 0, PLANE_Y2 = 1, PLANE_UV = 2, PLANE_Y_ALONE = 3 };

struct Out {
	int16_t *cy, *cu, *cv, *cy2;
	uint8_t *ymode, *uvmode, *seg, *hasc, *bmode;
	uint32_t* status;  // VP8G_ERR_TIMEOUT if a ring wait gives up (never expected; keeps the grid finite)
};

// Register tables.  Every memory access on the serial chain is pure latency (a scalar-cache round
// trip per token would dominate), so the tables consulted per token / per sub-block mode and the
// bitstream itself are held in VGPR lanes -- loaded once per frame, or one window ahead -- and
// read with v_readlane (lane index in an SGPR), a few cycles.
DEV uint32_t lane() { return threadIdx.x & 63u; }
DEV uint32_t rl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }

// RFC 6386 7 bool decoder in the host's formulation (host/vp8_bool.h): `value` holds the stream
// bits, compared at `bits`.  Refilled 32 bits at a time from a 512-byte window of the partition
// (two VGPRs of 64 big-endian dwords: `cur` at byte `base`, `nxt` after it, loaded one window
// ahead); bytes at or past `end` read as zero (the coder's padding), as in the host's byte-wise
// refill, so the compared values are identical.
struct DBool {
	uint64_t value;
	int bits;
	uint32_t range;  // range - 1 (saves the two +-1 of the split on the chain)
	uint32_t next, end;
	uint32_t base;       // window start (4-aligned)
	uint32_t cur, nxt;   // per lane: dword base/4 + lane, big-endian (cur); + 64, as loaded (nxt)
};

// The payload starts 4-B aligned in the bitstream buffer with >= 512 readable bytes after its end
// (a window is loaded only while the read position is inside the partition), so the loads need no
// guard (no exec-mask change on the chain); bytes past the end are masked in dfill.
DEV uint32_t win_load(const uint8_t* pl, uint32_t at) { return *(const uint32_t*)(pl + at + 4u * lane()); }

DEV void dinit(DBool& b, const uint8_t* pl, uint64_t value, int bits, uint32_t range, uint32_t next, uint32_t end) {
	b.value = value, b.bits = bits, b.range = range - 1u, b.next = next, b.end = end;
	b.base = next & ~3u;
	b.cur = __builtin_bswap32(win_load(pl, b.base));
	b.nxt = win_load(pl, b.base + 256u);
}

DEV void dfill(DBool& b, const uint8_t* pl) {
	const uint32_t pos = b.next;
	uint32_t v = 0;
	if (pos < b.end) {
		if (pos - b.base >= 256u) {  // slide the window (pos advances 4 bytes per refill)
			b.cur = __builtin_bswap32(b.nxt);  // byte swap only now: the load has long landed
			b.base += 256u;
			b.nxt = win_load(pl, b.base + 256u);
		}
		const uint32_t idx = (pos - b.base) >> 2, s = (pos & 3u) * 8u;
		const uint32_t hi = rl(b.cur, idx);
		const uint32_t lo = idx < 63u ? rl(b.cur, idx + 1u) : __builtin_bswap32(rl(b.nxt, 0));
		v = (uint32_t)(((((uint64_t)hi) << 32) | lo) >> (32u - s));
		const uint32_t n = b.end - pos;
		if (n < 4u) v &= 0xFFFFFFFFu << (32u - 8u * n);
	}
	b.value = (b.value << 32) | v;
	b.bits += 32;
	b.next = pos + 4u;
}

DEV uint32_t dread(DBool& b, const uint8_t* pl, uint32_t prob) {
	const uint32_t split = (b.range * prob) >> 8;  // RFC 6386 7.3 split - 1
	uint32_t bit, r;
	if ((uint32_t)(b.value >> b.bits) > split) {  // 64-bit shift + 32-bit compare: both scalar
		b.value -= (uint64_t)(split + 1u) << b.bits;
		r = b.range - split;  // new range (not minus 1)
		bit = 1u;
	} else {
		r = split + 1u;
		bit = 0u;
	}
	const int sh = __builtin_clz(r) - 24;
	b.range = (r << sh) - 1u;
	b.bits -= sh;
	if (b.bits < 0) dfill(b, pl);
	return bit;
}

// RFC 6386 11.2 / 9.3 trees as straight code (host: k_kf_ymode_tree, k_uv_mode_tree,
// k_bmode_tree, k_segment_tree)
DEV uint32_t read_ymode(DBool& b, const uint8_t* pl) {  // probs {145, 156, 163, 128}
	if (!dread(b, pl, 145)) return 4;                      // B_PRED
	if (!dread(b, pl, 156)) return dread(b, pl, 163);      // DC / V
	return 2u + dread(b, pl, 128);                         // H / TM
}
DEV uint32_t read_uvmode(DBool& b, const uint8_t* pl) {  // probs {142, 114, 183}
	if (!dread(b, pl, 142)) return 0;
	if (!dread(b, pl, 114)) return 1;
	return 2u + dread(b, pl, 183);
}
DEV uint32_t read_bmode(DBool& b, const uint8_t* pl, const Row& p) {
	if (!dread(b, pl, pb(p, 0))) return 0;  // B_DC
	if (!dread(b, pl, pb(p, 1))) return 1;  // B_TM
	if (!dread(b, pl, pb(p, 2))) return 2;  // B_VE
	if (!dread(b, pl, pb(p, 3))) {
		if (!dread(b, pl, pb(p, 4))) return 3;  // B_HE
		return dread(b, pl, pb(p, 5)) ? 6 : 5;  // B_VR : B_RD
	}
	if (!dread(b, pl, pb(p, 6))) return 4;  // B_LD
	if (!dread(b, pl, pb(p, 7))) return 7;  // B_VL
	return dread(b, pl, pb(p, 8)) ? 9 : 8;  // B_HU : B_HD
}
DEV uint32_t read_segment(DBool& b, const uint8_t* pl, uint32_t probs) {  // tree {2, 4, -0, -1, -2, -3}
	if (!dread(b, pl, probs & 255u)) return dread(b, pl, (probs >> 8) & 255u);
	return 2u + dread(b, pl, (probs >> 16) & 255u);
}

// DCT_CAT1..6 magnitude: base + extra bits (RFC 6386 13.2), probabilities as immediates
template <int N>
DEV uint32_t read_bits(DBool& b, const uint8_t* pl, const uint8_t (&p)[N]) {
	uint32_t e = 0;
#pragma unroll
	for (int i = 0; i < N; i++) e = 2u * e + dread(b, pl, p[i]);
	return e;
}
DEV uint32_t read_cat(DBool& b, const uint8_t* pl, uint32_t cat) {
	constexpr uint8_t p1[1] = {159}, p2[2] = {165, 145}, p3[3] = {173, 148, 140}, p4[4] = {176, 155, 140, 135};
	constexpr uint8_t p5[5] = {180, 157, 141, 134, 130};
	constexpr uint8_t p6[11] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129};
	switch (cat) {
		case 0: return 5u + read_bits(b, pl, p1);
		case 1: return 7u + read_bits(b, pl, p2);
		case 2: return 11u + read_bits(b, pl, p3);
		case 3: return 19u + read_bits(b, pl, p4);
		case 4: return 35u + read_bits(b, pl, p5);
		default: return 67u + read_bits(b, pl, p6);
	}
}

// Coefficient probabilities of one block type in lanes: `va` lane 2r + h = dword h (0, 1) of row r
// (r = band * 3 + ctx, 24 rows), `vb` lane r + vo = dword 2.
struct TypeTab {
	uint32_t va, vb, vo;
};

// One 4x4 block's tokens (RFC 6386 13; host/vp8_parse.c read_block): the non-zero values go to
// dst[natural position]; returns whether any value is non-zero.  Every lane stores the same value
// to the same address (no exec-mask juggling on the serial path).
DEV bool read_block(DBool& b, const uint8_t* pl, const TypeTab& t, uint32_t first, uint32_t ctx, int16_t* dst) {
	bool nz = false;
	uint32_t pos = first;
	uint32_t ri = nib(kBand4, pos) * 3u + ctx;
	bool skip_eob = false;
	while (true) {
		const uint32_t w0 = rl(t.va, 2u * ri);
		if (!skip_eob && !dread(b, pl, w0 & 255u)) break;  // EOB
		if (!dread(b, pl, (w0 >> 8) & 255u)) {                 // DCT_0: the next token has no EOB branch
			if (++pos == 16u) break;
			ri = nib(kBand4, pos) * 3u;
			skip_eob = true;
			continue;
		}
		uint32_t mag;
		if (!dread(b, pl, (w0 >> 16) & 255u)) {
			mag = 1u;
		} else {
			const uint32_t w1 = rl(t.va, 2u * ri + 1u);
			if (!dread(b, pl, w0 >> 24)) {
				mag = dread(b, pl, w1 & 255u) ? 3u + dread(b, pl, (w1 >> 8) & 255u) : 2u;
			} else {
				uint32_t cat;
				if (!dread(b, pl, (w1 >> 16) & 255u)) {
					cat = dread(b, pl, w1 >> 24);
				} else {
					const uint32_t w2 = rl(t.vb, ri + t.vo);
					if (!dread(b, pl, w2 & 255u)) cat = 2u + dread(b, pl, (w2 >> 8) & 255u);
					else cat = 4u + dread(b, pl, (w2 >> 16) & 255u);
				}
				mag = read_cat(b, pl, cat);
			}
		}
		const uint32_t neg = dread(b, pl, 128);
		dst[nib(kScan4, pos)] = (int16_t)(neg ? -(int)mag : (int)mag);
		nz = true;
		if (++pos == 16u) break;
		ri = nib(kBand4, pos) * 3u + (mag == 1u ? 1u : 2u);
		skip_eob = false;
	}
	return nz;
}

// Per-frame workgroup: one wave per arithmetic-coded chain (the chains are independent).
//   wave 0 ("modes") decodes partition 0 -- segment, skip flag, luma / chroma / sub-block modes --
//          and writes the mode arrays and, per MB, a flag byte (skip, has Y2) into an LDS ring;
//   waves 1..n ("tokens", one per token partition, RFC 6386 9.5) decode MB rows r = w, w + n, ...
//          from partition w as the ring fills.  With n > 1 the token waves form a row wavefront:
//          MB (r, c) needs the above contexts row r - 1 leaves at column c.
// Taking the modes off the token chain and splitting the tokens by rows shortens the frame's
// critical path; a single-partition frame has one token wave.
// Protocol (LDS only, one writer per word): the modes wave writes ring[m] and then prod = m + 1;
// token wave w publishes done[w] = index + 1 of the last MB it finished (all MBs once it runs
// out of rows).  A token wave waits for prod > m and for done[wave of row r - 1] past column c;
// the modes wave stays less than kRing MBs ahead of min(done).  LDS operations of a wave complete
// in order, so volatile accesses (no compiler reordering) suffice; s_sleep while waiting; waits
// are bounded (VP8G_ERR_TIMEOUT) so a broken stream cannot keep the grid alive.
constexpr uint32_t kRing = 8192;          // >= 8 MB rows of a 1024-MB-wide frame in flight
constexpr uint32_t kMaxParts = 8;
constexpr uint32_t kMaxPolls = 1u << 24;  // a few seconds of s_sleep
constexpr uint32_t kCtlWords = 1u + kMaxParts;
// LDS pointers typed as such: a volatile generic pointer would become flat accesses, whose
// completion the compiler tracks with vmcnt (so every poll would also wait for the wave's stores)
typedef __attribute__((address_space(3))) volatile uint32_t lds_u32;
typedef __attribute__((address_space(3))) volatile uint8_t lds_u8;

DEV void timeout(const Out& o) {
	if (lane() == 0) atomicOr(o.status, VP8G_ERR_TIMEOUT);
}

DEV void modes_wave(const Vp8gTokFrame& J, const uint8_t* pl, Out o, lds_u32* ctl, lds_u8* ring, lds_u32* above_b,
                    uint32_t nparts) {
	const uint32_t L = lane(), cols = J.mb_cols, rows = J.mb_rows;
	uint32_t bl[3], bh[3];  // sub-block mode rows 0..63 / 64..99 in lanes
#pragma unroll
	for (int x = 0; x < 3; x++) {
		bl[x] = kBmodeProbs.w[L][x];
		bh[x] = L < 36u ? kBmodeProbs.w[64u + L][x] : 0u;
	}
	const uint32_t flags = *(const uint32_t*)&J.seg_enabled;  // seg_enabled | seg_map_update | use_skip | skip_prob
	const bool seg_map = (flags & 0xFFu) && ((flags >> 8) & 0xFFu);
	const bool use_skip = (flags >> 16) & 0xFFu;
	const uint32_t skip_prob = flags >> 24;
	const uint32_t seg_probs = *(const uint32_t*)J.seg_probs;
	DBool hb;
	dinit(hb, pl, J.b_value, J.b_bits, J.b_range, J.b_next, J.p0_end);
	uint32_t m = 0, cons = 0, maxp = kMaxPolls;
	for (uint32_t r = 0; r < rows; r++) {
		uint32_t left_b = 0;  // right column's sub-block modes, 4 nibbles
		for (uint32_t c = 0; c < cols; c++, m++) {
			for (uint32_t polls = 0; m - cons >= kRing; polls++) {
				if (polls >= maxp) {  // sticky: after one timeout the wave never waits again
					if (maxp) timeout(o);
					maxp = 0;
					break;
				}
				__builtin_amdgcn_s_sleep(2);
				uint32_t lo = 0xFFFFFFFFu;
				for (uint32_t w = 0; w < nparts; w++) lo = min(lo, (uint32_t)__builtin_amdgcn_readfirstlane(ctl[1 + w]));
				cons = lo;
			}
			const uint64_t mb = J.mb_offset + m;
			const uint32_t ab = __builtin_amdgcn_readfirstlane(above_b[c]);
			const uint32_t seg = seg_map ? read_segment(hb, pl, seg_probs) : 0u;
			const uint32_t skip = use_skip ? dread(hb, pl, skip_prob) : 0u;
			const uint32_t ym = read_ymode(hb, pl);
			uint64_t bm;  // the MB's 16 sub-block modes, 4 bits each, raster order
			if (ym == 4u) {
				bm = 0;
				for (uint32_t i = 0; i < 16u; i++) {
					const uint32_t y = i >> 2, x = i & 3u;
					const uint32_t a = y ? nib(bm, i - 4u) : (ab >> (4u * x)) & 15u;
					const uint32_t l = x ? nib(bm, i - 1u) : (left_b >> (4u * y)) & 15u;
					const uint32_t ri = a * 10u + l;
					const Row p = ri < 64u ? Row{rl(bl[0], ri), rl(bl[1], ri), rl(bl[2], ri)}
					                       : Row{rl(bh[0], ri - 64u), rl(bh[1], ri - 64u), rl(bh[2], ri - 64u)};
					bm |= (uint64_t)read_bmode(hb, pl, p) << (4u * i);
				}
			} else {
				// implied sub-block context: DC->B_DC, V->B_VE, H->B_HE, TM->B_TM
				const uint32_t im = (0x1320u >> (4u * ym)) & 15u;
				bm = (uint64_t)im * 0x1111111111111111ull;
			}
			left_b = 0;
			for (uint32_t y = 0; y < 4u; y++) left_b |= nib(bm, 4u * y + 3u) << (4u * y);
			const uint32_t uvm = read_uvmode(hb, pl);
			if (L == 0) {
				above_b[c] = (uint32_t)(bm >> 48) & 0xFFFFu;
				ring[m & (kRing - 1u)] = (uint8_t)(skip | (ym != 4u ? 2u : 0u));
				ctl[0] = m + 1u;
			}
			o.seg[mb] = (uint8_t)seg;
			o.ymode[mb] = (uint8_t)ym;
			o.uvmode[mb] = (uint8_t)uvm;
			uint32_t bw[4];
			for (int i = 0; i < 4; i++) {
				const uint32_t q = (uint32_t)(bm >> (16 * i));
				bw[i] = (q & 15u) | ((q >> 4) & 15u) << 8 | ((q >> 8) & 15u) << 16 | ((q >> 12) & 15u) << 24;
			}
			if (L == 0) *(uint4*)(o.bmode + mb * 16u) = make_uint4(bw[0], bw[1], bw[2], bw[3]);
		}
	}
}

DEV void tokens_wave(const Vp8gTokFrame& J, const uint8_t* pl, Out o, lds_u32* ctl, lds_u8* ring, lds_u32* above,
                     uint32_t w, uint32_t nparts) {
	const uint32_t L = lane(), cols = J.mb_cols, rows = J.mb_rows;
	// coefficient rows of the 4 block types in lanes (TypeTab)
	const uint32_t* const cp = (const uint32_t*)J.coeff_probs;  // [4][24] rows of 3 dwords
	uint32_t va[4];
#pragma unroll
	for (int t = 0; t < 4; t++) va[t] = L < 48u ? cp[t * 72 + (L >> 1) * 3 + (L & 1u)] : 0u;
	uint32_t vb[2];
#pragma unroll
	for (int k = 0; k < 2; k++) vb[k] = (L & 31u) < 24u ? cp[(2 * k + (L >> 5)) * 72 + (L & 31u) * 3 + 2] : 0u;
	const TypeTab tt_y{va[PLANE_Y_AFTER_Y2], vb[0], 0}, tt_y2{va[PLANE_Y2], vb[0], 32}, tt_uv{va[PLANE_UV], vb[1], 0},
	    tt_yalone{va[PLANE_Y_ALONE], vb[1], 32};
	DBool tb;
	dinit(tb, pl, 0, -8, 255u, J.part_off[w], J.part_end[w]);
	dfill(tb, pl);
	const uint32_t prev = (w + nparts - 1u) % nparts;  // the wave of row r - 1
	uint32_t prod = 0, up = 0, maxp = kMaxPolls;
	for (uint32_t r = w; r < rows; r += nparts) {
		uint32_t left = 0;  // token contexts, bits as in above[]
		for (uint32_t c = 0; c < cols; c++) {
			const uint32_t m = r * cols + c;
			for (uint32_t polls = 0; m >= prod; polls++) {
				if (polls >= maxp) {
					if (maxp) timeout(o);
					maxp = 0;
					prod = m + 1u;
					break;
				}
				prod = __builtin_amdgcn_readfirstlane(ctl[0]);
				if (m >= prod) __builtin_amdgcn_s_sleep(1);
			}
			if (nparts > 1 && r > 0) {  // row wavefront: MB (r - 1, c) done
				for (uint32_t polls = 0; up < m - cols + 1u; polls++) {
					if (polls >= maxp) {
						if (maxp) timeout(o);
						maxp = 0;
						up = m;
						break;
					}
					up = __builtin_amdgcn_readfirstlane(ctl[1 + prev]);
					if (up < m - cols + 1u) __builtin_amdgcn_s_sleep(1);
				}
			}
			const uint32_t fl = __builtin_amdgcn_readfirstlane(ring[m & (kRing - 1u)]);
			const uint64_t mb = J.mb_offset + m;
			uint32_t ab = __builtin_amdgcn_readfirstlane(above[c]);
			const bool has_y2 = (fl & 2u) != 0;
			bool any = false;
			if (fl & 1u) {
				// no tokens: the contexts of the MB's blocks become 0; Y2's only if the MB has one
				const uint32_t clr = has_y2 ? 0x1FFu : 0xFFu;
				left &= ~clr;
				ab &= ~clr;
			} else {
				auto blk = [&](const TypeTab& tt, uint32_t first, uint32_t li, uint32_t ai, int16_t* dst) {
					const uint32_t ctx = ((left >> li) & 1u) + ((ab >> ai) & 1u);
					const bool nz = read_block(tb, pl, tt, first, ctx, dst);
					any |= nz;
					left = (left & ~(1u << li)) | ((uint32_t)nz << li);
					ab = (ab & ~(1u << ai)) | ((uint32_t)nz << ai);
				};
				if (has_y2) blk(tt_y2, 0, 8, 8, o.cy2 + mb * 16u);
				if (has_y2) {  // two loops: the table and the first position are constants in each
					for (uint32_t k = 0; k < 16u; k++) blk(tt_y, 1u, k >> 2, k & 3u, o.cy + (mb * 16u + k) * 16u);
				} else {
					for (uint32_t k = 0; k < 16u; k++) blk(tt_yalone, 0u, k >> 2, k & 3u, o.cy + (mb * 16u + k) * 16u);
				}
				for (uint32_t j = 0; j < 8u; j++) {
					const uint32_t p = j >> 2, jj = j & 3u;
					blk(tt_uv, 0, 4u + 2u * p + (jj >> 1), 4u + 2u * p + (jj & 1u), (p ? o.cv : o.cu) + (mb * 4u + jj) * 16u);
				}
			}
			if (L == 0) {
				above[c] = ab;
				if (nparts > 1 || (m & 63u) == 63u) ctl[1 + w] = m + 1u;
			}
			o.hasc[mb] = (uint8_t)any;
		}
	}
	if (L == 0) ctl[1 + w] = 0xFFFFFFFFu;  // out of rows: never the one anybody waits for
}

// LDS: ctl[kCtlWords] (prod, done[8]), ring[kRing] flag bytes, then per MB column the token
// contexts (bits 0..8: Y 0..3, U 4..5, V 6..7, Y2 8) and the bottom row's sub-block modes
// (4 nibbles; B_DC = 0 above the frame).
__global__ __launch_bounds__(64 * (1 + kMaxParts)) void m05_kernel(const Vp8gTokFrame* __restrict__ jobs,
                                                                   const uint8_t* __restrict__ bits, Out o) {
	extern __shared__ uint32_t sm[];
	const Vp8gTokFrame& J = jobs[blockIdx.x];
	const uint32_t cols = J.mb_cols, nparts = J.nparts;
	const uint32_t words = kCtlWords + kRing / 4u + 2u * cols;
	for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) sm[i] = 0;
	__syncthreads();
	lds_u32* const ctl = (lds_u32*)sm;
	lds_u8* const ring = (lds_u8*)(sm + kCtlWords);
	lds_u32* const above = (lds_u32*)(sm + kCtlWords + kRing / 4u);
	const uint8_t* pl = bits + J.data;
	const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
	if (wave == 0) modes_wave(J, pl, o, ctl, ring, above + cols, nparts);
	else if (wave <= nparts) tokens_wave(J, pl, o, ctl, ring, above, wave - 1u, nparts);
}

}  // namespace

VP8G_API int vp8g_m05_batch_device(const Vp8gTokFrame* h_jobs, const Vp8gTokFrame* d_jobs, uint32_t n,
                                   const uint8_t* d_bits, const Vp8gBatchArrays* arrays, void* hip_stream) {
	if (!h_jobs || !d_jobs || !d_bits || !arrays || !arrays->status || n == 0) {
		errno = EINVAL;
		return -1;
	}
	uint32_t max_cols = 0, max_parts = 1;
	for (uint32_t i = 0; i < n; i++) {
		const Vp8gTokFrame& j = h_jobs[i];
		bool ok = j.mb_cols > 0 && j.mb_cols <= 1024u && j.mb_rows > 0 && j.mb_rows <= 1024u && !(j.data & 3u) &&
		          j.b_next <= j.p0_end && j.b_bits >= 0 && j.b_bits <= 56 && j.b_range >= 128u && j.b_range <= 255u &&
		          (j.nparts == 1 || j.nparts == 2 || j.nparts == 4 || j.nparts == 8);
		for (uint32_t p = 0; ok && p < j.nparts; p++)
			ok = j.part_off[p] >= j.p0_end && j.part_end[p] >= j.part_off[p] && (p == 0 || j.part_off[p] >= j.part_end[p - 1]);
		if (!ok) {
			errno = EINVAL;
			return -1;
		}
		if (j.mb_cols > max_cols) max_cols = j.mb_cols;
		if (j.nparts > max_parts) max_parts = j.nparts;
	}
	Out o;
	o.cy = const_cast<int16_t*>(arrays->coeff_y);
	o.cu = const_cast<int16_t*>(arrays->coeff_u);
	o.cv = const_cast<int16_t*>(arrays->coeff_v);
	o.cy2 = const_cast<int16_t*>(arrays->coeff_y2);
	o.ymode = const_cast<uint8_t*>(arrays->ymode);
	o.uvmode = const_cast<uint8_t*>(arrays->uv_mode);
	o.seg = const_cast<uint8_t*>(arrays->segment_id);
	o.hasc = const_cast<uint8_t*>(arrays->has_coeff);
	o.bmode = const_cast<uint8_t*>(arrays->bmode);
	o.status = arrays->status;
	hipError_t e;
	{
		vp8g::GateScope gate((hipStream_t)hip_stream);  // (vp8g_device.h: no cross-workgroup launch beside it)
		e = gate.status();
		if (e == hipSuccess) {
			hipLaunchKernelGGL(m05_kernel, dim3(n), dim3(64u * (1u + max_parts)), (kCtlWords + kRing / 4u + 2u * max_cols) * 4u,
			                   (hipStream_t)hip_stream, d_jobs, d_bits, o);
			e = hipGetLastError();
		}
		if (e == hipSuccess) e = gate.done(false);
	}
	if (e != hipSuccess) {
		vp8g::set_error_text("m05 launch", e);
		errno = EIO;
		return -1;
	}
	return 0;
}
