// vp8g_m05.hip -- m05 on the device: per-macroblock modes and coefficient
// tokens of a batch of key frames, one wavefront per frame.
//
// VP8's arithmetic-coded partitions are serial chains (each bool's range depends on the previous
// one), and a key frame with one token partition has exactly two of them: partition 0 (modes) and
// the token partition.  There is no parallelism inside a frame, so the unit of parallelism is the
// frame: one 64-thread workgroup decodes one frame with wave-uniform code.  Every value is the
// same in all lanes (context words read from LDS go through readfirstlane), so the decoder state
// lives in scalar registers, the bool decoder runs on the scalar ALU and the bitstream comes in
// through scalar loads; lane 0 stores the results (vector stores only).  A batch of a few hundred
// frames gives every CU one or more frames.  The two chains are interleaved MB by MB (modes of MB
// m, then its tokens): they are independent streams read in the same raster order.
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
};

// RFC 6386 7 bool decoder in the host's formulation (host/vp8_bool.h): `value` holds the stream
// bits, compared at `bits`.  Refilled 32 bits at a time; bytes at or past `end` read as zero (the
// coder's padding), as in the host's byte-wise refill, so the compared values are identical.
struct DBool {
	uint64_t value;
	int bits;
	uint32_t range;
	uint32_t next, end;
};

// 4 big-endian stream bytes at payload offset pos (zero at and past end).  The payload starts
// 4-aligned in the bitstream buffer and is followed by >= 8 readable bytes.
DEV uint32_t be32_at(const uint8_t* pl, uint32_t pos, uint32_t end) {
	if (pos >= end) return 0u;
	const uint32_t al = pos & ~3u, sh = (pos & 3u) * 8u;
	const uint32_t* w = (const uint32_t*)(pl + al);
	const uint64_t x = ((uint64_t)w[1] << 32) | w[0];
	uint32_t v = (uint32_t)(x >> sh);
	const uint32_t n = end - pos;
	if (n < 4u) v &= 0xFFFFFFFFu >> (32u - 8u * n);
	return __builtin_bswap32(v);
}

DEV void dfill(DBool& b, const uint8_t* pl) {
	b.value = (b.value << 32) | be32_at(pl, b.next, b.end);
	b.bits += 32;
	b.next += 4u;
}

DEV uint32_t dread(DBool& b, const uint8_t* pl, uint32_t prob) {
	const uint32_t split = 1u + (((b.range - 1u) * prob) >> 8);
	uint32_t bit;
	if ((uint32_t)(b.value >> b.bits) >= split) {  // 64-bit shift + 32-bit compare: both scalar
		b.value -= (uint64_t)split << b.bits;
		b.range -= split;
		bit = 1u;
	} else {
		b.range = split;
		bit = 0u;
	}
	const int sh = __builtin_clz(b.range) - 24;
	b.range <<= sh;
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

// DCT_CAT1..6 extra bits (RFC 6386 13.2): probabilities packed 4 per dword
__constant__ uint32_t kCatProbs[6][3] = {
	{159u, 0u, 0u},
	{165u | 145u << 8, 0u, 0u},
	{173u | 148u << 8 | 140u << 16, 0u, 0u},
	{176u | 155u << 8 | 140u << 16 | 135u << 24, 0u, 0u},
	{180u | 157u << 8 | 141u << 16 | 134u << 24, 130u, 0u},
	{254u | 254u << 8 | 243u << 16 | 230u << 24, 196u | 177u << 8 | 153u << 16 | 140u << 24, 133u | 130u << 8 | 129u << 16},
};
DEV uint32_t read_cat(DBool& b, const uint8_t* pl, uint32_t cat) {
	const uint32_t nbits = cat < 5u ? cat + 1u : 11u;
	const uint32_t base = cat < 5u ? (3u + (2u << cat)) : 67u;  // 5 7 11 19 35 67
	uint32_t e = 0;
	for (uint32_t i = 0; i < nbits; i++) {
		const uint32_t p = (kCatProbs[cat][i >> 2] >> (8u * (i & 3u))) & 255u;
		e = 2u * e + dread(b, pl, p);
	}
	return base + e;
}

// One 4x4 block's tokens (RFC 6386 13; host/vp8_parse.c read_block): the non-zero values go to
// dst[natural position] (lane 0 stores); returns whether any value is non-zero.  `probs` points at
// the [8][3] rows of the block type (12 bytes each).
DEV bool read_block(DBool& b, const uint8_t* pl, const uint32_t* probs, uint32_t first, uint32_t ctx, int16_t* dst,
                    bool l0) {
	bool nz = false;
	uint32_t pos = first;
	uint32_t ri = nib(kBand4, pos) * 3u + ctx;
	bool skip_eob = false;
	while (true) {
		const Row p{probs[ri * 3u], probs[ri * 3u + 1u], probs[ri * 3u + 2u]};
		if (!skip_eob && !dread(b, pl, pb(p, 0))) break;  // EOB
		if (!dread(b, pl, pb(p, 1))) {                     // DCT_0: the next token has no EOB branch
			if (++pos == 16u) break;
			ri = nib(kBand4, pos) * 3u;
			skip_eob = true;
			continue;
		}
		uint32_t mag;
		if (!dread(b, pl, pb(p, 2))) {
			mag = 1u;
		} else if (!dread(b, pl, pb(p, 3))) {
			mag = dread(b, pl, pb(p, 4)) ? 3u + dread(b, pl, pb(p, 5)) : 2u;
		} else {
			uint32_t cat;
			if (!dread(b, pl, pb(p, 6))) cat = dread(b, pl, pb(p, 7));
			else if (!dread(b, pl, pb(p, 8))) cat = 2u + dread(b, pl, pb(p, 9));
			else cat = 4u + dread(b, pl, pb(p, 10));
			mag = read_cat(b, pl, cat);
		}
		const uint32_t neg = dread(b, pl, 128);
		if (l0) dst[nib(kScan4, pos)] = (int16_t)(neg ? -(int)mag : (int)mag);
		nz = true;
		if (++pos == 16u) break;
		ri = nib(kBand4, pos) * 3u + (mag == 1u ? 1u : 2u);
		skip_eob = false;
	}
	return nz;
}

// Per MB column in LDS, one dword: bits 0..8 token contexts (Y 0..3, U 4..5, V 6..7, Y2 8),
// bits 16..31 the bottom row's sub-block modes (4 nibbles; B_DC = 0 above the frame).
__global__ __launch_bounds__(64) void m05_kernel(const Vp8gTokFrame* __restrict__ jobs, const uint8_t* __restrict__ bits,
                                                 Out o) {
	extern __shared__ uint32_t above[];
	const Vp8gTokFrame& J = jobs[blockIdx.x];
	const uint32_t cols = J.mb_cols, rows = J.mb_rows;
	const bool l0 = threadIdx.x == 0;
	for (uint32_t i = threadIdx.x; i < cols; i += 64u) above[i] = 0;
	__syncthreads();
	const uint8_t* pl = bits + J.data;
	const uint32_t flags = *(const uint32_t*)&J.seg_enabled;  // seg_enabled | seg_map_update | use_skip | skip_prob
	const bool seg_map = (flags & 0xFFu) && ((flags >> 8) & 0xFFu);
	const bool use_skip = (flags >> 16) & 0xFFu;
	const uint32_t skip_prob = flags >> 24;
	const uint32_t seg_probs = *(const uint32_t*)J.seg_probs;
	const uint32_t* const cprobs = (const uint32_t*)J.coeff_probs;  // [4][8][3] rows of 3 dwords
	DBool hb{J.b_value, J.b_bits, J.b_range, J.b_next, J.p0_end};
	DBool tb{0, -8, 255u, J.tok_off, J.tok_end};
	dfill(tb, pl);
	for (uint32_t r = 0; r < rows; r++) {
		uint32_t left = 0;    // token contexts, bits as in above[]
		uint32_t left_b = 0;  // right column's sub-block modes, 4 nibbles
		for (uint32_t c = 0; c < cols; c++) {
			const uint64_t mb = J.mb_offset + (uint64_t)r * cols + c;
			uint32_t ab = __builtin_amdgcn_readfirstlane(above[c]);
			// ---- modes (partition 0; RFC 6386 11, 19.3)
			const uint32_t seg = seg_map ? read_segment(hb, pl, seg_probs) : 0u;
			const uint32_t skip = use_skip ? dread(hb, pl, skip_prob) : 0u;
			const uint32_t ym = read_ymode(hb, pl);
			uint64_t bm;  // the MB's 16 sub-block modes, 4 bits each, raster order
			if (ym == 4u) {
				bm = 0;
				for (uint32_t i = 0; i < 16u; i++) {
					const uint32_t y = i >> 2, x = i & 3u;
					const uint32_t a = y ? nib(bm, i - 4u) : (ab >> (16u + 4u * x)) & 15u;
					const uint32_t l = x ? nib(bm, i - 1u) : (left_b >> (4u * y)) & 15u;
					const uint32_t* w = kBmodeProbs.w[a * 10u + l];
					bm |= (uint64_t)read_bmode(hb, pl, Row{w[0], w[1], w[2]}) << (4u * i);
				}
			} else {
				// implied sub-block context: DC->B_DC, V->B_VE, H->B_HE, TM->B_TM
				const uint32_t im = (0x1320u >> (4u * ym)) & 15u;
				bm = (uint64_t)im * 0x1111111111111111ull;
			}
			const uint32_t bottom = (uint32_t)(bm >> 48) & 0xFFFFu;
			left_b = 0;
			for (uint32_t y = 0; y < 4u; y++) left_b |= nib(bm, 4u * y + 3u) << (4u * y);
			const uint32_t uvm = read_uvmode(hb, pl);
			// ---- tokens (token partition; RFC 6386 13)
			const bool has_y2 = ym != 4u;
			bool any = false;
			if (skip) {
				// no tokens: the contexts of the MB's blocks become 0; Y2's only if the MB has one
				const uint32_t clr = has_y2 ? 0x1FFu : 0xFFu;
				left &= ~clr;
				ab &= ~clr;
			} else {
				for (int k = has_y2 ? -1 : 0; k < 24; k++) {
					uint32_t type, first, li, ai;
					int16_t* dst;
					if (k < 0) {
						type = PLANE_Y2, first = 0, li = ai = 8;
						dst = o.cy2 + mb * 16u;
					} else if (k < 16) {
						type = has_y2 ? PLANE_Y_AFTER_Y2 : PLANE_Y_ALONE, first = has_y2 ? 1u : 0u;
						li = (uint32_t)k >> 2, ai = (uint32_t)k & 3u;
						dst = o.cy + (mb * 16u + (uint32_t)k) * 16u;
					} else {
						const uint32_t j = (uint32_t)k - 16u, p = j >> 2, jj = j & 3u;
						type = PLANE_UV, first = 0;
						li = 4u + 2u * p + (jj >> 1), ai = 4u + 2u * p + (jj & 1u);
						dst = (p ? o.cv : o.cu) + (mb * 4u + jj) * 16u;
					}
					const uint32_t ctx = ((left >> li) & 1u) + ((ab >> ai) & 1u);
					const bool nz = read_block(tb, pl, cprobs + type * 72u, first, ctx, dst, l0);
					any |= nz;
					left = (left & ~(1u << li)) | ((uint32_t)nz << li);
					ab = (ab & ~(1u << ai)) | ((uint32_t)nz << ai);
				}
			}
			ab = (ab & 0xFFFFu) | (bottom << 16);
			if (l0) {
				above[c] = ab;
				o.seg[mb] = (uint8_t)seg;
				o.ymode[mb] = (uint8_t)ym;
				o.uvmode[mb] = (uint8_t)uvm;
				o.hasc[mb] = (uint8_t)any;
				uint32_t bw[4];
				for (int i = 0; i < 4; i++) {
					const uint32_t q = (uint32_t)(bm >> (16 * i));
					bw[i] = (q & 15u) | ((q >> 4) & 15u) << 8 | ((q >> 8) & 15u) << 16 | ((q >> 12) & 15u) << 24;
				}
				*(uint4*)(o.bmode + mb * 16u) = make_uint4(bw[0], bw[1], bw[2], bw[3]);
			}
		}
	}
}

}  // namespace

VP8G_API int vp8g_m05_batch_device(const Vp8gTokFrame* h_jobs, const Vp8gTokFrame* d_jobs, uint32_t n,
                                   const uint8_t* d_bits, const Vp8gBatchArrays* arrays, void* hip_stream) {
	if (!h_jobs || !d_jobs || !d_bits || !arrays || n == 0) {
		errno = EINVAL;
		return -1;
	}
	uint32_t max_cols = 0;
	for (uint32_t i = 0; i < n; i++) {
		const Vp8gTokFrame& j = h_jobs[i];
		if (j.mb_cols == 0 || j.mb_cols > 1024u || j.mb_rows == 0 || j.mb_rows > 1024u || (j.data & 3u) ||
		    j.tok_end < j.tok_off || j.p0_end > j.tok_end || j.b_next > j.p0_end || j.b_bits < 0 || j.b_bits > 56 ||
		    j.b_range < 128u || j.b_range > 255u) {
			errno = EINVAL;
			return -1;
		}
		if (j.mb_cols > max_cols) max_cols = j.mb_cols;
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
	hipLaunchKernelGGL(m05_kernel, dim3(n), dim3(64), max_cols * 4u, (hipStream_t)hip_stream, d_jobs, d_bits, o);
	const hipError_t e = hipGetLastError();
	if (e != hipSuccess) {
		vp8g::set_error_text("m05 launch", e);
		errno = EIO;
		return -1;
	}
	return 0;
}
