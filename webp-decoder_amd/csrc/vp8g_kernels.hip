// vp8g_kernels.hip -- fused VP8 key-frame reconstruction + loop filter for CDNA4 (gfx950).
//
// Replaces the reference hot path src/m06_recon/vp8_recon.c:423-712 (per-MB dequant, iWHT,
// iDCT, intra prediction, reconstruction, crop) and src/m07_loopfilter/vp8_loopfilter.c:201-283
// (raster-order in-place deblocking), bit-exactly.
//
// Schedule:
//   * one workgroup = one frame; NW waves; wave w owns MB rows r = w, w+NW, ...
//   * MB(r,c) needs MB(r,c-1) and MB(r-1,c+1) done, for prediction AND for the loop filter
//     (SURVEY.md App. B), so each wave waits on an LDS progress word of the row above
//     (value r*C + cols_done, monotone within a frame) and publishes its own after every MB;
//   * the MB is reconstructed into a per-wave LDS tile and loop-filtered right away; the
//     unfiltered bottom row / right column needed for intra prediction are saved before
//     filtering (ctx_rec in the shared per-column context, kLeft per wave), and the bottom 4
//     filtered rows that the next MB row's top-edge filter still modifies travel through
//     ctx_lf.  Pixels are stored to HBM exactly once, when final: rows 0..11 of MB(r,c-1) after
//     LF(r,c), rows 12..15 after LF(r+1,c-1) by the wave below.
//   * residual work (dequant, iWHT, iDCT) depends on nothing spatial and runs before the
//     dependency wait; the next MB's coefficients are prefetched one MB ahead.
// Lane roles per MB: lanes 0..31 hold luma block b = lane/2 (rows 2h, 2h+1, h = lane&1) as
// loaded by one coalesced 16-B load per lane; 32..39 U, 40..47 V, 48..49 the Y2 block.
#include <stdint.h>

#include "vp8g_device.h"

#define DEV __device__ __forceinline__

// Diagnostic builds only (never in the shipped library): VP8G_STAMPS accumulates per-phase
// shader-clock cycles (s_memtime) into g_vp8g_stamps; VP8G_ABLATE skips phases (timing only,
// output wrong): 1 = loop filter, 2 = B_PRED steps, 4 = pixel stores, 8 = dependency wait.
#ifndef VP8G_ABLATE
#define VP8G_ABLATE 0
#endif
#ifdef VP8G_STAMPS
__device__ unsigned long long g_vp8g_stamps[16];
#define STAMP(i)                                                  \
	do {                                                          \
		const uint64_t t_ = __builtin_amdgcn_s_memtime();         \
		st_acc[i] += t_ - st_prev;                                \
		st_prev = t_;                                             \
	} while (0)
#else
#define STAMP(i) \
	do {         \
	} while (0)
#endif

namespace vp8g {
namespace {

// ---------------------------------------------------------------------------------------------
// B_PRED predictor table (RFC 6386 12.3; reference vp8_recon.c:218-358).  Edge array bytes in
// LDS: [0..3] = L3 L2 L1 L0, [7] = P (corner), [8..15] = A0..A7.  Entry = 3 byte positions +
// kind (0 avg3, 1 avg2, 2 copy).  Modes 0 (DC) and 1 (TM) are computed directly.
// ---------------------------------------------------------------------------------------------
struct BpTab {
	uint16_t v[256];
};
constexpr int epos(int e) { return e < 4 ? e : (e == 4 ? 7 : e + 3); }
constexpr uint16_t ent(int kind, int a, int b, int c) {
	return (uint16_t)(epos(a) | (epos(b) << 4) | (epos(c) << 8) | (kind << 12));
}
constexpr uint16_t A3(int a, int b, int c) { return ent(0, a, b, c); }
constexpr uint16_t A2(int a, int b) { return ent(1, a, b, b); }
constexpr uint16_t CP(int a) { return ent(2, a, a, a); }

constexpr BpTab make_bptab() {
	BpTab t{};
	const uint16_t vr[16] = {A2(4, 5), A2(5, 6), A2(6, 7), A2(7, 8), A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7), A3(6, 7, 8),
	                         A3(2, 3, 4), A2(4, 5), A2(5, 6), A2(6, 7), A3(1, 2, 3), A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7)};
	const uint16_t vl[16] = {A2(5, 6), A2(6, 7), A2(7, 8), A2(8, 9), A3(5, 6, 7), A3(6, 7, 8), A3(7, 8, 9), A3(8, 9, 10),
	                         A2(6, 7), A2(7, 8), A2(8, 9), A3(9, 10, 11), A3(6, 7, 8), A3(7, 8, 9), A3(8, 9, 10), A3(10, 11, 12)};
	const uint16_t hd[16] = {A2(3, 4), A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7), A2(2, 3), A3(2, 3, 4), A2(3, 4), A3(3, 4, 5),
	                         A2(1, 2), A3(1, 2, 3), A2(2, 3), A3(2, 3, 4), A2(0, 1), A3(0, 1, 2), A2(1, 2), A3(1, 2, 3)};
	const uint16_t hu[16] = {A2(3, 2), A3(3, 2, 1), A2(2, 1), A3(2, 1, 0), A2(2, 1), A3(2, 1, 0), A2(1, 0), A3(1, 0, 0),
	                         A2(1, 0), A3(1, 0, 0), CP(0), CP(0), CP(0), CP(0), CP(0), CP(0)};
	for (int p = 0; p < 16; p++) {
		const int r = p >> 2, c = p & 3;
		t.v[2 * 16 + p] = A3(4 + c, 5 + c, 6 + c);                                                  // B_VE
		t.v[3 * 16 + p] = r == 3 ? A3(1, 0, 0) : A3(4 - r, 3 - r, 2 - r);                           // B_HE
		t.v[4 * 16 + p] = A3(5 + r + c, 6 + r + c, (7 + r + c) > 12 ? 12 : (7 + r + c));            // B_LD
		t.v[5 * 16 + p] = A3(3 - r + c, 4 - r + c, 5 - r + c);                                      // B_RD
		t.v[6 * 16 + p] = vr[p];
		t.v[7 * 16 + p] = vl[p];
		t.v[8 * 16 + p] = hd[p];
		t.v[9 * 16 + p] = hu[p];
	}
	return t;
}
__constant__ BpTab kBpTab = make_bptab();

// ---------------------------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------------------------
// Intra-wave LDS ordering: a wave's LDS instructions execute in issue order, so only the
// compiler must be kept from reordering / caching across this point.
DEV void wave_lds_sync() { asm volatile("" ::: "memory"); }

DEV int sx16(int x) { return (int)(int16_t)x; }
DEV int sat8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
DEV int sclamp(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
DEV int iabs(int v) { return v < 0 ? -v : v; }
DEV int mul_s(int x) { return (x * 35468) >> 16; }          // x*sqrt(2)*sin(pi/8), RFC 14.4
DEV int mul_c(int x) { return x + ((x * 20091) >> 16); }    // x*sqrt(2)*cos(pi/8)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

DEV uint32_t bsum4(uint32_t w) { return __builtin_amdgcn_sad_u8(w, 0u, 0u); }
DEV int partner(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }  // lane ^ 1
DEV uint32_t u8(const uint8_t* p) { return *p; }
DEV uint32_t ld32(const uint8_t* p) { return *(const uint32_t*)p; }
DEV void st32(uint8_t* p, uint32_t v) { *(uint32_t*)p = v; }
DEV uint2 ld64(const uint8_t* p) { return *(const uint2*)p; }
DEV void st64(uint8_t* p, uint2 v) { *(uint2*)p = v; }
DEV uint32_t pack4(int a, int b, int c, int d) {
	return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}
DEV int ubyte(uint32_t w, int i) { return (int)((w >> (8 * i)) & 0xFFu); }
// byte q (0..15) of a 16-byte value held in 4 dwords
DEV int byte16(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, int q) {
	uint32_t lo = __builtin_amdgcn_perm(d1, d0, (uint32_t)(q & 7) * 0x01010101u);
	uint32_t hi = __builtin_amdgcn_perm(d3, d2, (uint32_t)(q & 7) * 0x01010101u);
	return (int)(((q & 8) ? hi : lo) & 0xFFu);
}

// Per-frame context (unfiltered bottom rows + filter-state bottom rows per MB column), in LDS
// or, for frames too wide for LDS, in device memory (read with L1-bypassing loads).
template <bool kG>
struct Ctx {
	uint8_t* lds;  // smem + offset (kG == false)
	uint8_t* g;    // device pointer (kG == true)
	DEV uint32_t rd(uint32_t off) const {
		if constexpr (kG) return __hip_atomic_load((uint32_t*)(g + off), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		else return ld32(lds + off);
	}
	DEV void wr(uint32_t off, uint32_t v) const {
		if constexpr (kG) *(uint32_t*)(g + off) = v;
		else st32(lds + off, v);
	}
	DEV void publish_fence() const {
		if constexpr (kG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	}
};
DEV uint32_t rec_off(uint32_t c) { return c * kCtxBytesPerCol; }
DEV uint32_t lf_off(uint32_t c) { return c * kCtxBytesPerCol + kCtxRecBytes; }

// ---------------------------------------------------------------------------------------------
// Loop filter on a line of pixels (RFC 6386 15.2-15.4; reference vp8_loopfilter.c:24-164).
// px[] is a 20-pixel line across the MB's edges: [0..3] = the neighbour (left or above),
// [4..19] = this MB; edges sit at q0 = 4 (MB edge), 8, 12, 16 (sub-block edges).
// ---------------------------------------------------------------------------------------------
template <int K>
DEV void lf_mb_edge(int* px, bool en, int lim, int I, int T) {  // normal filter, MB edge
	const int p3 = px[K - 4], p2 = px[K - 3], p1 = px[K - 2], p0 = px[K - 1];
	const int q0 = px[K], q1 = px[K + 1], q2 = px[K + 2], q3 = px[K + 3];
	const bool m = en && (iabs(p0 - q0) * 2 + (iabs(p1 - q1) >> 1) <= lim) && iabs(p3 - p2) <= I && iabs(p2 - p1) <= I &&
	               iabs(p1 - p0) <= I && iabs(q3 - q2) <= I && iabs(q2 - q1) <= I && iabs(q1 - q0) <= I;
	if (!m) return;
	const bool hev = iabs(p1 - p0) > T || iabs(q1 - q0) > T;
	const int w = sclamp(sclamp(p1 - q1) + 3 * (q0 - p0));
	if (hev) {
		px[K] = sat8(q0 - (sclamp(w + 4) >> 3));
		px[K - 1] = sat8(p0 + (sclamp(w + 3) >> 3));
	} else {
		int a = (27 * w + 63) >> 7;
		px[K - 1] = sat8(p0 + a);
		px[K] = sat8(q0 - a);
		a = (18 * w + 63) >> 7;
		px[K - 2] = sat8(p1 + a);
		px[K + 1] = sat8(q1 - a);
		a = (9 * w + 63) >> 7;
		px[K - 3] = sat8(p2 + a);
		px[K + 2] = sat8(q2 - a);
	}
}

template <int K>
DEV void lf_sub_edge(int* px, bool en, int lim, int I, int T) {  // normal filter, sub-block edge
	const int p3 = px[K - 4], p2 = px[K - 3], p1 = px[K - 2], p0 = px[K - 1];
	const int q0 = px[K], q1 = px[K + 1], q2 = px[K + 2], q3 = px[K + 3];
	const bool m = en && (iabs(p0 - q0) * 2 + (iabs(p1 - q1) >> 1) <= lim) && iabs(p3 - p2) <= I && iabs(p2 - p1) <= I &&
	               iabs(p1 - p0) <= I && iabs(q3 - q2) <= I && iabs(q2 - q1) <= I && iabs(q1 - q0) <= I;
	if (!m) return;
	const bool hev = iabs(p1 - p0) > T || iabs(q1 - q0) > T;
	const int a = sclamp(3 * (q0 - p0) + (hev ? sclamp(p1 - q1) : 0));
	const int f1 = sclamp(a + 4) >> 3, f2 = sclamp(a + 3) >> 3;
	px[K] = sat8(q0 - f1);
	px[K - 1] = sat8(p0 + f2);
	if (!hev) {
		const int a2 = (f1 + 1) >> 1;
		px[K + 1] = sat8(q1 - a2);
		px[K - 2] = sat8(p1 + a2);
	}
}

template <int K>
DEV void lf_simple_edge(int* px, bool en, int lim) {  // simple filter (luma only)
	const int p1 = px[K - 2], p0 = px[K - 1], q0 = px[K], q1 = px[K + 1];
	if (!(en && iabs(p0 - q0) * 2 + (iabs(p1 - q1) >> 1) <= lim)) return;
	const int a = sclamp(sclamp(p1 - q1) + 3 * (q0 - p0));
	px[K] = sat8(q0 - (sclamp(a + 4) >> 3));
	px[K - 1] = sat8(p0 + (sclamp(a + 3) >> 3));
}

// All edges of one line, in the reference order (MB edge, then sub-block edges).  `is_y`
// enables the luma-only edges at 12 and 16; chroma has its single inner edge at 8.
DEV void lf_line(int* px, bool simple, bool mb_edge, bool inner, bool is_y, int E, int I, int T) {
	if (simple) {
		lf_simple_edge<4>(px, mb_edge && is_y, (E + 2) * 2 + I);
		lf_simple_edge<8>(px, inner && is_y, E * 2 + I);
		lf_simple_edge<12>(px, inner && is_y, E * 2 + I);
		lf_simple_edge<16>(px, inner && is_y, E * 2 + I);
	} else {
		lf_mb_edge<4>(px, mb_edge, 2 * (E + 2) + I, I, T);
		lf_sub_edge<8>(px, inner, 2 * E + I, I, T);
		lf_sub_edge<12>(px, inner && is_y, 2 * E + I, I, T);
		lf_sub_edge<16>(px, inner && is_y, 2 * E + I, I, T);
	}
}

// ---------------------------------------------------------------------------------------------
// The fused kernel.
// ---------------------------------------------------------------------------------------------
template <int NW, bool kG>
__global__ __launch_bounds__(NW * 64) void frame_kernel(const Vp8gFrameDesc* __restrict__ descs, Vp8gBatchArrays A,
                                                        uint8_t* __restrict__ out, uint32_t ctx_cols,
                                                        uint8_t* __restrict__ gctx) {
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	const int lane0 = (int)(threadIdx.x & 63);
	const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
	const uint32_t f = blockIdx.x;

	for (int i = (int)threadIdx.x; i < 256; i += NW * 64) ((uint16_t*)(smem + kBpTable))[i] = kBpTab.v[i];
	if (threadIdx.x < 16) ((uint32_t*)(smem + kProgress))[threadIdx.x] = 0;
	__syncthreads();

	const Vp8gFrameDesc& D = descs[f];
	const uint32_t C = D.mb_cols, R = D.mb_rows;
	const uint32_t flags = D.flags;
	const bool lf_on = (flags & VP8G_F_LOOPFILTER) != 0;
	const bool simple = (flags & VP8G_F_SIMPLE) != 0;
	const bool lf_only = (flags & VP8G_F_LF_ONLY) != 0;
	const uint64_t mb0 = D.mb_offset;
	uint8_t* const outY = out + D.out_y;
	uint8_t* const outU = out + D.out_u;
	uint8_t* const outV = out + D.out_v;
	const uint32_t W = D.width, H = D.height, CW = (D.width + 1) >> 1, CH = (D.height + 1) >> 1;
	const uint32_t sy = D.stride_y, suv = D.stride_uv;

	uint8_t* const wv = smem + kHdrBytes + wave * kWaveBytes;
	uint8_t* const tY = wv + kLfY;
	uint8_t* const tU = wv + kLfU;
	uint8_t* const tV = wv + kLfV;
	uint8_t* const abY = wv + kAbY;
	uint8_t* const abUV = wv + kAbUV;
	uint8_t* const left = wv + kLeft;
	uint32_t* const prog = (uint32_t*)(smem + kProgress);
	const uint16_t* const bptab = (const uint16_t*)(smem + kBpTable);
	Ctx<kG> ctx;
	ctx.lds = smem + kHdrBytes + NW * kWaveBytes;
	ctx.g = kG ? gctx + (size_t)f * ctx_cols * kCtxBytesPerCol : nullptr;

	// coefficient source of a lane: 16 bytes = 8 int16 (two rows of one 4x4 block)
	auto coeff_ptr = [&](int ln, uint64_t m) -> const u32x4* {
		if (ln < 32) return (const u32x4*)(A.coeff_y + m * 256 + ln * 8);
		if (ln < 40) return (const u32x4*)(A.coeff_u + m * 64 + (ln - 32) * 8);
		if (ln < 48) return (const u32x4*)(A.coeff_v + m * 64 + (ln - 40) * 8);
		return (const u32x4*)(A.coeff_y2 + m * 16 + (ln - 48) * 8);
	};

#ifdef VP8G_STAMPS
	uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	uint64_t st_prev = __builtin_amdgcn_s_memtime();
#endif
	for (uint32_t r = (uint32_t)wave; r < R; r += NW) {
		const uint32_t y0 = r * 16, cy0 = r * 8;
		u32x4 nxt = {0u, 0u, 0u, 0u};
		if (lane0 < 50 && !lf_only) nxt = __builtin_nontemporal_load(coeff_ptr(lane0, mb0 + (uint64_t)r * C));

		for (uint32_t c = 0; c < C; c++) {
			const uint64_t m = mb0 + (uint64_t)r * C + c;
			// Lane-derived values are recomputed every MB from a laundered lane id: hoisting the
			// ~100 lane-dependent LDS addresses out of the loop would exhaust the VGPR budget.
			int lane = lane0;
			asm volatile("" : "+v"(lane));
			const bool is_yl = lane < 32, is_uvl = lane >= 32 && lane < 48, is_y2l = lane == 48 || lane == 49;
			const int h = lane & 1;
			const int yb = lane >> 1;          // luma block (lanes 0..31)
			const int uvk = (lane - 32) & 15;  // chroma lane index 0..15
			const int uvp = uvk >> 3;          // 0 = U, 1 = V
			const int uvb = (uvk & 7) >> 1;    // chroma block 0..3
			const bool loads = lane < 50 && !lf_only;

			const u32x4 cw = nxt;
			if (loads && c + 1 < C) nxt = __builtin_nontemporal_load(coeff_ptr(lane, m + 1));
			const int slot = (int)(c & 1);
			const uint32_t x0 = c * 16, cx0 = c * 8;

			// side info (uniform)
			const int ymode = __builtin_amdgcn_readfirstlane((int)A.ymode[m]);
			const int uvmode = __builtin_amdgcn_readfirstlane((int)A.uv_mode[m]);
			const int seg = __builtin_amdgcn_readfirstlane((int)A.segment_id[m]) & 3;
			const int hasc = A.has_coeff ? __builtin_amdgcn_readfirstlane((int)A.has_coeff[m]) : 0;
			const bool bpred = ymode == 4;

			// ------------------------------------------------ residual (no spatial dependency)
			int res[8];
			if (!lf_only) {
				int cf[8];
				cf[0] = (int)(int16_t)(cw.x & 0xFFFF);
				cf[1] = (int)(int16_t)(cw.x >> 16);
				cf[2] = (int)(int16_t)(cw.y & 0xFFFF);
				cf[3] = (int)(int16_t)(cw.y >> 16);
				cf[4] = (int)(int16_t)(cw.z & 0xFFFF);
				cf[5] = (int)(int16_t)(cw.z >> 16);
				cf[6] = (int)(int16_t)(cw.w & 0xFFFF);
				cf[7] = (int)(int16_t)(cw.w >> 16);
				const int16_t* dq = D.dq[seg];
				int fdc, fac;
				if (is_yl) fdc = dq[0], fac = dq[1];
				else if (is_uvl) fdc = dq[2], fac = dq[3];
				else fdc = dq[4], fac = dq[5];
				int v[8];
#pragma unroll
				for (int k = 0; k < 8; k++) v[k] = sx16(cf[k] * ((k == 0 && h == 0) ? fdc : fac));

				if (!bpred) {
					// inverse WHT of the Y2 block in lanes 48/49 -> 16 luma DCs (RFC 14.3)
					if (is_y2l) {
						int o[8];
#pragma unroll
						for (int k = 0; k < 8; k++) o[k] = partner(v[k]);
						int t[8];
#pragma unroll
						for (int i = 0; i < 4; i++) {
							const int r0 = h ? o[i] : v[i], r1 = h ? o[4 + i] : v[4 + i];
							const int r2 = h ? v[i] : o[i], r3 = h ? v[4 + i] : o[4 + i];
							const int a1 = r0 + r3, b1 = r1 + r2, c1 = r1 - r2, d1 = r0 - r3;
							t[i] = sx16(h ? a1 - b1 : a1 + b1);
							t[4 + i] = sx16(h ? d1 - c1 : c1 + d1);
						}
						uint32_t pk[4];
#pragma unroll
						for (int rr = 0; rr < 2; rr++) {
							const int* q = t + 4 * rr;
							const int a1 = q[0] + q[3], b1 = q[1] + q[2], c1 = q[1] - q[2], d1 = q[0] - q[3];
							const int o0 = sx16((a1 + b1 + 3) >> 3), o1 = sx16((c1 + d1 + 3) >> 3);
							const int o2 = sx16((a1 - b1 + 3) >> 3), o3 = sx16((d1 - c1 + 3) >> 3);
							pk[2 * rr] = (uint32_t)(o0 & 0xFFFF) | ((uint32_t)o1 << 16);
							pk[2 * rr + 1] = (uint32_t)(o2 & 0xFFFF) | ((uint32_t)o3 << 16);
						}
						*(uint4*)(wv + kWht + h * 16) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
					}
					wave_lds_sync();
					if (is_yl && h == 0) v[0] = (int)*(const int16_t*)(wv + kWht + yb * 2);
				}

				// any AC coefficient in the MB? (raw, before dequant: conservative)
				bool ac = false;
				if (lane < 48) {
#pragma unroll
					for (int k = 0; k < 8; k++) ac |= (k > 0 || h == 1) && cf[k] != 0;
				}
				if (__ballot(ac) != 0ull) {
					// inverse DCT, RFC 14.4 (vertical pass truncated to int16, then horizontal)
					int o[8];
#pragma unroll
					for (int k = 0; k < 8; k++) o[k] = partner(v[k]);
					int t[8];
#pragma unroll
					for (int i = 0; i < 4; i++) {
						const int r0 = h ? o[i] : v[i], r1 = h ? o[4 + i] : v[4 + i];
						const int r2 = h ? v[i] : o[i], r3 = h ? v[4 + i] : o[4 + i];
						const int a1 = r0 + r2, b1 = r0 - r2;
						const int c1 = mul_s(r1) - mul_c(r3), d1 = mul_c(r1) + mul_s(r3);
						t[i] = sx16(h ? b1 - c1 : a1 + d1);
						t[4 + i] = sx16(h ? a1 - d1 : b1 + c1);
					}
#pragma unroll
					for (int rr = 0; rr < 2; rr++) {
						const int* q = t + 4 * rr;
						const int a1 = q[0] + q[2], b1 = q[0] - q[2];
						const int c1 = mul_s(q[1]) - mul_c(q[3]), d1 = mul_c(q[1]) + mul_s(q[3]);
						res[4 * rr + 0] = sx16((a1 + d1 + 4) >> 3);
						res[4 * rr + 3] = sx16((a1 - d1 + 4) >> 3);
						res[4 * rr + 1] = sx16((b1 + c1 + 4) >> 3);
						res[4 * rr + 2] = sx16((b1 - c1 + 4) >> 3);
					}
				} else {
					// DC-only blocks: the transform output is (dc + 4) >> 3 everywhere
					const int pv0 = partner(v[0]);  // executed by every lane (DPP source must be live)
					const int dc = h ? pv0 : v[0];
					const int d = (dc + 4) >> 3;
#pragma unroll
					for (int k = 0; k < 8; k++) res[k] = d;
				}
			}

			STAMP(0);
			// ------------------------------------------------ wait for MB(r-1, c+1)
			if (r > 0 && !(VP8G_ABLATE & 8)) {
				const uint32_t need = (r - 1) * C + ((c + 2 < C) ? c + 2 : C);
				const uint32_t pw = (uint32_t)((wave + NW - 1) % NW);
				uint32_t spins = 0;
				uint64_t t0 = 0;
				while (__hip_atomic_load(prog + pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
					__builtin_amdgcn_s_sleep(1);
					if ((++spins & 1023u) == 0) {
						const uint64_t now = __builtin_amdgcn_s_memrealtime();
						if (t0 == 0) t0 = now;
						else if (now - t0 > 200000000ull) {  // 2 s at 100 MHz: give up, flag it
							if (lane == 0) atomicOr(A.status, VP8G_ERR_TIMEOUT);
							break;
						}
					}
				}
				asm volatile("" ::: "memory");
			}

			STAMP(1);
			// ------------------------------------------------ borders + loop-filter top strip
			if (!lf_only) {
				const bool top = r == 0;
				if (lane < 4) {  // luma above row
					st32(abY + 16 + 4 * lane, top ? 0x7F7F7F7Fu : ctx.rd(rec_off(c) + 4 * lane));
				} else if (lane == 4) {  // luma above-right (row above the MB, cols x+16..x+19)
					uint32_t v4;
					if (top) v4 = 0x7F7F7F7Fu;
					else if (c + 1 < C) v4 = ctx.rd(rec_off(c + 1));
					else v4 = (ctx.rd(rec_off(c) + 12) >> 24) * 0x01010101u;  // clamp to padded width
					st32(abY + 32, v4);
				} else if (lane < 9) {  // chroma above rows
					const int k = lane - 5, p = k >> 1, dw = k & 1;
					st32(abUV + 16 * p + 8 + 4 * dw, top ? 0x7F7F7F7Fu : ctx.rd(rec_off(c) + 16 + 8 * p + 4 * dw));
				} else if (lane < 17) {  // left columns at the frame's left edge: 129
					if (c == 0) st32(left + 4 * (lane - 9), 0x81818181u);
				} else if (lane == 17) {  // corners at the left edge: 127 on the top row, else 129
					if (c == 0) {
						const uint8_t pv = top ? 127 : 129;
						abY[15] = pv;
						abUV[7] = pv;
						abUV[23] = pv;
					}
				}
			}
			if (lf_on && r > 0 && lane >= 32 && lane < 48) {  // filter state of the MB above
				const int k = lane - 32;
				if (k < 8) {
					const int t = k >> 1, half = k & 1;
					const uint32_t o = lf_off(c) + t * 16 + half * 8;
					st64(tY + t * 32 + slot * 16 + half * 8, make_uint2(ctx.rd(o), ctx.rd(o + 4)));
				} else {
					const int p = (k - 8) >> 2, t = (k - 8) & 3;
					const uint32_t o = lf_off(c) + 64 + p * 32 + t * 8;
					st64((p ? tV : tU) + t * 16 + slot * 8, make_uint2(ctx.rd(o), ctx.rd(o + 4)));
				}
			}
			wave_lds_sync();

			STAMP(2);
			// ------------------------------------------------ prediction + reconstruction
			if (lf_only) {
				// loop-filter-only mode: the MB's pixels come from the padded input image
				const uint8_t* src = A.src;
				if (lane < 32) {  // luma: 16 rows x 2 halves
					const int row = lane >> 1, half = lane & 1;
					const uint8_t* s = src + D.src_y + (size_t)(y0 + row) * D.src_stride_y + x0 + half * 8;
					uint2 v2 = make_uint2(ld32(s), ld32(s + 4));
					st64(tY + (4 + row) * 32 + slot * 16 + half * 8, v2);
				} else if (lane < 48) {
					const int k = lane - 32, p = k >> 3, row = k & 7;
					const uint8_t* s = src + (p ? D.src_v : D.src_u) + (size_t)(cy0 + row) * D.src_stride_uv + cx0;
					st64((p ? tV : tU) + (4 + row) * 16 + slot * 8, make_uint2(ld32(s), ld32(s + 4)));
				}
			} else {
				const bool have_above = r > 0, have_left = c > 0;
				if (!bpred || is_uvl) {
					// whole-block predictors (RFC 12.2; reference vp8_recon.c:152-212, 533-560, 605-651)
					if (lane < 48) {
						const bool yl = is_yl;
						const int mode = yl ? (ymode > 4 ? 0 : ymode) : (uvmode > 3 ? 0 : uvmode);
						const uint8_t* ab = yl ? abY + 16 : abUV + 16 * uvp + 8;
						const uint8_t* lc = yl ? left : left + 16 + 8 * uvp;
						const int blk = yl ? yb : uvb;
						const int py = yl ? 4 * (blk >> 2) + 2 * h : 4 * (blk >> 1) + 2 * h;
						const int pxo = yl ? 4 * (blk & 3) : 4 * (blk & 1);
						int dcv = 128;
						if (mode == 0) {
							uint32_t sa = 0, sl = 0;
							if (yl) {
								sa = bsum4(ld32(ab)) + bsum4(ld32(ab + 4)) + bsum4(ld32(ab + 8)) + bsum4(ld32(ab + 12));
								sl = bsum4(ld32(lc)) + bsum4(ld32(lc + 4)) + bsum4(ld32(lc + 8)) + bsum4(ld32(lc + 12));
							} else {
								sa = bsum4(ld32(ab)) + bsum4(ld32(ab + 4));
								sl = bsum4(ld32(lc)) + bsum4(ld32(lc + 4));
							}
							const int sh = yl ? 4 : 3;
							if (have_above && have_left) dcv = (int)(sa + sl + (1u << sh)) >> (sh + 1);
							else if (have_left) dcv = (int)(sl + (1u << (sh - 1))) >> sh;
							else if (have_above) dcv = (int)(sa + (1u << (sh - 1))) >> sh;
						}
						const uint32_t aw = ld32(ab + pxo);
						const int P = (int)u8(ab - 1);
						uint8_t* dst = yl ? tY + (4 + py) * 32 + slot * 16 + pxo
						                  : (uvp ? tV : tU) + (4 + py) * 16 + slot * 8 + pxo;
						const int dstride = yl ? 32 : 16;
#pragma unroll
						for (int rr = 0; rr < 2; rr++) {
							const int L = (int)u8(lc + py + rr);
							int px4[4];
#pragma unroll
							for (int k = 0; k < 4; k++) {
								const int a = ubyte(aw, k);
								const int pred = mode == 1 ? a : (mode == 2 ? L : (mode == 3 ? sat8(L + a - P) : dcv));
								px4[k] = sat8(pred + res[4 * rr + k]);
							}
							st32(dst + rr * dstride, pack4(px4[0], px4[1], px4[2], px4[3]));
						}
					}
				}
				if (bpred && !(VP8G_ABLATE & 2)) {
					// B_PRED: 16 sub-blocks along the 2i+j wavefront (10 steps, <= 2 sub-blocks
					// each), using already reconstructed pixels (reference vp8_recon.c:454-530)
					int16_t* rs = (int16_t*)(wv + kResid);
					if (is_yl) {
						uint4 pk;
						pk.x = (uint32_t)(res[0] & 0xFFFF) | ((uint32_t)res[1] << 16);
						pk.y = (uint32_t)(res[2] & 0xFFFF) | ((uint32_t)res[3] << 16);
						pk.z = (uint32_t)(res[4] & 0xFFFF) | ((uint32_t)res[5] << 16);
						pk.w = (uint32_t)(res[6] & 0xFFFF) | ((uint32_t)res[7] << 16);
						*(uint4*)(wv + kResid + lane * 16) = pk;
					}
					const uint4 bm = *(const uint4*)(A.bmode + m * 16);
					const uint32_t bmw[4] = {(uint32_t)__builtin_amdgcn_readfirstlane((int)bm.x),
					                         (uint32_t)__builtin_amdgcn_readfirstlane((int)bm.y),
					                         (uint32_t)__builtin_amdgcn_readfirstlane((int)bm.z),
					                         (uint32_t)__builtin_amdgcn_readfirstlane((int)bm.w)};
					wave_lds_sync();
					const int g = (lane >> 4) & 1, p = lane & 15;
					uint8_t* edge = wv + kEdge + g * 16;
					for (int s = 0; s < 10; s++) {
						const int ilo = s <= 3 ? 0 : (s - 2) >> 1;
						const int i = ilo + g, j = s - 2 * i;
						const bool valid = lane < 32 && i <= 3 && j >= 0 && j <= 3;
						// (1) gather the 13 edge pixels of each sub-block of this step
						if (valid && p <= 12) {
							const int e = p;
							const uint8_t* srcp;
							if (e < 4) {
								const int yl = 4 * i + 3 - e;
								srcp = (j == 0) ? left + yl : tY + (4 + yl) * 32 + slot * 16 + 4 * j - 1;
							} else if (e == 4) {
								srcp = (i == 0) ? abY + 16 + 4 * j - 1
								                : ((j == 0) ? left + 4 * i - 1 : tY + (3 + 4 * i) * 32 + slot * 16 + 4 * j - 1);
							} else {
								const int k = e - 5;
								if (j == 3 && k >= 4) srcp = abY + 32 + (k - 4);
								else srcp = (i == 0) ? abY + 16 + 4 * j + k : tY + (3 + 4 * i) * 32 + slot * 16 + 4 * j + k;
							}
							edge[e < 4 ? e : (e == 4 ? 7 : e + 3)] = *srcp;
						}
						wave_lds_sync();
						// (2) predict + add residual, one pixel per lane
						if (valid) {
							const uint4 E = *(const uint4*)edge;
							const int b = 4 * i + j;
							const int mode = (int)((bmw[b >> 2] >> (8 * (b & 3))) & 0xFFu);
							const int rr = p >> 2, cc = p & 3;
							int pred;
							if (mode == 0) {
								pred = (int)(bsum4(E.x) + bsum4(E.z) + 4) >> 3;
							} else if (mode == 1) {
								pred = sat8(ubyte(E.x, 3 - rr) + ubyte(E.z, cc) - ubyte(E.y, 3));
							} else if (mode <= 9) {
								const uint32_t t = bptab[mode * 16 + p];
								const int xa = byte16(E.x, E.y, E.z, E.w, (int)(t & 15));
								const int xb = byte16(E.x, E.y, E.z, E.w, (int)((t >> 4) & 15));
								const int xc = byte16(E.x, E.y, E.z, E.w, (int)((t >> 8) & 15));
								const uint32_t kind = t >> 12;
								pred = kind == 0 ? (xa + 2 * xb + xc + 2) >> 2 : (kind == 1 ? (xa + xb + 1) >> 1 : xa);
							} else {
								pred = 128;
							}
							const int rv = rs[b * 16 + p];
							tY[(4 + 4 * i + rr) * 32 + slot * 16 + 4 * j + cc] = (uint8_t)sat8(pred + rv);
						}
						wave_lds_sync();
					}
				}
			}
			wave_lds_sync();

			STAMP(3);
			// ------------------------------------------------ save unfiltered context
			if (!lf_only) {
				if (lane < 4) {  // bottom rows -> ctx_rec[c] for the next MB row
					if (r + 1 < R) {
						const uint8_t* t = lane < 2 ? tY + 19 * 32 + slot * 16 + 8 * lane
						                            : (lane == 2 ? tU : tV) + 11 * 16 + slot * 8;
						const uint32_t o = rec_off(c) + 8 * lane;  // Y 0..15, U 16..23, V 24..31
						ctx.wr(o, ld32(t));
						ctx.wr(o + 4, ld32(t + 4));
					}
				} else if (lane == 4) {  // corner for the next MB
					abY[15] = abY[31];
					abUV[7] = abUV[15];
					abUV[23] = abUV[31];
				} else if (lane >= 32) {  // right column -> left column of the next MB
					const int k = lane - 32;
					if (k < 16) left[k] = tY[(4 + k) * 32 + slot * 16 + 15];
					else if (k < 24) left[k] = tU[(4 + k - 16) * 16 + slot * 8 + 7];
					else left[k] = tV[(4 + k - 24) * 16 + slot * 8 + 7];
				}
			}
			wave_lds_sync();

			STAMP(4);
			// ------------------------------------------------ loop filter MB(r, c)
			if (lf_on && !(VP8G_ABLATE & 1)) {
				const uint8_t* lp = D.lf[seg][bpred ? 1 : 0];
				const int E = lp[0], I = lp[1], T = lp[2];
				if (E != 0) {
					const bool inner = hasc != 0 || bpred;
					// vertical edges: one line per lane along a pixel row (Y 16, U 8, V 8)
					if (lane < 32) {
						const bool isy = lane < 16;
						int px[20];
						if (isy) {
							uint8_t* rowp = tY + (4 + lane) * 32;
#pragma unroll
							for (int k = 0; k < 5; k++) {
								const uint32_t w4 = ld32(rowp + 4 * ((slot * 4 - 1 + k) & 7));
#pragma unroll
								for (int b = 0; b < 4; b++) px[4 * k + b] = ubyte(w4, b);
							}
						} else {
							const int k2 = lane - 16, p = k2 >> 3, row = k2 & 7;
							uint8_t* rowp = (p ? tV : tU) + (4 + row) * 16;
#pragma unroll
							for (int k = 0; k < 3; k++) {
								const uint32_t w4 = ld32(rowp + 4 * ((slot * 2 - 1 + k) & 3));
#pragma unroll
								for (int b = 0; b < 4; b++) px[4 * k + b] = ubyte(w4, b);
							}
#pragma unroll
							for (int k = 12; k < 20; k++) px[k] = 0;
						}
						lf_line(px, simple, c > 0, inner, isy, E, I, T);
						if (isy) {
							uint8_t* rowp = tY + (4 + lane) * 32;
#pragma unroll
							for (int k = 0; k < 5; k++)
								st32(rowp + 4 * ((slot * 4 - 1 + k) & 7), pack4(px[4 * k], px[4 * k + 1], px[4 * k + 2], px[4 * k + 3]));
						} else if (!simple) {
							const int k2 = lane - 16, p = k2 >> 3, row = k2 & 7;
							uint8_t* rowp = (p ? tV : tU) + (4 + row) * 16;
#pragma unroll
							for (int k = 0; k < 3; k++)
								st32(rowp + 4 * ((slot * 2 - 1 + k) & 3), pack4(px[4 * k], px[4 * k + 1], px[4 * k + 2], px[4 * k + 3]));
						}
					}
					wave_lds_sync();
					// horizontal edges: one line per lane down a pixel column
					if (lane < 32) {
						const bool isy = lane < 16;
						int px[20];
						uint8_t* colp;
						int stride;
						if (isy) {
							colp = tY + slot * 16 + lane;
							stride = 32;
						} else {
							const int k2 = lane - 16, p = k2 >> 3;
							colp = (p ? tV : tU) + slot * 8 + (k2 & 7);
							stride = 16;
						}
						const int n = isy ? 20 : 12;
#pragma unroll
						for (int k = 0; k < 20; k++) px[k] = k < n ? (int)colp[k * stride] : 0;
						lf_line(px, simple, r > 0, inner, isy, E, I, T);
						if (isy || !simple) {
#pragma unroll
							for (int k = 1; k < 19; k++)
								if (k < n) colp[k * stride] = (uint8_t)px[k];
						}
					}
					wave_lds_sync();
				}
			}

			STAMP(5);
			// ------------------------------------------------ store final pixels
			// 8-byte chunk store with crop; falls back to bytes at the right edge / misalignment
			auto put8 = [&](uint8_t* plane, uint32_t stride, uint32_t vis_w, uint32_t vis_h, uint32_t row, uint32_t col,
			                uint2 v) {
				if (row >= vis_h || col >= vis_w || (VP8G_ABLATE & 4)) return;
				uint8_t* d = plane + (size_t)row * stride + col;
				const uint32_t n = vis_w - col;
				if (n >= 8 && (((uintptr_t)d) & 7) == 0) {
					*(uint2*)d = v;
				} else {
					const uint32_t cnt = n < 8 ? n : 8;
					for (uint32_t k = 0; k < cnt; k++) d[k] = (uint8_t)(((k < 4 ? v.x : v.y) >> (8 * (k & 3))) & 0xFF);
				}
			};
			if (!lf_on) {
				// unfiltered: MB(r, c) is final as soon as it is reconstructed
				if (lane < 32) {
					const int row = lane >> 1, half = lane & 1;
					put8(outY, sy, W, H, y0 + row, x0 + half * 8, ld64(tY + (4 + row) * 32 + slot * 16 + half * 8));
				} else if (lane < 48) {
					const int k = lane - 32, p = k >> 3, row = k & 7;
					put8(p ? outV : outU, suv, CW, CH, cy0 + row, cx0, ld64((p ? tV : tU) + (4 + row) * 16 + slot * 8));
				}
			} else {
				const bool last_row = r + 1 == R;
				// flush one finished MB column `cc` held in ring slot `sl` (rows 0..11 luma, 0..3
				// chroma final; the bottom 4 rows go to ctx_lf for the row below, or out if last row)
				auto flush_col = [&](uint32_t ccol, int sl) {
					const uint32_t xx = ccol * 16, cxx = ccol * 8;
					if (lane >= 8 && lane < 32) {
						const int k = lane - 8, row = k >> 1, half = k & 1;
						put8(outY, sy, W, H, y0 + row, xx + half * 8, ld64(tY + (4 + row) * 32 + sl * 16 + half * 8));
					} else if (lane >= 32 && lane < 40) {
						const int k = lane - 32, t = k >> 1, half = k & 1;
						const uint2 v2 = ld64(tY + (16 + t) * 32 + sl * 16 + half * 8);
						if (last_row) put8(outY, sy, W, H, y0 + 12 + t, xx + half * 8, v2);
						else {
							const uint32_t o = lf_off(ccol) + t * 16 + half * 8;
							ctx.wr(o, v2.x);
							ctx.wr(o + 4, v2.y);
						}
					} else if (lane >= 48 && lane < 56) {
						const int k = lane - 48, p = k >> 2, t = k & 3;
						put8(p ? outV : outU, suv, CW, CH, cy0 + t, cxx, ld64((p ? tV : tU) + (4 + t) * 16 + sl * 8));
					} else if (lane >= 56) {
						const int k = lane - 56, p = k >> 2, t = k & 3;
						const uint2 v2 = ld64((p ? tV : tU) + (8 + t) * 16 + sl * 8);
						if (last_row) put8(p ? outV : outU, suv, CW, CH, cy0 + 4 + t, cxx, v2);
						else {
							const uint32_t o = lf_off(ccol) + 64 + p * 32 + t * 8;
							ctx.wr(o, v2.x);
							ctx.wr(o + 4, v2.y);
						}
					}
				};
				// rows 12..15 of the MB above are final now (LF(r,c) was their last writer)
				if (r > 0) {
					if (lane < 8) {
						const int t = lane >> 1, half = lane & 1;
						put8(outY, sy, W, H, y0 - 4 + t, x0 + half * 8, ld64(tY + t * 32 + slot * 16 + half * 8));
					} else if (lane >= 40 && lane < 48) {
						const int k = lane - 40, p = k >> 2, t = k & 3;
						put8(p ? outV : outU, suv, CW, CH, cy0 - 4 + t, cx0, ld64((p ? tV : tU) + t * 16 + slot * 8));
					}
				}
				if (c > 0) flush_col(c - 1, slot ^ 1);
				if (c + 1 == C) flush_col(c, slot);
			}
			wave_lds_sync();

			STAMP(6);
			// ------------------------------------------------ publish progress
			ctx.publish_fence();
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			if (lane == 0) __hip_atomic_store(prog + wave, r * C + c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
			STAMP(7);
		}
	}
#ifdef VP8G_STAMPS
	if (lane0 == 0)
		for (int i = 0; i < 8; i++) atomicAdd(&g_vp8g_stamps[i], (unsigned long long)st_acc[i]);
#endif
}

template <int NW, bool kG>
hipError_t launch_t(const Vp8gFrameDesc* d_descs, uint32_t n, const Vp8gBatchArrays& arrays, uint8_t* d_out,
                    uint32_t ctx_cols, uint8_t* gctx, hipStream_t stream) {
	const size_t lds = lds_bytes(NW, ctx_cols, kG);
	auto fn = frame_kernel<NW, kG>;
	if (lds > 65536) {
		hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
		if (e != hipSuccess) return e;
	}
	hipLaunchKernelGGL(fn, dim3(n), dim3(NW * 64), lds, stream, d_descs, arrays, d_out, ctx_cols, gctx);
	return hipGetLastError();
}

}  // namespace

#ifdef VP8G_STAMPS
extern "C" __attribute__((visibility("default"))) int vp8g_debug_stamps(unsigned long long* out, int reset) {
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vp8g_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
	if (reset) {
		unsigned long long z[16] = {0};
		if (hipMemcpyToSymbol(HIP_SYMBOL(g_vp8g_stamps), z, sizeof(z)) != hipSuccess) return -1;
	}
	return 0;
}
#endif

hipError_t launch_frames(const Vp8gFrameDesc* d_descs, uint32_t n_frames, const Vp8gBatchArrays& arrays,
                         uint8_t* d_out, uint32_t ctx_cols, uint32_t max_mb_rows, uint8_t* global_ctx,
                         hipStream_t stream, uint32_t waves_hint) {
	if (n_frames == 0) return hipSuccess;
	static const uint32_t kSupported[] = {1, 2, 4, 8, 12, 16};
	uint32_t want = waves_hint ? waves_hint : 16;
	if (want > max_mb_rows) want = max_mb_rows;  // no point in more waves than MB rows
	uint32_t nw = 1;
	for (uint32_t s : kSupported)
		if (s <= want) nw = s;
	const bool g = global_ctx != nullptr;
#define VP8G_CASE(N)                                                                                         \
	case N:                                                                                                  \
		return g ? launch_t<N, true>(d_descs, n_frames, arrays, d_out, ctx_cols, global_ctx, stream)        \
		         : launch_t<N, false>(d_descs, n_frames, arrays, d_out, ctx_cols, nullptr, stream);
	switch (nw) {
		VP8G_CASE(1)
		VP8G_CASE(2)
		VP8G_CASE(4)
		VP8G_CASE(8)
		VP8G_CASE(12)
		default:
		VP8G_CASE(16)
	}
#undef VP8G_CASE
}

}  // namespace vp8g
