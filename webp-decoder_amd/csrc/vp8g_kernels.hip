// vp8g_kernels.hip -- fused VP8 key-frame reconstruction + loop filter for CDNA4 (gfx950).
//
// Replaces the reference hot path src/m06_recon/vp8_recon.c:423-712 (per-MB dequant, iWHT,
// iDCT, intra prediction, reconstruction, crop) and src/m07_loopfilter/vp8_loopfilter.c:201-283
// (raster-order in-place deblocking), bit-exactly.  Design notes: DESIGN.md §3.
//
// Schedule:
//   * one workgroup = one frame; NW waves; wave w owns MB row PAIRS k = w, w+NW, ...;
//   * a wave works on two macroblocks at once: lanes 0..31 on MB(2k, t), lanes 32..63 on
//     MB(2k+1, t-2) at step t -- the 2-column skew is exactly the VP8 dependency (MB(r,c) needs
//     MB(r,c-1) and MB(r-1,c+1), for intra prediction AND for the raster-order loop filter,
//     SURVEY.md App. B), so the lower half's inputs were finished by the upper half one step
//     earlier in the same wave;
//   * between waves: an LDS progress word per wave (pair*(C+2) + steps done, monotone); the
//     upper half of pair k needs pair k-1's lower half 2 columns ahead of it;
//   * each half reconstructs its MB into a per-half LDS tile and loop-filters it right away;
//     the unfiltered bottom row / right column needed for prediction are saved first (ctx_rec,
//     per column, shared; kLeft, per half) and the bottom 4 rows the next row's top-edge
//     filter still modifies travel through ctx_lf.  Pixels go to HBM once, when final.
// Lane roles inside a half (ln = lane & 31):
//   residual: ln 0..15 = luma block ln, 16..19 = U blocks, 20..23 = V blocks, 24 = Y2; one
//             lane holds a whole 4x4 block (two 16-B loads) and transforms it in registers;
//   loop filter: ln 0..15 = luma rows (V-pass) / columns (H-pass), 16..23 U, 24..31 V;
//   B_PRED: 16 lanes per sub-block, two sub-blocks per step of the 2i+j wavefront.
// All per-pixel arithmetic is branch-free (selects, v_med3, v_sad); the only divergent
// control flow is lane-role selection of addresses.
#include <stdint.h>

#include "vp8g_device.h"

#define DEV __device__ __forceinline__

// Diagnostic builds only (never in the shipped library): VP8G_STAMPS accumulates per-phase
// shader-clock cycles (s_memtime) into g_vp8g_stamps; VP8G_ABLATE skips phases (timing only,
// output wrong): 1 = loop filter, 2 = B_PRED steps, 4 = pixel stores, 8 = dependency wait.
// Wave issue priority per phase (s_setprio 0..3): residual, wait, borders, whole-block
// prediction, B_PRED, loop filter, flush, publish.  Four waves share a SIMD, each in some phase
// of its step: the latency-bound phases (chains of dependent LDS round trips, above all the
// 10-step B_PRED wavefront) issue ahead of the throughput-bound ones (the residual transform
// and the loop filter, long runs of independent VALU), which then fill the gaps.  Measured on
// 512 x 4K (tools/abn.sh, one box): all 0 -> 17.7 ms; B_PRED 2 -> 17.2; this table -> 15.6.
#ifndef VP8G_PRIO_TABLE
#define VP8G_PRIO_TABLE 0, 2, 2, 3, 3, 1, 2, 2
#endif
#ifndef VP8G_PRIO_LF  // loop filter: gather (LDS round trip), edge arithmetic
#define VP8G_PRIO_LF 1, 1
#endif
#ifndef VP8G_PRIO_WHT  // the iWHT's two LDS round trips inside the residual phase
#define VP8G_PRIO_WHT 2
#endif
constexpr int kPrioTab[11] = {VP8G_PRIO_TABLE, VP8G_PRIO_LF, VP8G_PRIO_WHT};
#define PRIO(ph) __builtin_amdgcn_s_setprio(kPrioTab[ph])
// PRIO_AFTER(ph, prev...): PRIO(ph), elided when it would not change the level set by any of the
// phases that can come right before it (7 of the 15 s_setprio per step with the default table)
template <int ph, int... prev>
__device__ __forceinline__ void prio_after() {
	if constexpr (((kPrioTab[ph] != kPrioTab[prev]) || ...)) __builtin_amdgcn_s_setprio(kPrioTab[ph]);
}
#define PRIO_AFTER(ph, ...) prio_after<ph, __VA_ARGS__>()
#ifndef VP8G_ABLATE
#define VP8G_ABLATE 0
#endif
// (Rejected experiments -- their numbers are in DESIGN.md §6 -- were removed in round 5; the shipped
// paths are unconditional now.  The remaining switches are the diagnostics above and below.)
// Bound of one dependency wait in s_memrealtime ticks (100 MHz): 2 s.  Test builds shorten it and
// make one wave never publish its progress (VP8G_TEST_STALL_WAVE) to check that a stalled producer
// ends the launch promptly with VP8G_ERR_TIMEOUT (tests/test_gpu_batch.py).
#ifndef VP8G_WAIT_TICKS
#define VP8G_WAIT_TICKS 200000000ull
#endif
#ifndef VP8G_WAIT_SLEEP  // s_sleep units (64 clocks each) between polls of a dependency wait
#define VP8G_WAIT_SLEEP 1
#endif
#ifndef VP8G_TEST_STALL_WAVE
#define VP8G_TEST_STALL_WAVE (-1)
#endif
#ifdef VP8G_STAMPS
__device__ unsigned long long g_vp8g_stamps[16];
__device__ unsigned long long g_vp8g_wave_times[64];  // frame 0: per wave {start, end} s_memrealtime
__device__ unsigned long long g_vp8g_wave_info[512 * 16 * 2];  // blocks < 512: per wave {HW_ID | XCC_ID << 32, end - start}
#define STAMP(i)                                          \
	do {                                                  \
		const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
		st_acc[i] += t_ - st_prev;                        \
		st_prev = t_;                                     \
	} while (0)
#elif defined(VP8G_MARKS)
#define STAMP(i) asm volatile(";MARK_" #i)  // static per-phase instruction counts (tools/section_counts.py)
#define SUBMARK(i) asm volatile(";MARK_" #i)
#else
#define STAMP(i) \
	do {         \
	} while (0)
#endif
#ifndef SUBMARK
#define SUBMARK(i) \
	do {           \
	} while (0)
#endif

namespace vp8g {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;
constexpr int kBS = 4 * kTP - 8;  // B_PRED: tile offset from sub-block (i, j) to (i + 1, j - 2)  // global-memory vector (never flat)

// ---------------------------------------------------------------------------------------------
// B_PRED predictor table (RFC 6386 12.3; reference vp8_recon.c:218-358).  A lane predicting one
// pixel of a 4x4 sub-block holds the sub-block's edge as 16 bytes E: [0..3] = L0..L3 (left
// column, top down), [4..6] = 128, [7] = P (corner), [8..15] = A0..A7 (above + above-right).
// Every directional mode is avg3(x, y, z) = (x + 2y + z + 2) >> 2 of three edge bytes (avg2(x, y)
// = avg3(x, y, x), a copy = avg3(x, x, x)), so an entry is just three byte positions, stored
// as v_perm selectors (pos & 7) plus a byte mask picking the high half (pos >= 8) of E: one
// perm pair + one bfi fetches all three, one signed v_dot4 over the bytes biased by -128 weighs
// them (avg3 weights (1, 2, 1); TM_PRED = sat8(L + A - P) is the same dot with weights
// (1, -1, 1) over the positions (L_r, P, A_c)); DC_PRED is a direct sum.
// Entry kBpModes-1 (all positions 128) serves out-of-range modes.
// Edge index notation of the builders: 0..3 = L3..L0, 4 = P, 5..12 = A0..A7.
// ---------------------------------------------------------------------------------------------
struct BpTab {
	uint32_t v[kBpModes * 16 * (kBpEntry / 4)];
};
constexpr int epos(int e) { return e < 4 ? 3 - e : (e == 4 ? 7 : e + 3); }
struct Tri {
	int a, b, c;  // byte positions in E
};
constexpr Tri A3(int a, int b, int c) { return Tri{epos(a), epos(b), epos(c)}; }
constexpr Tri A2(int a, int b) { return Tri{epos(a), epos(b), epos(a)}; }
constexpr Tri CP(int a) { return Tri{epos(a), epos(a), epos(a)}; }

constexpr BpTab make_bptab() {
	BpTab t{};
	const Tri vr[16] = {A2(4, 5), A2(5, 6), A2(6, 7), A2(7, 8), A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7), A3(6, 7, 8),
	                    A3(2, 3, 4), A2(4, 5), A2(5, 6), A2(6, 7), A3(1, 2, 3), A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7)};
	const Tri vl[16] = {A2(5, 6), A2(6, 7), A2(7, 8), A2(8, 9), A3(5, 6, 7), A3(6, 7, 8), A3(7, 8, 9), A3(8, 9, 10),
	                    A2(6, 7), A2(7, 8), A2(8, 9), A3(9, 10, 11), A3(6, 7, 8), A3(7, 8, 9), A3(8, 9, 10), A3(10, 11, 12)};
	const Tri hd[16] = {A2(3, 4), A3(3, 4, 5), A3(4, 5, 6), A3(5, 6, 7), A2(2, 3), A3(2, 3, 4), A2(3, 4), A3(3, 4, 5),
	                    A2(1, 2), A3(1, 2, 3), A2(2, 3), A3(2, 3, 4), A2(0, 1), A3(0, 1, 2), A2(1, 2), A3(1, 2, 3)};
	const Tri hu[16] = {A2(3, 2), A3(3, 2, 1), A2(2, 1), A3(2, 1, 0), A2(2, 1), A3(2, 1, 0), A2(1, 0), A3(1, 0, 0),
	                    A2(1, 0), A3(1, 0, 0), CP(0), CP(0), CP(0), CP(0), CP(0), CP(0)};
	for (int m = 0; m < kBpModes; m++)
		for (int p = 0; p < 16; p++) {
			const int r = p >> 2, c = p & 3;
			Tri e{4, 4, 4};  // 128 (DC_PRED is computed directly; out-of-range modes)
			switch (m) {
				case 1: e = Tri{r, 7, 8 + c}; break;                                      // B_TM: L_r, P, A_c
				case 2: e = A3(4 + c, 5 + c, 6 + c); break;                               // B_VE
				case 3: e = r == 3 ? A3(1, 0, 0) : A3(4 - r, 3 - r, 2 - r); break;        // B_HE
				case 4: e = A3(5 + r + c, 6 + r + c, (7 + r + c) > 12 ? 12 : (7 + r + c)); break;  // B_LD
				case 5: e = A3(3 - r + c, 4 - r + c, 5 - r + c); break;                   // B_RD
				case 6: e = vr[p]; break;
				case 7: e = vl[p]; break;
				case 8: e = hd[p]; break;
				case 9: e = hu[p]; break;
				default: break;
			}
			const int pos[3] = {e.a, e.b, e.c};
			uint32_t sel = 12u << 24, mask = 0;  // byte 3: constant 0
			for (int k = 0; k < 3; k++) {
				sel |= (uint32_t)(pos[k] & 7) << (8 * k);
				if (pos[k] >= 8) mask |= 0xFFu << (8 * k);
			}
			// weights (signed bytes) and bias / shift of the one dot-product formula:
			// value = (sdot4(E_xyz - 128, w) + bias) >> sh  (avg3: (1, 2, 1), 514, 2; TM: (1, -1, 1), 128, 0)
			const bool tm = m == 1;
			t.v[(m * 16 + p) * 4] = sel;
			t.v[(m * 16 + p) * 4 + 1] = mask | ((tm ? 0u : 2u) << 24);  // byte 3: the shift (x3's byte 3 is unused)
			t.v[(m * 16 + p) * 4 + 2] = tm ? 0x0001FF01u : 0x00010201u;
			t.v[(m * 16 + p) * 4 + 3] = tm ? 128u : 514u;
		}
	return t;
}
__constant__ BpTab kBpTab = make_bptab();

// Border setup roles of lanes 0..19 (see "borders"): dst offset in the half area [11:0], source
// offset in the unfiltered context row [19:12], kind [21:20] (0 above, 1 left fill, 2 corner).
struct BorderTab {
	uint32_t v[32];
};
constexpr uint32_t BE(int dst, int src, int kind) { return (uint32_t)dst | ((uint32_t)src << 12) | ((uint32_t)kind << 20); }
constexpr BorderTab make_bordertab() {
	BorderTab t{};
	for (int ln = 0; ln < 32; ln++) {
		if (ln < 4) t.v[ln] = BE(kAbY + 16 + 4 * ln, 4 * ln, 0);
		else if (ln == 4) t.v[ln] = BE(kAbY + 32, 0, 0);
		else if (ln < 9) {
			const int q = ln - 5;
			t.v[ln] = BE(kAbUV + 8 + 16 * (q >> 1) + 4 * (q & 1), 16 + 8 * (q >> 1) + 4 * (q & 1), 0);
		} else if (ln < 17) t.v[ln] = BE(kLeft + 4 * (ln - 9), 0, 1);
		else if (ln == 17) t.v[ln] = BE(kAbY + 12, 19, 2);  // corner P from the old abY[31]
		else if (ln < 20) t.v[ln] = BE(kAbUV + 4 + 16 * (ln - 18), 11, 2);  // from abUV[15] / abUV[31]
		else {
			// ln 20..31: copy of the MB above's filter-state rows (ctx_lf) into the tile -- luma rows
			// 0..3 (ln 20..23, 16 B, bit 22) or U / V rows 0..3 (8 B): tile offset at slot 0 (slot 1:
			// +16 / +8), source offset in the context column
			const bool ly = ln < 24;
			const int tr = ly ? ln - 20 : (ln - 24) & 3, p = (ln - 24) >> 2;
			t.v[ln] = BE(ly ? kLfY + tr * kTP : kLfUV + p * kCV + tr * kTP, kCtxRecBytes + (ly ? tr * 16 : 64 + p * 32 + tr * 8), 3) |
			          (ly ? 1u << 22 : 0u);
		}
	}
	return t;
}
__constant__ BorderTab kBorderTab = make_bordertab();

// Whole-block predictor roles of lanes 0..23 (offsets from the half's area):
// v[2 ln] = above-row base | own above word << 11 | is-luma << 22 | last block row << 23 | last
// block column << 24 | offset in the ctx_rec column << 25; v[2 ln + 1] = left-column base |
// destination in the tile at slot 0 << 11 | block row << 22.
struct PredRoleTab {
	uint32_t v[64];
};
constexpr PredRoleTab make_predroletab() {
	PredRoleTab t{};
	for (int ln = 0; ln < 24; ln++) {
		const bool yl = ln < 16;
		const int p = yl ? 0 : (ln - 16) >> 2;
		const int blk = yl ? ln : (ln & 3);
		const int bx = yl ? (blk & 3) : (blk & 1), by = yl ? (blk >> 2) : (blk >> 1);
		const int ab = yl ? kAbY + 16 : kAbUV + 16 * p + 8;
		const int lc = yl ? kLeft : kLeft + 16 + 8 * p;
		const int dst = yl ? kLfY + (4 + 4 * by) * kTP + 4 * bx : kLfUV + p * kCV + (4 + 4 * by) * kTP + 4 * bx;
		const int rec = yl ? 4 * bx : 16 + 8 * p + 4 * bx;
		const int last = yl ? 3 : 1;
		t.v[2 * ln] = (uint32_t)ab | ((uint32_t)(ab + 4 * bx) << 11) | ((yl ? 1u : 0u) << 22) | ((by == last ? 1u : 0u) << 23) |
		              ((bx == last ? 1u : 0u) << 24) | ((uint32_t)rec << 25);
		t.v[2 * ln + 1] = (uint32_t)lc | ((uint32_t)dst << 11) | ((uint32_t)by << 22);
	}
	return t;
}
__constant__ PredRoleTab kPredRoleTab = make_predroletab();
static_assert(kLeft + 32 < 2048 && kAbUV + 40 < 2048 && kLfUV + kCV + 20 * kTP < 2048, "11-bit role offsets");


// ---------------------------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------------------------
// Intra-wave LDS ordering: a wave's LDS instructions execute in issue order, so only the
// compiler must be kept from reordering / caching across this point.
DEV void wave_lds_sync() { asm volatile("" ::: "memory"); }

DEV int sx16(int x) { return (int)(int16_t)x; }
DEV int sat8(int v) { return min(max(v, 0), 255); }  // v_med3_i32
DEV int sclamp(int v) { return min(max(v, -128), 127); }
// sclamp(sclamp(x) + k) >> 3 for k = 3, 4 (RFC 15.2 common_adjust), as one v_med3 with inline
// bounds after the shift: both forms give (x + k) >> 3 clamped to [-16, 15]
DEV int fshift(int x, int k) { return min(max((x + k) >> 3, -16), 15); }
DEV int ad(int a, int b) { return (int)__builtin_amdgcn_sad_u16((uint32_t)a, (uint32_t)b, 0u); }  // |a-b| for 0 <= a,b < 65536
DEV int max3i(int a, int b, int c) { return max(a, max(b, c)); }
// v_max3_u32 pinned (the compiler re-associates max chains into more two-input maxes)
DEV int max3u(int a, int b, int c) {
	int r;
	asm("v_max3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
	return r;
}
DEV int mul_s(int x) { return (x * 35468) >> 16; }        // x*sqrt(2)*sin(pi/8), RFC 14.4
DEV int mul_c(int x) { return x + ((x * 20091) >> 16); }  // x*sqrt(2)*cos(pi/8)
DEV uint32_t bsum4(uint32_t w) { return __builtin_amdgcn_sad_u8(w, 0u, 0u); }
DEV uint32_t ld32(const uint8_t* p) { return *(const uint32_t*)p; }
DEV void st32(uint8_t* p, uint32_t v) { *(uint32_t*)p = v; }
DEV u32x2 ld64(const uint8_t* p) { return *(const u32x2*)p; }
DEV void st64(uint8_t* p, u32x2 v) { *(u32x2*)p = v; }
// a chroma tile 8-B piece (4-B aligned unless kC8)
DEV u32x2 ldc64(const uint8_t* p) {
	if constexpr (kC8) return ld64(p);
	else return u32x2{ld32(p), ld32(p + 4)};
}
DEV void stc64(uint8_t* p, u32x2 v) {
	if constexpr (kC8) st64(p, v);
	else st32(p, v.x), st32(p + 4, v.y);
}
DEV u32x4 ld128(const uint8_t* p) { return *(const u32x4*)p; }
DEV void st128(uint8_t* p, u32x4 v) { *(u32x4*)p = v; }
DEV uint32_t pack4(int a, int b, int c, int d) {
	return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}
// four bytes (each < 256) into a dword: three dependent v_lshl_or_b32 (asm: the compiler's own
// form of pack4 takes about five instructions)
DEV uint32_t pack4b(int a, int b, int c, int d) {
	uint32_t r0, r1, r2;
	asm("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(r0) : "v"(b), "v"(a));
	asm("v_lshl_or_b32 %0, %1, 16, %2" : "=v"(r1) : "v"(c), "v"(r0));
	asm("v_lshl_or_b32 %0, %1, 24, %2" : "=v"(r2) : "v"(d), "v"(r1));
	return r2;
}
DEV int ubyte(uint32_t w, int i) { return (int)((w >> (8 * i)) & 0xFFu); }
DEV uint32_t lo16(int a, int b) { return (uint32_t)(a & 0xFFFF) | ((uint32_t)b << 16); }
// packed int16 pairs (wrapping, as the reference's int16 stores)
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
DEV u16x2 as_p(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
DEV uint32_t as_w(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
DEV uint32_t pk_add(uint32_t a, uint32_t b) { return as_w(as_p(a) + as_p(b)); }
DEV uint32_t pk_sub(uint32_t a, uint32_t b) { return as_w(as_p(a) - as_p(b)); }
DEV uint32_t pk_mul(uint32_t a, uint32_t b) { return as_w(as_p(a) * as_p(b)); }
typedef int16_t s16x2 __attribute__((ext_vector_type(2)));
DEV uint32_t pk_clamp255(uint32_t x) {  // each int16 half clamped to [0, 255] (v_pk_max_i16 + v_pk_min_i16)
	s16x2 v = __builtin_bit_cast(s16x2, x);
	v = __builtin_elementwise_min(__builtin_elementwise_max(v, s16x2{0, 0}), s16x2{255, 255});
	return __builtin_bit_cast(uint32_t, v);
}
// both int16 halves of x saturated to u8, in bytes 0 / 1 (v_sat_pk_u8_i16, one VOP1 instead of the
// v_pk_max_i16 + v_pk_min_i16 clamp and a byte-gathering v_perm)
DEV uint32_t sat_pk(uint32_t x) {
	uint32_t r;
	asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(x));
	return r;
}
DEV int lo_s16(uint32_t x) { return (int)(int16_t)(x & 0xFFFFu); }
DEV int hi_s16(uint32_t x) { return (int)(int16_t)(x >> 16); }
DEV uint32_t pack2(int a, int b) { return __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x05040100u); }
// floor(x * c / 65536) of each int16 half
DEV uint32_t mulhi2(uint32_t x, int c) {
	return __builtin_amdgcn_perm((uint32_t)(hi_s16(x) * c), (uint32_t)(lo_s16(x) * c), 0x07060302u);
}
DEV uint32_t mul_s2(uint32_t x) { return pk_add(x, mulhi2(x, 35468 - 65536)); }  // mul_s of both halves, mod 2^16
DEV uint32_t mul_c2(uint32_t x) { return pk_add(x, mulhi2(x, 20091)); }
// c ? a : b per lane, as two v_cndmask (opaque to the optimiser)
DEV uint64_t vsel(bool c, uint64_t a, uint64_t b) {
	const uint64_t mk = __builtin_amdgcn_ballot_w64(c);
	uint32_t lo, hi;
	asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(lo) : "v"((uint32_t)b), "v"((uint32_t)a), "s"(mk));
	asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(b >> 32)), "v"((uint32_t)(a >> 32)), "s"(mk));
	return ((uint64_t)hi << 32) | lo;
}
// Output stores through buffer resources.  A lane with nothing to store this round passes
// kNoStore, an offset past the end of the plane, and the hardware's range check drops it: the
// store instructions of a step are then issued on every path.  (Stores behind a branch would make
// the compiler's vmcnt bookkeeping assume a path without stores, and the next step's wait for its
// prefetched coefficients -- loaded before these stores -- would also wait for every store of this
// step to be acknowledged: a full drain of the store queue per step, ~10 % of the kernel time.)
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr uint32_t kNoStore = 0x80000000u;
constexpr uint32_t kFlCtxBias = 512u;  // (fast flush: keeps the per-lane ctx_lf offsets non-negative)
DEV Rsrc plane_rsrc(uint8_t* base, uint32_t bytes) {
	// (inputs laundered through readfirstlane: built inside the chain's frame loop, the resource was
	// otherwise kept in VGPRs and every store became a waterfall loop)
	const uint64_t b = (uint64_t)(uintptr_t)base;
	const uint64_t bu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
	                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
	return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)bu, (short)0, __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}
// Cache policy of the output pixel stores: sc1, write-through.  A 128-B output line collects its
// 16-B (luma) / 8-B (chroma) row pieces over 8 / 16 MB steps; stored plainly, the partial lines sat
// dirty in the XCD's L2 (4 MB: about the launch's whole in-flight set), were evicted half written
// and refilled (3x the algorithmic write bytes).  sc1 stores leave L2 at once and
// drop the line, so they neither occupy L2 nor need a refill (A/B uhd4 -1.5 %, fhd4 -2.4 %,
// byte-identical; `nt` stores, which keep the line, were +120 %).
#ifndef VP8G_STORE_AUX
#define VP8G_STORE_AUX 16
#endif
constexpr int kCpolSc1 = 16;   // cache-policy bits of a buffer access: sc1 (device-coherent, bypasses the CU's L1)
constexpr int kSnapBatch = 8;  // mirror split: 16-B snapshot loads per lane in flight
DEV void bst128(Rsrc r, uint32_t off, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, VP8G_STORE_AUX); }
DEV void bst64(Rsrc r, uint32_t off, u32x2 v) { __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, VP8G_STORE_AUX); }

// single-byte LDS access that the load/store vectoriser leaves alone
DEV int ldb(const uint8_t* p) { return (int)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT); }
DEV void stb(uint8_t* p, int v) { __hip_atomic_store(p, (uint8_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT); }
DEV int rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Per-frame context (unfiltered bottom rows + filter-state bottom rows per MB column), in LDS
// or, for frames too wide for LDS, in device memory (read with L1-bypassing loads).
template <bool kG>
struct Ctx {
	uint8_t* lds;
	uint8_t* g;
	DEV uint32_t rd(uint32_t off) const {
		if constexpr (kG) return __hip_atomic_load((uint32_t*)(g + off), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		else return ld32(lds + off);
	}
	DEV u32x2 rd64(uint32_t off) const {
		if constexpr (kG) return u32x2{rd(off), rd(off + 4)};
		else return ld64(lds + off);
	}
	DEV u32x4 rd128(uint32_t off) const {
		if constexpr (kG) return u32x4{rd(off), rd(off + 4), rd(off + 8), rd(off + 12)};
		else return ld128(lds + off);
	}
	DEV void wr8(uint32_t off, uint32_t v) const {
		if constexpr (kG) g[off] = (uint8_t)v;
		else lds[off] = (uint8_t)v;
	}
	DEV void wr32(uint32_t off, uint32_t v) const {
		if constexpr (kG) *(uint32_t*)(g + off) = v;
		else st32(lds + off, v);
	}
	DEV void wr64(uint32_t off, u32x2 v) const {
		if constexpr (kG) *(u32x2*)(g + off) = v;
		else st64(lds + off, v);
	}
	DEV void wr128(uint32_t off, u32x4 v) const {
		if constexpr (kG) *(u32x4*)(g + off) = v;
		else st128(lds + off, v);
	}
	DEV void publish_fence() const {
		if constexpr (kG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	}
};
// (24-bit multiplies: v_mul_lo_u32 is a quarter-rate instruction; all operands here are < 2^24)
DEV uint32_t rec_off(uint32_t c) { return __umul24(c, (uint32_t)kCtxBytesPerCol); }
DEV uint32_t lf_off(uint32_t c) { return __umul24(c, (uint32_t)kCtxBytesPerCol) + kCtxRecBytes; }

// ---------------------------------------------------------------------------------------------
// Loop filter on a line of pixels (RFC 6386 15.2-15.4; reference vp8_loopfilter.c:24-164),
// branch-free, on unpacked bytes: a line is px[0..19] = the neighbour's last 4 pixels (left or
// above) and this MB's 16 (chroma: 8); the edge at 4j (j = 1 MB edge, 2..4 sub-block edges) has
// p3..p0 = px[4j-4..4j-1], q0..q3 = px[4j..4j+3].  Lines are gathered / scattered with LDS byte
// loads and stores at immediate offsets, so no vector instruction is spent on (un)packing.
// ---------------------------------------------------------------------------------------------
// normal-filter edge mask (RFC 15.3 filter_yes + interior limits) and high-edge-variance
DEV void edge_mask(const int* x, bool en, int lim, int I, int T, bool& m, bool& hev) {
	const int hm = max(ad(x[2], x[3]), ad(x[5], x[4]));  // max(|p1-p0|, |q1-q0|), shared with hev
	const int interior = max3u(max3u(ad(x[0], x[1]), ad(x[1], x[2]), ad(x[7], x[6])), ad(x[6], x[5]), hm);
	const bool fy = ad(x[3], x[4]) * 2 + (ad(x[2], x[5]) >> 1) <= lim;
	m = en & fy & (interior <= I);
	hev = hm > T;
}

// m ? v : 0 (the compiler makes it an exec-masked branch around the filter arithmetic; a forced
// v_cndmask select measured +0.5...+1.8 %)
DEV int sel0(bool m, int v) { return m ? v : 0; }

// Masking: the filter input (the common-adjust value) is zeroed where the edge mask is off, which
// makes every tap 0 ((0 + 4) >> 3 = (0 + 3) >> 3 = (0 + 63) >> 7 = 0), so one select per edge
// replaces one per delta and the pixel updates sat8(pixel +- delta) run unconditionally.
DEV void lf_mb_edge(int* x, bool en, int lim, int I, int T) {  // normal, MB edge
	bool m, hev;
	edge_mask(x, en, lim, I, T, m, hev);
	const int p2 = x[1], p1 = x[2], p0 = x[3], q0 = x[4], q1 = x[5], q2 = x[6];
	const int w = sclamp(sel0(m, sclamp(p1 - q1) + __mul24(q0 - p0, 3)));
	const int f1 = sclamp(w + 4) >> 3, f2 = sclamp(w + 3) >> 3;
	const int a27 = (27 * w + 63) >> 7, a18 = (18 * w + 63) >> 7, a9 = (9 * w + 63) >> 7;
	const int d0p = hev ? f2 : a27, d0q = hev ? f1 : a27;
	const int d1 = hev ? 0 : a18, d2 = hev ? 0 : a9;
	x[3] = sat8(p0 + d0p);
	x[4] = sat8(q0 - d0q);
	x[2] = sat8(p1 + d1);
	x[5] = sat8(q1 - d1);
	x[1] = sat8(p2 + d2);
	x[6] = sat8(q2 - d2);
}

DEV void lf_sub_edge(int* x, bool en, int lim, int I, int T) {  // normal, sub-block edge
	bool m, hev;
	edge_mask(x, en, lim, I, T, m, hev);
	const int p1 = x[2], p0 = x[3], q0 = x[4], q1 = x[5];
	const int a = sel0(m, __mul24(q0 - p0, 3) + (hev ? sclamp(p1 - q1) : 0));
	const int f1 = fshift(a, 4), f2 = fshift(a, 3);
	const int a2 = hev ? 0 : (f1 + 1) >> 1;
	x[4] = sat8(q0 - f1);
	x[3] = sat8(p0 + f2);
	x[5] = sat8(q1 - a2);
	x[2] = sat8(p1 + a2);
}

DEV void lf_simple_edge(int* x, bool en, int lim) {  // simple filter (luma only)
	const int p1 = x[2], p0 = x[3], q0 = x[4], q1 = x[5];
	const bool m = en & (ad(p0, q0) * 2 + (ad(p1, q1) >> 1) <= lim);
	const int a = sclamp(p1 - q1) + __mul24(q0 - p0, 3);  // (branched over where no lane filters)
	x[4] = m ? sat8(q0 - fshift(a, 4)) : q0;
	x[3] = m ? sat8(p0 + fshift(a, 3)) : p0;
}

// All edges of one line, in the reference order (MB edge, then sub-block edges).  `is_y`
// enables the luma-only edges at 12 and 16; chroma has its single inner edge at 8.
template <bool kSimple>
DEV void lf_line(int* px, bool mb_edge, bool inner, bool is_y, int E, int I, int T) {
	if constexpr (kSimple) {
		lf_simple_edge(px + 0, mb_edge & is_y, (E + 2) * 2 + I);
		lf_simple_edge(px + 4, inner & is_y, E * 2 + I);
		lf_simple_edge(px + 8, inner & is_y, E * 2 + I);
		lf_simple_edge(px + 12, inner & is_y, E * 2 + I);
	} else {
		lf_mb_edge(px + 0, mb_edge, 2 * (E + 2) + I, I, T);
		lf_sub_edge(px + 4, inner, 2 * E + I, I, T);
		lf_sub_edge(px + 8, inner & is_y, 2 * E + I, I, T);
		lf_sub_edge(px + 12, inner & is_y, 2 * E + I, I, T);
	}
}

// Gather 20 bytes from LDS into 20 VGPRs: px[0..3] = a[0..3], px[4..19] = b[o .. o + 15*st] (byte
// loads at immediate offsets in one asm block that ends with its own lgkmcnt wait; separate C++
// loads get merged into wide loads plus unpacking, or carry a zero-extension per byte)
template <int kA, int kB>  // byte pitch of the a-run and the b-run
DEV void gather20(const uint8_t* a, const uint8_t* b, int* px) {
	const uint32_t la = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)a;
	const uint32_t lb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)b;
#define G1(i, base, off) "ds_read_u8 %" #i ", %" base " offset:" #off "\n"
	asm volatile(
	    "ds_read_u8 %0, %20\n"
	    "ds_read_u8 %1, %20 offset:%22\n"
	    "ds_read_u8 %2, %20 offset:%23\n"
	    "ds_read_u8 %3, %20 offset:%24\n"
	    "ds_read_u8 %4, %21\n"
	    "ds_read_u8 %5, %21 offset:%25\n"
	    "ds_read_u8 %6, %21 offset:%26\n"
	    "ds_read_u8 %7, %21 offset:%27\n"
	    "ds_read_u8 %8, %21 offset:%28\n"
	    "ds_read_u8 %9, %21 offset:%29\n"
	    "ds_read_u8 %10, %21 offset:%30\n"
	    "ds_read_u8 %11, %21 offset:%31\n"
	    "ds_read_u8 %12, %21 offset:%32\n"
	    "ds_read_u8 %13, %21 offset:%33\n"
	    "ds_read_u8 %14, %21 offset:%34\n"
	    "ds_read_u8 %15, %21 offset:%35\n"
	    "ds_read_u8 %16, %21 offset:%36\n"
	    "ds_read_u8 %17, %21 offset:%37\n"
	    "ds_read_u8 %18, %21 offset:%38\n"
	    "ds_read_u8 %19, %21 offset:%39\n"
	    "s_waitcnt lgkmcnt(0)"
	    : "=&v"(px[0]), "=&v"(px[1]), "=&v"(px[2]), "=&v"(px[3]), "=&v"(px[4]), "=&v"(px[5]), "=&v"(px[6]),
	      "=&v"(px[7]), "=&v"(px[8]), "=&v"(px[9]), "=&v"(px[10]), "=&v"(px[11]), "=&v"(px[12]), "=&v"(px[13]),
	      "=&v"(px[14]), "=&v"(px[15]), "=&v"(px[16]), "=&v"(px[17]), "=&v"(px[18]), "=&v"(px[19])
	    : "v"(la), "v"(lb), "i"(kA), "i"(2 * kA), "i"(3 * kA), "i"(kB), "i"(2 * kB), "i"(3 * kB), "i"(4 * kB),
	      "i"(5 * kB), "i"(6 * kB), "i"(7 * kB), "i"(8 * kB), "i"(9 * kB), "i"(10 * kB), "i"(11 * kB), "i"(12 * kB),
	      "i"(13 * kB), "i"(14 * kB), "i"(15 * kB)
	    : "memory");
#undef G1
#pragma unroll
	for (int i = 0; i < 20; i++) __builtin_assume((uint32_t)px[i] < 256u);  // bytes: lets 24-bit multiplies through
}

// Both passes of the loop filter over this lane's line of the MB held in LDS.  Lanes 0..15:
// luma rows / columns; 16..23 U, 24..31 V.  Bytes that may change: 1..17 (luma), 1..9 (chroma).
// The line addresses of a lane: Lp / Mp the left neighbour's 4 pixels / this MB's pixels of its
// row (vertical-edge pass), colp the top of its column (horizontal-edge pass, tile row 0).
struct LfLine {
	uint8_t* Lp;
	uint8_t* Mp;
	uint8_t* colp;
};
template <bool kSimple>
DEV void lf_mb(const LfLine& L, int ln, bool en, bool mb_v, bool mb_h, bool inner, int E, int I, int T) {
	const bool isy = ln < 16;
	const bool wr = en && (isy || !kSimple);
	int px[20];
	// vertical edges: one line per lane along a pixel row; the neighbour's 4 pixels sit at the
	// other end of the 2-MB ring when slot == 0
	{
		// (ldb/stb: relaxed wave-scope atomics keep the byte accesses single ds_read_u8 /
		// ds_write_b8 -- merged wide accesses cost vector instructions to (un)pack)
		uint8_t* const Lp = L.Lp;
		uint8_t* const Mp = L.Mp;
		PRIO_AFTER(8, 5);
		gather20<1, 1>(Lp, Mp, px);
		PRIO_AFTER(9, 8);
		lf_line<kSimple>(px, en && mb_v, en && inner, isy, E, I, T);
		// the row written back as dwords -- bytes the filter leaves alone are rewritten unchanged;
		// 3 / 5 LDS stores instead of 9 / 17 byte stores, for ~15 packing instructions
		if (wr) {
			st32(Lp, pack4b(px[0], px[1], px[2], px[3]));
			st32(Mp, pack4b(px[4], px[5], px[6], px[7]));
			st32(Mp + 4, pack4b(px[8], px[9], px[10], px[11]));
			if (isy) {
				st32(Mp + 8, pack4b(px[12], px[13], px[14], px[15]));
				st32(Mp + 12, pack4b(px[16], px[17], px[18], px[19]));
			}
		}
	}
	wave_lds_sync();
	// horizontal edges: one line per lane down a pixel column (tile rows 0..19, pitch kTP)
	{
		uint8_t* const colp = L.colp;
		PRIO_AFTER(8, 9);
		gather20<kTP, kTP>(colp, colp + 4 * kTP, px);
		PRIO_AFTER(9, 8);
		lf_line<kSimple>(px, en && mb_h, en && inner, isy, E, I, T);
		if (wr) {
#pragma unroll
			for (int i = 1; i < 10; i++) stb(colp + kTP * i, px[i]);
			if (isy) {
#pragma unroll
				for (int i = 10; i < 18; i++) stb(colp + kTP * i, px[i]);
			}
		}
	}
	wave_lds_sync();
}

// one lane's 32 bytes of coefficients (or side info) for the next step
struct Pref {
	u32x4 a, b;
	uint32_t side;
};

// ---------------------------------------------------------------------------------------------
// The fused kernel.
// ---------------------------------------------------------------------------------------------
// Occupancy target: two workgroups (frames) per CU at NW <= 8 (2*NW waves per CU); one
// workgroup of 12 or 16 waves per CU for batches smaller than the CU count (pick_waves).  Either
// way at most 4 waves per SIMD, i.e. the full 128-VGPR budget.
template <int NW>
constexpr int min_waves_per_simd() {
	return NW >= 6 ? 4 : (NW >= 2 ? (2 * NW) / 4 : 1);
}

// Split mode (kS, small batches): a frame's MB row pairs are dealt over `nsplit` workgroups
// ("parts") of NW waves each -- global wave g = part * NW + wave owns pairs g, g + nsplit*NW, ...
// Inside a part the waves hand off through LDS as above.  Across parts (wave 0 of part j waits on
// wave NW-1 of part j-1) the hand-off is a mailbox in device memory, one channel per part, laid
// out like ctx (rec + lf per column): the producer copies each column's finished ctx entry with
// write-through (sc1) stores, drains them (vmcnt(0)) and then stores its progress word with an
// agent-scope atomic; the consumer polls that word and reads the mailbox with sc1 loads, one step
// ahead of use (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 payload + drained flag).
// Requires every part of a frame to be resident at once: the host splits only batches of at most
// one part per CU.
// The frame workgroup blockIdx.x decodes under the cost-balanced launch order (pick_order in
// vp8g_device.h): the position p of this workgroup in the sorted batch, then the frame at that
// position -- a histogram of the n frames' cost classes gives p's class c and its rank r among
// the frames of class c, and a block-wide ballot scan over the frames finds the r-th frame of
// class c in index order (a stable sort, without sorting).  Runs before the workgroup's LDS is
// initialised and uses its first bytes as scratch; ends with a barrier.
template <int NT>
DEV uint32_t ordered_frame(const Vp8gFrameDesc* descs, uint32_t n, uint32_t F, uint8_t* scratch) {
	uint32_t* const hist = (uint32_t*)scratch;          // kCostClasses words
	uint32_t* const wcnt = hist + kCostClasses;          // NT / 64 words
	uint32_t* const found = wcnt + NT / 64;
	const uint32_t tid = threadIdx.x, w = blockIdx.x;
	const uint32_t S = min(n - F, F);
	// the first F workgroups take the F heaviest frames, the next S the S lightest (lightest first,
	// so the heaviest frame shares its CU with the lightest), the rest the middle, heaviest first
	const uint32_t p = w < F ? w : (w < F + S ? n - 1u - (w - F) : w - S);
	for (uint32_t i = tid; i < kCostClasses; i += NT) hist[i] = 0u;
	if (tid == 0) *found = w < n ? w : 0u;  // (every position is matched; this only keeps the read defined)
	__syncthreads();
	for (uint32_t i = tid; i < n; i += NT) atomicAdd(&hist[cost_class(descs[i])], 1u);
	__syncthreads();
	uint32_t acc = 0, cls = 0, r = 0;
	for (int c = (int)kCostClasses - 1; c >= 0; c--) {  // descending cost
		const uint32_t h = hist[c];
		if (p >= acc && p < acc + h) cls = (uint32_t)c, r = p - acc;
		acc += h;
	}
	const int wv = (int)(tid >> 6), lane = (int)(tid & 63);
	uint32_t base = 0;  // frames of class cls before this chunk (block-uniform)
	for (uint32_t c0 = 0; c0 < n; c0 += NT) {
		const uint32_t i = c0 + tid;
		const bool m = i < n && cost_class(descs[i]) == cls;
		const uint64_t b = __ballot(m);
		if (lane == 0) wcnt[wv] = (uint32_t)__popcll(b);
		__syncthreads();
		uint32_t off = base, tot = 0;
		for (int q = 0; q < NT / 64; q++) {
			const uint32_t cq = wcnt[q];
			off += q < wv ? cq : 0u;
			tot += cq;
		}
		if (m && off + (uint32_t)__popcll(b & ((1ull << lane) - 1ull)) == r) *found = i;
		__syncthreads();
		base += tot;
		if (base > r) break;
	}
	const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane((int)*found);
	__syncthreads();
	return f;
}

// Chain mode (kC, batches with more frames than CUs): ONE workgroup of NW = 16 waves per CU
// decodes a list of frames as one continuous chain of MB row pairs -- global pair g of the list
// (the frames' pairs one after another) belongs to wave g % NW -- so no wave idles at a frame's
// end while another frame of the CU still has rows, and a heavy frame never runs alone on half
// the CU.  Two frames are in flight at once: frame j of the list uses LDS slot j & 1 (its
// per-column context and its dequant / loop-filter tables); pair 0 of frame j waits until frame
// j - 2, the slot's previous user, has finished its last pair (which implies all of its pairs:
// pair k's last steps wait for pair k - 1 to complete).  The list of workgroup b: the frames at
// positions b, 2W-1-b, 2W+b, 4W-1-b, ... of the batch sorted by descending cost class (snake
// order: every CU gets one of the heaviest and one of the lightest frames per two rounds), sorted
// in the prologue by wave 0 (stable counting sort over the cost classes in LDS scratch).
// Progress words encode global pair * 2048 + steps done (C <= 1024, so steps <= 1026).
constexpr uint32_t kProgShift = 11;
// Mirror split (launch_chain with split, batches of at most two frames per workgroup): each frame is
// cut at pair h = ceil(pairs / 2) into a top segment (pairs [0, h), decoded by the frame's own
// workgroup, first in its list) and a bottom segment (pairs [h, pairs), decoded LAST by the mirror
// workgroup W-1-b).  Every workgroup thus decodes half of its own frames and half of its mirror's,
// which evens out the pairing of heavy and light frames (two 4K frames per CU cannot balance four
// fixture kinds).  The top segment's last pair, after its last step, copies the frame's context
// slot (the row above the bottom segment, C x 160 B) to a snapshot in device memory (sc1 stores,
// drained) and stores the launch's epoch in the frame's flag; the bottom segment's first pair,
// when it claims its slot, waits for that flag and copies the snapshot into the slot.  Tops never
// wait across workgroups and bottoms come after every top of their list, so no cycle exists, and a
// top finishes in the first half of its workgroup's work, long before its bottom starts.
constexpr uint32_t kSegTop = 1u, kSegBottom = 2u, kSegMask = 0x3FFFFFFFu;  // list entry: frame | tag << 30

template <int NW, bool kG, bool kS, bool kC>
__global__ __launch_bounds__(NW * 64, min_waves_per_simd<NW>()) void frame_kernel(const Vp8gFrameDesc* __restrict__ descs, Vp8gBatchArrays A,
                                                        uint8_t* __restrict__ out, uint32_t ctx_cols,
                                                        uint8_t* __restrict__ gctx, uint32_t nsplit,
                                                        uint8_t* __restrict__ mbox, uint32_t* __restrict__ gprog,
                                                        uint32_t ord_first, uint32_t n_chain) {
	static_assert(!kC || !kS, "chain mode never splits frames into parts");
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	const int lane0 = (int)(threadIdx.x & 63);
	const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
	const uint32_t K = kS ? nsplit : 1u;
	const uint32_t nfr = kS ? gridDim.x / K : gridDim.x;
	const uint32_t slot_bytes = ctx_cols * (uint32_t)kCtxBytesPerCol;
	uint8_t* const ctx_base = smem + kHdrBytes + NW * kWaveBytes;
	// (kC) after the two context slots (global context: after the cost sort's scratch)
	// (kC, ord_first bit 2: two frames interleaved, four context slots)
	const bool il = kC && (ord_first & 4u) != 0;
	uint32_t* const chain_list = (uint32_t*)(ctx_base + (kG ? ((4u * (kCostClasses + n_chain) + 15u) & ~15u) : (il ? 4u : 2u) * slot_bytes));
	uint32_t m_chain = 1;  // (kC) frames in this workgroup's list
	uint32_t f;
	if constexpr (kC) {
		// ---- this workgroup's frame list (see above); ord_first != 0: cost-sorted positions
		const uint32_t Wg = gridDim.x, b = blockIdx.x, n = n_chain;
		if (wave == 0) {
			uint32_t* const hist = (uint32_t*)ctx_base;  // scratch (the context slots, written later)
			uint32_t* const sorted = hist + kCostClasses;
			const uint64_t lt = (1ull << lane0) - 1ull;
			if (ord_first & 1u) {
				for (int i = lane0; i < (int)kCostClasses; i += 64) hist[i] = 0u;
				wave_lds_sync();
				for (int pass = 0; pass < 2; pass++) {
					for (uint32_t c0 = 0; c0 < n; c0 += 64) {
						const uint32_t i = c0 + (uint32_t)lane0;
						const bool valid = i < n;
						const uint32_t cls = valid ? cost_class(descs[i]) : 0u;
						uint64_t rem = __ballot(valid);
						while (rem) {  // one distinct class per iteration (peeled by its first lane)
							const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cls, (int)__builtin_ctzll(rem));
							const uint64_t mk = __ballot(valid && cls == c);
							const uint32_t base = hist[c];
							wave_lds_sync();
							if (pass == 1 && ((mk >> lane0) & 1ull)) sorted[base + (uint32_t)__popcll(mk & lt)] = i;
							if (lane0 == (int)__builtin_ctzll(mk)) hist[c] = base + (uint32_t)__popcll(mk);
							wave_lds_sync();
							rem &= ~mk;
						}
					}
					if (pass == 0) {  // counts -> start positions, heaviest class first
						if (lane0 == 0) {
							uint32_t acc = 0;
							for (int c = (int)kCostClasses - 1; c >= 0; c--) {
								const uint32_t h = hist[c];
								hist[c] = acc;
								acc += h;
							}
						}
						wave_lds_sync();
					}
				}
			}
			// snake positions of workgroup b (increasing in j), empty descriptors left out.  Mirror
			// split (ord_first bit 1): workgroup b decodes the top halves of its own frames, then the
			// bottom halves of workgroup W-1-b's frames (entry tags, kSegTop / kSegBottom)
			uint32_t cnt = 0;
			auto add_list = [&](uint32_t bb, uint32_t tag) {
				for (uint32_t j0 = 0;; j0 += 64) {
					const uint32_t j = j0 + (uint32_t)lane0;
					const uint32_t pos = j * Wg + ((j & 1u) ? Wg - 1u - bb : bb);
					const bool valid = pos < n;
					if (__ballot(valid) == 0ull) break;
					const uint32_t fi = valid ? ((ord_first & 1u) ? sorted[pos] : pos) : 0u;
					const bool keep = valid && descs[fi].mb_cols != 0 && descs[fi].mb_rows != 0 && (tag != kSegBottom || descs[fi].mb_rows > 2u);
					const uint64_t mk = __ballot(keep);
					if (keep) chain_list[cnt + (uint32_t)__popcll(mk & lt)] = fi | (tag << 30);
					cnt += (uint32_t)__popcll(mk);
				}
			};
			const bool split = (ord_first & 2u) != 0;
			add_list(b, split ? kSegTop : 0u);
			if (split) add_list(Wg - 1u - b, kSegBottom);
			if (lane0 == 0) *(uint32_t*)(smem + kMisc) = cnt;
		}
		__syncthreads();
		m_chain = (uint32_t)__builtin_amdgcn_readfirstlane((int)*(const uint32_t*)(smem + kMisc));
		f = m_chain ? (uint32_t)__builtin_amdgcn_readfirstlane((int)chain_list[0]) & kSegMask : 0u;
	} else {
		f = kS ? blockIdx.x % nfr : (ord_first ? ordered_frame<NW * 64>(descs, nfr, ord_first, smem) : blockIdx.x);
	}
	const uint32_t part = kS ? blockIdx.x / nfr : 0u;

	for (int i = (int)threadIdx.x; i < kBpModes * 16 * (kBpEntry / 4); i += NW * 64) ((uint32_t*)(smem + kBpTable))[i] = kBpTab.v[i];
	if (threadIdx.x < 64) ((uint32_t*)(smem + kRoleTab))[threadIdx.x] = kPredRoleTab.v[threadIdx.x];
	uint32_t bt_l = kBorderTab.v[lane0 & 31];  // this lane's border-setup role (loop-invariant)
	// dequant / loop-filter tables of a frame into its slot (chain mode: by the wave of the frame's pair 0)
	auto put_tables = [&](const Vp8gFrameDesc& Df, uint32_t tabo, int l) {
		// dequant factors as (dc, ac) int16 pairs, [class][segment] (one 16-B read per lane
		// fetches a class's four segments before the segment is known)
		if (l < 24) {
			const int sg = l / 6, k = l % 6, cl = k >> 1;
			((int16_t*)(smem + kDqTable + tabo))[(cl * 4 + sg) * 2 + (k & 1)] = Df.dq[sg][k];
		}
		if (l < 32) smem[kLfTable + tabo + l] = Df.lf[l >> 3][(l >> 2) & 1][l & 3];
	};
	if constexpr (!kC) put_tables(descs[f], 0u, (int)threadIdx.x);
	if (threadIdx.x < 16) ((uint32_t*)(smem + kProgress))[threadIdx.x] = 0;
	__syncthreads();
	if (kC && m_chain == 0) return;

	// ---- the current frame (chain mode: reloaded when the wave's next pair is in another frame)
	const Vp8gFrameDesc* Dp;
	uint32_t C, R, flags, W, H, CW, CH, sy, suv, vofs, yal, ual, npairs, CP2, tabo;
	uint64_t mb0;
	uint8_t* outY;
	uint8_t* outU;
	Ctx<kG> ctx;
	auto set_frame = [&](uint32_t fi, uint32_t slot) {
		Dp = descs + fi;
		const Vp8gFrameDesc& D = *Dp;
		C = D.mb_cols, R = D.mb_rows;
		flags = D.flags;
		mb0 = D.mb_offset;
		outY = out + D.out_y;
		outU = out + D.out_u;
		W = D.width, H = D.height, CW = (D.width + 1) >> 1, CH = (D.height + 1) >> 1;
		sy = D.stride_y, suv = D.stride_uv;
		vofs = (uint32_t)(D.out_v - D.out_u);  // V plane relative to U (< 2^32 by construction)
		yal = (uint32_t)(uintptr_t)outY, ual = (uint32_t)(uintptr_t)outU;  // alignment tests
		ctx.lds = ctx_base + slot * slot_bytes;
		ctx.g = kG ? gctx + (size_t)fi * ctx_cols * kCtxBytesPerCol : nullptr;
		npairs = (R + 1) >> 1;
		CP2 = C + 2;
		tabo = slot * (uint32_t)kTabStride;
	};
	set_frame(f, 0u);
	uint32_t flags_l = flags;  // (laundered per step)
	uint32_t* const prog = (uint32_t*)(smem + kProgress);
	const uint32_t GW = K * NW, gw = part * NW + (uint32_t)wave;
	const size_t chan = (size_t)ctx_cols * kCtxBytesPerCol;
	const uint32_t pin = (part + K - 1) % K;  // the part holding this part's wave-0 predecessors
	uint8_t* const mb_in = kS ? mbox + (f * K + pin) * chan : nullptr;
	uint8_t* const mb_out = kS ? mbox + (f * K + part) * chan : nullptr;
	uint32_t* const gp_in = kS ? gprog + f * K + pin : nullptr;
	uint32_t* const gp_out = kS ? gprog + f * K + part : nullptr;

#ifdef VP8G_STAMPS
	// phases 0..7 as below; sub-phases (round 5): 13 the wait for the prefetched coefficients, 10 side
	// info, 11 iWHT (within the residual), 12 whole-block prediction (within recon); 8 and 9 hold the
	// launch clocks
	uint64_t st_acc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
	uint64_t st_prev = __builtin_amdgcn_s_memtime();
	if (blockIdx.x == 0 && lane0 == 0 && wave < 32) g_vp8g_wave_times[2 * wave] = __builtin_amdgcn_s_memrealtime();
	const uint64_t st_t0 = __builtin_amdgcn_s_memrealtime();
#endif

	// Loads for one lane of one step: coefficient blocks (ln 0..24), bmode (25), side bytes (26..29).
	// Straight-line: every lane issues the same three loads from a per-pair row base (hoisted, see
	// below) plus its column; columns outside the frame are clamped (their data is never used).
	// Loop-filter-only frames read the descriptor instead of the absent coefficient arrays: a
	// path without these loads would make the compiler's wait-count analysis fall back to
	// vmcnt(0) on the next step's use of the side bytes, i.e. wait for this very prefetch.
	auto prefetch = [&](int lane, uint64_t cbase, uint64_t sbase, uint32_t csh, int tt) -> Pref {
		Pref p;
		const int hh = lane >> 5, ln = lane & 31;
		const uint32_t cn = (uint32_t)min(max(tt - 2 * hh, 0), (int)C - 1);
		const gu32x4* src = (const gu32x4*)(cbase + ((uint64_t)cn << csh));
		// (default cache policy: non-temporal loads measured 1 % slower and cost 11 % more HBM
		// writes -- streamed coefficients then crowd out the partially written output lines in L2)
		p.a = *src;
		p.b = *(ln == 25 ? src : src + 1);
		p.side = ((const __attribute__((address_space(1))) uint8_t*)sbase)[cn];
		return p;
	};

	// Set once a dependency wait has timed out: the wave finishes without waiting again (its output
	// is garbage and the status word says so), so a stalled producer costs one bound, not one per step.
	bool dead = false;
	// bounded wait until the progress word of wave pw reaches `need`
	auto wait_prog = [&](uint32_t pw, uint32_t need, bool xin_, uint32_t* pa = nullptr) {
		uint32_t spins = 0;
		uint64_t t0 = 0;
		uint32_t* const pw_ = (pa ? pa : prog) + pw;
		while (((kS && xin_) ? __hip_atomic_load(gp_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
		             : __hip_atomic_load(pw_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < need) {
			__builtin_amdgcn_s_sleep(VP8G_WAIT_SLEEP);
			if ((++spins & 1023u) == 0) {
				const uint64_t now = __builtin_amdgcn_s_memrealtime();
				if (t0 == 0) t0 = now;
				else if (now - t0 > (uint64_t)VP8G_WAIT_TICKS) {  // give up, flag it, and never wait again
					if (lane0 == 0) atomicOr(A.status, VP8G_ERR_TIMEOUT);
					dead = true;
					break;
				}
			}
		}
		asm volatile("" ::: "memory");
	};
	// (chain, mirror split) bounded wait until a bottom segment's snapshot flag holds this launch's epoch
	auto wait_flag = [&](uint32_t* flag, uint32_t epoch) {
		uint32_t spins = 0;
		uint64_t t0 = 0;
		while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
			__builtin_amdgcn_s_sleep(2);
			if ((++spins & 255u) == 0) {
				const uint64_t now = __builtin_amdgcn_s_memrealtime();
				if (t0 == 0) t0 = now;
				else if (now - t0 > (uint64_t)VP8G_WAIT_TICKS) {
					if (lane0 == 0) atomicOr(A.status, VP8G_ERR_TIMEOUT);
					dead = true;
					break;
				}
			}
		}
		asm volatile("" ::: "memory");
	};
	auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
	// chain mode: list index of the wave's current frame, its first global pair, and the last global
	// pair (with its step count) of the frames one and two list positions back
	// (Only these few scalars are carried around the chain's frame loop; every other frame value is
	// re-derived per pair from the laundered frame index: frame values carried as loop PHIs were
	// taken for divergent, kept in VGPRs, and every output store became a waterfall loop.)
	// (chain: list entries carry a segment tag, see kSegTop; a segment is pairs [k0, k0 + its pairs))
	auto pairs_of = [&](uint32_t fi) { return (descs[fi].mb_rows + 1u) >> 1; };
	auto seg_k0 = [&](uint32_t e) { return (e >> 30) == kSegBottom ? (pairs_of(e & kSegMask) + 1u) >> 1 : 0u; };
	auto seg_pairs = [&](uint32_t e) {
		const uint32_t np = pairs_of(e & kSegMask), tag = e >> 30;
		return tag == 0u ? np : (tag == kSegTop ? (np + 1u) >> 1 : np >> 1);
	};
	uint32_t jf = 0, gbase = 0, ecur = kC ? uni(chain_list[0]) : f, np_c = kC ? seg_pairs(ecur) : npairs;
	// (interleave) pairs per frame -- every frame of the batch has the same size
	const uint32_t ilP = il ? uni(pairs_of(ecur & kSegMask)) : 0u;
	for (uint32_t g = gw;; g += GW) {
		uint32_t k;
		bool has_pred;        // the pair above is decoded by this workgroup (else: frame top, or a bottom segment's snapshot)
		bool snap_out = false;  // (kC) the top segment's last pair: context -> snapshot after its last step
		uint32_t fcur = f;
		uint32_t dg = 1;      // global pairs back to the pair above (2 when two frames run interleaved)
		if (il) {
			// Two frames at a time: list entries 2m, 2m + 1 form group m, whose 2P global pairs alternate
			// between them (pair k of frame 2m + e is global pair m * 2P + 2k + (e ^ (m & 1)), its pair
			// above two global pairs back, i.e. two waves back); an odd last entry runs alone.  2P is even,
			// so a wave keeps its parity's role in every group: the swap on odd groups hands the even and
			// the odd waves the snake's heavy and light list positions in turn (without it the even waves
			// took every heavy frame, fhd4 +8 %).  Frame j uses context slot j & 3: its first pair waits
			// for frame j - 4's last pair.
			const uint32_t gp = 2u * ilP, m = g / gp, off = g - m * gp;
			if (m >= (m_chain >> 1)) {  // the odd tail frame, sequential
				if (m > (m_chain >> 1) || !(m_chain & 1u) || off >= ilP) break;
				jf = 2u * m, k = off, dg = 1u;
			} else {
				jf = 2u * m + ((off ^ m) & 1u), k = off >> 1, dg = 2u;
			}
			jf = uni(jf), k = uni(k), dg = uni(dg);
			ecur = uni(chain_list[jf]);
			fcur = ecur & kSegMask;
			set_frame(fcur, jf & 3u);
			has_pred = k > 0;
			if (k == 0) {
				if (jf >= 4u && !dead) {
					const uint32_t j4 = jf - 4u, last4 = (j4 >> 1) * gp + 2u * (ilP - 1u) + ((j4 ^ (j4 >> 1)) & 1u);
					const uint32_t T4 = 2u * (ilP - 1u) + 1u < R ? C + 2u : C;
					wait_prog(last4 % NW, (last4 << kProgShift) + T4, false);
				}
				put_tables(*Dp, tabo, lane0);
				wave_lds_sync();
			} else if (!dead) {
				wait_prog((uint32_t)((wave + NW - dg) % NW), ((g - dg) << kProgShift) + 1u, false);
			}
		} else if constexpr (kC) {
			while (g >= gbase + np_c) {  // advance to the segment holding global pair g
				gbase += np_c;
				if (++jf >= m_chain) break;
				ecur = uni(chain_list[jf]);
				np_c = seg_pairs(ecur);
			}
			if (jf >= m_chain) break;
			jf = uni(jf), gbase = uni(gbase), ecur = uni(ecur);
			fcur = ecur & kSegMask;
			set_frame(fcur, jf & 1u);
			const uint32_t tag = ecur >> 30, k0 = seg_k0(ecur);
			k = k0 + (g - gbase);
			has_pred = g > gbase;
			snap_out = tag == kSegTop && g + 1u == gbase + np_c && np_c < npairs;
			if (g == gbase) {
				// claim slot jf & 1: segment jf - 2 must be done with it, i.e. its last pair (global
				// index gbase - pairs(jf - 1) - 1) must have published all T2 of its steps
				if (jf >= 2 && !dead) {
					const uint32_t e2 = uni(chain_list[jf - 2u]), f2 = e2 & kSegMask;
					const uint32_t last2 = gbase - seg_pairs(uni(chain_list[jf - 1u])) - 1u;
					const uint32_t kl2 = seg_k0(e2) + seg_pairs(e2) - 1u, R2 = descs[f2].mb_rows, C2 = descs[f2].mb_cols;
					const uint32_t T2 = 2u * kl2 + 1u < R2 ? C2 + 2u : C2;
					wait_prog(last2 % NW, (last2 << kProgShift) + T2, false);
				}
				if (tag == kSegBottom) {
					// the rows above come from the top segment's snapshot (another workgroup); with the
					// context in device memory the snapshot is the frame's context itself
					uint32_t* const flag = gprog + fcur;
					if (!dead) wait_flag(flag, nsplit);
					// (16-B agent-coherent loads, kSnapBatch per lane in flight: one round trip per batch instead
					// of one per 1 KB -- the chain's next pairs wait for this copy)
					const uint32_t nb = C * (uint32_t)kCtxBytesPerCol;
					const Rsrc rsn = plane_rsrc(gctx + (size_t)fcur * slot_bytes, nb);
					for (uint32_t o0 = (uint32_t)lane0 * 16u; !kG && o0 < nb; o0 += 1024u * kSnapBatch) {
						u32x4 v[kSnapBatch];
#pragma unroll
						for (int i = 0; i < kSnapBatch; i++) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rsn, (int)(o0 + 1024u * i), 0, kCpolSc1);
#pragma unroll
						for (int i = 0; i < kSnapBatch; i++)
							if (o0 + 1024u * i < nb) st128(ctx.lds + o0 + 1024u * i, v[i]);
					}
				}
				put_tables(*Dp, tabo, lane0);
				wave_lds_sync();
			} else if (!dead) {
				// step 0's dependency wait, before its residual: the residual reads the dequant table
				// that the segment's first pair writes when it claims the slot (pair g - 1 past step 0
				// implies the first pair past it, and that pair writes its tables before its first publish)
				wait_prog((uint32_t)((wave + NW - 1) % NW), ((g - 1u) << kProgShift) + 1u, false);
			}
		} else {
			k = g;
			if (k >= npairs) break;
			has_pred = k > 0;
		}
		// output planes (built per pair: a buffer resource carried around the chain's frame loop
		// would be a loop PHI the backend cannot keep in SGPRs)
		const Rsrc rY = plane_rsrc(outY, sy * H), rC = plane_rsrc(outU, vofs + suv * CH);
		const bool xin = kS && wave == 0 && k > 0;             // predecessor pair in another part
		const bool xout = kS && wave == NW - 1 && k + 1 < npairs;  // successor pair in another part
		u32x4 mbx = u32x4{0u, 0u, 0u, 0u};                     // mailbox prefetch (xin: lanes 0..9)
		const uint32_t rA = 2 * k;
		const bool two = rA + 1 < R;
		const uint32_t T = two ? CP2 : C;
		[[maybe_unused]] const bool lf_on = (flags & VP8G_F_LOOPFILTER) != 0;
		[[maybe_unused]] const bool simple = (flags & VP8G_F_SIMPLE) != 0;
		const bool lf_only = (flags & VP8G_F_LF_ONLY) != 0;
		// Per-lane row bases of this pair (lane roles: ln 0..24 one 32-B coefficient block each --
		// Y 0..15, U 16..19, V 20..23, Y2 24 (and 26..31, duplicates) -- ln 25 the 16 B_PRED modes;
		// side bytes ln&3: ymode, uv_mode, segment_id, has_coeff for lanes 26..29).  MB m's data
		// sits at cbase + (column << csh).
		uint64_t cbase, sbase;
		uint32_t csh;
		{
			const int hh = lane0 >> 5, ln = lane0 & 31;
			const uint64_t mrow = mb0 + __umul24(rA + (two ? (uint32_t)hh : 0u), C);
			const bool isb = ln == 25;
			const uint32_t sh = ln < 16 ? 9u : (ln < 24 ? 7u : (isb ? 4u : 5u));
			const uint32_t boff = ln < 16 ? (uint32_t)ln * 32u : (ln < 24 ? (uint32_t)(ln & 3) * 32u : 0u);
			// (vsel: explicit v_cndmask -- a select among struct fields by a lane-dependent index
			// would otherwise compile to a per-lane load from the kernel-argument block)
			const uint64_t base = vsel(ln < 16, (uint64_t)A.coeff_y,
			                           vsel(ln < 20, (uint64_t)A.coeff_u,
			                                vsel(ln < 24, (uint64_t)A.coeff_v, vsel(isb, (uint64_t)A.bmode, (uint64_t)A.coeff_y2))));
			cbase = lf_only ? (uint64_t)descs : base + (mrow << sh) + boff;
			csh = lf_only ? 0u : sh;
			const int q = ln & 3;
			sbase = vsel(q == 2, (uint64_t)A.ymode, vsel(q == 3, (uint64_t)A.uv_mode, vsel(q == 0, (uint64_t)A.segment_id, (uint64_t)A.has_coeff))) + mrow;
		}
		// Per-lane flush geometry of this pair (loop-filtered frames): lane ln of a half stores
		// luma tile row ln (0..19) and chroma plane ln / 12, tile row ln % 12 of some column;
		// image row = MB row origin + tile row - 4 (negative rows wrap and fail the crop test).
		uint32_t fl_offY, fl_offC, fl_bits, fl_srcY = 0u, fl_srcC = 0u;
		// loop-filter line addresses of this lane (rows for the vertical-edge pass, columns for the
		// horizontal-edge pass), relative to the wave's LDS area: slot 0 in bits 0..15, slot 1 in 16..31
		uint32_t lf_vp, lf_hp;
		{
			const int hh = lane0 >> 5, ln = lane0 & 31;
			const bool isy = ln < 16;
			const uint32_t cp = (uint32_t)(ln >> 3) & 1u, hb = (uint32_t)(kHdrBytes + (hh ? kHalfBytes : 0));
			const uint32_t rowp = hb + (isy ? (uint32_t)(kLfY + (4 + ln) * kTP) : (uint32_t)kLfUV + (4u + (uint32_t)(ln & 7)) * kTP + cp * kCV);
			const uint32_t col = hb + (isy ? (uint32_t)(kLfY + ln) : (uint32_t)kLfUV + cp * kCV + (uint32_t)(ln & 7));
			const uint32_t d = isy ? 16u : 8u;
			lf_vp = rowp | ((rowp + d) << 16);
			lf_hp = col | ((col + d) << 16);
		}
		const bool fl_fast = lf_on && W == 16u * C && ((yal | sy) & 15u) == 0 && ((ual | suv | vofs) & 7u) == 0;
		{
			const int hh = lane0 >> 5, ln = lane0 & 31;
			const uint32_t rr = rA + (uint32_t)hh;
			const bool row_ok = hh == 0 || two;
			const uint32_t prowY = rr * 16u + (uint32_t)ln - 4u;
			const int pc = ln >= 12 ? 1 : 0, kc = ln - 12 * pc;
			const uint32_t prowC = rr * 8u + (uint32_t)kc - 4u;
			fl_offY = __umul24(prowY, sy);
			fl_offC = (pc ? vofs : 0u) + __umul24(prowC, suv);
			const bool nlast = rr + 1 < R;
			fl_bits = (row_ok && ln < 20 && prowY < H ? 1u : 0u) | (ln >= 16 && nlast ? 2u : 0u) |
			          4u | (row_ok && ln < 24 && prowC < CH ? 8u : 0u) |
			          (kc >= 8 && nlast ? 16u : 0u) | 32u;
			// Whole-piece frames (fl_fast): every row piece of a column inside the frame is a full,
			// aligned 16-B / 8-B store.  The offsets then fold the lane's column shift (the left MB for
			// tile rows >= 4) in, and a lane that never stores to HBM this pair (outside the crop, or
			// its rows go to ctx_lf) gets a base past the plane end: per step offset = base + t * 16
			// (chroma t * 8), taken when the MB is active and the column exists.
			// The tile source of a lane's piece, by column parity (slot = t & 1): even | odd << 16,
			// relative to the wave's LDS area.  The ctx_lf destination of the rows the next MB row still
			// filters (luma ln 16..19; chroma tile rows 8..11, marked by bit 30) at t = 0, replacing
			// fl_bits, or ~0u: offset + t * 160 once the column exists.
			if (fl_fast) {
				const bool topY = ln < 4, topC = kc < 4;
				const uint32_t sh = 2u * (uint32_t)hh + (topY ? 0u : 1u);
				const uint32_t shc = 2u * (uint32_t)hh + (topC ? 0u : 1u);
				const uint32_t hb = (uint32_t)(kHdrBytes + (hh ? kHalfBytes : 0));
				const uint32_t sY = hb + kLfY + (uint32_t)ln * kTP, sC = hb + kLfUV + (uint32_t)(pc * kCV + kc * kTP);
				fl_srcY = (sY + (topY ? 0u : 16u)) | ((sY + (topY ? 16u : 0u)) << 16);
				fl_srcC = (sC + (topC ? 0u : 8u)) | ((sC + (topC ? 8u : 0u)) << 16);
				// lf_off(t - 2hh - 1) - t * 160 + kFlCtxBias (>= 0: sh <= 3)
				const uint32_t lc0 = kFlCtxBias - sh * (uint32_t)kCtxBytesPerCol + (uint32_t)kCtxRecBytes;
				const uint32_t lcY = lc0 + ((uint32_t)ln - 16u) * 16u;
				const uint32_t lcC = lc0 + 64u + (uint32_t)pc * 32u + ((uint32_t)kc - 8u) * 8u;
				fl_offY = (fl_bits & 1u) && !(fl_bits & 2u) ? fl_offY - sh * 16u : kNoStore;
				fl_offC = (fl_bits & 8u) && !(fl_bits & 16u) ? fl_offC - shc * 8u : kNoStore;
				fl_bits = (fl_bits & 3u) == 3u ? lcY : ((fl_bits & 24u) == 24u ? (lcC | 0x40000000u) : ~0u);  // (bit 2 / 16 alone: lanes 20..31)
			}
		}
		// The step's 32 bytes per lane, loaded one step ahead.  One variable carried around the loop
		// and reloaded right after its last use (the dequantisation), so no register copy -- which
		// would have to wait for the loads to land -- sits at the end of the step.
		Pref cur = prefetch(lane0, cbase, sbase, csh, 0);
		// two dropped stores (kNoStore): the loop entry then has as many vector-memory operations
		// after the prefetch as every step has (its two output stores), so the first use of the
		// prefetched data waits for the loads alone, never for stores (see kNoStore)
		bst128(rY, kNoStore, u32x4{0u, 0u, 0u, 0u});
		bst64(rC, kNoStore, u32x2{0u, 0u});
		flags_l = (uint32_t)__builtin_amdgcn_readfirstlane((int)flags);  // (the chain's frame loop makes it a PHI)
		// Per-half side info of a step, broadcast from the prefetched bytes of lanes 26..29 / 58..61 (and
		// the 16 B_PRED modes from lane 25 / 57) with ds_bpermute (LDS crossbar, no LDS memory), at the
		// top of the step.  (Round 5 fetched it at the end of the previous step, after the loop filter,
		// to take its round trip off the step's start: +6.3 %, r05f -- the work moved in front of the
		// publish delays the next wave, whose dependency wait is on that publish.)
		struct Side {
			int ymode, uvmode, seg, hasc;
			u32x4 bmw;
		};
		// the four segments' dequant factors of a lane's class in one 16-B read, the segment's pair picked
		// by two v_cndmask levels once the side info is known
		auto load_dq4 = [&](int ln_) -> u32x4 { return *(const u32x4*)(smem + kDqTable + tabo + 16 * (ln_ < 16 ? 0 : (ln_ < 24 ? 1 : 2))); };
		auto pick_dq = [&](const u32x4& dq4, int seg_) -> uint32_t {
			const uint64_t m1 = __builtin_amdgcn_ballot_w64((seg_ & 1) != 0), m2 = __builtin_amdgcn_ballot_w64((seg_ & 2) != 0);
			uint32_t lo, hi, r;
			asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(lo) : "v"(dq4.x), "v"(dq4.y), "s"(m1));
			asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(hi) : "v"(dq4.z), "v"(dq4.w), "s"(m1));
			asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(lo), "v"(hi), "s"(m2));
			return r;
		};
		auto fetch_side = [&](int lane_) -> Side {
			const int hh_ = lane_ >> 5;
			const int sdl = (hh_ ? 58 : 26) * 4, bml = (hh_ ? 57 : 25) * 4;
			Side sd;
			sd.ymode = __builtin_amdgcn_ds_bpermute(sdl, (int)cur.side);
			sd.uvmode = __builtin_amdgcn_ds_bpermute(sdl + 4, (int)cur.side);
			sd.seg = __builtin_amdgcn_ds_bpermute(sdl + 8, (int)cur.side) & 3;
			sd.hasc = __builtin_amdgcn_ds_bpermute(sdl + 12, (int)cur.side);
			sd.bmw = u32x4{(uint32_t)__builtin_amdgcn_ds_bpermute(bml, (int)cur.a.x), (uint32_t)__builtin_amdgcn_ds_bpermute(bml, (int)cur.a.y),
			               (uint32_t)__builtin_amdgcn_ds_bpermute(bml, (int)cur.a.z), (uint32_t)__builtin_amdgcn_ds_bpermute(bml, (int)cur.a.w)};
			return sd;
		};

		for (uint32_t t = 0; t < T; t++) {
			// Lane-derived values are recomputed every step from a laundered lane id: hoisting the
			// lane-dependent LDS addresses out of the loop would exhaust the VGPR budget.
			int lane = lane0;
			asm volatile("" : "+v"(lane));
			// The same for the loop-invariant per-lane words and the frame flags: comparisons on them
			// would otherwise be hoisted as 64-bit lane masks, which exhaust the SGPRs and are spilled
			// to VGPR lanes (a v_readlane pair, plus a hazard wait, per use per step).
			asm volatile("" : "+v"(bt_l), "+v"(fl_bits), "+s"(flags_l));
			asm volatile("" : "+v"(fl_srcY), "+v"(fl_srcC));
			asm volatile("" : "+v"(lf_vp), "+v"(lf_hp));
			const bool lf_on = (flags_l & VP8G_F_LOOPFILTER) != 0;
			const bool simple = (flags_l & VP8G_F_SIMPLE) != 0;
			const bool lf_only = (flags_l & VP8G_F_LF_ONLY) != 0;
			const int hh = lane >> 5, ln = lane & 31;
			const uint32_t r = rA + (uint32_t)hh;
			const int c = (int)t - 2 * hh;
			const bool act = (hh == 0 || two) && c >= 0 && c < (int)C;
			const uint32_t cu = (uint32_t)c;
			const int slot = c & 1;
			uint8_t* const hv = smem + kHdrBytes + wave * kWaveBytes + (hh ? kHalfBytes : 0);  // this half's area
			uint8_t* const tY = hv + kLfY;
			uint8_t* const tC = hv + kLfUV;  // chroma: U at +0, V at +kCV, row pitch kTP
			uint8_t* const abY = hv + kAbY;
			[[maybe_unused]] uint8_t* const abUV = hv + kAbUV;  // (the predictor role word carries it)
			uint8_t* const left = hv + kLeft;

			// per-half side info, held by lanes 26..29 / 58..61: fetched with ds_bpermute (LDS
			// crossbar, no LDS memory) instead of readlane + per-half select
			// (the four segments' dequant factors of this lane's class, read before the side info is known)
#ifdef VP8G_STAMPS
			// (stamps build: the wait for this step's prefetched coefficients timed on its own, sub-phase 13;
			// vmcnt(2): all but the previous step's two output stores)
			asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
			STAMP(13);
#endif
			// (the four segments' dequant factors of this lane's class, read before the side info is known)
			const u32x4 dq4 = load_dq4(ln);
			// (the half's 16 B_PRED modes come from lane 25 / 57, used by the B_PRED phase)
			const Side side = fetch_side(lane);
			const int ymode = side.ymode, uvmode = side.uvmode, seg = side.seg, hasc = side.hasc;
			const u32x4 bmw = side.bmw;
			const bool bpred = ymode == 4;
			const uint32_t y0 = r * 16, cy0 = r * 8, x0 = cu * 16, cx0 = cu * 8;

			STAMP(10);
			// ---------------------------------------------- residual (no spatial dependency)
			SUBMARK(30);
			PRIO(0);
			// Computed before the dependency wait.  Each block stays in its lane's registers (rs[],
			// packed int16 pairs) for the whole-block predictors of the same lane; the luma blocks
			// are also parked in LDS (kResid) for the B_PRED pixel lanes.
			uint32_t rs[8];
			if (lf_only) {
#pragma unroll
				for (int i = 0; i < 8; i++) rs[i] = 0u;
			} else {
				// Packed int16 pairs: w[2r + h] = row r, columns 2h, 2h+1.  Dequantisation and the
				// vertical pass wrap mod 2^16 exactly like the reference's int16 stores; the
				// horizontal pass (whose (x + 4) >> 3 needs the full-precision sum) runs in 32 bits.
				const uint32_t fdcac = pick_dq(dq4, seg);  // (dc, ac) int16 pair
				const uint32_t facac = __builtin_amdgcn_perm(fdcac, fdcac, 0x03020302u);
				uint32_t w[8] = {pk_mul(cur.a.x, fdcac), pk_mul(cur.a.y, facac), pk_mul(cur.a.z, facac), pk_mul(cur.a.w, facac),
				                 pk_mul(cur.b.x, facac), pk_mul(cur.b.y, facac), pk_mul(cur.b.z, facac), pk_mul(cur.b.w, facac)};
				const bool anyac = ((w[0] >> 16) | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) != 0u;
				// Y2 (non-B_PRED): inverse WHT (RFC 14.3), 16 DCs to LDS.  Lanes 26..29 hold the Y2
				// coefficients too (their prefetch duplicates lane 24's load): the vertical pass runs
				// packed in lanes 26 / 27 (column pairs 0-1 / 2-3), the horizontal pass one row per
				// lane in 26..29, through kWht.
				if (__ballot(act && !bpred) != 0ull) {
					PRIO(10);
					const bool wl = ln >= 26 && ln < 30;
					{
						const int h = ln & 1;
						const uint32_t r0 = h ? w[1] : w[0], r1 = h ? w[3] : w[2], r2 = h ? w[5] : w[4], r3 = h ? w[7] : w[6];
						const uint32_t a1 = pk_add(r0, r3), b1 = pk_add(r1, r2), c1 = pk_sub(r1, r2), d1 = pk_sub(r0, r3);
						if (ln == 26 || ln == 27) {
							uint8_t* const q = hv + kWht + 4 * h;
							st32(q, pk_add(a1, b1));
							st32(q + 8, pk_add(c1, d1));
							st32(q + 16, pk_sub(a1, b1));
							st32(q + 24, pk_sub(d1, c1));
						}
					}
					wave_lds_sync();
					if (wl) {
						uint8_t* const q = hv + kWht + 8 * (ln - 26);
						const u32x2 t = ld64(q);
						const int q0 = lo_s16(t.x), q1 = hi_s16(t.x), q2 = lo_s16(t.y), q3 = hi_s16(t.y);
						const int a1 = q0 + q3 + 3, b1 = q1 + q2, c1 = q1 - q2, d1 = q0 - q3 + 3;
						st64(q, u32x2{pack2((a1 + b1) >> 3, (c1 + d1) >> 3), pack2((a1 - b1) >> 3, (d1 - c1) >> 3)});
					}
					wave_lds_sync();
					if (ln < 16 && !bpred) w[0] = (w[0] & 0xFFFF0000u) | *(const uint16_t*)(hv + kWht + 2 * ln);
					PRIO(0);
				}
				STAMP(11);
				// inverse DCT (RFC 14.4), the whole block per lane.  DC-only shortcut when no lane of the wave
				// has an AC coefficient ((dc+4)>>3 everywhere, exact); a column-pair-0 transform when no
				// block of the wave has coefficients in columns 2-3.  (Round 3 compacted the AC blocks two
				// lanes per block through LDS: +1.6 %, removed)
				const uint64_t mac = __ballot(anyac && ln < 24 && act);
				auto dc_fill = [&]() {
					const int d = (lo_s16(w[0]) + 4) >> 3;
#pragma unroll
					for (int i = 0; i < 8; i++) rs[i] = pack2(d, d);
				};
				auto vpass = [&](uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t* o) {  // two columns
					const uint32_t a1 = pk_add(r0, r2), b1 = pk_sub(r0, r2);
					const uint32_t c1 = pk_sub(mul_s2(r1), mul_c2(r3)), d1 = pk_add(mul_c2(r1), mul_s2(r3));
					o[0] = pk_add(a1, d1);
					o[3] = pk_sub(a1, d1);
					o[1] = pk_add(b1, c1);
					o[2] = pk_sub(b1, c1);
				};
				if (mac == 0ull) {
					dc_fill();
				} else if (__ballot(act && ln < 24 && (w[1] | w[3] | w[5] | w[7]) != 0u) == 0ull) {
					// Columns 2 and 3 of every block of the wave are zero (the vertical pass leaves them
					// zero): the vertical pass of column pair 0 only, and the horizontal pass with
					// x2 = x3 = 0 -- a1 = b1 = x0 + 4, c1 = mul_s(x1), d1 = mul_c(x1)
					uint32_t oh[4];
					vpass(w[0], w[2], w[4], w[6], oh);
					int c1[4], d1[4];
#pragma unroll
					for (int r = 0; r < 4; r++) {
						const int x1 = hi_s16(oh[r]);
						c1[r] = mul_s(x1), d1[r] = mul_c(x1);
					}
#pragma unroll
					for (int r = 0; r < 4; r++) {
						const int x0 = lo_s16(oh[r]) + 4;
						rs[2 * r] = pack2((x0 + d1[r]) >> 3, (x0 + c1[r]) >> 3);
						rs[2 * r + 1] = pack2((x0 - c1[r]) >> 3, (x0 - d1[r]) >> 3);
					}
				} else {
					uint32_t o[8];
#pragma unroll
					for (int h = 0; h < 2; h++) {  // vertical pass, two columns per op
						uint32_t oh[4];
						vpass(w[h], w[2 + h], w[4 + h], w[6 + h], oh);
#pragma unroll
						for (int r = 0; r < 4; r++) o[2 * r + h] = oh[r];
					}
					// horizontal pass: the multiplications first (columns 1, 3), then the sums with columns 0, 2
					int c1[4], d1[4];
#pragma unroll
					for (int r = 0; r < 4; r++) {
						const int x1 = hi_s16(o[2 * r]), x3 = hi_s16(o[2 * r + 1]);
						c1[r] = mul_s(x1) - mul_c(x3), d1[r] = mul_c(x1) + mul_s(x3);
					}
#pragma unroll
					for (int r = 0; r < 4; r++) {
						const int x0 = lo_s16(o[2 * r]), x2 = lo_s16(o[2 * r + 1]);
						const int a1 = x0 + x2 + 4, b1 = x0 - x2 + 4;
						rs[2 * r] = pack2((a1 + d1[r]) >> 3, (b1 + c1[r]) >> 3);
						rs[2 * r + 1] = pack2((b1 - c1[r]) >> 3, (a1 - d1[r]) >> 3);
					}
				}
				if (ln < 16 && bpred) {  // (only the B_PRED pixel lanes of a B_PRED half read it)
					uint8_t* rp = hv + kResid + ln * 32;
					st128(rp, u32x4{rs[0], rs[1], rs[2], rs[3]});
					st128(rp + 16, u32x4{rs[4], rs[5], rs[6], rs[7]});
				}
			}
			// next step's coefficients into the same registers (the dequantisation above was cur's last
			// use; one definition on every path, so the loop carries it without copies)
			// (round 5: issued right after the dequantisation instead, ahead of the iWHT and iDCT: +0.6 /
			// +1.0 %, r05h)
			cur = prefetch(lane, cbase, sbase, csh, (int)t + 1);
			STAMP(0);

			// ---------------------------------------------- wait: pair k-1's lower row 2 cols ahead
			PRIO(1);
			if (has_pred && !dead && !(VP8G_ABLATE & 8)) {
				// (one column more lag across parts: the mailbox is read a step ahead of use)
				const uint32_t lag = xin ? 5u : 4u;
				const uint32_t ahead = (t + lag < CP2) ? t + lag : CP2;
				if (xin) wait_prog(0u, (k - 1) * CP2 + ahead, true);
				else wait_prog((uint32_t)((wave + NW - dg) % NW), ((g - dg) << kProgShift) + ahead, false);
			}
			if (kS && xin) {
				// mailbox -> this part's LDS ctx: rec[t + 1] and lf[t] now (loaded last step; at t = 0
				// rec[0], rec[1], lf[0] directly), then the loads for the next step (lane roles: ln 0..1
				// the 32-B rec entry, 2..9 the 128-B lf entry, as 16-B pieces)
				auto mload = [&](uint32_t col, uint32_t o) -> u32x4 {
					const uint32_t* q = (const uint32_t*)(mb_in + (size_t)col * kCtxBytesPerCol + o);
					return u32x4{__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
					             __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
					             __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
					             __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
				};
				const uint32_t o = 16u * (uint32_t)(lane0 & 15);  // byte offset in the column entry
				if (t == 0) {
					// ln 0..9: column 0 (rec + lf), 10..11: rec of column 1
					const uint32_t col = lane0 < 10 ? 0u : 1u, oo = lane0 < 10 ? o : o - 160u;
					if (lane0 < 12 && col < C) st128(ctx.lds + col * kCtxBytesPerCol + oo, mload(col, oo));
				} else {
					const uint32_t col = lane0 < 2 ? t + 1 : t;
					if (lane0 < 10 && col < C) st128(ctx.lds + col * kCtxBytesPerCol + o, mbx);
				}
				const uint32_t ncol = lane0 < 2 ? t + 2 : t + 1;
				if (lane0 < 10 && ncol < C) mbx = mload(ncol, o);
				wave_lds_sync();
			}
			STAMP(1);

			// ---------------------------------------------- borders + loop-filter top strip
			PRIO_AFTER(2, 1);
			const u32x2 prole = ld64(smem + kRoleTab + 8 * ln);  // (used by the predictor; rides the border loads' round trip)
			if (act) {
				const bool top = r == 0;
				if (lf_only) {
					// loop-filter-only mode: the MB's pixels come from the padded input image
					const uint8_t* src = A.src;
					if (ln < 16) {
						const uint8_t* s = src + Dp->src_y + (size_t)(y0 + ln) * Dp->src_stride_y + x0;
						uint8_t* const td = tY + (4 + ln) * kTP + slot * 16;
						st64(td, u32x2{ld32(s), ld32(s + 4)});
						st64(td + 8, u32x2{ld32(s + 8), ld32(s + 12)});
					} else {
						const int p = (ln - 16) >> 3, row = ln & 7;
						const uint8_t* s = src + (p ? Dp->src_v : Dp->src_u) + (size_t)(cy0 + row) * Dp->src_stride_uv + cx0;
						stc64(tC + p * kCV + (4 + row) * kTP + slot * 8, u32x2{ld32(s), ld32(s + 4)});
					}
				} else {
					// One 4-byte store per lane 0..19 (kBorderTab: destination, context source, kind):
					// ln 0..3 luma above row, 4 luma above-right (cols x+16..x+19; in the last column
					// the padded width's last byte, replicated), 5..8 chroma above rows -- 127 on the
					// top row; 9..16 left columns at the frame's left edge (129); 17..19 the corners
					// there (byte 3 of the word: 127 on the top row, else 129).
					const uint32_t bt = bt_l;
					const bool clampc = ln == 4 && cu + 1 == C;
					const uint32_t rsrc = rec_off(cu + ((ln == 4 && !clampc) ? 1u : 0u)) + (clampc ? 12u : ((bt >> 12) & 0xFFu));
					const uint32_t ldv = ctx.rd(rsrc);
					const uint32_t kind = (bt >> 20) & 3u;
					const uint32_t vabove = top ? 0x7F7F7F7Fu : (clampc ? __builtin_amdgcn_perm(ldv, ldv, 0x03030303u) : ldv);
					// corner: at the left edge a constant, else the previous MB's above row's last byte
					// (still in the above-row buffer: read before this step's stores replace it)
					const uint32_t oldb = hv[(bt & 0xFFFu) + ((bt >> 12) & 0xFFu)];
					const uint32_t vcorner = c == 0 ? (top ? 0x7F000000u : 0x81000000u) : oldb << 24;
					const uint32_t v = kind == 0 ? vabove : (kind == 1 ? 0x81818181u : vcorner);
					if (ln < 20 && (kind != 1 || c == 0)) st32(hv + (bt & 0xFFFu), v);
				}
				if (lf_on && !top && ln >= 20) {  // filter state of the MB above (both modes; roles in kBorderTab)
					const uint32_t bt = bt_l;
					const bool ly = (bt >> 22) & 1u;
					const uint32_t lo = rec_off(cu) + ((bt >> 12) & 0xFFu);
					uint8_t* const td = hv + (bt & 0xFFFu) + (slot ? (ly ? 16u : 8u) : 0u);
					// (both halves of a luma row loaded before either store: one LDS round trip, not two)
					const u32x2 s0 = ctx.rd64(lo), s1 = ctx.rd64(lo + 8);
					if (ly) st64(td, s0), st64(td + 8, s1);
					else stc64(td, s0);
				}
			}
			wave_lds_sync();
			STAMP(2);

			// ---------------------------------------------- prediction + reconstruction
			PRIO(3);
			if (!lf_only) {
				if (act && ln < 24 && (ln >= 16 || !bpred)) {
					// whole-block predictors (RFC 12.2; reference vp8_recon.c:152-212, 533-560, 605-651),
					// one 4x4 block per lane, branch-free: every mode is sat8(L' + A' + K) with
					// L' = L & mL, A' = A & mA (DC: K = dc value; V: mA; H: mL; TM: both, K = -P)
					const bool yl = (prole.x >> 22) & 1u;
					const uint8_t* ab = hv + (prole.x & 0x7FFu);
					const uint8_t* lc = hv + (prole.y & 0x7FFu);
					const int mode = yl ? (ymode > 4 ? 0 : ymode) : (uvmode > 3 ? 0 : uvmode);
					const u32x2 a01 = ld64(ab), a23 = ld64(ab + 8), l01 = ld64(lc), l23 = ld64(lc + 8);
					const uint32_t aw = ld32(hv + __builtin_amdgcn_ubfe(prole.x, 11u, 11u));
					const uint32_t lw = ld32(lc + 4u * __builtin_amdgcn_ubfe(prole.y, 22u, 2u));
					const int P = (int)ab[-1];
					const uint32_t sa2 = __builtin_amdgcn_sad_u8(a01.y, 0u, __builtin_amdgcn_sad_u8(a01.x, 0u, 0u));
					const uint32_t sl2 = __builtin_amdgcn_sad_u8(l01.y, 0u, __builtin_amdgcn_sad_u8(l01.x, 0u, 0u));
					const uint32_t sa4 = __builtin_amdgcn_sad_u8(a23.y, 0u, __builtin_amdgcn_sad_u8(a23.x, 0u, sa2));
					const uint32_t sl4 = __builtin_amdgcn_sad_u8(l23.y, 0u, __builtin_amdgcn_sad_u8(l23.x, 0u, sl2));
					const bool ha = r > 0, hl = c > 0;
					const uint32_t sum = (ha ? (yl ? sa4 : sa2) : 0u) + (hl ? (yl ? sl4 : sl2) : 0u);
					const int shift = (yl ? 3 : 2) + (ha ? 1 : 0) + (hl ? 1 : 0);  // 16 or 8 samples per edge
					// (no branch around the sums: every load of the predictor issued in one LDS round trip)
					int dcv;
					asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(dcv) : "v"(128), "v"((int)((sum + (1u << (shift - 1))) >> shift)),
					    "s"(__builtin_amdgcn_ballot_w64(ha || hl)));
					// two pixels per op as int16 pairs (|residual| < 2^14, so nothing wraps)
					const uint32_t mA = (mode == 1 || mode == 3) ? 0x00FF00FFu : 0u;
					const uint32_t mL = (mode == 2 || mode == 3) ? 0x00FF00FFu : 0u;
					const int K = (mode == 3 ? -P : 0) + (mode == 0 ? dcv : 0);
					const uint32_t K2 = __builtin_amdgcn_perm((uint32_t)K, (uint32_t)K, 0x05040100u);  // K in both halves
					uint8_t* dst = hv + __builtin_amdgcn_ubfe(prole.y, 11u, 11u) + (slot ? (yl ? 16u : 8u) : 0u);
					const uint32_t* const rw = rs;  // this lane's own block
					const uint32_t A01 = pk_add(__builtin_amdgcn_perm(aw, aw, 0x0C010C00u) & mA, K2);
					const uint32_t A23 = pk_add(__builtin_amdgcn_perm(aw, aw, 0x0C030C02u) & mA, K2);
					uint32_t wv[4];
					// only TM_PRED's predictor can leave [0, 255]: its clamp runs when some lane uses it
					// (the final clamp + byte packing by two v_sat_pk_u8_i16 and one shift-or)
					auto pack_row = [&](uint32_t q01, uint32_t q23) -> uint32_t { return sat_pk(q01) | (sat_pk(q23) << 16); };
					if (__ballot(mode == 3) != 0ull) {
#pragma unroll
						for (int rr = 0; rr < 4; rr++) {
							const uint32_t L2 = __builtin_amdgcn_perm(lw, lw, 0x0C000C00u + 0x00010001u * rr) & mL;
							wv[rr] = pack_row(pk_add(pk_clamp255(pk_add(L2, A01)), rw[2 * rr]), pk_add(pk_clamp255(pk_add(L2, A23)), rw[2 * rr + 1]));
						}
					} else {
#pragma unroll
						for (int rr = 0; rr < 4; rr++) {
							const uint32_t L2 = __builtin_amdgcn_perm(lw, lw, 0x0C000C00u + 0x00010001u * rr) & mL;
							wv[rr] = pack_row(pk_add(pk_add(L2, A01), rw[2 * rr]), pk_add(pk_add(L2, A23), rw[2 * rr + 1]));
						}
					}
#pragma unroll
					for (int rr = 0; rr < 4; rr++) st32(dst + rr * kTP, wv[rr]);
					// the MB's unfiltered bottom row -> ctx_rec[c] (the next MB row's above row) and its
					// right column -> the left column of the next MB (reference vp8_recon.c:395-421)
					if ((prole.x >> 23) & 1u) ctx.wr32(rec_off(cu) + (prole.x >> 25), wv[3]);
					if ((prole.x >> 24) & 1u) {
						const uint32_t c01 = __builtin_amdgcn_perm(wv[1], wv[0], 0x0C0C0703u);
						const uint32_t c23 = __builtin_amdgcn_perm(wv[3], wv[2], 0x0C0C0703u);
						st32(const_cast<uint8_t*>(lc) + 4u * __builtin_amdgcn_ubfe(prole.y, 22u, 2u), __builtin_amdgcn_perm(c23, c01, 0x05040100u));
					}
				}
				wave_lds_sync();
				STAMP(12);
				SUBMARK(20);
				const bool bp_lane = act && bpred;
				if (__ballot(bp_lane) != 0ull && !(VP8G_ABLATE & 2)) {
					PRIO_AFTER(4, 3);
					// B_PRED: 16 sub-blocks along the 2i+j wavefront (10 steps, <= 2 sub-blocks each;
					// lanes 0..15 / 16..31 of a half = group g take sub-block (i0 + g, s - 2 i0 - 2 g)),
					// one pixel per lane, from already reconstructed pixels (reference
					// vp8_recon.c:454-530).  Fully unrolled: every per-step offset is a constant, the
					// per-lane parts are hoisted.  Edge sources (reference vp8_recon.c:464-504): the row
					// above is the MB's above row when i == 0 and the tile otherwise, A4..A7 of the
					// last sub-block column come from the MB above (abY + 32), the left column of
					// sub-block column j is at kLeft - 16 j (kColY, written here by the lanes of
					// pixel column 3), P is the byte before the above row (i == 0) or the left column.
					const int g = (ln >> 4) & 1, p = ln & 15, rr = p >> 2, cc = p & 3;
					uint8_t* const tpix = tY + slot * 16 + 4 * kTP + kBS * g + kTP * rr + cc;  // + kBS i0 + 4 s
					const uint8_t* const tA = tY + slot * 16 + 3 * kTP + kBS * g;             // + kBS i0 + 4 s
					const uint8_t* const aE = g ? tA : abY + 16;                              // i0 == 0: + 4 s
					uint8_t* const lB = left + 36 * g;                                        // + 36 i0 - 16 s
					const int16_t* const rsp = (const int16_t*)(hv + kResid) + p + 32 * g;    // + 16 b0
					const u32x4* const tabp = (const u32x4*)(smem + kBpTable) + p * (kBpEntry / 16);  // + 16 mode entries
					const bool col3 = cc == 3;
					// (one exec region for the whole wavefront: group 0 has a sub-block at every step and
					// group 1 at steps 2..7, so only steps 0, 1, 8, 9 narrow the lanes again)
					if (bp_lane) {
#pragma unroll
					for (int s = 0; s < 10; s++) {
						const int i0 = s <= 3 ? 0 : (s - 2) >> 1;
						const int j0 = s - 2 * i0;  // g = 0: (i0, j0); g = 1: (i0 + 1, j0 - 2)
						const bool v0 = j0 <= 3, v1 = i0 + 1 <= 3 && j0 >= 2;
						const bool valid = g ? v1 : v0;
						if (valid) {
							const int b0 = 4 * i0 + j0;
							const int mb0 = v0 ? (int)((bmw[b0 >> 2] >> (8 * (b0 & 3))) & 0xFFu) : 0;
							const int mb1 = v1 ? (int)((bmw[(b0 + 2) >> 2] >> (8 * ((b0 + 2) & 3))) & 0xFFu) : 0;
							const int mode = min(g ? mb1 : mb0, kBpModes - 1);
							const uint8_t* const arow = i0 == 0 ? aE + 4 * s : tA + kBS * i0 + 4 * s;
							// above-right: the MB above's row when this sub-block is in column 3
							const bool r3_0 = j0 == 3, r3_1 = j0 == 5;
							const uint8_t* const a47p = (r3_0 || r3_1) ? ((g ? r3_1 : r3_0) ? abY + 32 : arow + 4) : arow + 4;
							uint8_t* const lb = lB + 36 * i0 - 16 * s;
							const uint8_t* const pp = i0 == 0 ? (g ? lb - 1 : arow - 1) : lb - 1;
							const uint32_t a03 = ld32(arow), a47 = ld32(a47p), lw = ld32(lb);
							const uint32_t pv = *pp;
							const u32x4 tb = tabp[16 * (kBpEntry / 16) * mode];
							const int rv = rsp[16 * b0];
							const uint32_t ey = (pv << 24) | 0x808080u;
							const uint32_t lo = __builtin_amdgcn_perm(ey, lw, tb.x);
							const uint32_t hi = __builtin_amdgcn_perm(a47, a03, tb.x);
							const uint32_t x3 = (hi & tb.y) | (lo & ~tb.y);  // bytes 0..2 = x, y, z
							// directional modes and TM in one signed dot product over the byte-biased edge
							const int vdir = sat8(__builtin_amdgcn_sdot4((int)(x3 ^ 0x00808080u), (int)tb.z, (int)tb.w, false) >>
							                      (tb.y >> 24));
							const int vdc = (int)((__builtin_amdgcn_sad_u8(a03, 0u, __builtin_amdgcn_sad_u8(lw, 0u, 4u))) >> 3);
							const int pred = mode == 0 ? vdc : vdir;
							const int px = sat8(pred + rv);
							tpix[kBS * i0 + 4 * s] = (uint8_t)px;
							// right pixel column of a sub-block: left column of the next sub-block column (in
							// sub-block column 3: of the next MB); the MB's bottom row -> ctx_rec[c]
							const bool j3 = g ? j0 == 5 : j0 == 3;
							if (col3) (j3 ? left + 4 * (i0 + g) + rr : lb - 16 + rr)[0] = (uint8_t)px;
							if (i0 + g == 3 && rr == 3) ctx.wr8(rec_off(cu) + 4 * (g ? j0 - 2 : j0) + cc, (uint32_t)px);
						}
						wave_lds_sync();
					}
					}
				}
			}
			wave_lds_sync();
			STAMP(3);

			// (the unfiltered bottom row / right column were saved by the prediction lanes; the
			// corner for the next MB is taken at its border setup)
			STAMP(4);

			// ---------------------------------------------- loop filter MB(r, c)
			PRIO(5);
			if (lf_on && !(VP8G_ABLATE & 1)) {
				const uint8_t* lp = smem + kLfTable + tabo + seg * 8 + (bpred ? 4 : 0);
				const int E = lp[0], I = lp[1], Tt = lp[2];
				const bool en = act && E != 0;
				if (__ballot(en) != 0ull) {
					const bool inner = hasc != 0 || bpred;
					// (per-pair lane words: tile offsets at slot 0 | slot 1 << 16, from the wave's area)
					LfLine L;
					{
						const uint32_t sl16 = (t & 1u) << 4;
						uint8_t* const wv = smem + wave * kWaveBytes;
						L.Mp = wv + __builtin_amdgcn_ubfe(lf_vp, sl16, 16u);
						L.Lp = L.Mp + (slot ? -4 : (ln < 16 ? 28 : 12));
						L.colp = wv + __builtin_amdgcn_ubfe(lf_hp, sl16, 16u);
					}
					if (simple) lf_mb<true>(L, ln, en, c > 0, r > 0, inner, E, I, Tt);
					else lf_mb<false>(L, ln, en, c > 0, r > 0, inner, E, I, Tt);
				}
			}
			STAMP(5);

			// ---------------------------------------------- store final pixels
			PRIO(6);
			// One row piece per lane (luma 16 B, chroma 8 B) from LDS to the output plane or, for the
			// bottom rows the next MB row still filters, to ctx_lf.  Straight-line: the crop / odd
			// alignment case (a partial row piece at the right edge) is a rare wave-uniform branch.
			// Rounds are plane-uniform (luma 16-B pieces / chroma 8-B pieces), so plane pointers,
			// strides and crop limits stay scalar.
			// 32-bit offsets from the (uniform) plane bases, so stores use the SGPR-base address form
			auto emitY = [&](bool ok, uint32_t prow, uint32_t col, const uint8_t* src, u32x2 lo, u32x2 hi) {
				const uint32_t colpx = col * 16u;
				const uint32_t off = __umul24(prow, sy) + colpx;
				const bool vis = ok && prow < H && !(VP8G_ABLATE & 4);
				const bool full = colpx + 16u <= W;
				bst128(rY, vis && full ? off : kNoStore, u32x4{lo.x, lo.y, hi.x, hi.y});
				if (__ballot(vis && !full) != 0ull) {
					if (vis && !full) {
						const uint32_t n = W - colpx, cnt = n < 16u ? n : 16u;
						for (uint32_t q = 0; q < cnt; q++) outY[off + q] = src[q];
					}
				}
			};
			auto emitC = [&](bool ok, int p, uint32_t prow, uint32_t col, const uint8_t* src, u32x2 lo) {
				const uint32_t colpx = col * 8u;
				const uint32_t off = (p ? vofs : 0u) + __umul24(prow, suv) + colpx;  // from outU
				const bool vis = ok && prow < CH && !(VP8G_ABLATE & 4);
				const bool full = colpx + 8u <= CW;
				bst64(rC, vis && full ? off : kNoStore, lo);
				if (__ballot(vis && !full) != 0ull) {
					if (vis && !full) {
						const uint32_t n = CW - colpx, cnt = n < 8u ? n : 8u;
						for (uint32_t q = 0; q < cnt; q++) outU[off + q] = src[q];
					}
				}
			};
			// This step's row piece of each lane for the two store rounds (luma 16 B, chroma 8 B):
			// computed on either path, stored once after the join (see kNoStore).  A piece that is
			// visible but cut by the right edge, or not aligned, goes byte by byte (rare branch).
			uint32_t offY = kNoStore, offC = kNoStore, poffY = 0, poffC = 0, pcntY = 0, pcntC = 0;
			u32x2 yl0, yl1, cl0;
			const uint8_t* srcY;
			const uint8_t* srcC;
			if (!lf_on) {
				// unfiltered: MB(r, c) is final as soon as it is reconstructed; lanes 0..15 store luma
				// rows, 16..31 chroma rows
				const bool yl = ln < 16;
				srcY = tY + (4 + (ln & 15)) * kTP + slot * 16;
				const int p = (ln >> 3) & 1, row = ln & 7;
				srcC = tC + p * kCV + (4 + row) * kTP + slot * 8;
				yl0 = ld64(srcY), yl1 = ld64(srcY + 8), cl0 = ldc64(srcC);
				{
					const uint32_t colpx = cu * 16u, prow = y0 + (uint32_t)(ln & 15);
					const uint32_t off = __umul24(prow, sy) + colpx;
					const bool vis = act && yl && prow < H && !(VP8G_ABLATE & 4);
					const bool full = colpx + 16u <= W;
					offY = vis && full ? off : kNoStore;
					poffY = off, pcntY = vis && !full ? min(W - colpx, 16u) : 0u;
				}
				{
					const uint32_t colpx = cu * 8u, prow = cy0 + (uint32_t)row;
					const uint32_t off = (p ? vofs : 0u) + __umul24(prow, suv) + colpx;
					const bool vis = act && !yl && prow < CH && !(VP8G_ABLATE & 4);
					const bool full = colpx + 8u <= CW;
					offC = vis && full ? off : kNoStore;
					poffC = off, pcntC = vis && !full ? min(CW - colpx, 8u) : 0u;
				}
			}
			else if (fl_fast) {
				// whole-piece frame: the folded per-pair offsets and tile sources (see fl_fast); the rows
				// the next MB row still filters go to ctx_lf instead (fl_bits = their ctx_lf offset)
				const uint32_t sl16 = (t & 1u) << 4;  // slot = c & 1 = t & 1
				uint8_t* const wv = smem + wave * kWaveBytes;
				const bool okc = act && (ln < 4 || c > 0);
				srcY = wv + __builtin_amdgcn_ubfe(fl_srcY, sl16, 16u);
				yl0 = ld64(srcY), yl1 = ld64(srcY + 8);
				const uint32_t lcx = fl_bits, t160 = t * (uint32_t)kCtxBytesPerCol - kFlCtxBias;
				if (okc && lcx < 0x40000000u) ctx.wr128(lcx + t160, u32x4{yl0.x, yl0.y, yl1.x, yl1.y});
				offY = okc ? fl_offY + t * 16u : kNoStore;
				const int kr = ln < 12 ? ln : ln - 12;
				const bool okcc = act && (kr < 4 || c > 0);
				srcC = wv + __builtin_amdgcn_ubfe(fl_srcC, sl16, 16u);
				cl0 = ldc64(srcC);
				if (okcc && (int)lcx > 0x3FFFFFFF) ctx.wr64(lcx + (t160 - 0x40000000u), cl0);
				offC = okcc ? fl_offC + t * 8u : kNoStore;
#if VP8G_ABLATE & 16
				// diagnostic (output wrong): the same stores of the same lanes, linearised per wave half, so
				// each step's pieces fill whole consecutive lines -- the traffic and time without partial lines
				{
					const uint32_t linR = ((H * sy) / (2 * NW)) & ~1023u, linRc = ((vofs + suv * CH) / (2 * NW)) & ~1023u;
					const uint32_t reg = (uint32_t)(wave * 2 + hh), st = k * T + t;
					offY = offY == kNoStore ? kNoStore : reg * linR + (st * 512u + (uint32_t)ln * 16u) % linR;
					offC = offC == kNoStore ? kNoStore : reg * linRc + (st * 256u + (uint32_t)ln * 8u) % linRc;
				}
#endif
			}
			else {
				{  // luma: ln 0..3 the MB above's bottom rows (this column, final now); 4..19 the left MB
					const bool top = ln < 4;
					const uint32_t col = top ? cu : cu - 1;
					srcY = tY + ln * kTP + (top ? slot : slot ^ 1) * 16;
					yl0 = ld64(srcY), yl1 = ld64(srcY + 8);
					const bool ok = act && (fl_bits & 1u) && (top || c > 0);
					const bool to_ctx = ok && (fl_bits & 2u);
					if (to_ctx) ctx.wr128(lf_off(col) + (ln - 16) * 16, u32x4{yl0.x, yl0.y, yl1.x, yl1.y});
#if VP8G_ABLATE & 16  // diagnostic: same stores, linearised per half (whole lines; output wrong)
					const uint32_t linR = (H * sy) / (2 * NW) & ~1023u;
					const uint32_t colpx = col * 16u, off = (uint32_t)(wave * 2 + hh) * linR + ((k * T + t) * 512u + (uint32_t)ln * 16u) % linR;
#else
					const uint32_t colpx = col * 16u, off = fl_offY + colpx;
#endif
					const bool vis = ok && !to_ctx && !(VP8G_ABLATE & 4);
					const bool full = (fl_bits & 4u) && colpx + 16u <= W;
					offY = vis && full ? off : kNoStore;
					poffY = off, pcntY = vis && !full ? min(W - colpx, 16u) : 0u;
				}
				{  // chroma: plane ln / 12, tile row ln % 12 (same split)
					const int p = ln >= 12 ? 1 : 0, kr = ln - 12 * p;
					const bool top = kr < 4;
					const uint32_t col = top ? cu : cu - 1;
					srcC = tC + p * kCV + kr * kTP + (top ? slot : slot ^ 1) * 8;
					cl0 = ldc64(srcC);
					const bool ok = act && (fl_bits & 8u) && (top || c > 0);
					const bool to_ctx = ok && (fl_bits & 16u);
					if (to_ctx) ctx.wr64(lf_off(col) + 64 + p * 32 + (kr - 8) * 8, cl0);
#if VP8G_ABLATE & 16
					const uint32_t linRc = (CH * suv) / (2 * NW) & ~1023u;
					const uint32_t colpx = col * 8u, off = (uint32_t)(wave * 2 + hh) * linRc + ((k * T + t) * 256u + (uint32_t)ln * 8u) % linRc;
#else
					const uint32_t colpx = col * 8u, off = fl_offC + colpx;
#endif
					const bool vis = ok && !to_ctx && !(VP8G_ABLATE & 4);
					const bool full = (fl_bits & 32u) && colpx + 8u <= CW;
					offC = vis && full ? off : kNoStore;
					poffC = off, pcntC = vis && !full ? min(CW - colpx, 8u) : 0u;
				}
			}
			auto pixel_stores = [&]() {
				bst128(rY, offY, u32x4{yl0.x, yl0.y, yl1.x, yl1.y});
				bst64(rC, offC, cl0);
				if (__ballot(pcntY | pcntC) != 0ull) {
					for (uint32_t q = 0; q < pcntY; q++) outY[poffY + q] = srcY[q];
					for (uint32_t q = 0; q < pcntC; q++) outU[poffC + q] = srcC[q];
				}
			};
			// (round 5: issued after the publish instead, which the next wave waits on: +5.9 %, r05g -- the
			// compiler then drains every outstanding store, vmcnt(0), at the top of each step)
			pixel_stores();
			if (lf_on) {
				const bool last_row = r + 1 == R;
				// tile row t of a column holds image row (MB row origin) + t - 4; rows >= 16 (luma) /
				// >= 8 (chroma) are the bottom 4 rows the next MB row still filters: to ctx_lf unless
				// this is the last MB row
				auto flushY = [&](bool ok, int trow, uint32_t col, int sl) {
					const uint8_t* src = tY + trow * kTP + sl * 16;
					const u32x2 lo = ld64(src), hi = ld64(src + 8);
					const bool to_ctx = ok && trow >= 16 && !last_row;
					if (to_ctx) ctx.wr128(lf_off(col) + (trow - 16) * 16, u32x4{lo.x, lo.y, hi.x, hi.y});
					emitY(ok && !to_ctx, y0 + trow - 4, col, src, lo, hi);
				};
				auto flushC = [&](bool ok, int p, int trow, uint32_t col, int sl) {
					const uint8_t* src = tC + p * kCV + trow * kTP + sl * 8;
					const u32x2 lo = ldc64(src);
					const bool to_ctx = ok && trow >= 8 && !last_row;
					if (to_ctx) ctx.wr64(lf_off(col) + 64 + p * 32 + (trow - 8) * 8, lo);
					emitC(ok && !to_ctx, p, cy0 + trow - 4, col, src, lo);
				};
				SUBMARK(21);
				if (__ballot(act && cu + 1 == C) != 0ull) {  // last column: its own rows are final too
					const bool own = act && cu + 1 == C;
					flushY(own && ln < 16, 4 + ln, cu, slot);
					flushC(own && ln < 16, ln >> 3, 4 + (ln & 7), cu, slot);
				}
			}
			wave_lds_sync();
			STAMP(6);

			if (kC && snap_out && t + 1u == T) {
				// top segment of a mirror-split frame, last step of its last pair: every column's context
				// is final -> snapshot (write-through stores, drained) -> flag = this launch's epoch
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
				const uint32_t nb = C * (uint32_t)kCtxBytesPerCol;
				const Rsrc rsn = plane_rsrc(gctx + (size_t)fcur * slot_bytes, nb);
				for (uint32_t o0 = (uint32_t)lane0 * 16u; !kG && o0 < nb; o0 += 1024u * kSnapBatch) {
					u32x4 v[kSnapBatch];
#pragma unroll
					for (int i = 0; i < kSnapBatch; i++) v[i] = ld128(ctx.lds + min(o0 + 1024u * i, nb - 16u));
#pragma unroll
					for (int i = 0; i < kSnapBatch; i++)  // (sc1: write-through to the device-coherent level; lanes past the end dropped)
						__builtin_amdgcn_raw_buffer_store_b128(v[i], rsn, (int)(o0 + 1024u * i), 0, kCpolSc1);
				}
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				if (lane0 == 0) __hip_atomic_store(gprog + fcur, nsplit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
			// ---------------------------------------------- publish progress
			PRIO_AFTER(7, 6);
			ctx.publish_fence();
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			if (kS && xout) {
				// the ctx entries this step finished (rec of column t - 2, lf of column t - 3, and at the
				// last step lf of column C - 1) -> mailbox, write-through; drained before the flag
				const int cl = lane0 < 2 ? (int)t - 2 : (lane0 < 10 ? (int)t - 3 : (t + 1 == T ? (int)C - 1 : -1));
				const uint32_t o = lane0 < 2 ? 16u * (uint32_t)lane0 : 32u + 16u * (uint32_t)((lane0 - 2) & 7);
				if (lane0 < 18 && cl >= 0 && cl < (int)C) {
					const u32x4 v = ld128(ctx.lds + (uint32_t)cl * kCtxBytesPerCol + o);
					uint32_t* q = (uint32_t*)(mb_out + (size_t)cl * kCtxBytesPerCol + o);
					__hip_atomic_store(q, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					__hip_atomic_store(q + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					__hip_atomic_store(q + 2, v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					__hip_atomic_store(q + 3, v.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				}
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				if (lane == 0) __hip_atomic_store(gp_out, k * CP2 + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
			if (lane == 0 && wave != VP8G_TEST_STALL_WAVE)
				__hip_atomic_store(prog + wave, (g << kProgShift) + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
			STAMP(7);
		}
	}
#ifdef VP8G_STAMPS
	if (lane0 == 0)
		for (int i = 0; i < 14; i++)
			if (i != 8 && i != 9) atomicAdd(&g_vp8g_stamps[i], (unsigned long long)st_acc[i]);
	if (f == 0 && lane0 == 0 && wave < 32) g_vp8g_wave_times[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
	if (blockIdx.x < 512 && wave < 16 && lane0 == 0) {
		uint32_t hw, xcc;
		asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
		asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
		g_vp8g_wave_info[2 * (blockIdx.x * 16 + wave)] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
		g_vp8g_wave_info[2 * (blockIdx.x * 16 + wave) + 1] = __builtin_amdgcn_s_memrealtime() - st_t0;
	}
	if (f == 0 && lane0 == 0 && wave == 0) {
		g_vp8g_stamps[8] = __builtin_amdgcn_s_memtime();
		g_vp8g_stamps[9] = __builtin_amdgcn_s_memrealtime();
	}
#endif
}

#include "vp8g_quad.inc"

// The dynamic-LDS limit of a kernel instantiation, set once to the whole of the CU's LDS (the
// kernel has no static LDS): concurrent launches from several threads then never race a smaller
// value set by another thread between its own set and launch.
template <int NW, bool kG, bool kS, bool kC>
hipError_t lds_attr() {
	static const hipError_t e =
	    hipFuncSetAttribute((const void*)frame_kernel<NW, kG, kS, kC>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds);
	return e;
}

template <int NW, bool kG, bool kS>
hipError_t launch_t(const Vp8gFrameDesc* d_descs, uint32_t n, const Vp8gBatchArrays& arrays, uint8_t* d_out,
                    uint32_t ctx_cols, uint8_t* gctx, uint32_t nsplit, uint8_t* mbox, uint32_t* gprog, hipStream_t stream,
                    uint32_t ord_first = 0) {
	const size_t lds = lds_bytes(NW, ctx_cols, kG);
	auto fn = frame_kernel<NW, kG, kS, false>;
	if (lds > 65536) {
		hipError_t e = lds_attr<NW, kG, kS, false>();
		if (e != hipSuccess) return e;
	}
	hipLaunchKernelGGL(fn, dim3(n * (kS ? nsplit : 1u)), dim3(NW * 64), lds, stream, d_descs, arrays, d_out, ctx_cols, gctx,
	                   nsplit, mbox, gprog, kS ? 0u : ord_first, 0u);
	return hipGetLastError();
}

}  // namespace

#ifdef VP8G_STAMPS
extern "C" __attribute__((visibility("default"))) int vp8g_debug_wave_times(unsigned long long* out) {
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vp8g_wave_times), sizeof(unsigned long long) * 64) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int vp8g_debug_wave_info(unsigned long long* out) {
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vp8g_wave_info), sizeof(unsigned long long) * 512 * 16 * 2) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int vp8g_debug_stamps(unsigned long long* out, int reset) {
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vp8g_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
	if (reset) {
		unsigned long long z[16] = {0};
		if (hipMemcpyToSymbol(HIP_SYMBOL(g_vp8g_stamps), z, sizeof(z)) != hipSuccess) return -1;
	}
	return 0;
}
#endif

int device_cus() {
	static const int n_cus = [] {
		int dev = 0, n = 0;
		if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
			n = 0;
		return n;
	}();
	return n_cus;
}

uint32_t pick_waves(uint32_t waves_hint, uint32_t max_mb_rows, uint32_t n_frames) {
	static const uint32_t kSupported[] = {1, 2, 4, 8, 12, 16};
	// default: 8 waves (two frames per CU) when the batch fills the chip; a batch with at most
	// one frame per CU gets 16 waves per frame instead (twice the MB row pairs in flight)
	const int n_cus = device_cus();
	uint32_t want = waves_hint ? waves_hint : (n_cus > 0 && n_frames <= (uint32_t)n_cus ? 16u : 8u);
	const uint32_t pairs = (max_mb_rows + 1) / 2;
	if (want > pairs) want = pairs;  // no point in more waves than MB row pairs
	uint32_t nw = 1;
	for (uint32_t s : kSupported)
		if (s <= want) nw = s;
	return nw;
}

uint32_t pick_split(uint32_t split_hint, uint32_t n_frames, uint32_t nw, uint32_t max_mb_rows) {
	if (nw != 8 && nw != 16) return 1;  // split kernels exist for these only
	const int n_cus = device_cus();
	const uint32_t pairs = (max_mb_rows + 1) / 2;
	uint32_t k = split_hint ? split_hint : (n_cus > 0 ? (uint32_t)n_cus / (n_frames ? n_frames : 1u) : 1u);
	if (k > kMaxSplit) k = kMaxSplit;
	while (k > 1 && (k - 1) * nw >= pairs) k--;  // every part gets at least one pair
	// all parts of all frames must be resident together: at most one part per CU
	if (n_cus <= 0 || (uint64_t)n_frames * k > (uint64_t)n_cus) k = 1;
	return k ? k : 1;
}

uint32_t pick_order(const Vp8gFrameDesc* h_descs, uint32_t n_frames, uint32_t nsplit) {
	static const bool off = [] {  // VP8G_ORDER=0: launch in batch order (A/B experiments)
		const char* e = getenv("VP8G_ORDER");
		return e && e[0] == '0';
	}();
#ifdef VP8G_NO_ORDER  // diagnostic build: batch order always
	return 0;
#endif
	const int n_cus = device_cus();
	if (off || nsplit > 1 || n_cus <= 0 || n_frames <= (uint32_t)n_cus) return 0;
	const uint32_t c0 = cost_class(h_descs[0]);
	for (uint32_t i = 1; i < n_frames; i++)
		if (cost_class(h_descs[i]) != c0) return (uint32_t)n_cus;
	return 0;  // uniform batch: the order would be the identity
}

uint32_t pick_chain(const Vp8gFrameDesc* h_descs, uint32_t n_frames, uint32_t ctx_cols, bool* ordered, bool quad) {
#ifndef VP8G_CHAIN_DEFAULT  // (A/B builds: -DVP8G_CHAIN_DEFAULT=0)
#define VP8G_CHAIN_DEFAULT -1
#endif
	static const int mode = [] {  // VP8G_CHAIN=0: never (A/B experiments), =1: also for batches <= the CU count
		const char* e = getenv("VP8G_CHAIN");
		return e ? atoi(e) : VP8G_CHAIN_DEFAULT;
	}();
	*ordered = false;
	const int n_cus = device_cus();
	if (mode == 0 || n_cus <= 0 || n_frames == 0 || (mode < 0 && n_frames <= (uint32_t)n_cus)) return 0;
	const uint32_t slots = (uint32_t)n_cus * (uint32_t)kChainWgPerCu;
	const uint32_t wg = n_frames < slots ? n_frames : slots;
	const uint32_t list_max = (n_frames + wg - 1) / wg;
	if (ctx_cols > 1024 || (size_t)(quad ? 1 : kChainWgPerCu) * chain_lds_bytes(ctx_cols, list_max, n_frames, false, quad) > (size_t)kMaxLds)
		return 0;
	// cost-class placement when the classes differ and the sort scratch fits the context slots
	const uint32_t c0 = cost_class(h_descs[0]);
	bool differ = false;
	for (uint32_t i = 1; i < n_frames && !differ; i++) differ = cost_class(h_descs[i]) != c0;
	*ordered = differ && (size_t)4 * (kCostClasses + n_frames) <= chain_ctx_lds(ctx_cols, n_frames, false, quad) && pick_order(h_descs, n_frames, 1) != 0;
	return wg;
}

bool pick_chain_split(uint32_t n_frames, uint32_t ctx_cols, uint32_t workgroups, bool ordered, bool quad) {
#ifndef VP8G_SPLITCHAIN_DEFAULT  // (A/B builds: -DVP8G_SPLITCHAIN_DEFAULT=0 / 1)
#define VP8G_SPLITCHAIN_DEFAULT -1
#endif
	static const int mode = [] {  // VP8G_SPLITCHAIN=0: never, =1: whenever it fits (A/B experiments, tests)
		const char* e = getenv("VP8G_SPLITCHAIN");
		return e ? atoi(e) : VP8G_SPLITCHAIN_DEFAULT;
	}();
	if (mode == 0 || workgroups == 0) return false;
	const uint32_t list_max = (n_frames + workgroups - 1) / workgroups;
	if ((size_t)(quad ? 1 : kChainWgPerCu) * chain_lds_bytes(ctx_cols, 2 * list_max, n_frames, false, quad) > (size_t)kMaxLds) return false;
	return mode > 0 || (ordered && list_max <= 2);
}

bool pick_chain_interleave(const Vp8gFrameDesc* h_descs, uint32_t n_frames, uint32_t ctx_cols, uint32_t workgroups, bool split,
                           bool quad) {
#ifndef VP8G_CHAIN_IL_DEFAULT  // (A/B builds: -DVP8G_CHAIN_IL_DEFAULT=0)
#define VP8G_CHAIN_IL_DEFAULT -1
#endif
	static const int mode = [] {  // VP8G_CHAIN_IL=0: never, =1: wherever it fits (A/B experiments, tests)
		const char* e = getenv("VP8G_CHAIN_IL");
		return e ? atoi(e) : VP8G_CHAIN_IL_DEFAULT;
	}();
	if (mode == 0 || (kChainG && !quad) || split || workgroups == 0 || n_frames < 2 * workgroups) return false;
	for (uint32_t i = 1; i < n_frames; i++)
		if (h_descs[i].mb_cols != h_descs[0].mb_cols || h_descs[i].mb_rows != h_descs[0].mb_rows) return false;
	if (h_descs[0].mb_rows < 2) return false;
	const uint32_t list_max = (n_frames + workgroups - 1) / workgroups;
	return (size_t)(quad ? 1 : kChainWgPerCu) * chain_lds_bytes(ctx_cols, list_max, n_frames, true, quad) <= (size_t)kMaxLds;
}

bool quad_supported(const Vp8gFrameDesc* h_descs, uint32_t n_frames) {
	// every frame but loop-filter-only ones (frames without whole row pieces take the quad kernel's
	// byte path at the right edge / for unaligned planes)
	for (uint32_t i = 0; i < n_frames; i++)
		if (h_descs[i].mb_cols != 0 && h_descs[i].mb_rows != 0 && (h_descs[i].flags & VP8G_F_LF_ONLY)) return false;
	return true;
}

bool whole_pieces(const Vp8gFrameDesc* h_descs, uint32_t n_frames) {
	// every 16-B luma / 8-B chroma row piece inside its frame and aligned (the output base is at least
	// 16-B aligned): the quad kernel's lean instantiation
	for (uint32_t i = 0; i < n_frames; i++) {
		const Vp8gFrameDesc& d = h_descs[i];
		if (d.mb_cols == 0 || d.mb_rows == 0) continue;
		if (d.width != 16u * d.mb_cols || ((d.out_y | d.stride_y) & 15u) != 0 || ((d.out_u | d.stride_uv | (d.out_v - d.out_u)) & 7u) != 0)
			return false;
	}
	return true;
}

bool pick_quad(const Vp8gFrameDesc* h_descs, uint32_t n_frames) {
#ifndef VP8G_QUAD_DEFAULT  // (A/B builds: -DVP8G_QUAD_DEFAULT=0, the two-rows-per-wave chain)
#define VP8G_QUAD_DEFAULT 1
#endif
	static const int mode = [] {  // VP8G_QUAD=0: never (A/B experiments)
		const char* e = getenv("VP8G_QUAD");
		return e ? atoi(e) : VP8G_QUAD_DEFAULT;
	}();
	return mode != 0 && quad_supported(h_descs, n_frames);
}

hipError_t launch_chain(const Vp8gFrameDesc* d_descs, uint32_t n_frames, const Vp8gBatchArrays& arrays, uint8_t* d_out,
                        uint32_t ctx_cols, hipStream_t stream, uint32_t workgroups, bool ordered, bool split, uint8_t* snap,
                        uint32_t* flags, uint32_t epoch, bool interleave, bool quad, bool whole) {
	if (n_frames == 0) return hipSuccess;
	if ((split && (!snap || !flags)) || (kChainG && !snap) || (interleave && split)) return hipErrorInvalidValue;
	const uint32_t list_max = (n_frames + workgroups - 1) / workgroups;
	const size_t lds = chain_lds_bytes(ctx_cols, split ? 2 * list_max : list_max, n_frames, interleave, quad);
	if (quad) {  // four MB rows per wave; the snapshot buffer holds every frame's context
		if (!snap) return hipErrorInvalidValue;
		static const hipError_t eq1 =
		    hipFuncSetAttribute((const void*)quad_kernel<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds);
		static const hipError_t eq0 =
		    hipFuncSetAttribute((const void*)quad_kernel<16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds);
		if (eq1 != hipSuccess) return eq1;
		if (eq0 != hipSuccess) return eq0;
		auto fq = whole ? quad_kernel<16, true> : quad_kernel<16, false>;
		hipLaunchKernelGGL(fq, dim3(workgroups), dim3(16 * 64), lds, stream, d_descs, arrays, d_out, ctx_cols, snap,
		                   split ? epoch : 1u, split ? flags : nullptr, (ordered ? 1u : 0u) | (split ? 2u : 0u) | (interleave ? 4u : 0u),
		                   n_frames);
		return hipGetLastError();
	}
	auto fn = frame_kernel<kChainWaves, kChainG, false, true>;
	hipError_t e = lds_attr<kChainWaves, kChainG, false, true>();
	if (e != hipSuccess) return e;
	// (chain kernel arguments: gctx = snapshots -- with the context in device memory, the frames'
	// contexts, n_frames x ctx_cols x kCtxBytesPerCol --, gprog = flags, nsplit = epoch,
	// ord_first = ordered | split << 1)
	hipLaunchKernelGGL(fn, dim3(workgroups), dim3(kChainWaves * 64), lds, stream, d_descs, arrays, d_out, ctx_cols,
	                   split || kChainG ? snap : nullptr, split ? epoch : 1u, nullptr, split ? flags : nullptr,
	                   (ordered ? 1u : 0u) | (split ? 2u : 0u) | (interleave ? 4u : 0u), n_frames);
	return hipGetLastError();
}

hipError_t launch_frames(const Vp8gFrameDesc* d_descs, uint32_t n_frames, const Vp8gBatchArrays& arrays,
                         uint8_t* d_out, uint32_t ctx_cols, uint32_t max_mb_rows, uint8_t* global_ctx,
                         hipStream_t stream, uint32_t waves_hint, uint32_t nsplit, uint8_t* mbox, uint32_t* gprog,
                         uint32_t ord_first) {
	if (n_frames == 0) return hipSuccess;
	if (ord_first >= n_frames) ord_first = 0;  // (the order maps positions >= ord_first; needs n > ord_first)
	const uint32_t nw = pick_waves(waves_hint, max_mb_rows, n_frames);
	const bool g = global_ctx != nullptr;
	if (nsplit > 1 && !g && (nw == 8 || nw == 16)) {
		if (!mbox || !gprog) return hipErrorInvalidValue;
		return nw == 8 ? launch_t<8, false, true>(d_descs, n_frames, arrays, d_out, ctx_cols, nullptr, nsplit, mbox, gprog, stream)
		               : launch_t<16, false, true>(d_descs, n_frames, arrays, d_out, ctx_cols, nullptr, nsplit, mbox, gprog, stream);
	}
#define VP8G_CASE(N)                                                                                                          \
	case N:                                                                                                                   \
		return g ? launch_t<N, true, false>(d_descs, n_frames, arrays, d_out, ctx_cols, global_ctx, 1, nullptr, nullptr, stream, \
		                                    ord_first)                                                                        \
		         : launch_t<N, false, false>(d_descs, n_frames, arrays, d_out, ctx_cols, nullptr, 1, nullptr, nullptr, stream, ord_first);
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
