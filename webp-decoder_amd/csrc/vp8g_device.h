// vp8g_device.h -- internal interface between the C-ABI shim and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "vp8g.h"

namespace vp8g {

// Per-half-wave LDS scratch (bytes).  A wave works on two macroblocks at once, one per 32-lane
// half; each half owns one of these areas.  16-B aligned where a 16-B access is made.
// Filter tiles (luma 20 rows, chroma 12 rows, one pitch: the horizontal-edge pass reads every
// plane's lines with one set of immediate row offsets), each row a ring of two MB columns (slot =
// mb_col & 1).  Their placement sets the LDS bank conflicts of the loop filter's byte gathers
// (tools/lds_banks.py): 32 lines per 32-lane half -- 16 luma, 8 U and 8 V rows in the vertical-edge
// pass -- should spread over the 32 banks.  With the chroma tile 4 bytes off 8-B alignment the
// chroma 8-B pieces are accessed as two dwords (kC8).
#ifndef VP8G_TP
#define VP8G_TP 40
#endif
#ifndef VP8G_UV
#define VP8G_UV 804
#endif
#ifndef VP8G_CV
#define VP8G_CV 64
#endif
constexpr int kTP = VP8G_TP;    // tile row pitch
constexpr int kLfY = 0;         // luma filter tile: 20 rows x kTP (4 rows above + 16 MB rows; two MB
                                // columns as a ring at +0 / +16)
constexpr int kLfUV = VP8G_UV;  // chroma tile: 12 rows x kTP (4 above + 8 MB rows); per row U at +0,
constexpr int kCV = VP8G_CV;    // V at +kCV, each a ring of two 8-B MB columns
constexpr bool kC8 = kLfUV % 8 == 0 && kTP % 8 == 0 && kCV % 8 == 0;  // chroma 8-B pieces 8-B aligned
// V rows may sit rows away from their U rows (kCV >= kTP: V row r shares a physical row with U row
// r + kCV / kTP, in bytes kCV % kTP ..+16): with kCV = 64 at pitch 40 (V at 24..39 of the next row)
// the 32 rows a vertical-edge gather touches -- 16 luma, 8 U, 8 V -- fall on 32 distinct banks
// (tools/lds_banks.py), where U and V side by side (kCV = 16) met two rows per bank.
static_assert(kLfUV >= 20 * kTP && kCV % kTP >= 16 && kCV % kTP + 16 <= kTP, "tile layout");
constexpr int kUVBytes = 12 * kTP > kCV + 11 * kTP + 16 ? 12 * kTP : kCV + 11 * kTP + 16;  // chroma tile span
constexpr int kAbY = (kLfUV + kUVBytes + 15) & ~15;  // luma above row: [15] corner P, [16..31] A, [32..35] above-right
constexpr int kAbUV = kAbY + 48;   // chroma above rows: U P@7 A@8..15, V P@23 A@24..31
constexpr int kColY = kAbUV + 32;  // B_PRED: luma columns 11, 7, 3 of the MB (16 B each, in that order),
                                   // so that the left column of sub-block column j is at kLeft - 16 j
constexpr int kLeft = kColY + 48;  // unfiltered left columns: Y 0..15, U 16..23, V 24..31
constexpr int kResid = kLeft + 32;  // luma residual of the MB (for B_PRED): 16 blocks x 16 int16
constexpr int kWht = kResid + 512;  // 16 int16 luma DCs out of the inverse WHT
constexpr int kHalfBytes = kWht + 32;
constexpr int kWaveBytes = 2 * kHalfBytes;

// Workgroup header.
constexpr int kProgress = 0;      // 16 x u32 progress words (one per wave)
constexpr int kBpTable = 64;      // B_PRED predictor table: 11 modes x 16 px x {perm selectors, byte
                                  // mask, dot weights, bias | shift}
constexpr int kBpModes = 11;      // modes 0..9 + one constant-128 entry for out-of-range modes
constexpr int kBpEntry = 16;      // bytes per (mode, pixel) entry
constexpr int kDqTable = kBpTable + kBpModes * 16 * kBpEntry;  // 4 segments x 6 int16 dequant factors
constexpr int kLfTable = kDqTable + 48;                 // 4 segments x 2 (B_PRED?) x {E, I, T, 0}
constexpr int kTabStride = 80;                          // per frame slot (chain mode: two slots, four interleaved)
constexpr int kTabSlots = 4;
constexpr int kMisc = kDqTable + kTabSlots * kTabStride;  // chain mode: list length
constexpr int kRoleTab = kMisc + 16;                    // whole-block predictor lane roles: 32 lanes x 8 B
constexpr int kHdrBytes = kRoleTab + 256;

// Shared per-MB-column context (one frame per workgroup).
constexpr int kCtxRecBytes = 32;   // unfiltered bottom row: Y 16, U 8, V 8 (intra prediction)
constexpr int kCtxLfBytes = 128;   // bottom 4 rows, filter state: Y 4x16, U 4x8, V 4x8 (loop filter)
constexpr int kCtxBytesPerCol = kCtxRecBytes + kCtxLfBytes;

constexpr int kMaxLds = 163840;

// Launch order (cost-balanced placement).  A frame's time is set by its size and by how much its
// loop filter filters (profiles/r02b_wave_placement.json: 4K frames at filter level 2 take 11.2 ms,
// at 40-63 14.8 ms); workgroups b and b + CUs share a CU.  cost_class is a coarse log2 of
// MBs x (64 + the frame's largest MB-edge limit 2E + I, halved for the simple filter): 4 classes
// per octave, 0..127, higher = heavier.
constexpr uint32_t kCostClasses = 128;
__host__ __device__ inline uint32_t cost_class(const Vp8gFrameDesc& d) {
	uint32_t s = 0;
	if (d.flags & VP8G_F_LOOPFILTER) {
		for (int g = 0; g < 4; g++)
			for (int b = 0; b < 2; b++) {
				const uint32_t v = 2u * d.lf[g][b][0] + d.lf[g][b][1];
				s = v > s ? v : s;
			}
		if (d.flags & VP8G_F_SIMPLE) s >>= 1;
	}
	const uint64_t cost = (uint64_t)d.mb_cols * d.mb_rows * (64u + s);  // < 2^27 for valid frames
	if (cost < 4u) return 0u;  // an empty (all-zero) descriptor: a no-op slot, the lightest class
	if (cost >= (1ull << 31)) return kCostClasses - 1u;
	const uint32_t lg = 63u - (uint32_t)__builtin_clzll(cost);
	return 4u * lg + (uint32_t)((cost >> (lg - 2u)) & 3u);
}

inline size_t lds_bytes(int waves, uint32_t ctx_cols, bool global_ctx) {
	return (size_t)kHdrBytes + (size_t)waves * kWaveBytes + (global_ctx ? 0 : (size_t)ctx_cols * kCtxBytesPerCol);
}
// Chain mode (one 16-wave workgroup per CU decoding a list of frames, vp8g_kernels.hip): two
// context slots and the list (at most list_max frames).
// Experiment builds: VP8G_CHAIN_G = 1 keeps the chain's per-column context in device memory (one
// region per frame; the LDS then holds only the cost sort's scratch), which lets VP8G_CHAIN_WPC
// workgroups of VP8G_CHAIN_NW waves share a CU (e.g. 2 x 12 waves at 6 waves per SIMD).
#ifndef VP8G_CHAIN_NW
#define VP8G_CHAIN_NW 16
#endif
#ifndef VP8G_CHAIN_G
#define VP8G_CHAIN_G 0
#endif
#ifndef VP8G_CHAIN_WPC
#define VP8G_CHAIN_WPC 1
#endif
constexpr int kChainWaves = VP8G_CHAIN_NW;
constexpr bool kChainG = VP8G_CHAIN_G != 0;
constexpr int kChainWgPerCu = VP8G_CHAIN_WPC;
// LDS context area of a chain workgroup: the two context slots (four when two frames run
// interleaved, see pick_chain_interleave), or (global context) the cost sort's scratch of
// kCostClasses + n_frames words
// Four MB rows per wave (the quad chain kernel, vp8g_quad.inc): a wave's LDS is four
// quarter areas (the half layout without the iWHT scratch) and four 3-column context rings; the
// context between waves lives in device memory (the snapshot buffer, one region per frame), so the
// quad chain's LDS does not depend on the frame width.  Chosen per batch (pick_quad).
#ifndef VP8G_QPAD  // (experiment: quarter stride padding; 4 puts quarters 1 and 3 on the odd LDS banks)
#define VP8G_QPAD 0
#endif
constexpr int kQuarterBytes = kWht + VP8G_QPAD;              // tile, borders, B_PRED buffers, residual park
constexpr int kRingBytes = 3 * kCtxBytesPerCol;              // three MB columns of context
constexpr int kQRings = kHdrBytes + 4 * kQuarterBytes;       // wave-relative: ring h at + h * kRingBytes
constexpr int kQWaveBytes = 4 * kQuarterBytes + 4 * kRingBytes;
constexpr int kQList = kHdrBytes + 16 * kQWaveBytes;         // the chain list (after 16 wave areas)
inline size_t chain_ctx_lds(uint32_t ctx_cols, uint32_t n_frames, bool il = false, bool quad = false) {
	if (quad) return (size_t)16 * kQWaveBytes;  // (the cost sort's scratch sits in the wave areas)
	return kChainG ? ((size_t)4 * (kCostClasses + n_frames) + 15) & ~(size_t)15
	               : (il ? 4 : 2) * (size_t)ctx_cols * kCtxBytesPerCol;
}
inline size_t chain_lds_bytes(uint32_t ctx_cols, uint32_t list_max, uint32_t n_frames, bool il = false, bool quad = false) {
	if (quad) return (size_t)kQList + 4 * (size_t)list_max;
	return (size_t)kHdrBytes + (size_t)kChainWaves * kWaveBytes + chain_ctx_lds(ctx_cols, n_frames, il) + 4 * (size_t)list_max;
}

// Process-wide launch gate (vp8g_shim.hip).  Launch modes whose workgroups wait on each other across
// CUs -- split parts (launch_frames with nsplit > 1) and the chain's mirror split -- need every
// workgroup of the launch resident at once.  Beside another kernel of this library (an earlier
// asynchronous batch on another stream, a pipeline chunk, a device-m05 or writer kernel) some of
// them could wait for CUs that the others hold while they spin; two such launches side by side
// would both run into the bounded wait and fail with VP8G_ERR_TIMEOUT.  So every kernel launch of
// the library is enqueued inside a GateScope, which holds one process-wide mutex from the decision
// to the last enqueue:
//   * the scope's stream is first ordered after a cross-workgroup launch still in flight on
//     another stream (hipStreamWaitEvent), so nothing starts beside one;
//   * may_cross() is true only when no launch of the library is in flight on any other stream
//     (hipEventQuery of each stream's last recorded launch), so a cross-workgroup launch never
//     starts beside another kernel;
//   * done(crossed) records the launch's completion event for the next caller.
// Kernels launched by the caller's own code on other streams are outside the gate.
class GateScope {
   public:
	explicit GateScope(hipStream_t s);
	~GateScope();
	GateScope(const GateScope&) = delete;
	GateScope& operator=(const GateScope&) = delete;
	hipError_t status() const { return err_; }
	bool may_cross() const { return may_cross_; }
	hipError_t done(bool crossed);

   private:
	hipStream_t s_;
	hipError_t err_ = hipSuccess;
	bool may_cross_ = false;
};

// Launch the fused recon(+LF) kernel.  `global_ctx` != nullptr selects the variant whose
// per-column context lives in device memory (frames too wide for LDS); it must hold
// n_frames * ctx_cols * kCtxBytesPerCol bytes.
// nsplit > 1 (LDS context, 8 or 16 waves only): each frame is worked on by nsplit workgroups
// that hand off through `mbox` (n_frames * nsplit * ctx_cols * kCtxBytesPerCol bytes) and
// `gprog` (n_frames * nsplit words, zeroed before the launch).
hipError_t launch_frames(const Vp8gFrameDesc* d_descs, uint32_t n_frames, const Vp8gBatchArrays& arrays,
                         uint8_t* d_out, uint32_t ctx_cols, uint32_t max_mb_rows, uint8_t* global_ctx,
                         hipStream_t stream, uint32_t waves_hint, uint32_t nsplit, uint8_t* mbox, uint32_t* gprog,
                         uint32_t ord_first = 0);
// ord_first != 0 (unsplit launches of more than ord_first frames): workgroup w decodes the frame at
// position p(w) of the batch sorted by descending cost_class (stable): the first F = ord_first
// workgroups the F heaviest frames, the next S = min(n - F, F) the S lightest in reverse (so the
// heaviest frame shares its CU with the lightest), the rest the middle positions heaviest first.
// pick_order returns F = the CU count when that is worth it (classes differ, more frames than
// CUs), else 0.
uint32_t pick_order(const Vp8gFrameDesc* h_descs, uint32_t n_frames, uint32_t nsplit);

// Chain mode for n_frames frames on this device: the workgroup count (0 = not applicable: too few
// frames, a context too wide for two LDS slots, or VP8G_CHAIN=0), and whether the frames are
// placed by cost class (*ordered; needs the sort scratch to fit the context slots).
uint32_t pick_chain(const Vp8gFrameDesc* h_descs, uint32_t n_frames, uint32_t ctx_cols, bool* ordered, bool quad = false);
// Mirror split of a chain launch (vp8g_kernels.hip, kSegTop): worth it for ordered batches of at most
// two frames per workgroup (VP8G_SPLITCHAIN=0 / 1 forces it off / on), and the doubled list must fit.
bool pick_chain_split(uint32_t n_frames, uint32_t ctx_cols, uint32_t workgroups, bool ordered, bool quad = false);
// Two-frame interleave of a chain launch (vp8g_kernels.hip): the frames of a workgroup's list run two
// at a time with their MB row pairs alternating (the pair above is two global pairs back), which
// halves the chain's fill and drain.  Needs every frame of the batch the same size, four context
// slots in LDS and no mirror split (VP8G_CHAIN_IL=0 / 1 forces it off / on where it fits).
bool pick_chain_interleave(const Vp8gFrameDesc* h_descs, uint32_t n_frames, uint32_t ctx_cols, uint32_t workgroups, bool split,
                           bool quad = false);
// The quad chain kernel for this batch: no frame is loop-filter-only (quad_supported), and VP8G_QUAD
// is not 0 (A/B experiments).  whole_pieces: every frame has whole, aligned 16-B / 8-B row pieces, so
// launch_chain(..., whole = true) takes the kernel's lean instantiation (the general one adds a byte
// path for pieces cut by the right edge or unaligned planes).  A quad launch needs
// `snap` (every frame's context, n_frames * ctx_cols * kCtxBytesPerCol bytes) in every mode.
bool quad_supported(const Vp8gFrameDesc* h_descs, uint32_t n_frames);
bool pick_quad(const Vp8gFrameDesc* h_descs, uint32_t n_frames);
bool whole_pieces(const Vp8gFrameDesc* h_descs, uint32_t n_frames);
// split: `snap` holds n_frames * ctx_cols * kCtxBytesPerCol bytes, `flags` n_frames words that hold
// no value equal to `epoch` (a per-launch counter) before the launch.
hipError_t launch_chain(const Vp8gFrameDesc* d_descs, uint32_t n_frames, const Vp8gBatchArrays& arrays, uint8_t* d_out,
                        uint32_t ctx_cols, hipStream_t stream, uint32_t workgroups, bool ordered, bool split = false,
                        uint8_t* snap = nullptr, uint32_t* flags = nullptr, uint32_t epoch = 0, bool interleave = false,
                        bool quad = false, bool whole = false);

constexpr uint32_t kMaxSplit = 8;
int device_cus();
// Workgroups per frame for this batch: split_hint if non-zero, else CUs / frames, capped at
// kMaxSplit and at one part per CU overall (all parts must be co-resident), 1 if not possible.
uint32_t pick_split(uint32_t split_hint, uint32_t n_frames, uint32_t nw, uint32_t max_mb_rows);

// Waves per workgroup the launcher would use for this batch (for LDS sizing decisions):
// waves_hint if non-zero, else 8, or 16 when n_frames <= the device's CU count.
uint32_t pick_waves(uint32_t waves_hint, uint32_t max_mb_rows, uint32_t n_frames);

// vp8g_make_frame_desc; dense_coeffs = false skips the check of the coeff_* pointers (packed
// frames: the coefficients reach the device through the expansion kernel).
int make_desc(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, int filtered, uint64_t mb_offset, uint64_t out_offset,
              Vp8gFrameDesc* out, bool dense_coeffs);

// Planes in the yuv420_alloc layout; init = false leaves them uninitialised (outputs a D2H
// overwrites completely).
int alloc_planes(Yuv420Image* img, uint32_t width, uint32_t height, bool init);

// Record a HIP failure for vp8g_last_error() (calling thread).
void set_error_text(const char* where, hipError_t e);

}  // namespace vp8g
