// vp8g_shim.hip -- the C-ABI boundary (include/vp8g.h): the reference's m06/m07 entry points and
// the additive batch API, implemented on top of the gfx950 kernels in vp8g_kernels.hip.
//
// Host-side work done here, once per frame (not per MB):
//   * dequantisation factors per segment     -- reference src/m06_recon/vp8_recon.c:57-76
//   * loop-filter level / interior / hev per (segment, B_PRED?) -- src/m07_loopfilter/vp8_loopfilter.c:166-199
//   * frame geometry and output placement, H2D of the nine Vp8DecodedFrame arrays, D2H of I420.
// Errors follow the reference: 0, or -1 with errno (EINVAL bad arguments, ENOMEM allocation);
// HIP failures add EIO (text in vp8g_last_error()).  There is no CPU fallback.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "vp8g_device.h"

#define VP8G_API extern "C" __attribute__((visibility("default")))

namespace {

thread_local char g_err[256];
// launch mode of the calling thread's last reconstruction launch (vp8g_last_launch_mode)
thread_local uint32_t g_mode = 0;

void set_err(const char* where, hipError_t e) {
	snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
}

// RFC 6386 14.1 dequantisation tables (same values as the host front end's vp8_tables.inc)
const int16_t kDcQ[128] = {
    4,   5,   6,   7,   8,   9,   10,  10,  11,  12,  13,  14,  15,  16,  17,  17,  18,  19,  20,  20,  21,  21,
    22,  22,  23,  23,  24,  25,  25,  26,  27,  28,  29,  30,  31,  32,  33,  34,  35,  36,  37,  37,  38,  39,
    40,  41,  42,  43,  44,  45,  46,  46,  47,  48,  49,  50,  51,  52,  53,  54,  55,  56,  57,  58,  59,  60,
    61,  62,  63,  64,  65,  66,  67,  68,  69,  70,  71,  72,  73,  74,  75,  76,  76,  77,  78,  79,  80,  81,
    82,  83,  84,  85,  86,  87,  88,  89,  91,  93,  95,  96,  98,  100, 101, 102, 104, 106, 108, 110, 112, 114,
    116, 118, 122, 124, 126, 128, 130, 132, 134, 136, 138, 140, 143, 145, 148, 151, 154, 157};
const int16_t kAcQ[128] = {
    4,   5,   6,   7,   8,   9,   10,  11,  12,  13,  14,  15,  16,  17,  18,  19,  20,  21,  22,  23,  24,  25,
    26,  27,  28,  29,  30,  31,  32,  33,  34,  35,  36,  37,  38,  39,  40,  41,  42,  43,  44,  45,  46,  47,
    48,  49,  50,  51,  52,  53,  54,  55,  56,  57,  58,  60,  62,  64,  66,  68,  70,  72,  74,  76,  78,  80,
    82,  84,  86,  88,  90,  92,  94,  96,  98,  100, 102, 104, 106, 108, 110, 112, 114, 116, 119, 122, 125, 128,
    131, 134, 137, 140, 143, 146, 149, 152, 155, 158, 161, 164, 167, 170, 173, 177, 181, 185, 189, 193, 197, 201,
    205, 209, 213, 217, 221, 225, 229, 234, 239, 245, 249, 254, 259, 264, 269, 274, 279, 284};

inline int qidx(int q) { return q < 0 ? 0 : (q > 127 ? 127 : q); }

void fill_dequant(const Vp8DecodedFrame* d, Vp8gFrameDesc* out) {
	for (int s = 0; s < 4; s++) {
		int q = d->q_index;
		if (d->segmentation_enabled) q = d->segmentation_abs ? d->seg_quant_idx[s] : q + d->seg_quant_idx[s];
		int y2ac = kAcQ[qidx(q + d->y2_ac_delta_q)] * 155 / 100;
		int uvdc = kDcQ[qidx(q + d->uv_dc_delta_q)];
		out->dq[s][0] = kDcQ[qidx(q + d->y1_dc_delta_q)];
		out->dq[s][1] = kAcQ[qidx(q)];
		out->dq[s][2] = (int16_t)(uvdc > 132 ? 132 : uvdc);
		out->dq[s][3] = kAcQ[qidx(q + d->uv_ac_delta_q)];
		out->dq[s][4] = (int16_t)(2 * kDcQ[qidx(q + d->y2_dc_delta_q)]);
		out->dq[s][5] = (int16_t)(y2ac < 8 ? 8 : y2ac);
	}
}

// returns 1 if any (segment, mode) combination has a non-zero filter level
int fill_loopfilter(const Vp8DecodedFrame* d, Vp8gFrameDesc* out) {
	int any = 0;
	for (int s = 0; s < 4; s++) {
		for (int bp = 0; bp < 2; bp++) {
			int lvl = d->lf_level;
			if (d->segmentation_enabled) lvl = d->segmentation_abs ? d->seg_lf_level[s] : lvl + d->seg_lf_level[s];
			lvl = lvl < 0 ? 0 : (lvl > 63 ? 63 : lvl);
			if (d->lf_delta_enabled) {
				lvl += d->lf_ref_delta[0];
				if (bp) lvl += d->lf_mode_delta[0];
				lvl = lvl < 0 ? 0 : (lvl > 63 ? 63 : lvl);
			}
			int il = lvl;
			if (d->lf_sharpness) {
				il >>= (d->lf_sharpness > 4) ? 2 : 1;
				if (il > 9 - d->lf_sharpness) il = 9 - d->lf_sharpness;
			}
			if (il < 1) il = 1;
			out->lf[s][bp][0] = (uint8_t)lvl;
			out->lf[s][bp][1] = (uint8_t)il;
			out->lf[s][bp][2] = (uint8_t)((lvl >= 40) ? 2 : (lvl >= 15 ? 1 : 0));
			out->lf[s][bp][3] = 0;
			any |= lvl != 0;
		}
	}
	return any;
}

// The arrays the reference's m06/m07 read (vp8_recon.c:423-712, vp8_loopfilter.c:166-283): like the
// reference, segment_id only when segmentation is enabled (a missing map reads as segment 0) and
// has_coeff may be NULL; mb_total is never read (mb_cols * mb_rows sizes everything).
bool frame_ok(const Vp8DecodedFrame* d) {
	return d && d->mb_cols && d->mb_rows && d->mb_cols <= 1024 && d->mb_rows <= 1024 &&
	       (d->segment_id || !d->segmentation_enabled) && d->ymode && d->uv_mode && d->bmode && d->coeff_y2 && d->coeff_y &&
	       d->coeff_u && d->coeff_v;
}
inline uint64_t mb_count(const Vp8DecodedFrame* d) { return (uint64_t)d->mb_cols * d->mb_rows; }

inline uint64_t align256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

// Device-side state of one call: its stream, device buffers (grown on demand, kept for the next
// call) and status word.  The reference's entry points are reentrant, so concurrent callers must be
// safe: a call leases one of up to kMaxCtx contexts (a pool guarded by a mutex; a caller waits only
// when every context is in use), so up to kMaxCtx threads decode at once, each on its own stream.
struct DevState {
	bool ready = false;
	hipStream_t stream = nullptr;
	uint8_t* in = nullptr;
	size_t in_cap = 0;
	uint8_t* out = nullptr;
	size_t out_cap = 0;
	uint8_t* desc = nullptr;
	size_t desc_cap = 0;
	uint8_t* gctx = nullptr;
	size_t gctx_cap = 0;
	uint8_t* mbox = nullptr;  // split-mode hand-off mailboxes + progress words (host APIs only)
	size_t mbox_cap = 0;
	uint8_t* snap = nullptr;  // mirror-split chain launches: per-frame context snapshots + flags
	size_t snap_cap = 0;
	uint8_t* sflags = nullptr;
	size_t sflags_cap = 0;
	uint32_t epoch = 0;  // launch counter for the snapshot flags
	uint32_t* status = nullptr;
	// (device batch API: the call returns before its kernel ends; the next lease of this context
	// orders its work on the context's buffers after that kernel)
	hipEvent_t done = nullptr;
	bool pending = false;
};
constexpr int kMaxCtx = 8;
struct DevPool {
	std::mutex mu;
	std::condition_variable cv;
	DevState ctx[kMaxCtx];
	bool busy[kMaxCtx] = {};
};
DevPool g_pool;
struct Lease {
	DevState* d;
	int i;
	Lease() {
		std::unique_lock<std::mutex> lk(g_pool.mu);
		for (;;) {
			for (i = 0; i < kMaxCtx && g_pool.busy[i]; i++) {
			}
			if (i < kMaxCtx) break;
			g_pool.cv.wait(lk);
		}
		g_pool.busy[i] = true;
		d = &g_pool.ctx[i];
	}
	~Lease() {
		std::lock_guard<std::mutex> lk(g_pool.mu);
		g_pool.busy[i] = false;
		g_pool.cv.notify_one();
	}
	Lease(const Lease&) = delete;
	Lease& operator=(const Lease&) = delete;
};

// The process-wide launch gate (vp8g_device.h, GateScope): each stream's last launch of the library
// and the last cross-workgroup launch, as events.
struct GateEntry {
	hipStream_t s;
	hipEvent_t ev;
	bool live;
};
struct Gate {
	std::recursive_mutex mu;  // (the pipeline's chunk scope encloses vp8g_m05_batch_device's own)
	std::vector<GateEntry> last;
	hipEvent_t xev = nullptr;
	hipStream_t xs = nullptr;
	bool xpending = false;
};
Gate g_gate;

// Device memory held by all contexts (the buffers below), so that concurrent large callers do not
// accumulate eight working sets: growing past half of the device's memory first releases the buffers
// of idle contexts.
std::atomic<size_t> g_held{0};


}  // namespace

vp8g::GateScope::GateScope(hipStream_t s) : s_(s) {
	g_gate.mu.lock();
	const hipError_t before = hipPeekAtLastError();
	if (g_gate.xpending) {
		const hipError_t q = hipEventQuery(g_gate.xev);
		if (q == hipSuccess) g_gate.xpending = false;
		else if (g_gate.xs != s) err_ = hipStreamWaitEvent(s, g_gate.xev, 0);
	}
	may_cross_ = !g_gate.xpending || g_gate.xs == s;
	for (GateEntry& x : g_gate.last) {
		if (!x.live || x.s == s) continue;
		if (hipEventQuery(x.ev) == hipSuccess) x.live = false;
		else may_cross_ = false;  // in flight (or unknown): no cross-workgroup launch beside it
	}
	// (hipErrorNotReady of the queries must not read as a launch failure later, so it is cleared.  HIP
	// keeps one last-error slot per thread: a caller's error pending before the gate stays pending
	// only when no query replaced it; after a query that returned hipErrorNotReady it is already gone,
	// and clearing the slot then loses nothing more)
	if (before == hipSuccess || hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
}

vp8g::GateScope::~GateScope() { g_gate.mu.unlock(); }

hipError_t vp8g::GateScope::done(bool crossed) {
	GateEntry* slot = nullptr;
	for (GateEntry& x : g_gate.last)
		if (x.s == s_ || (!slot && !x.live)) slot = &x;
	if (!slot) {
		GateEntry x{s_, nullptr, false};
		hipError_t e = hipEventCreateWithFlags(&x.ev, hipEventDisableTiming);
		if (e != hipSuccess) return e;
		g_gate.last.push_back(x);
		slot = &g_gate.last.back();
	}
	slot->s = s_;
	hipError_t e = hipEventRecord(slot->ev, s_);
	if (e != hipSuccess) return e;
	slot->live = true;
	if (crossed) {
		if (!g_gate.xev && (e = hipEventCreateWithFlags(&g_gate.xev, hipEventDisableTiming)) != hipSuccess) return e;
		if ((e = hipEventRecord(g_gate.xev, s_)) != hipSuccess) return e;
		g_gate.xs = s_;
		g_gate.xpending = true;
	}
	return hipSuccess;
}

namespace {

// Grow a buffer of context g.  The context's last asynchronous launch (device batch API) may still
// read its buffers: it completes before one is freed.  Past half of the device's memory held by all
// contexts, the idle contexts' buffers are released first.
hipError_t grow(DevState& g, uint8_t** p, size_t* cap, size_t need);
void release_buffers(DevState& g) {
	uint8_t** const bufs[] = {&g.in, &g.out, &g.desc, &g.gctx, &g.mbox, &g.snap, &g.sflags};
	size_t* const caps[] = {&g.in_cap, &g.out_cap, &g.desc_cap, &g.gctx_cap, &g.mbox_cap, &g.snap_cap, &g.sflags_cap};
	for (int i = 0; i < 7; i++) {
		if (*bufs[i]) (void)hipFree(*bufs[i]);
		*bufs[i] = nullptr;
		g_held.fetch_sub(*caps[i]);
		*caps[i] = 0;
	}
}
void trim_idle(const DevState* keep) {
	// The idle contexts are taken (marked busy) under the pool lock and released outside it: waiting
	// for their last asynchronous launch and hipFree (which synchronises the device) must not block
	// every other thread's lease for the length of a batch.
	bool took[kMaxCtx] = {};
	{
		std::lock_guard<std::mutex> lk(g_pool.mu);
		for (int i = 0; i < kMaxCtx; i++) {
			const DevState& o = g_pool.ctx[i];
			if (g_pool.busy[i] || &o == keep || !o.ready) continue;
			g_pool.busy[i] = took[i] = true;
		}
	}
	for (int i = 0; i < kMaxCtx; i++) {
		if (!took[i]) continue;
		DevState& o = g_pool.ctx[i];
		if (o.pending) {
			if (hipEventSynchronize(o.done) != hipSuccess) continue;
			o.pending = false;
		}
		release_buffers(o);
	}
	std::lock_guard<std::mutex> lk(g_pool.mu);
	for (int i = 0; i < kMaxCtx; i++)
		if (took[i]) g_pool.busy[i] = false;
	g_pool.cv.notify_all();
}
hipError_t grow(DevState& g, uint8_t** p, size_t* cap, size_t need) {
	if (need <= *cap) return hipSuccess;
	if (g.pending) {
		hipError_t e = hipEventSynchronize(g.done);
		if (e != hipSuccess) return e;
	}
	if (*p) (void)hipFree(*p);
	g_held.fetch_sub(*cap);
	*p = nullptr;
	*cap = 0;
	const size_t n = need + need / 4;
	size_t fr = 0, tot = 0;
	if (hipMemGetInfo(&fr, &tot) == hipSuccess && g_held.load() + n > tot / 2) trim_idle(&g);
	hipError_t e = hipMalloc((void**)p, n);
	if (e == hipSuccess) {
		*cap = n;
		g_held.fetch_add(n);
	}
	return e;
}

hipError_t dev_init(DevState& g) {
	if (g.ready) return hipSuccess;
	hipError_t e = hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking);
	if (e != hipSuccess) return e;
	e = hipMalloc((void**)&g.status, 256);
	if (e != hipSuccess) return e;
	g.ready = true;
	return hipSuccess;
}

// Sub-array layout of one batch inside the device input buffer.
struct InLayout {
	uint64_t y, u, v, y2, ym, uvm, seg, hasc, bm, src, total;
};
InLayout in_layout(uint64_t mbs, uint64_t src_bytes) {
	InLayout L;
	uint64_t o = 0;
	L.y = o, o = align256(o + mbs * 512);
	L.u = o, o = align256(o + mbs * 128);
	L.v = o, o = align256(o + mbs * 128);
	L.y2 = o, o = align256(o + mbs * 32);
	L.ym = o, o = align256(o + mbs);
	L.uvm = o, o = align256(o + mbs);
	L.seg = o, o = align256(o + mbs);
	L.hasc = o, o = align256(o + mbs);
	L.bm = o, o = align256(o + mbs * 16);
	L.src = o, o = align256(o + src_bytes);
	L.total = o;
	return L;
}

#define HIP_TRY(expr, where)          \
	do {                              \
		hipError_t e_ = (expr);       \
		if (e_ != hipSuccess) {       \
			set_err(where, e_);       \
			errno = EIO;              \
			return -1;                \
		}                             \
	} while (0)

// VP8G_SPLIT=<k>: workgroups per frame (1 = never split); unset: automatic for the host APIs.
uint32_t split_env() {
	const char* e = getenv("VP8G_SPLIT");
	return e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
}

// Launch over device-resident data with the buffers of the leased context g.  `may_split`: the
// call completes (stream synchronised) before its lease ends.  Launch modes whose workgroups wait on
// each other across CUs (split parts, the chain's mirror split) need every workgroup of the launch
// resident: they are chosen only when the launch gate (vp8g_device.h, GateScope) reports no other
// launch of the library in flight, and every later launch on another stream is ordered after them.
int run_locked(DevState& g_dev, const std::vector<Vp8gFrameDesc>& descs, const Vp8gBatchArrays& arr, uint8_t* d_out, hipStream_t s,
               uint32_t waves_hint, uint8_t* d_descs, bool may_split) {
	uint32_t max_cols = 0, max_rows = 0;
	for (const auto& d : descs) {
		if (d.mb_cols > max_cols) max_cols = d.mb_cols;
		if (d.mb_rows > max_rows) max_rows = d.mb_rows;
	}
	const uint32_t n = (uint32_t)descs.size();
	g_mode = 0u;  // (a call that fails before its launch reports no mode, not the previous call's)
	if (g_dev.pending) {  // the previous (asynchronous) launch on this context's buffers comes first
		HIP_TRY(hipStreamWaitEvent(s, g_dev.done, 0), "hipStreamWaitEvent");
	}
	if (!waves_hint) {
		const char* e = getenv("VP8G_WAVES");  // override of the default waves per workgroup
		if (e) waves_hint = (uint32_t)strtoul(e, nullptr, 10);
	}
	const uint32_t env = split_env();
	// Buffers for every mode this call could pick, before the gate (growing may wait for this context's
	// previous launch, or release idle contexts' buffers).  A call that the gate then keeps from the
	// cross-workgroup modes (another launch in flight) holds mailbox / snapshot memory it did not use
	// this time: the price of never allocating inside the gate, bounded by trim_idle.
	uint32_t nw = vp8g::pick_waves(waves_hint, max_rows, n);
	const bool try_split = (may_split || env > 1) && env != 1 && !waves_hint;
	const uint32_t nw_split = try_split && vp8g::pick_split(env, n, 8, max_rows) > 1 ? 8u : nw;
#ifdef VP8G_FORCE_GCTX  // diagnostic: per-column context in device memory for every frame
	const bool big = true;
#else
	const bool big = vp8g::lds_bytes((int)nw, max_cols, false) > (size_t)vp8g::kMaxLds;
#endif
	const bool big_split = vp8g::lds_bytes((int)nw_split, max_cols, false) > (size_t)vp8g::kMaxLds;
	uint8_t* gctx = nullptr;
	if (big) {
		const size_t need = descs.size() * (size_t)max_cols * vp8g::kCtxBytesPerCol;
		HIP_TRY(grow(g_dev, &g_dev.gctx, &g_dev.gctx_cap, need), "hipMalloc(ctx)");
		gctx = g_dev.gctx;
	}
	const uint32_t k_want = !big_split && try_split ? vp8g::pick_split(env, n, nw_split, max_rows) : 1u;
	if (k_want > 1) {
		const size_t mb = (size_t)n * k_want * max_cols * vp8g::kCtxBytesPerCol, pb = (size_t)n * k_want * sizeof(uint32_t);
		HIP_TRY(grow(g_dev, &g_dev.mbox, &g_dev.mbox_cap, mb + pb), "hipMalloc(mailbox)");
	}
	bool ordered = false;
	const bool quad = !big && !waves_hint && vp8g::pick_quad(descs.data(), n);  // (four MB rows per wave)
	const uint32_t wg = !big && !waves_hint ? vp8g::pick_chain(descs.data(), n, max_cols, &ordered, quad) : 0u;
	const bool split_want = wg && vp8g::pick_chain_split(n, max_cols, wg, ordered, quad);
	if (wg && (vp8g::kChainG || quad))  // (experiment builds: the chain's context in device memory, in the snapshot buffer)
		HIP_TRY(grow(g_dev, &g_dev.snap, &g_dev.snap_cap, (size_t)n * max_cols * vp8g::kCtxBytesPerCol), "hipMalloc(context)");
	if (split_want) {
		HIP_TRY(grow(g_dev, &g_dev.snap, &g_dev.snap_cap, (size_t)n * max_cols * vp8g::kCtxBytesPerCol), "hipMalloc(snapshots)");
		const size_t old_cap = g_dev.sflags_cap;
		HIP_TRY(grow(g_dev, &g_dev.sflags, &g_dev.sflags_cap, (size_t)n * sizeof(uint32_t)), "hipMalloc(flags)");
		if (g_dev.sflags_cap != old_cap) g_dev.epoch = 0;  // (fresh flags: zeroed below)
	}
	g_dev.pending = false;

	vp8g::GateScope gate(s);
	HIP_TRY(gate.status(), "hipStreamWaitEvent(gate)");
	const bool alone = gate.may_cross();
	// small batches on the host APIs: 8-wave parts, up to kMaxSplit per frame (measured on one 4K
	// frame: 8 waves x 8 parts 3.9 ms per call, 16 waves x 1..8 parts 8.1..4.7 ms)
	const uint32_t k = alone && k_want > 1 ? k_want : 1u;
	bool crossed = k > 1;
	g_mode = k > 1 ? VP8G_MODE_SPLIT_PARTS : 0u;
	if (k > 1) {
		const size_t mb = (size_t)n * k * max_cols * vp8g::kCtxBytesPerCol, pb = (size_t)n * k * sizeof(uint32_t);
		HIP_TRY(hipMemsetAsync(g_dev.mbox + mb, 0, pb, s), "memset(progress)");
		HIP_TRY(vp8g::launch_frames((const Vp8gFrameDesc*)d_descs, n, arr, d_out, max_cols, max_rows, nullptr, s, nw_split, k, g_dev.mbox,
		                            (uint32_t*)(g_dev.mbox + mb), 0),
		        "launch");
	} else if (wg) {  // more frames than CUs: one 16-wave chain of frames per CU
		// mirror split (vp8g_kernels.hip, kSegTop): snapshot flags of a fresh epoch
		const bool split = alone && split_want;
		if (split && (g_dev.epoch == 0 || ++g_dev.epoch == 0)) {  // (epoch 0 = the zeroed flags: never used)
			g_dev.epoch = 1;
			HIP_TRY(hipMemsetAsync(g_dev.sflags, 0, g_dev.sflags_cap, s), "memset(flags)");
		}
		crossed = split;
		const bool il = vp8g::pick_chain_interleave(descs.data(), n, max_cols, wg, split, quad);  // (1080p batches: two frames interleaved)
		g_mode = VP8G_MODE_CHAIN | (split ? VP8G_MODE_MIRROR_SPLIT : 0u) | (il ? VP8G_MODE_INTERLEAVE : 0u) | (quad ? VP8G_MODE_QUAD : 0u);
		HIP_TRY(vp8g::launch_chain((const Vp8gFrameDesc*)d_descs, n, arr, d_out, max_cols, s, wg, ordered, split, g_dev.snap,
		                           (uint32_t*)g_dev.sflags, g_dev.epoch, il, quad,
		                           quad && vp8g::whole_pieces(descs.data(), n) && ((uintptr_t)d_out & 15u) == 0),
		        "launch");
	} else {
		const uint32_t ord = vp8g::pick_order(descs.data(), n, 1);  // cost-balanced placement (vp8g_device.h)
		HIP_TRY(vp8g::launch_frames((const Vp8gFrameDesc*)d_descs, n, arr, d_out, max_cols, max_rows, gctx, s, nw, 1, nullptr, nullptr, ord),
		        "launch");
	}
	HIP_TRY(gate.done(crossed), "hipEventRecord(gate)");
	return 0;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Reference entry points
// ---------------------------------------------------------------------------------------------

VP8G_API int yuv420_alloc(Yuv420Image* img, uint32_t width, uint32_t height) {
	return vp8g::alloc_planes(img, width, height, true);
}

// Planes as yuv420_alloc lays them out; init = false leaves them uninitialised, for outputs the
// D2H overwrites completely (the fill would be a second full pass over fresh pages).
int vp8g::alloc_planes(Yuv420Image* img, uint32_t width, uint32_t height, bool init) {
	if (!img || width == 0 || height == 0) {
		errno = EINVAL;
		return -1;
	}
	memset(img, 0, sizeof(*img));
	img->width = width;
	img->height = height;
	img->stride_y = width;
	img->stride_uv = (width + 1) / 2;
	const size_t ysz = (size_t)width * height, uvsz = (size_t)img->stride_uv * ((height + 1) / 2);
	img->y = (uint8_t*)malloc(ysz);
	img->u = (uint8_t*)malloc(uvsz);
	img->v = (uint8_t*)malloc(uvsz);
	if (!img->y || !img->u || !img->v) {
		free(img->y);
		free(img->u);
		free(img->v);
		memset(img, 0, sizeof(*img));
		errno = ENOMEM;
		return -1;
	}
	if (init) {
		memset(img->y, 0, ysz);
		memset(img->u, 128, uvsz);
		memset(img->v, 128, uvsz);
	}
	return 0;
}

VP8G_API void yuv420_free(Yuv420Image* img) {
	if (!img) return;
	free(img->y);
	free(img->u);
	free(img->v);
	memset(img, 0, sizeof(*img));
}

VP8G_API uint64_t vp8g_i420_size(uint32_t w, uint32_t h) {
	return (uint64_t)w * h + 2 * (uint64_t)((w + 1) / 2) * ((h + 1) / 2);
}

VP8G_API int vp8g_make_frame_desc(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, int filtered, uint64_t mb_offset,
                                  uint64_t out_offset, Vp8gFrameDesc* out) {
	return vp8g::make_desc(kf, d, filtered, mb_offset, out_offset, out, true);
}

int vp8g::make_desc(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, int filtered, uint64_t mb_offset,
                    uint64_t out_offset, Vp8gFrameDesc* out, bool dense_coeffs) {
	if (!out || !d || !d->mb_cols || !d->mb_rows || d->mb_cols > 1024 || d->mb_rows > 1024 ||
	    (dense_coeffs && !frame_ok(d))) {
		errno = EINVAL;
		return -1;
	}
	memset(out, 0, sizeof(*out));
	out->mb_cols = d->mb_cols;
	out->mb_rows = d->mb_rows;
	out->width = kf ? kf->width : d->mb_cols * 16;
	out->height = kf ? kf->height : d->mb_rows * 16;
	if (out->width == 0 || out->height == 0 || out->width > d->mb_cols * 16 || out->height > d->mb_rows * 16) {
		errno = EINVAL;
		return -1;
	}
	out->stride_y = out->width;
	out->stride_uv = (out->width + 1) / 2;
	out->mb_offset = mb_offset;
	out->out_y = out_offset;
	out->out_u = out->out_y + (uint64_t)out->stride_y * out->height;
	out->out_v = out->out_u + (uint64_t)out->stride_uv * ((out->height + 1) / 2);
	fill_dequant(d, out);
	const int any_lf = fill_loopfilter(d, out);
	if (filtered && any_lf) out->flags |= VP8G_F_LOOPFILTER;
	if (d->lf_use_simple) out->flags |= VP8G_F_SIMPLE;
	return 0;
}

VP8G_API int vp8g_decode_batch_device(const Vp8gFrameDesc* h_descs, const Vp8gFrameDesc* d_descs, uint32_t n,
                                      const Vp8gBatchArrays* arrays, uint8_t* d_out, void* stream, uint32_t waves) {
	if (!h_descs || !d_descs || !arrays || !d_out || !arrays->status) {
		errno = EINVAL;
		return -1;
	}
	for (uint32_t i = 0; i < n; i++)  // (all-zero descriptors are allowed: empty slots, no work)
		if (h_descs[i].mb_cols > 1024 || h_descs[i].mb_rows > 1024 || (!h_descs[i].mb_cols != !h_descs[i].mb_rows)) {
			errno = EINVAL;
			return -1;
		}
	std::vector<Vp8gFrameDesc> v(h_descs, h_descs + n);
	Lease lease;
	DevState& g = *lease.d;
	if (!g.done) HIP_TRY(hipEventCreateWithFlags(&g.done, hipEventDisableTiming), "hipEventCreate");
	if (run_locked(g, v, *arrays, d_out, (hipStream_t)stream, waves, (uint8_t*)d_descs, false) != 0) return -1;
	HIP_TRY(hipEventRecord(g.done, (hipStream_t)stream), "hipEventRecord");
	g.pending = true;
	return 0;
}

VP8G_API int vp8g_reconstruct_batch(const Vp8KeyFrameHeader* const* kfs, const Vp8DecodedFrame* const* frames, uint32_t n,
                                    int filtered, Yuv420Image* outs) {
	if (!kfs || !frames || !outs || n == 0) {
		errno = EINVAL;
		return -1;
	}
	std::vector<Vp8gFrameDesc> descs(n);
	uint64_t mbs = 0, outb = 0;
	for (uint32_t i = 0; i < n; i++) {
		if (!kfs[i] || vp8g_make_frame_desc(kfs[i], frames[i], filtered, mbs, outb, &descs[i]) != 0) {
			errno = EINVAL;
			return -1;
		}
		mbs += mb_count(frames[i]);
		outb = align256(outb + vp8g_i420_size(kfs[i]->width, kfs[i]->height));
	}
	for (uint32_t i = 0; i < n; i++) {
		if (vp8g::alloc_planes(&outs[i], kfs[i]->width, kfs[i]->height, false) != 0) {
			for (uint32_t k = 0; k < i; k++) yuv420_free(&outs[k]);
			return -1;
		}
	}
	Lease lease;
	DevState& g_dev = *lease.d;
	auto fail = [&](void) {
		for (uint32_t k = 0; k < n; k++) yuv420_free(&outs[k]);
		errno = EIO;
		return -1;
	};
#define TRY(expr, where)              \
	do {                              \
		hipError_t e_ = (expr);       \
		if (e_ != hipSuccess) {       \
			set_err(where, e_);       \
			return fail();            \
		}                             \
	} while (0)
	TRY(dev_init(g_dev), "init");
	const InLayout L = in_layout(mbs, 0);
	TRY(grow(g_dev, &g_dev.in, &g_dev.in_cap, L.total), "hipMalloc(in)");
	TRY(grow(g_dev, &g_dev.out, &g_dev.out_cap, outb ? outb : 256), "hipMalloc(out)");
	TRY(grow(g_dev, &g_dev.desc, &g_dev.desc_cap, n * sizeof(Vp8gFrameDesc)), "hipMalloc(desc)");
	hipStream_t s = g_dev.stream;
	uint8_t* in = g_dev.in;
	for (uint32_t i = 0; i < n; i++) {
		const Vp8DecodedFrame* d = frames[i];
		const uint64_t o = descs[i].mb_offset, k = mb_count(d);
		TRY(hipMemcpyAsync(in + L.y + o * 512, d->coeff_y, k * 512, hipMemcpyHostToDevice, s), "H2D");
		TRY(hipMemcpyAsync(in + L.u + o * 128, d->coeff_u, k * 128, hipMemcpyHostToDevice, s), "H2D");
		TRY(hipMemcpyAsync(in + L.v + o * 128, d->coeff_v, k * 128, hipMemcpyHostToDevice, s), "H2D");
		TRY(hipMemcpyAsync(in + L.y2 + o * 32, d->coeff_y2, k * 32, hipMemcpyHostToDevice, s), "H2D");
		TRY(hipMemcpyAsync(in + L.ym + o, d->ymode, k, hipMemcpyHostToDevice, s), "H2D");
		TRY(hipMemcpyAsync(in + L.uvm + o, d->uv_mode, k, hipMemcpyHostToDevice, s), "H2D");
		if (d->segment_id) TRY(hipMemcpyAsync(in + L.seg + o, d->segment_id, k, hipMemcpyHostToDevice, s), "H2D");
		else TRY(hipMemsetAsync(in + L.seg + o, 0, k, s), "memset");
		if (d->has_coeff) TRY(hipMemcpyAsync(in + L.hasc + o, d->has_coeff, k, hipMemcpyHostToDevice, s), "H2D");
		else TRY(hipMemsetAsync(in + L.hasc + o, 0, k, s), "memset");
		TRY(hipMemcpyAsync(in + L.bm + o * 16, d->bmode, k * 16, hipMemcpyHostToDevice, s), "H2D");
	}
	TRY(hipMemcpyAsync(g_dev.desc, descs.data(), n * sizeof(Vp8gFrameDesc), hipMemcpyHostToDevice, s), "H2D");
	TRY(hipMemsetAsync(g_dev.status, 0, 4, s), "memset");
	Vp8gBatchArrays arr;
	arr.coeff_y = (const int16_t*)(in + L.y);
	arr.coeff_u = (const int16_t*)(in + L.u);
	arr.coeff_v = (const int16_t*)(in + L.v);
	arr.coeff_y2 = (const int16_t*)(in + L.y2);
	arr.ymode = in + L.ym;
	arr.uv_mode = in + L.uvm;
	arr.segment_id = in + L.seg;
	arr.has_coeff = in + L.hasc;
	arr.bmode = in + L.bm;
	arr.src = nullptr;
	arr.status = g_dev.status;
	if (run_locked(g_dev, descs, arr, g_dev.out, s, 0, g_dev.desc, true) != 0) return fail();
	for (uint32_t i = 0; i < n; i++) {
		const Vp8gFrameDesc& d = descs[i];
		const size_t ysz = (size_t)d.stride_y * d.height, uvsz = (size_t)d.stride_uv * ((d.height + 1) / 2);
		TRY(hipMemcpyAsync(outs[i].y, g_dev.out + d.out_y, ysz, hipMemcpyDeviceToHost, s), "D2H");
		TRY(hipMemcpyAsync(outs[i].u, g_dev.out + d.out_u, uvsz, hipMemcpyDeviceToHost, s), "D2H");
		TRY(hipMemcpyAsync(outs[i].v, g_dev.out + d.out_v, uvsz, hipMemcpyDeviceToHost, s), "D2H");
	}
	uint32_t status = 0;
	TRY(hipMemcpyAsync(&status, g_dev.status, 4, hipMemcpyDeviceToHost, s), "D2H");
	TRY(hipStreamSynchronize(s), "sync");
	if (status != 0) {
		snprintf(g_err, sizeof(g_err), "kernel status 0x%x (dependency wait timed out)", status);
		return fail();
	}
#undef TRY
	return 0;
}

VP8G_API int vp8_reconstruct_keyframe_yuv(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* decoded, Yuv420Image* out) {
	if (!kf || !decoded || !out) {
		errno = EINVAL;
		return -1;
	}
	return vp8g_reconstruct_batch(&kf, &decoded, 1, 0, out);
}

VP8G_API int vp8_reconstruct_keyframe_yuv_filtered(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* decoded,
                                                   Yuv420Image* out) {
	if (!kf || !decoded || !out) {
		errno = EINVAL;
		return -1;
	}
	return vp8g_reconstruct_batch(&kf, &decoded, 1, 1, out);
}

VP8G_API int vp8_loopfilter_apply_keyframe(Yuv420Image* img, const Vp8DecodedFrame* d) {
	if (!img || !d) {
		errno = EINVAL;
		return -1;
	}
	if (img->width != d->mb_cols * 16u || img->height != d->mb_rows * 16u || !img->y || !img->u || !img->v ||
	    !d->ymode || (!d->segment_id && d->segmentation_enabled) || d->mb_cols > 1024 || d->mb_rows > 1024) {
		errno = EINVAL;
		return -1;
	}
	Vp8gFrameDesc desc;
	memset(&desc, 0, sizeof(desc));
	desc.mb_cols = d->mb_cols;
	desc.mb_rows = d->mb_rows;
	desc.width = img->width;
	desc.height = img->height;
	desc.stride_y = img->width;
	desc.stride_uv = img->width / 2;
	desc.out_y = 0;
	desc.out_u = (uint64_t)img->width * img->height;
	desc.out_v = desc.out_u + (uint64_t)desc.stride_uv * (img->height / 2);
	if (!fill_loopfilter(d, &desc)) return 0; /* every MB level is 0: nothing to filter */
	desc.flags = VP8G_F_LOOPFILTER | VP8G_F_LF_ONLY | (d->lf_use_simple ? VP8G_F_SIMPLE : 0);
	const uint64_t frame_bytes = desc.out_v + (uint64_t)desc.stride_uv * (img->height / 2);
	desc.src_y = 0;
	desc.src_u = desc.out_u;
	desc.src_v = desc.out_v;
	desc.src_stride_y = desc.stride_y;
	desc.src_stride_uv = desc.stride_uv;
	std::vector<Vp8gFrameDesc> descs(1, desc);
	const uint64_t k = mb_count(d);
	Lease lease;
	DevState& g_dev = *lease.d;
	HIP_TRY(dev_init(g_dev), "init");
	const InLayout L = in_layout(k, frame_bytes);
	HIP_TRY(grow(g_dev, &g_dev.in, &g_dev.in_cap, L.total), "hipMalloc(in)");
	HIP_TRY(grow(g_dev, &g_dev.out, &g_dev.out_cap, frame_bytes), "hipMalloc(out)");
	HIP_TRY(grow(g_dev, &g_dev.desc, &g_dev.desc_cap, sizeof(Vp8gFrameDesc)), "hipMalloc(desc)");
	hipStream_t s = g_dev.stream;
	uint8_t* in = g_dev.in;
	const uint32_t cw = img->width / 2, ch = img->height / 2;
	HIP_TRY(hipMemcpyAsync(in + L.ym, d->ymode, k, hipMemcpyHostToDevice, s), "H2D");
	if (d->segment_id) HIP_TRY(hipMemcpyAsync(in + L.seg, d->segment_id, k, hipMemcpyHostToDevice, s), "H2D");
	else HIP_TRY(hipMemsetAsync(in + L.seg, 0, k, s), "memset");
	if (d->has_coeff) HIP_TRY(hipMemcpyAsync(in + L.hasc, d->has_coeff, k, hipMemcpyHostToDevice, s), "H2D");
	else HIP_TRY(hipMemsetAsync(in + L.hasc, 0, k, s), "memset");
	uint8_t* src = in + L.src;
	HIP_TRY(hipMemcpy2DAsync(src, img->width, img->y, img->stride_y, img->width, img->height, hipMemcpyHostToDevice, s), "H2D");
	HIP_TRY(hipMemcpy2DAsync(src + desc.src_u, cw, img->u, img->stride_uv, cw, ch, hipMemcpyHostToDevice, s), "H2D");
	HIP_TRY(hipMemcpy2DAsync(src + desc.src_v, cw, img->v, img->stride_uv, cw, ch, hipMemcpyHostToDevice, s), "H2D");
	HIP_TRY(hipMemcpyAsync(g_dev.desc, &desc, sizeof(desc), hipMemcpyHostToDevice, s), "H2D");
	HIP_TRY(hipMemsetAsync(g_dev.status, 0, 4, s), "memset");
	Vp8gBatchArrays arr;
	memset(&arr, 0, sizeof(arr));
	arr.ymode = in + L.ym;
	arr.uv_mode = in + L.ym;
	arr.segment_id = in + L.seg;
	arr.has_coeff = in + L.hasc;
	arr.bmode = nullptr;
	arr.src = src;
	arr.status = g_dev.status;
	if (run_locked(g_dev, descs, arr, g_dev.out, s, 0, g_dev.desc, true) != 0) return -1;
	HIP_TRY(hipMemcpy2DAsync(img->y, img->stride_y, g_dev.out, img->width, img->width, img->height, hipMemcpyDeviceToHost, s),
	        "D2H");
	HIP_TRY(hipMemcpy2DAsync(img->u, img->stride_uv, g_dev.out + desc.out_u, cw, cw, ch, hipMemcpyDeviceToHost, s), "D2H");
	HIP_TRY(hipMemcpy2DAsync(img->v, img->stride_uv, g_dev.out + desc.out_v, cw, cw, ch, hipMemcpyDeviceToHost, s), "D2H");
	uint32_t status = 0;
	HIP_TRY(hipMemcpyAsync(&status, g_dev.status, 4, hipMemcpyDeviceToHost, s), "D2H");
	HIP_TRY(hipStreamSynchronize(s), "sync");
	if (status != 0) {
		snprintf(g_err, sizeof(g_err), "kernel status 0x%x", status);
		errno = EIO;
		return -1;
	}
	return 0;
}

VP8G_API const char* vp8g_last_error(void) { return g_err; }

VP8G_API uint32_t vp8g_last_launch_mode(void) { return g_mode; }

void vp8g::set_error_text(const char* where, hipError_t e) { set_err(where, e); }

VP8G_API uint32_t vp8g_abi_version(void) { return VP8G_ABI_VERSION; }
