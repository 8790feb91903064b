// vp8g_pipeline.hip -- end-to-end batch decode, .webp bytes -> I420 in host memory
// (vp8g_decode_webp_batch, include/vp8g.h).
//
//   worker threads   container + key-frame header + m05 (host/vp8_parse.c, reentrant) into the
//                    packed wire format, frames handed out in order from an atomic counter and
//                    kept at most a window ahead of the device
//   this thread      groups finished frames into chunks; per chunk: H2D of the side arrays, the
//                    block masks and the non-zero values (~5x less than dense int16), expansion
//                    to the dense SoA the recon kernel reads, the fused recon(+LF) kernel, D2H
//                    into the callers' images.  Chunk slots alternate (two per chunk kind), so the device work and
//                    the copies of one chunk overlap the entropy decoding of the next ones.
//
// With VP8G_BATCH_DEVICE_M05 the workers only parse the container, the
// frame header and the first partition's frame-level fields (vp8f_token_header_memory); the
// chunk uploads the compressed VP8 payloads themselves (the smallest possible wire format), and
// m05 runs on the device (vp8g_m05.hip, one wavefront per frame) straight into the dense SoA.
//
// The reference decodes one file per process (src/main.c:591-705: m01..m05 then m06/m07); its
// m05 keeps global state (vp8_tokens.c:382, :625), which is why it cannot be threaded as is.
#include <errno.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../host/vp8_front.h"
#include "vp8g_device.h"

#define VP8G_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr uint32_t kChunkFrames = 32;          // frames per host-m05 chunk (at most; tools/chunk_sweep.py: 32 shortens the tail)
constexpr uint64_t kChunkMbs = 2u << 20;       // macroblocks per chunk (at most, unless one frame is bigger)
// device m05: one workgroup per frame and a chunk's m05 time is its slowest frame's, so a chunk
// wants as many frames as the chip runs at once (~1500 at full scalar-unit load): 1024 4K frames,
// ~1.2 KB of device buffers per MB (coefficients, side arrays, I420 out) = ~41 GB per slot
constexpr uint32_t kTokChunkFrames = 1024;
constexpr uint64_t kTokChunkMbs = 34u << 20;
constexpr uint32_t kNb = VP8G_PK_BLOCKS;

// Packed -> dense coefficients.  32 lanes per MB; lane b < 25 owns block b (Y 0..15, U 0..3,
// V 0..3, Y2).  Its values start at the MB's offset plus the popcounts of the blocks before it
// (a 32-lane inclusive scan); position i takes value rank popcount(mask & ((1 << i) - 1)).
__global__ __launch_bounds__(256) void expand_kernel(const uint16_t* __restrict__ masks, const uint32_t* __restrict__ mb_off,
                                                     const int16_t* __restrict__ vals, uint32_t n_mb, int16_t* __restrict__ cy,
                                                     int16_t* __restrict__ cu, int16_t* __restrict__ cv,
                                                     int16_t* __restrict__ cy2) {
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	const uint32_t mb = t >> 5, b = t & 31u;
	if (mb >= n_mb) return;  // whole 32-lane groups leave together
	const uint32_t m = b < kNb ? masks[(size_t)mb * kNb + b] : 0u;
	const uint32_t cnt = __popc(m);
	uint32_t incl = cnt;
#pragma unroll
	for (int d = 1; d < 32; d <<= 1) {
		const uint32_t v = __shfl_up(incl, (unsigned)d, 32);
		if (b >= (uint32_t)d) incl += v;
	}
	if (b >= kNb) return;
	const int16_t* src = vals + mb_off[mb] + (incl - cnt);
	uint32_t w[8];
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const uint32_t k0 = 2 * i, k1 = 2 * i + 1;
		uint32_t lo = 0, hi = 0;
		if ((m >> k0) & 1u) lo = (uint16_t)src[__popc(m & ((1u << k0) - 1u))];
		if ((m >> k1) & 1u) hi = (uint16_t)src[__popc(m & ((1u << k1) - 1u))];
		w[i] = lo | (hi << 16);
	}
	int16_t* dst = b < 16u   ? cy + ((size_t)mb * 16u + b) * 16u
	               : b < 20u ? cu + ((size_t)mb * 4u + (b - 16u)) * 16u
	               : b < 24u ? cv + ((size_t)mb * 4u + (b - 20u)) * 16u
	                         : cy2 + (size_t)mb * 16u;
	uint4* d4 = (uint4*)dst;
	d4[0] = make_uint4(w[0], w[1], w[2], w[3]);
	d4[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

inline uint64_t al256(uint64_t x) { return (x + 255u) & ~(uint64_t)255u; }
// bitstream slot of a payload: 16-B aligned start, >= 512 bytes of slack (the device bool
// decoder loads its 256-byte windows one ahead, up to 512 bytes past a partition's end)
inline uint64_t bits_slot(uint32_t psize) { return ((uint64_t)psize + 512u + 15u) & ~(uint64_t)15u; }

// Host half of a device-m05 frame.
struct TokJob {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame hdr;  // header fields only (no arrays)
	Vp8gTokFrame tf;
	uint64_t poff;  // VP8 payload in the file
	uint32_t psize;
};

// The library's one background releaser of host frames (the last chunks' packed frames, freed
// after a call returns: see defer_release).  Owned, and joined when the library is unloaded or
// the process exits, so no thread runs library code after that.
struct Freer {
	std::mutex mu;
	std::condition_variable cv;
	std::vector<std::vector<Vp8gPackedFrame>> q;
	bool stop = false;
	std::thread th;
	void post(std::vector<Vp8gPackedFrame>&& v) {
		std::lock_guard<std::mutex> lk(mu);
		if (!th.joinable()) th = std::thread([this] { run(); });
		q.push_back(std::move(v));
		cv.notify_one();
	}
	void run() {
		std::unique_lock<std::mutex> lk(mu);
		for (;;) {
			cv.wait(lk, [this] { return stop || !q.empty(); });
			if (q.empty()) return;  // (stop with nothing queued)
			std::vector<Vp8gPackedFrame> v = std::move(q.back());
			q.pop_back();
			lk.unlock();
			for (Vp8gPackedFrame& p : v) vp8f_packed_free(&p);
			lk.lock();
		}
	}
	~Freer() {
		{
			std::lock_guard<std::mutex> lk(mu);
			stop = true;
		}
		cv.notify_one();
		if (th.joinable()) th.join();
	}
};
Freer g_freer;

uint32_t default_threads() {
	cpu_set_t set;
	if (sched_getaffinity(0, sizeof(set), &set) == 0) {
		const int n = CPU_COUNT(&set);
		if (n > 0) return (uint32_t)n;
	}
	const unsigned h = std::thread::hardware_concurrency();
	return h ? h : 1u;
}

// Frames handed from the workers to the device thread, in the order `order` (positions), each
// either decoded on the host into the packed format or only header-parsed for device m05 (dev[i]).
struct Feed {
	const ByteSpan* files = nullptr;
	uint32_t n = 0;
	std::vector<uint8_t> dev;       // frame i: m05 on the device (workers fill tj[i], else pk[i])
	std::vector<uint32_t> order;    // position -> frame index
	unsigned fflags = 0;  // front-end flags (VP8F_MULTI_PARTITION)
	std::vector<Vp8gPackedFrame> pk;
	std::vector<TokJob> tj;
	std::vector<int> err;
	std::unique_ptr<uint8_t[]> ready;
	std::atomic<uint32_t> next{0};
	uint32_t limit = 0;  // workers may start positions < limit (guarded by mu)
	bool abort = false;
	std::mutex mu;
	std::condition_variable cv_ready, cv_limit;

	void work() {
		for (;;) {
			const uint32_t pos = next.fetch_add(1);
			if (pos >= n) return;
			{
				std::unique_lock<std::mutex> lk(mu);
				cv_limit.wait(lk, [&] { return pos < limit || abort; });
				if (abort) return;
			}
			const uint32_t i = order[pos];
			int stage = 0, e = 0;
			if (!files[i].data) e = EINVAL;
			else if (dev[i]) {
				TokJob& j = tj[i];
				if (vp8f_token_header_memory(files[i].data, files[i].size, &j.kf, &j.hdr, &j.tf, &j.poff, &j.psize, &stage,
				                             fflags) != 0)
					e = errno ? errno : EINVAL;
			} else if (vp8f_decode_packed_memory(files[i].data, files[i].size, &pk[i], &stage, fflags) != 0)
				e = errno ? errno : EINVAL;
			{
				std::lock_guard<std::mutex> lk(mu);
				err[i] = e;
				ready[i] = 1;
			}
			cv_ready.notify_all();
		}
	}
	void wait_ready(uint32_t i) {
		std::unique_lock<std::mutex> lk(mu);
		cv_ready.wait(lk, [&] { return ready[i] != 0; });
	}
	void set_limit(uint32_t l) {
		{
			std::lock_guard<std::mutex> lk(mu);
			if (l > limit) limit = l;
		}
		cv_limit.notify_all();
	}
	void stop() {
		{
			std::lock_guard<std::mutex> lk(mu);
			abort = true;
		}
		cv_limit.notify_all();
	}
};

// One chunk's device buffer and the host state that must live until its copies are done.
struct D2H {
	void* dst;
	const void* src;
	size_t bytes;
};
struct Slot {
	uint8_t* buf = nullptr;
	size_t cap = 0;
	hipEvent_t done = nullptr;     // the chunk's D2H finished (copy stream)
	hipEvent_t kdone = nullptr;    // the chunk's kernels finished (compute stream)
	bool busy = false;
	std::vector<uint32_t> frames;  // frame indices of the chunk (packed data freed when the slot is reused)
	std::vector<Vp8gFrameDesc> descs;
	std::vector<Vp8gTokFrame> jobs;  // device m05
	uint32_t status = 0;
	std::vector<D2H> d2h;          // the chunk's downloads (issued by a Copier)
	bool issued = false;           // the Copier has issued them and recorded `done` (guarded by its mutex)
	hipError_t copy_err = hipSuccess;
};

// Downloads into the callers' images are pageable-memory copies, which HIP completes
// synchronously in the calling thread -- after waiting for the chunk's kernels.  Issued from
// the thread that launches chunks, one long device-m05 chunk's download would hold up every
// later launch (host-m05 chunks that are ready, the next device chunk).  Each Copier owns a
// thread and a stream and issues the downloads of the chunks queued to it, in order.
struct Copier {
	std::thread th;
	std::mutex mu;
	std::condition_variable cv;
	std::vector<Slot*> q;
	size_t head = 0;
	bool quit = false;
	hipStream_t stream = nullptr;

	void run() {
		for (;;) {
			Slot* s;
			{
				std::unique_lock<std::mutex> lk(mu);
				cv.wait(lk, [&] { return head < q.size() || quit; });
				if (quit) return;
				s = q[head++];
			}
			// fresh output images fault their pages in during the copy, one 4-KB page at a time in
			// this thread; populate them first, while the chunk's kernels still run
			for (const D2H& c : s->d2h) prefault(c.dst, c.bytes);
			hipError_t e = hipStreamWaitEvent(stream, s->kdone, 0);
			for (const D2H& c : s->d2h)
				if (e == hipSuccess) e = hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToHost, stream);
			if (e == hipSuccess) e = hipEventRecord(s->done, stream);
			{
				std::lock_guard<std::mutex> lk(mu);
				s->issued = true;
				s->copy_err = e;
			}
			cv.notify_all();
		}
	}
	static void prefault(void* p, size_t bytes) {
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
		static const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
		const uintptr_t a = ((uintptr_t)p + pg - 1) & ~(pg - 1), e = ((uintptr_t)p + bytes) & ~(pg - 1);
		if (e > a) (void)madvise((void*)a, e - a, MADV_POPULATE_WRITE);  // (best effort: older kernels say EINVAL)
	}
	void push(Slot* s) {
		{
			std::lock_guard<std::mutex> lk(mu);
			s->issued = false;
			q.push_back(s);
		}
		cv.notify_all();
	}
	hipError_t wait_issued(Slot* s) {
		std::unique_lock<std::mutex> lk(mu);
		cv.wait(lk, [&] { return s->issued; });
		return s->copy_err;
	}
	void stop() {
		{
			std::lock_guard<std::mutex> lk(mu);
			quit = true;
		}
		cv.notify_all();
		if (th.joinable()) th.join();
	}
};

struct ChunkLayout {
	uint64_t ym, uvm, seg, hasc, bm, masks, mboff, vals, cy, cu, cv, cy2, bits, jobs, desc, status, gctx, mbox, gprog, out,
	    total;
};

hipError_t grow(Slot& s, size_t need) {
	if (need <= s.cap) return hipSuccess;
	if (s.buf) (void)hipFree(s.buf);
	s.buf = nullptr;
	s.cap = 0;
	const size_t n = need + need / 4;
	hipError_t e = hipMalloc((void**)&s.buf, n);
	if (e == hipSuccess) s.cap = n;
	return e;
}

// Which frames run m05 on the device and in which order the workers take them.  Without
// VP8G_BATCH_DEVICE_M05 every frame is decoded on the host, in index order.  With it the device
// runs m05 as one workgroup per frame, so the device part lasts as long as its heaviest frame
// (latency ~ kDevNsPerByte x payload bytes) plus the download of all its images, while the host
// threads would otherwise only parse headers.  So the heaviest frames go to the host threads
// (~ kHostNsPerByte x bytes each, `threads` at a time): the k heaviest, for the k that minimises
// max(host time, device time) (VP8G_HYBRID=0 turns this off).  Device frames come
// first, so their chunk launches while the host threads decode the heavy ones.
constexpr double kDevNsPerByte = 850.0;    // device m05 latency per payload byte, 4K fixtures
constexpr double kHostNsPerByte = 50.0;    // host m05 into the packed format, per payload byte and thread
constexpr double kD2HNsPerByte = 0.085;    // download into fresh pageable images (~12 GB/s)
// (rates measured on the box: tools/e2e_probe.py chunk traces, tools/hybrid_sweep.py; profiles/r02_hybrid.json)
void plan_frames(const ByteSpan* files, uint32_t n, bool tok, uint32_t threads, std::vector<uint8_t>& dev,
                 std::vector<uint32_t>& order) {
	dev.assign(n, tok ? 1 : 0);
	order.resize(n);
	for (uint32_t i = 0; i < n; i++) order[i] = i;
	const char* hv = getenv("VP8G_HYBRID");
	if (!tok || (hv && atoi(hv) == 0)) return;
	double dev_per_b = kDevNsPerByte, host_per_b = kHostNsPerByte, d2h_per_b = kD2HNsPerByte;
	if (const char* e = getenv("VP8G_DEV_NS_PER_BYTE")) dev_per_b = atof(e);  // calibration knobs
	if (const char* e = getenv("VP8G_HOST_NS_PER_BYTE")) host_per_b = atof(e);
	if (const char* e = getenv("VP8G_D2H_NS_PER_BYTE")) d2h_per_b = atof(e);
	std::vector<double> outb(n, 0.0);  // I420 bytes (0 for a file whose header does not parse: it fails anyway)
	for (uint32_t i = 0; i < n; i++) {
		WebPContainer c;
		Vp8KeyFrameHeader kf;
		if (files[i].data && webp_parse_simple_lossy(files[i], &c) == 0 &&
		    vp8_parse_keyframe_header(ByteSpan{files[i].data + c.vp8_chunk_offset, c.vp8_chunk_size}, &kf) == 0)
			outb[i] = (double)vp8g_i420_size(kf.width, kf.height);
	}
	std::vector<uint32_t> by_size(order);
	std::stable_sort(by_size.begin(), by_size.end(), [&](uint32_t x, uint32_t y) { return files[x].size > files[y].size; });
	double dev_out = 0;
	for (uint32_t i = 0; i < n; i++) dev_out += outb[i];
	const double thr = threads ? (double)threads : 1.0;
	double host_ns = 0, best = dev_per_b * (double)files[by_size[0]].size + d2h_per_b * dev_out;
	uint32_t best_k = 0;
	for (uint32_t k = 1; k <= n; k++) {  // the k heaviest on the host
		const uint32_t f = by_size[k - 1];
		host_ns += host_per_b * (double)files[f].size / thr;
		dev_out -= outb[f];
		const double dev_ns = (k < n ? dev_per_b * (double)files[by_size[k]].size : 0.0) + d2h_per_b * dev_out;
		const double t = host_ns > dev_ns ? host_ns : dev_ns;
		if (t < best) best = t, best_k = k;
	}
	for (uint32_t k = 0; k < best_k; k++) dev[by_size[k]] = 0;
	uint32_t p = 0;
	for (uint32_t i = 0; i < n; i++)
		if (dev[i]) order[p++] = i;
	for (uint32_t k = 0; k < n; k++)
		if (!dev[by_size[k]]) order[p++] = by_size[k];
}

}  // namespace

VP8G_API int vp8g_plan_batch(const ByteSpan* files, uint32_t n, uint32_t threads, uint32_t flags, uint8_t* dev,
                             uint32_t* order) {
	if (!files || !dev || !order || n == 0 || (flags & ~(VP8G_BATCH_DEVICE_M05 | VP8G_BATCH_MULTI_PARTITION))) {
		errno = EINVAL;
		return -1;
	}
	std::vector<uint8_t> d;
	std::vector<uint32_t> o;
	uint32_t thr = threads ? threads : default_threads();
	if (thr > n) thr = n;  // (as vp8g_decode_webp_batch_ex)
	plan_frames(files, n, (flags & VP8G_BATCH_DEVICE_M05) != 0, thr, d, o);
	memcpy(dev, d.data(), n);
	memcpy(order, o.data(), n * sizeof(uint32_t));
	return 0;
}

VP8G_API int vp8g_decode_webp_batch_ex(const ByteSpan* files, uint32_t n, int filtered, uint32_t threads, uint32_t flags,
                                       Yuv420Image* outs, int* status) {
	if (!files || !outs || n == 0 || (flags & ~(VP8G_BATCH_DEVICE_M05 | VP8G_BATCH_MULTI_PARTITION))) {
		errno = EINVAL;
		return -1;
	}
	const bool tok = (flags & VP8G_BATCH_DEVICE_M05) != 0;
	uint32_t chunk_frames_pk = kChunkFrames, chunk_frames_tok = kTokChunkFrames;
	if (const char* e = getenv("VP8G_CHUNK_FRAMES")) {  // test knob: smaller chunks
		const long v = atol(e);
		if (v > 0 && (uint64_t)v < chunk_frames_pk) chunk_frames_pk = (uint32_t)v;
		if (v > 0 && (uint64_t)v < chunk_frames_tok) chunk_frames_tok = (uint32_t)v;
	}
	uint64_t chunk_mbs_tok = kTokChunkMbs, chunk_mbs_pk = kChunkMbs;
	{
		// four chunk slots (two per chunk kind): host-m05 chunks ~1.5 KB per MB, device-m05 chunks
		// ~1.3 KB per MB (+ payloads).  All four stay within ~3/8 of the free device memory, so a
		// device shared with other work gets smaller chunks instead of a failed allocation (EIO for
		// every frame); the device-m05 slots get what the (small) host-m05 slots leave.  (Round 5:
		// the old cap, free / 16384 MBs for every slot, cut 768 device frames into two m05 launches
		// on a 288-GB card; the second one then waited behind the first whenever their streams
		// shared a hardware queue -- DESIGN.md §12.)
		size_t fr = 0, tot = 0;
		if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr) {
			const uint64_t budget = (uint64_t)fr / 8u * 3u;
			const uint64_t floor_mbs = 1u << 15;  // one 4K frame and change
			const uint64_t cap_pk = budget / (4u * 1536u);
			if (cap_pk < chunk_mbs_pk) chunk_mbs_pk = cap_pk > floor_mbs ? cap_pk : floor_mbs;
			const uint64_t pk_bytes = 2u * chunk_mbs_pk * 1536u;
			const uint64_t cap_tok = budget > pk_bytes ? (budget - pk_bytes) / (2u * 1331u) : 0u;
			if (cap_tok < chunk_mbs_tok) chunk_mbs_tok = cap_tok > floor_mbs ? cap_tok : floor_mbs;
		}
	}
	for (uint32_t i = 0; i < n; i++) memset(&outs[i], 0, sizeof(outs[i]));
	if (!threads) threads = default_threads();
	if (threads > n) threads = n;

	Feed feed;
	feed.files = files;
	feed.n = n;
	feed.fflags = (flags & VP8G_BATCH_MULTI_PARTITION) ? VP8F_MULTI_PARTITION : 0u;
	feed.pk.assign(n, Vp8gPackedFrame{});
	if (tok) feed.tj.assign(n, TokJob{});
	feed.err.assign(n, 0);
	feed.ready.reset(new uint8_t[n]());
	plan_frames(files, n, tok, threads, feed.dev, feed.order);
	// VP8G_PIPE_TRACE=1: one stderr line per chunk (kind, frames, MBs, launch / retire times; diagnostics)
	const bool trace = getenv("VP8G_PIPE_TRACE") && atoi(getenv("VP8G_PIPE_TRACE")) != 0;
	const auto t_start = std::chrono::steady_clock::now();
	auto ms_now = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count(); };
	if (trace) {
		uint32_t nd = 0;
		for (uint32_t i = 0; i < n; i++) nd += feed.dev[i];
		fprintf(stderr, "[pipe] n=%u threads=%u device_frames=%u host_frames=%u chunk_mbs_tok=%llu chunk_mbs_pk=%llu\n", n,
		        threads, nd, n - nd, (unsigned long long)chunk_mbs_tok, (unsigned long long)chunk_mbs_pk);
	}
	const uint32_t chunk_frames = tok ? chunk_frames_tok : chunk_frames_pk;
	const uint32_t window = 2 * chunk_frames > 4 * threads ? 2 * chunk_frames : 4 * threads;
	feed.limit = window;
	std::vector<std::thread> pool;
	pool.reserve(threads);
	for (uint32_t t = 0; t < threads; t++) pool.emplace_back([&feed] { feed.work(); });

	// uploads and kernels on one stream per chunk slot (a long device-m05 chunk and the next
	// chunk's kernels overlap); downloads by the Copiers: chunk k's D2H overlaps chunk k+1's kernels
	// slots 0/1 alternate between device-m05 chunks, 2/3 between host-m05 chunks, so a hybrid batch's
	// host chunks never wait for the (long) device-m05 chunk's slot
	hipStream_t streams[4] = {nullptr, nullptr, nullptr, nullptr};
	Copier copiers[2];  // downloads of host-m05 chunks / device-m05 chunks
	Slot slots[4];
	uint32_t nchunk[2] = {0, 0};  // chunks so far per kind (host, device)
	uint32_t released = 0;  // positions whose frames' host data is freed (all below this one)
	const char* where = nullptr;
	hipError_t he = hipSuccess;
	// The host frames of the last chunks are released by the background freer (g_freer) once the
	// call has its results: freeing them is when glibc trims the heap those frames grew (GBs of packed data,
	// ~0.3 s at 1024 4K frames), work the caller need not wait for.
	bool defer_release = false;
	std::vector<Vp8gPackedFrame> late;
	auto release = [&](Slot& s) {
		for (uint32_t i : s.frames)
			if (!feed.dev[i]) {
				if (defer_release) {
					late.push_back(feed.pk[i]);
					memset(&feed.pk[i], 0, sizeof(feed.pk[i]));
				} else {
					vp8f_packed_free(&feed.pk[i]);
				}
			}
		s.frames.clear();
	};
	auto kf_of = [&](uint32_t i) -> const Vp8KeyFrameHeader& { return feed.dev[i] ? feed.tj[i].kf : feed.pk[i].kf; };
	auto f_of = [&](uint32_t i) -> const Vp8DecodedFrame& { return feed.dev[i] ? feed.tj[i].hdr : feed.pk[i].f; };
	auto finish_slot = [&](Slot& s) -> bool {  // wait for a slot's chunk; false on a device failure
		if (!s.busy) return true;
		s.busy = false;
		const double tw = trace ? ms_now() : 0.0;
		if ((he = copiers[&s - slots < 2 ? 1 : 0].wait_issued(&s)) != hipSuccess) {
			where = "D2H";
			return false;
		}
		if ((he = hipEventSynchronize(s.done)) != hipSuccess) {
			where = "sync";
			return false;
		}
		if (trace) fprintf(stderr, "[pipe] slot %d retired at %.1f ms (waited %.1f ms)\n", (int)(&s - slots), ms_now(), ms_now() - tw);
		const double tr = trace ? ms_now() : 0.0;
		release(s);
		if (trace) fprintf(stderr, "[pipe] slot %d host data freed in %.1f ms\n", (int)(&s - slots), ms_now() - tr);
		if (s.status != 0) {
			where = "kernel status";
			he = hipErrorLaunchFailure;
			return false;
		}
		return true;
	};

#define PTRY(expr, w)                \
	do {                             \
		if ((he = (expr)) != hipSuccess) { \
			where = w;               \
			goto fail;               \
		}                            \
	} while (0)

	// The device-m05 slots' streams (0, 1) at the lowest stream priority, the others at the default:
	// HIP keeps a pool of hardware queues per priority, so a host-m05 chunk never sits in one hardware
	// queue behind a device-m05 kernel (~0.5-1.5 s, one frame's serial bool decoding) -- streams
	// beyond GPU_MAX_HW_QUEUES share queues, and work on a shared queue runs in order.
	{
		int least = 0, greatest = 0;
		if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
		for (int i = 0; i < 4; i++)
			PTRY(i < 2 ? hipStreamCreateWithPriority(&streams[i], hipStreamNonBlocking, least)
			           : hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking),
			     "stream");
	}
	for (Copier& c : copiers) {
		PTRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "stream");
		c.th = std::thread([&c] { c.run(); });
	}
	for (Slot& s : slots) {
		PTRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "event");
		PTRY(hipEventCreateWithFlags(&s.kdone, hipEventDisableTiming), "event");
	}

	{
		uint32_t a = 0;
		while (a < n) {
			// -- gather the next chunk: consecutive positions of one kind (device m05 or host m05),
			// in order, as they finish
			std::vector<uint32_t> idx;
			uint64_t mbs = 0, vals = 0, bitsb = 0, outb = 0;
			uint32_t b = a, max_cols = 0, max_rows = 0;
			const bool ctok = feed.dev[feed.order[a]] != 0;  // this chunk's kind
			const uint32_t cframes = ctok ? chunk_frames_tok : chunk_frames_pk;
			const uint64_t cmbs = ctok ? chunk_mbs_tok : chunk_mbs_pk;
			while (b < n && b - a < cframes && (feed.dev[feed.order[b]] != 0) == ctok) {
				const uint32_t fi = feed.order[b];
				feed.wait_ready(fi);
				if (feed.err[fi] == 0) {
					const Vp8DecodedFrame& f = f_of(fi);
					if (!idx.empty() && mbs + f.mb_total > cmbs) break;
					idx.push_back(fi);
					mbs += f.mb_total;
					if (ctok) bitsb += bits_slot(feed.tj[fi].psize);
					else vals += feed.pk[fi].n_values;
					outb = al256(outb + vp8g_i420_size(kf_of(fi).width, kf_of(fi).height));
					if (f.mb_cols > max_cols) max_cols = f.mb_cols;
					if (f.mb_rows > max_rows) max_rows = f.mb_rows;
				}
				b++;
			}
			const uint32_t si = (ctok ? 0u : 2u) + (nchunk[ctok ? 1 : 0]++ & 1u);
			Slot& s = slots[si];
			hipStream_t stream = streams[si];
			if (!finish_slot(s)) goto fail;
			if (idx.empty()) {
				a = b;
				continue;
			}
			const uint32_t nf = (uint32_t)idx.size();
			// -- launch geometry (the choices vp8g_reconstruct_batch makes)
			// Split mode (a frame over several co-resident workgroups that spin on each other) only
			// for a chunk that is the call's only one: chunks on the other slots' streams -- a long
			// device-m05 kernel, the other host slot -- could hold the CUs a part is waiting for.
			const bool alone = a == 0 && b == n;
			uint32_t nw = vp8g::pick_waves(0, max_rows, nf);
			if (alone && vp8g::pick_split(0, nf, 8, max_rows) > 1) nw = 8;
			const bool big = vp8g::lds_bytes((int)nw, max_cols, false) > (size_t)vp8g::kMaxLds;
			const uint32_t k_plan = big || !alone ? 1u : vp8g::pick_split(0, nf, nw, max_rows);
			ChunkLayout L;
			uint64_t o = 0;
			L.ym = o, o = al256(o + mbs);
			L.uvm = o, o = al256(o + mbs);
			L.seg = o, o = al256(o + mbs);
			L.hasc = o, o = al256(o + mbs);
			L.bm = o, o = al256(o + mbs * 16);
			L.masks = o, o = al256(o + (ctok ? 0 : mbs * kNb * 2));
			L.mboff = o, o = al256(o + (ctok ? 0 : mbs * 4));
			L.vals = o, o = al256(o + (ctok ? 0 : vals * 2 + 64));  // +64: the expansion may address one past the end
			L.cy = o, o = al256(o + mbs * 512);
			L.cu = o, o = al256(o + mbs * 128);
			L.cv = o, o = al256(o + mbs * 128);
			L.cy2 = o, o = al256(o + mbs * 32);
			L.bits = o, o = al256(o + bitsb);
			L.jobs = o, o = al256(o + (ctok ? nf * sizeof(Vp8gTokFrame) : 0));
			L.desc = o, o = al256(o + nf * sizeof(Vp8gFrameDesc));
			L.status = o, o = al256(o + 4);
			// (every frame's column context: the global-context variant for frames too wide for LDS, and
			// the quad chain kernel, whose rows hand over through device memory)
			L.gctx = o, o = al256(o + (uint64_t)nf * max_cols * vp8g::kCtxBytesPerCol);
			L.mbox = o, o = al256(o + (k_plan > 1 ? (uint64_t)nf * k_plan * max_cols * vp8g::kCtxBytesPerCol : 0));
			L.gprog = o, o = al256(o + (k_plan > 1 ? (uint64_t)nf * k_plan * 4 : 0));
			L.out = o, o = al256(o + outb);
			L.total = o;
			const double tg = trace ? ms_now() : 0.0;
			PTRY(grow(s, L.total), "hipMalloc(chunk)");
			if (trace) fprintf(stderr, "[pipe] slot %u buffer %.1f GB ready at %.1f ms (%.1f ms)\n", si, L.total / 1e9, ms_now(), ms_now() - tg);
			uint8_t* d = s.buf;
			// -- descriptors and output images
			s.descs.assign(nf, Vp8gFrameDesc{});
			if (ctok) {
				s.jobs.resize(nf);
				uint64_t mo = 0, bo = 0, oo = 0;
				for (uint32_t j = 0; j < nf; j++) {
					TokJob& t = feed.tj[idx[j]];
					if (vp8g::make_desc(&t.kf, &t.hdr, filtered, mo, oo, &s.descs[j], false) != 0 ||
					    vp8g::alloc_planes(&outs[idx[j]], t.kf.width, t.kf.height, false) != 0) {
						feed.err[idx[j]] = errno ? errno : EINVAL;  // (cannot happen for a frame the header parse accepted)
						s.descs[j].flags = 0;
					}
					s.jobs[j] = t.tf;
					s.jobs[j].data = bo;
					s.jobs[j].mb_offset = mo;
					PTRY(hipMemcpyAsync(d + L.bits + bo, files[idx[j]].data + t.poff, t.psize, hipMemcpyHostToDevice, stream),
					     "H2D");
					mo += t.hdr.mb_total;
					bo += bits_slot(t.psize);
					oo = al256(oo + vp8g_i420_size(t.kf.width, t.kf.height));
				}
				PTRY(hipMemcpyAsync(d + L.jobs, s.jobs.data(), nf * sizeof(Vp8gTokFrame), hipMemcpyHostToDevice, stream), "H2D");
			} else {
				uint64_t mo = 0, vo = 0, oo = 0;
				for (uint32_t j = 0; j < nf; j++) {
					Vp8gPackedFrame& p = feed.pk[idx[j]];
					if (vp8g::make_desc(&p.kf, &p.f, filtered, mo, oo, &s.descs[j], false) != 0 ||
					    vp8g::alloc_planes(&outs[idx[j]], p.kf.width, p.kf.height, false) != 0) {
						feed.err[idx[j]] = errno ? errno : EINVAL;  // (cannot happen for a frame m05 accepted)
						s.descs[j].flags = 0;
					}
					// chunk-relative value offsets
					if (vo)
						for (uint32_t m = 0; m < p.f.mb_total; m++) p.mb_off[m] += (uint32_t)vo;
					const uint64_t mt = p.f.mb_total;
					PTRY(hipMemcpyAsync(d + L.ym + mo, p.f.ymode, mt, hipMemcpyHostToDevice, stream), "H2D");
					PTRY(hipMemcpyAsync(d + L.uvm + mo, p.f.uv_mode, mt, hipMemcpyHostToDevice, stream), "H2D");
					PTRY(hipMemcpyAsync(d + L.seg + mo, p.f.segment_id, mt, hipMemcpyHostToDevice, stream), "H2D");
					PTRY(hipMemcpyAsync(d + L.hasc + mo, p.f.has_coeff, mt, hipMemcpyHostToDevice, stream), "H2D");
					PTRY(hipMemcpyAsync(d + L.bm + mo * 16, p.f.bmode, mt * 16, hipMemcpyHostToDevice, stream), "H2D");
					PTRY(hipMemcpyAsync(d + L.masks + mo * kNb * 2, p.masks, mt * kNb * 2, hipMemcpyHostToDevice, stream), "H2D");
					PTRY(hipMemcpyAsync(d + L.mboff + mo * 4, p.mb_off, mt * 4, hipMemcpyHostToDevice, stream), "H2D");
					if (p.n_values)
						PTRY(hipMemcpyAsync(d + L.vals + vo * 2, p.values, p.n_values * 2, hipMemcpyHostToDevice, stream), "H2D");
					mo += mt;
					vo += p.n_values;
					oo = al256(oo + vp8g_i420_size(p.kf.width, p.kf.height));
				}
			}
			s.frames = idx;
			if (trace)
				fprintf(stderr, "[pipe] chunk %s slot %u frames=%u mbs=%llu launched at %.1f ms\n", ctok ? "device-m05" : "host-m05", si,
				        nf, (unsigned long long)mbs, ms_now());
			PTRY(hipMemcpyAsync(d + L.desc, s.descs.data(), nf * sizeof(Vp8gFrameDesc), hipMemcpyHostToDevice, stream), "H2D");
			PTRY(hipMemsetAsync(d + L.status, 0, 4, stream), "memset");
			// -- expansion (or device m05) + recon(+LF), inside the process-wide launch gate
			// (vp8g_device.h): the split mode only when no other launch of the library is in flight
			{
				vp8g::GateScope gate(stream);
				PTRY(gate.status(), "hipStreamWaitEvent(gate)");
				const uint32_t k = k_plan > 1 && gate.may_cross() ? k_plan : 1u;
				if (k > 1) PTRY(hipMemsetAsync(d + L.gprog, 0, (size_t)nf * k * 4, stream), "memset");
				Vp8gBatchArrays arr;
				arr.coeff_y = (const int16_t*)(d + L.cy);
				arr.coeff_u = (const int16_t*)(d + L.cu);
				arr.coeff_v = (const int16_t*)(d + L.cv);
				arr.coeff_y2 = (const int16_t*)(d + L.cy2);
				arr.ymode = d + L.ym;
				arr.uv_mode = d + L.uvm;
				arr.segment_id = d + L.seg;
				arr.has_coeff = d + L.hasc;
				arr.bmode = d + L.bm;
				arr.src = nullptr;
				arr.status = (uint32_t*)(d + L.status);
				if (ctok) {
					PTRY(hipMemsetAsync(d + L.cy, 0, L.cy2 + mbs * 32 - L.cy, stream), "memset");
					if (vp8g_m05_batch_device(s.jobs.data(), (const Vp8gTokFrame*)(d + L.jobs), nf, d + L.bits, &arr, stream) != 0) {
						he = hipGetLastError();
						if (he == hipSuccess) he = hipErrorInvalidValue;
						where = "m05 launch";
						goto fail;
					}
				} else {
					const uint64_t threads_x = mbs * 32;
					hipLaunchKernelGGL(expand_kernel, dim3((uint32_t)((threads_x + 255) / 256)), dim3(256), 0, stream,
					                   (const uint16_t*)(d + L.masks), (const uint32_t*)(d + L.mboff),
					                   (const int16_t*)(d + L.vals), (uint32_t)mbs, (int16_t*)(d + L.cy), (int16_t*)(d + L.cu),
					                   (int16_t*)(d + L.cv), (int16_t*)(d + L.cy2));
					PTRY(hipGetLastError(), "expand launch");
				}
				bool ordered = false;
				const bool quad = !big && k == 1 && vp8g::pick_quad(s.descs.data(), nf);  // (four MB rows per wave)
				const uint32_t wg = big || k > 1 || (vp8g::kChainG && !quad) ? 0u : vp8g::pick_chain(s.descs.data(), nf, max_cols, &ordered, quad);
				if (wg)  // more frames than CUs: one 16-wave chain of frames per CU
					PTRY(vp8g::launch_chain((const Vp8gFrameDesc*)(d + L.desc), nf, arr, d + L.out, max_cols, stream, wg, ordered, false,
					                        quad ? d + L.gctx : nullptr, nullptr, 0u, false, quad,
					                        quad && vp8g::whole_pieces(s.descs.data(), nf)),
					     "recon launch");
				else
					PTRY(vp8g::launch_frames((const Vp8gFrameDesc*)(d + L.desc), nf, arr, d + L.out, max_cols, max_rows,
					                         big ? d + L.gctx : nullptr, stream, nw, k, k > 1 ? d + L.mbox : nullptr,
					                         k > 1 ? (uint32_t*)(d + L.gprog) : nullptr),
					     "recon launch");
				PTRY(gate.done(k > 1), "hipEventRecord(gate)");
			}
			// -- D2H into the callers' images, by this kind's Copier once the kernels are done
			PTRY(hipEventRecord(s.kdone, stream), "event");
			s.d2h.clear();
			for (uint32_t j = 0; j < nf; j++) {
				const Vp8gFrameDesc& fd = s.descs[j];
				Yuv420Image& img = outs[idx[j]];
				if (!img.y) continue;
				const size_t ysz = (size_t)fd.stride_y * fd.height, uvsz = (size_t)fd.stride_uv * ((fd.height + 1) / 2);
				s.d2h.push_back({img.y, d + L.out + fd.out_y, ysz});
				s.d2h.push_back({img.u, d + L.out + fd.out_u, uvsz});
				s.d2h.push_back({img.v, d + L.out + fd.out_v, uvsz});
			}
			s.d2h.push_back({&s.status, d + L.status, 4});
			copiers[ctok ? 1 : 0].push(&s);
			s.busy = true;
			released = b;
			feed.set_limit(released + window);
			a = b;
		}
		defer_release = true;
		for (Slot& s : slots)
			if (!finish_slot(s)) goto fail;
		defer_release = false;
	}
	if (trace) fprintf(stderr, "[pipe] all chunks retired at %.1f ms\n", ms_now());

	for (auto& t : pool) t.join();
	pool.clear();
	for (Copier& c : copiers) c.stop();
	for (Slot& s : slots) {
		if (s.done) (void)hipEventDestroy(s.done);
		if (s.kdone) (void)hipEventDestroy(s.kdone);
		if (s.buf) (void)hipFree(s.buf);
	}
	for (hipStream_t st : streams) (void)hipStreamDestroy(st);
	for (Copier& c : copiers) (void)hipStreamDestroy(c.stream);
	if (trace) fprintf(stderr, "[pipe] buffers freed at %.1f ms\n", ms_now());
	if (!late.empty()) {  // (started last: its heap trimming would contend with the device-memory frees above)
		g_freer.post(std::move(late));
	}
	{
		int first = 0;
		for (uint32_t i = 0; i < n; i++) {
			if (!feed.dev[i]) vp8f_packed_free(&feed.pk[i]);  // failed frames (the others were freed per chunk)
			if (status) status[i] = feed.err[i];
			if (feed.err[i] && !first) first = feed.err[i];
			if (feed.err[i]) yuv420_free(&outs[i]);
		}
		if (first) {
			errno = first;
			return -1;
		}
	}
	return 0;

fail:
	feed.stop();
	for (auto& t : pool) t.join();
	for (Vp8gPackedFrame& p : late) vp8f_packed_free(&p);
	for (Copier& c : copiers) c.stop();
	for (hipStream_t st : streams)
		if (st) (void)hipStreamSynchronize(st);
	for (Copier& c : copiers)
		if (c.stream) (void)hipStreamSynchronize(c.stream);
	vp8g::set_error_text(where ? where : "pipeline", he);
	for (Slot& s : slots) {
		if (s.done) (void)hipEventDestroy(s.done);
		if (s.kdone) (void)hipEventDestroy(s.kdone);
		if (s.buf) (void)hipFree(s.buf);
	}
	for (hipStream_t st : streams)
		if (st) (void)hipStreamDestroy(st);
	for (Copier& c : copiers)
		if (c.stream) (void)hipStreamDestroy(c.stream);
	for (uint32_t i = 0; i < n; i++) {
		if (!feed.dev[i]) vp8f_packed_free(&feed.pk[i]);
		yuv420_free(&outs[i]);
		if (status) status[i] = EIO;
	}
	errno = EIO;
	return -1;
#undef PTRY
}

VP8G_API int vp8g_decode_webp_batch(const ByteSpan* files, uint32_t n, int filtered, uint32_t threads, Yuv420Image* outs,
                                    int* status) {
	return vp8g_decode_webp_batch_ex(files, n, filtered, threads, 0, outs, status);
}
