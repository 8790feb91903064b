// vp8g_digest.hip -- per-frame 64-bit digest of the cropped I420 outputs, on the device.
//
// Parity over a whole device-resident batch without copying pixels back: one launch reads every
// frame's output once (HBM-bound, ~1 ms per 512 x 4K) and leaves one 64-bit word per frame, which
// the caller compares with the digest of the reference decoder's I420 for the same input
// (tests/golden/digests.json) or gathers across ranks (vp8g_dist).  The reference has no
// equivalent; its gates compare whole files (scripts/m7_compare_yuv_filtered_with_oracle.sh:66).
//
// Definition (also restated in numpy as vp8g.digest64, and in DESIGN.md §5): the frame's I420
// bytes B[0..L) (Y rows, then U, then V, each at stride = row width -- exactly the file the
// reference CLI writes, src/main.c:681-687) as little-endian 64-bit words w_i, the last one
// zero-padded;  D = L*K + sum_i mix(w_i + (i + 1)*K)  (mod 2^64), K = 0x9E3779B97F4A7C15, mix =
// the splitmix64 finaliser.  A sum of position-keyed mixes is order-sensitive like a hash and
// fully parallel: blocks reduce their words and add into the frame's word with 64-bit atomics
// (integer adds commute, so the result does not depend on scheduling).
#include <errno.h>
#include <stdio.h>

#include <vector>

#include "vp8g_device.h"

#define VP8G_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr uint64_t kK = 0x9E3779B97F4A7C15ull;
constexpr uint32_t kChunk = 65536;  // bytes per workgroup
constexpr int kThreads = 256;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

// grid: x = 64-KB chunk of a frame, y = frame
__global__ __launch_bounds__(kThreads) void digest_kernel(const Vp8gFrameDesc* __restrict__ descs, const uint8_t* __restrict__ out,
                                                          unsigned long long* __restrict__ dig) {
	const Vp8gFrameDesc& D = descs[blockIdx.y];
	const uint64_t base = D.out_y;
	const uint64_t len = D.out_v + (uint64_t)D.stride_uv * ((D.height + 1) / 2) - D.out_y;
	const uint64_t c0 = (uint64_t)blockIdx.x * kChunk;
	if (c0 >= len) return;
	const uint64_t c1 = c0 + kChunk < len ? c0 + kChunk : len;
	const uint8_t* p = out + base;
	uint64_t acc = 0;
	const bool aligned = (base & 15u) == 0;
	// 16 bytes (two words) per lane per iteration; chunk starts are multiples of 16
	for (uint64_t o = c0 + 16u * threadIdx.x; o < c1; o += 16u * kThreads) {
		uint64_t w0, w1;
		if (aligned && o + 16 <= len) {
			const uint4 v = *(const uint4*)(p + o);
			w0 = (uint64_t)v.x | ((uint64_t)v.y << 32);
			w1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
		} else {  // frame tail or unaligned frame start: byte loads, zero padding
			w0 = w1 = 0;
			for (int b = 0; b < 16; b++) {
				const uint64_t x = o + (uint64_t)b < len ? p[o + b] : 0u;
				if (b < 8) w0 |= x << (8 * b);
				else w1 |= x << (8 * (b - 8));
			}
		}
		const uint64_t i0 = o >> 3;
		acc += mix64(w0 + (i0 + 1) * kK);
		if (o + 8 < len) acc += mix64(w1 + (i0 + 2) * kK);
	}
	// wave reduction, then one add per wave
	for (int s = 32; s > 0; s >>= 1) {
		const uint32_t lo = __shfl_xor((uint32_t)acc, s), hi = __shfl_xor((uint32_t)(acc >> 32), s);
		acc += (uint64_t)lo | ((uint64_t)hi << 32);
	}
	if ((threadIdx.x & 63) == 0) {
		if (blockIdx.x == 0 && threadIdx.x == 0) acc += len * kK;
		atomicAdd(dig + blockIdx.y, (unsigned long long)acc);
	}
}

}  // namespace

VP8G_API int vp8g_frame_digests(const Vp8gFrameDesc* h_descs, const Vp8gFrameDesc* d_descs, uint32_t n, const uint8_t* d_out,
                                uint64_t* d_digests, void* stream) {
	if (!h_descs || !d_descs || !d_out || !d_digests) {
		errno = EINVAL;
		return -1;
	}
	if (n == 0) return 0;
	if (n > 65535) {  // grid.y limit
		errno = EINVAL;
		return -1;
	}
	uint64_t max_len = 0;
	for (uint32_t i = 0; i < n; i++) {
		const Vp8gFrameDesc& d = h_descs[i];
		const uint64_t cw = (d.width + 1) / 2, ch = (d.height + 1) / 2;
		// the digest covers the contiguous cropped I420 layout vp8g_make_frame_desc produces
		if (d.stride_y != d.width || d.stride_uv != cw || d.out_u != d.out_y + (uint64_t)d.width * d.height ||
		    d.out_v != d.out_u + cw * ch) {
			errno = EINVAL;
			return -1;
		}
		const uint64_t len = (uint64_t)d.width * d.height + 2 * cw * ch;
		if (len > max_len) max_len = len;
	}
	hipStream_t s = (hipStream_t)stream;
	vp8g::GateScope gate(s);  // (vp8g_device.h: no cross-workgroup launch beside it)
	hipError_t e = gate.status();
	if (e == hipSuccess) e = hipMemsetAsync(d_digests, 0, (size_t)n * 8, s);
	if (e == hipSuccess) {
		const uint32_t chunks = (uint32_t)((max_len + kChunk - 1) / kChunk);
		hipLaunchKernelGGL(digest_kernel, dim3(chunks, n), dim3(kThreads), 0, s, d_descs, d_out,
		                   (unsigned long long*)d_digests);
		e = hipGetLastError();
	}
	if (e == hipSuccess) e = gate.done(false);
	if (e != hipSuccess) {
		vp8g::set_error_text("digest", e);
		errno = EIO;
		return -1;
	}
	return 0;
}
