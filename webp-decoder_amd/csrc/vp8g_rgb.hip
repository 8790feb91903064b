// vp8g_rgb.hip -- m08 / m09 on the GPU: "fancy" 4:2:0 upsampled I420 -> RGB24 and the exact
// PPM / PNG files the reference writes (src/m08_yuv2rgb_ppm/yuv2rgb_ppm.c, src/m09_png/yuv2rgb_png.c).
//
// The output FILE is the unit of work: it is cut into VP8G_ENC_SPAN-byte spans (32 KB), one
// workgroup task each (a workgroup loops over tasks).
//   enc_write_kernel (every format) writes a span's bytes straight to HBM: one thread per 12-pixel
//     chunk of a row (six pixel pairs, each pair sharing four chroma samples and the 9:3:3:1
//     diagonals; one unaligned 8-byte load per chroma row and plane with the edge columns
//     replicated, one 12-byte luma load; 36 bytes out with unaligned 8-byte stores), plus the few
//     layout bytes (PPM header; PNG signature / IHDR / IDAT header / zlib header, the 5-byte
//     stored-block headers, the IEND trailer).  No LDS and no barriers: the waves of a CU overlap
//     their memory latency freely.
//   crc_kernel (PNG) re-reads each span, 32 contiguous bytes per thread, folds them into a CRC-32
//     (slice-by-8 tables in LDS) and Adler-32 partial sums, and combines the 1024 thread partials
//     (lane shuffles inside a wave, GF(2) shift operators as nibble tables) into one per span.
//   png_finish_kernel (one workgroup per PNG) combines the span partials with host-precomputed
//     operators and writes the Adler-32 and the IDAT CRC.
// Every byte of every file is produced on the device.
//
// CRC algebra (reflected CRC-32, polynomial 0xEDB88320): the raw register update is linear, so
// with Z_n = "feed n zero bytes", crc_raw(A || B) = Z_|B|(crc_raw(A)) ^ crc_raw(B), leading zero
// bytes change nothing, and crc32(M) = ~(crc_raw(M) ^ Z_|M|(0xFFFFFFFF)).  Spans are CRC'd over
// the whole span with every byte outside the IDAT CRC range (and the 4 Adler bytes, patched in at
// the end) read as zero; the padded total is shifted back by Z_-d.  The host precomputes the
// operators (32 columns each).
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "vp8g_device.h"

#define VP8G_API extern "C" __attribute__((visibility("default")))
#define DEV __device__ __forceinline__

namespace {

constexpr uint32_t kSpan = VP8G_ENC_SPAN;
constexpr int kThreads = 1024;                     // task kernel
constexpr uint32_t kPerThread = kSpan / kThreads;  // 32 contiguous file bytes per thread
constexpr int kFinThreads = 256;                   // PNG finishing kernel
constexpr int kFinLevels = 8;                      // log2(kFinThreads)
constexpr uint32_t kChunk = 12;                     // pixels of a row per thread and iteration (36 bytes)
constexpr uint32_t kUnits = kChunk / 2;            // pixel-pair units m .. m + kUnits touched by a chunk
constexpr uint32_t kMod = 65521u;                  // Adler-32
constexpr uint32_t kBlk = 65535u;                  // stored-deflate block payload
constexpr uint32_t kBlkFile = kBlk + 5u;           // ... plus its header
constexpr uint32_t kPngPrefix = 43u;               // signature 8, IHDR 25, IDAT len/type 8, zlib 2
constexpr uint32_t kPngRaw0 = kPngPrefix + 5u;     // file offset of the first pixel-stream byte
constexpr uint32_t kCrcStart = 37u;                // IDAT CRC covers the chunk type + data
static_assert(kSpan % kThreads == 0 && kPerThread % 16 == 0, "span layout");

// Tables shared by every task (48 KB): CRC-32 slice-by-8 tables T0..T7, then the nibble tables
// (tab[base + 128 i + 16 j + v] = Z(v << 4j)) of the operators that move a thread's CRC to the end
// of the span: per lane L, Z_{(63 - L) * 32} (to the end of its wave's 2 KB), per wave w,
// Z_{(15 - w) * 2048} (to the end of the span).  The span CRC is then a plain XOR over lanes and
// waves: one 8-lookup operator per thread instead of a 10-level tree of them.
constexpr int kSlice = 8;
constexpr int kNibBase = kSlice * 256;
constexpr int kWaves = kThreads / 64;
constexpr int kLaneOps = kNibBase;
constexpr int kWaveOps = kLaneOps + 64 * 128;
constexpr int kTabWords = kWaveOps + kWaves * 128;

struct CrcLds {
	uint32_t tab[kTabWords];
	uint32_t red[2][3][kThreads / 64];  // per-wave partials, double-buffered by task parity
};

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

// ---- device helpers ----------------------------------------------------------------------
// reference yuv2rgb_ppm.c:19-42: libwebp VP8YuvToRgb (14-bit fixed point, clip of v >> 6)
// Clamp before the shift (same result as clip(v >> 6)): the shift-then-clamp form of two
// neighbouring channels is selected as v_ashr_pk_u8_i32, whose result here kept the old upper 16
// bits of its destination register, which then leaked into the packed colour word.
DEV uint32_t clip6(int v) { return (uint32_t)min(max(v, 0), 16383) >> 6; }
DEV uint32_t yuv_rgb(int y, int u, int v) {  // packed r | g << 8 | b << 16
	const int yy = (y * 19077) >> 8;
	const uint32_t r = clip6(yy + ((v * 26149) >> 8) - 14234);
	const uint32_t g = clip6(yy - ((u * 6419) >> 8) - ((v * 13320) >> 8) + 8708);
	const uint32_t b = clip6(yy + ((u * 33050) >> 8) - 17685);
	return r | (g << 8) | (b << 16);
}

// One unit = pixels {2k-1, 2k} of a row (reference yuv2rgb_ppm.c:44-121): it blends chroma columns
// k-1 and k of the two chroma rows around the pixel row (at the edges both columns are one, which
// gives the 3:1 edge formula exactly).  (tl, t) = row a, (l, u) = row b; near_a = the pixel row is
// nearer row a.  Returns the two pixels' colours.
DEV void pair_rgb(bool near_a, int tlu, int tu, int lu, int uu, int tlv, int tv, int lv, int uv, int y_odd, int y_even,
                  uint32_t& c_odd, uint32_t& c_even) {
	const int au = tlu + tu + lu + uu + 8, av = tlv + tv + lv + uv + 8;
	const int d12u = (au + 2 * (tu + lu)) >> 3, d03u = (au + 2 * (tlu + uu)) >> 3;
	const int d12v = (av + 2 * (tv + lv)) >> 3, d03v = (av + 2 * (tlv + uv)) >> 3;
	c_odd = yuv_rgb(y_odd, near_a ? (d12u + tlu) >> 1 : (d03u + lu) >> 1, near_a ? (d12v + tlv) >> 1 : (d03v + lv) >> 1);
	c_even = yuv_rgb(y_even, near_a ? (d03u + tu) >> 1 : (d12u + uu) >> 1, near_a ? (d03v + tv) >> 1 : (d12v + uv) >> 1);
}

// file offset of pixel-stream byte p (PNG: stored blocks of kBlk bytes behind 5-byte headers)
DEV uint32_t png_file_of_raw(uint32_t p) { return kPngRaw0 + p + 5u * (p / kBlk); }
// first pixel-stream byte at or after file offset q, clamped to n
DEV uint32_t raw_of_file(const Vp8gEncDesc& d, uint32_t q) {
	if (d.format != VP8G_ENC_PNG) return q <= d.prefix_len ? 0u : min(q - d.prefix_len, d.raw_len);
	if (q <= kPngRaw0) return 0u;
	const uint32_t z = q - kPngPrefix, k = z / kBlkFile, o = z - k * kBlkFile;
	return min(k * kBlk + (o < 5u ? 0u : o - 5u), d.raw_len);
}

DEV uint32_t byte_of2(u32x2 v, int i) { return ((i < 4 ? v.x : v.y) >> (8 * (i & 3))) & 255u; }
DEV uint32_t byte_of3(u32x3 v, int i) { return ((i < 4 ? v.x : (i < 8 ? v.y : v.z)) >> (8 * (i & 3))) & 255u; }
DEV uint32_t crc_byte(const uint32_t* t0, uint32_t c, uint32_t b) { return t0[(c ^ b) & 255u] ^ (c >> 8); }
DEV uint32_t crc_dword2(const uint32_t* t, uint32_t c, uint32_t w0, uint32_t w1) {  // slice-by-8, 8 bytes
	c ^= w0;
	return t[1792 + (c & 255u)] ^ t[1536 + ((c >> 8) & 255u)] ^ t[1280 + ((c >> 16) & 255u)] ^ t[1024 + (c >> 24)] ^
	       t[768 + (w1 & 255u)] ^ t[512 + ((w1 >> 8) & 255u)] ^ t[256 + ((w1 >> 16) & 255u)] ^ t[w1 >> 24];
}
DEV uint32_t nib_apply(const uint32_t* nt, uint32_t v) {  // GF(2) operator via 8 nibble tables
	uint32_t r = 0;
#pragma unroll
	for (int j = 0; j < 8; j++) r ^= nt[j * 16 + ((v >> (4 * j)) & 15u)];
	return r;
}
DEV uint32_t mod_add(uint32_t a, uint32_t b) {  // (a + b) mod 65521 for a, b < 65521
	const uint32_t t = a + b;
	return t >= kMod ? t - kMod : t;
}
DEV uint32_t op_apply(const uint32_t* col, uint32_t v) {  // GF(2) operator by columns
	uint32_t r = 0;
#pragma unroll
	for (int i = 0; i < 32; i++) r ^= ((v >> i) & 1u) ? col[i] : 0u;
	return r;
}

// 8 chroma samples, columns m1 .. m1 + 7 of one row (m1 >= -1), with the edge rule of the
// upsampler (reference yuv2rgb_ppm.c:44-121: column -1 reads column 0, columns >= cw read cw - 1):
// one unaligned 8-byte load inside the row, then the missing edge bytes replicated.  cw >= 8.
DEV uint64_t chroma8(const uint8_t* row, int m1, int cw) {
	const int s = min(max(m1, 0), cw - 8);
	uint64_t v = *(const uint64_t*)(row + s);  // unaligned: gfx950 runs in unaligned mode (tools/ubench/unaligned.hip)
	const int dl = m1 - s;                     // -1 (left edge), 0 (inside), 1..7 (right edge)
	if (dl < 0) v = (v << 8) | (v & 0xFFu);
	if (dl > 0) v = (v >> (8 * dl)) | (((v >> 56) * 0x0101010101010101ull) << (64 - 8 * dl));
	return v;
}
DEV uint32_t byte8(uint64_t v, int i) { return (uint32_t)(v >> (8 * i)) & 255u; }

// Pixel bytes of the span [F0, F0 + kSpan) of image d's file, written straight into the file:
// thread tid of NT takes chunks of kChunk pixels of a row (chunk index = row * chunks per row +
// column chunk) and stores its 36 bytes with unaligned 8-byte stores (full lines form in L2 from
// the neighbouring threads).  A chunk that straddles two spans is written whole by both, with
// the same bytes.  (Assembling each wave's run in LDS for aligned 16-byte stores was measured
// slower: the extra registers cost more occupancy than the coalescing gained.)
template <int NT>
DEV void span_pixels(const Vp8gEncDesc& d, bool png, uint32_t F0, uint32_t tid, const uint8_t* __restrict__ src,
                     uint8_t* __restrict__ file) {
	const uint32_t p_lo = raw_of_file(d, F0), p_hi = raw_of_file(d, F0 + kSpan);
	if (p_lo >= p_hi) return;
	const uint32_t W = d.width, SB = d.row_bytes, f = png ? 1u : 0u;
	const uint32_t cw = (W + 1u) >> 1, ch = (d.height + 1u) >> 1;
	const uint32_t CPR = (W + kChunk - 1u) / kChunk;  // chunks per row
	const uint32_t ylo = p_lo / SB, rlo = p_lo - ylo * SB, xlo = rlo < f ? 0u : (rlo - f) / 3u;
	const uint32_t yhi = (p_hi - 1u) / SB, rhi = p_hi - 1u - yhi * SB, xhi = rhi < f ? 0u : (rhi - f) / 3u;
	const uint32_t g_first = ylo * CPR + xlo / kChunk, g_last = yhi * CPR + xhi / kChunk;
	const uint8_t* Y = src + d.src_y;
	const uint8_t* U = src + d.src_u;
	const uint8_t* V = src + d.src_v;
	auto file_of = [&](uint32_t pi) { return png ? kPngRaw0 + pi + 5u * (pi / kBlk) : d.prefix_len + pi; };
	for (uint32_t gc = g_first + tid; gc <= g_last; gc += NT) {
		const uint32_t y = gc / CPR, x0 = (gc - y * CPR) * kChunk, m = x0 >> 1;
		// chroma rows (reference yuv2rgb_ppm.c:178-202): row 0 uses row 0 twice; row y sits between
		// a = (y-1)/2 and b = min(a+1, ch-1), nearer a when y is odd
		const uint32_t a = y ? (y - 1u) >> 1 : 0u, b = y ? min(a + 1u, ch - 1u) : 0u;
		const bool near_a = y == 0 || (y & 1u);
		const uint32_t rowp = y * SB;
		if (png && x0 == 0) file[file_of(rowp)] = 0;  // the scanline's filter byte (0 = none)
		const uint32_t p0 = rowp + f + 3u * x0;          // raw offset of the chunk's first pixel byte
		if (x0 + kChunk <= W && cw >= 8u) {
			// units m .. m+6 (unit k = pixels 2k-1, 2k) over chroma columns m-1 .. m+6 of rows a, b;
			// pixel x0 + 2i is the even pixel of unit m+i, x0 + 2i - 1 the odd pixel of unit m+i
			const int m1 = (int)m - 1;
			const uint64_t ua = chroma8(U + a * d.stride_uv, m1, (int)cw), ub = chroma8(U + b * d.stride_uv, m1, (int)cw);
			const uint64_t va = chroma8(V + a * d.stride_uv, m1, (int)cw), vb = chroma8(V + b * d.stride_uv, m1, (int)cw);
			const u32x3 yl = *(const u32x3*)(Y + y * d.stride_y + x0);
			uint32_t c[kChunk];
#pragma unroll
			for (int i = 0; i <= (int)kUnits; i++) {
				uint32_t c_odd, c_even;
				const int yo = i ? (int)byte_of3(yl, 2 * i - 1) : 0, ye = i < (int)kUnits ? (int)byte_of3(yl, 2 * i) : 0;
				pair_rgb(near_a, (int)byte8(ua, i), (int)byte8(ua, i + 1), (int)byte8(ub, i), (int)byte8(ub, i + 1),
				         (int)byte8(va, i), (int)byte8(va, i + 1), (int)byte8(vb, i), (int)byte8(vb, i + 1), yo, ye, c_odd, c_even);
				if (i) c[2 * i - 1] = c_odd;
				if (i < (int)kUnits) c[2 * i] = c_even;
			}
			// 12 pixels -> 36 bytes -> 9 dwords (4 pixels = 3 dwords)
			uint32_t w[9];
#pragma unroll
			for (int k = 0; k < 3; k++) {
				w[3 * k + 0] = c[4 * k] | (c[4 * k + 1] << 24);
				w[3 * k + 1] = (c[4 * k + 1] >> 8) | (c[4 * k + 2] << 16);
				w[3 * k + 2] = (c[4 * k + 2] >> 16) | (c[4 * k + 3] << 8);
			}
			if (!png || p0 / kBlk == (p0 + 3u * kChunk - 1u) / kBlk) {
				// unaligned 8-byte stores (gfx950 runs in unaligned mode, tools/ubench/unaligned.hip)
				uint8_t* o = file + file_of(p0);
#pragma unroll
				for (int k = 0; k < 4; k++) *(u32x2*)(o + 8 * k) = u32x2{w[2 * k], w[2 * k + 1]};
				*(uint32_t*)(o + 32) = w[8];
			} else {  // a stored-block header falls inside the chunk: byte by byte
#pragma unroll
				for (uint32_t i = 0; i < 3u * kChunk; i++) file[file_of(p0 + i)] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
			}
			continue;
		}
		// generic chunk (a row's last, partial chunk; images narrower than 15 pixels): pixel by pixel
		const uint32_t xe = min(x0 + kChunk, W);
		for (uint32_t x = x0; x < xe; x++) {
			const uint32_t k = (x + 1u) >> 1;  // unit: pixels 2k-1 (odd x) and 2k (even x)
			const uint32_t cl = k ? k - 1u : 0u, cr = min(k, cw - 1u);
			const uint32_t ra = a * d.stride_uv, rb = b * d.stride_uv;
			uint32_t c_odd, c_even;
			const int yv = Y[y * d.stride_y + x];
			pair_rgb(near_a, U[ra + cl], U[ra + cr], U[rb + cl], U[rb + cr], V[ra + cl], V[ra + cr], V[rb + cl], V[rb + cr], yv, yv,
			         c_odd, c_even);
			const uint32_t col = (x & 1u) ? c_odd : c_even;
			const uint32_t pb = rowp + f + 3u * x;
#pragma unroll
			for (uint32_t i = 0; i < 3; i++) file[file_of(pb + i)] = (uint8_t)(col >> (8 * i));
		}
	}
}

// ---- PNG checksum kernel: one workgroup task per 32 KB span of a PNG file already written by
// enc_write_kernel; 32 contiguous bytes per thread folded into a CRC-32 (slice-by-8 tables in LDS)
// and Adler-32 partial sums, then combined over the span (below).
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void crc_kernel(
    const Vp8gEncDesc* __restrict__ D, uint32_t n, uint32_t total, const uint8_t* __restrict__ out,
    uint32_t* __restrict__ part, const uint32_t* __restrict__ tables) {
	__shared__ CrcLds L;
	const uint32_t tid = threadIdx.x;
	for (uint32_t i = tid; i < (uint32_t)kTabWords; i += kThreads) L.tab[i] = tables[i];
	__syncthreads();
	// The next task's 32 bytes per thread are loaded before the current task is folded and reduced,
	// so the HBM latency of a task overlaps the previous task's work.
	auto fetch = [&](uint32_t g, uint32_t& im, uint32_t* v) {
		while (im + 1 < n && D[im + 1].span0 <= g) im++;  // tasks are numbered image by image
		const Vp8gEncDesc& dd = D[im];
		const uint32_t q = (g - dd.span0) * kSpan + tid * kPerThread, fl = (uint32_t)dd.file_len;
		const bool use = dd.format == VP8G_ENC_PNG;
#pragma unroll
		for (uint32_t i = 0; i < kPerThread / 16u; i++) {
			const uint4 x = use && q + 16u * i < fl ? *(const uint4*)(out + dd.out + q + 16u * i) : make_uint4(0, 0, 0, 0);
			v[4 * i] = x.x, v[4 * i + 1] = x.y, v[4 * i + 2] = x.z, v[4 * i + 3] = x.w;
		}
	};
	uint32_t img = 0, img_next = 0, tcount = 0;
	uint32_t nxt[kPerThread / 4u];
	if (blockIdx.x < total) fetch(blockIdx.x, img_next, nxt);
	for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
		img = img_next;
		uint32_t bw[kPerThread / 4u];
#pragma unroll
		for (uint32_t i = 0; i < kPerThread / 4u; i++) bw[i] = nxt[i];
		if (g + gridDim.x < total) fetch(g + gridDim.x, img_next, nxt);
		const Vp8gEncDesc& d = D[img];
		if (d.format != VP8G_ENC_PNG) continue;
		const uint32_t F0 = (g - d.span0) * kSpan;  // file offset of this span
		const uint32_t q0 = F0 + tid * kPerThread;
		{
			uint32_t c = 0, s0 = 0, s1 = 0;
			const uint32_t N = d.raw_len;
			const uint32_t z0 = q0 - kPngPrefix, k0 = z0 / kBlkFile, o0 = z0 - k0 * kBlkFile;
			const uint32_t p0 = k0 * kBlk + o0 - 5u;
			const bool fast = q0 >= kPngRaw0 && o0 >= 5u && o0 + kPerThread <= kBlkFile && p0 + kPerThread <= N;
			if (fast) {
				// all 32 bytes are pixel-stream bytes of one stored block (inside the CRC range)
				uint32_t sj = 0;
#pragma unroll
				for (uint32_t i = 0; i < kPerThread / 4u; i += 2) {
					const uint32_t w0 = bw[i], w1 = bw[i + 1];
					c = crc_dword2(L.tab, c, w0, w1);
					s0 = __builtin_amdgcn_sad_u8(w1, 0u, __builtin_amdgcn_sad_u8(w0, 0u, s0));
					sj = __builtin_amdgcn_udot4(w0, 0x03020100u + 0x04040404u * i, sj, false);
					sj = __builtin_amdgcn_udot4(w1, 0x03020100u + 0x04040404u * (i + 1), sj, false);
				}
				// Adler b-sum: sum over bytes of (N - p) r_p = (N - p0) s0 - sum j r_j (mod 65521)
				const uint32_t w0 = (N - p0) % kMod;
				s1 = ((w0 * s0) % kMod + kMod - sj % kMod) % kMod;
				s0 %= kMod;
			} else if (q0 < d.zend + 4u) {
				const uint32_t crc_end = d.zend - 4u, raw_end = png_file_of_raw(N - 1u) + 1u;
#pragma unroll
				for (uint32_t j = 0; j < kPerThread; j++) {
					const uint32_t q = q0 + j, v = (bw[j >> 2] >> (8 * (j & 3))) & 255u;
					c = crc_byte(L.tab, c, (q >= kCrcStart && q < crc_end) ? v : 0u);
					if (q >= kPngRaw0 && q < raw_end) {
						const uint32_t z = q - kPngPrefix, k = z / kBlkFile, o = z - k * kBlkFile;
						if (o >= 5u) {
							const uint32_t p = k * kBlk + o - 5u;
							s0 = (s0 + v) % kMod;
							s1 = (s1 + ((N - p) % kMod) * v) % kMod;
						}
					}
				}
			} else {
				// past the CRC range: zero bytes (the padded tail of the last span)
#pragma unroll
				for (uint32_t i = 0; i < kPerThread / 4u; i += 2) c = crc_dword2(L.tab, c, 0u, 0u);
			}
			// -- 3. span CRC = XOR over threads t of Z_{(1023 - t) * 32}(crc_t): each lane moves its CRC
			// to the end of its wave's 2 KB and the wave XOR-reduces; wave 0 moves the 16 wave CRCs to
			// the end of the span and XOR-reduces them.  The Adler partials are plain sums (< 2^27 over
			// a span), reduced mod 65521 once at the end.
			const uint32_t lane = tid & 63u, wv = tid >> 6, par = tcount & 1u;
			c = nib_apply(L.tab + kLaneOps + lane * 128u, c);
#pragma unroll
			for (int l = 0; l < 6; l++) {
				c ^= __shfl_xor(c, 1 << l, 64);
				s0 += __shfl_xor(s0, 1 << l, 64);
				s1 += __shfl_xor(s1, 1 << l, 64);
			}
			if (lane == 0) L.red[par][0][wv] = c, L.red[par][1][wv] = s0, L.red[par][2][wv] = s1;
			__syncthreads();
			if (wv == 0) {
				c = lane < 16u ? nib_apply(L.tab + kWaveOps + lane * 128u, L.red[par][0][lane]) : 0u;
				s0 = lane < 16u ? L.red[par][1][lane] : 0u;
				s1 = lane < 16u ? L.red[par][2][lane] : 0u;
#pragma unroll
				for (int l = 0; l < 4; l++) {
					c ^= __shfl_xor(c, 1 << l, 16);
					s0 += __shfl_xor(s0, 1 << l, 16);
					s1 += __shfl_xor(s1, 1 << l, 16);
				}
				if (lane == 0) {
					uint32_t* pp = part + 4u * g;
					pp[0] = c;
					pp[1] = s0 % kMod;
					pp[2] = s1 % kMod;
				}
			}
			tcount++;
		}
	}
}

// ---- write kernel (every format): the file bytes of one 32 KB span per workgroup task, straight
// to HBM -- pixel bytes with unaligned 8-byte stores (full lines form in L2 from neighbouring
// threads), layout bytes one by one.  No LDS image and no barriers, so the waves of a CU overlap
// their loads freely.
constexpr int kPlainThreads = 256;
__global__ __launch_bounds__(kPlainThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void enc_write_kernel(const Vp8gEncDesc* __restrict__ D, uint32_t n,
                                                                  uint32_t total, const uint8_t* __restrict__ src,
                                                                  uint8_t* __restrict__ out) {
	const uint32_t tid = threadIdx.x;
	uint32_t img = 0;
	for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
		while (img + 1 < n && D[img + 1].span0 <= g) img++;  // tasks are numbered image by image
		const Vp8gEncDesc& d = D[img];
		const bool png = d.format == VP8G_ENC_PNG;
		const uint32_t F0 = (g - d.span0) * kSpan;
		uint8_t* file = out + d.out;
		span_pixels<kPlainThreads>(d, png, F0, tid, src, file);
		if (tid < 64) {
			// prefix (PPM header / PNG signature + IHDR + IDAT header + zlib header)
			if (tid < d.prefix_len && tid >= F0 && tid < F0 + kSpan) file[tid] = d.prefix[tid];
		} else if (png && tid < 74) {
			// stored-block headers: at most two blocks meet a span
			const uint32_t j = tid - 64, kc = (F0 >= kPngPrefix ? (F0 - kPngPrefix) / kBlkFile : 0u) + j / 5u;
			const uint32_t q = kPngPrefix + kc * kBlkFile + j % 5u;
			const uint32_t nblk = (d.raw_len + kBlk - 1u) / kBlk;
			if (kc < nblk && q >= F0 && q < F0 + kSpan) {
				const uint32_t len = min(kBlk, d.raw_len - kc * kBlk);
				const uint32_t hdr[5] = {kc + 1u == nblk ? 1u : 0u, len & 255u, len >> 8, ~len & 255u, (~len >> 8) & 255u};
				file[q] = (uint8_t)hdr[j % 5u];
			}
		} else if (png && tid >= 96 && tid < 116) {
			// Adler-32 and CRC placeholders (written by the finishing launch), IEND chunk
			const uint32_t i = tid - 96, q = d.zend - 4u + i;
			const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};
			if (q >= F0 && q < F0 + kSpan) file[q] = i < 8 ? 0 : iend[i - 8];
		}
	}
}

// ---- PNG finishing kernel: one workgroup per image ---------------------------------------
__global__ __launch_bounds__(kFinThreads) void png_finish_kernel(const Vp8gEncDesc* __restrict__ D,
                                                              const uint32_t* __restrict__ part, uint8_t* __restrict__ out,
                                                              const uint32_t* __restrict__ tables) {
	__shared__ uint32_t red[3][kFinThreads];
	const Vp8gEncDesc& d = D[blockIdx.x];
	if (d.format != VP8G_ENC_PNG) return;
	const uint32_t tid = threadIdx.x, G = d.nspans, m = (G + kFinThreads - 1u) / kFinThreads, pad = m * kFinThreads - G;
	// Horner over this thread's m consecutive spans (front-padded with zero spans: neutral)
	uint32_t c = 0, s0 = 0, s1 = 0;
	for (uint32_t i = 0; i < m; i++) {
		const int gi = (int)(tid * m + i) - (int)pad;
		c = op_apply(d.crc_ops[0], c);
		if (gi >= 0) {
			const uint32_t* pp = part + 4u * (d.span0 + (uint32_t)gi);
			c ^= pp[0];
			s0 = (s0 + pp[1]) % kMod;
			s1 = (s1 + pp[2]) % kMod;
		}
	}
	red[0][tid] = c;
	red[1][tid] = s0;
	red[2][tid] = s1;
	for (int l = 0; l < kFinLevels; l++) {
		__syncthreads();
		if (tid < (uint32_t)(kFinThreads >> (l + 1))) {
			const uint32_t lo = tid << (l + 1), hi = lo + (1u << l);
			red[0][lo] = op_apply(d.crc_ops[1 + l], red[0][lo]) ^ red[0][hi];
			red[1][lo] = (red[1][lo] + red[1][hi]) % kMod;
			red[2][lo] = (red[2][lo] + red[2][hi]) % kMod;
		}
	}
	__syncthreads();
	if (tid == 0) {
		const uint32_t a = (1u + red[1][0]) % kMod, b = (d.raw_len % kMod + red[2][0]) % kMod;
		const uint32_t adler = (b << 16) | a;
		const uint8_t ab[4] = {(uint8_t)(adler >> 24), (uint8_t)(adler >> 16), (uint8_t)(adler >> 8), (uint8_t)adler};
		uint32_t craw = op_apply(d.crc_ops[9], red[0][0]);  // un-pad: Z_-d
		uint32_t ca = 0;
		for (int i = 0; i < 4; i++) ca = crc_byte(tables, ca, ab[i]);
		const uint32_t crc = ~(craw ^ ca ^ d.crc_init);
		uint8_t* f = out + d.out + d.zend - 4u;
		for (int i = 0; i < 4; i++) f[i] = ab[i];
		f[4] = (uint8_t)(crc >> 24), f[5] = (uint8_t)(crc >> 16), f[6] = (uint8_t)(crc >> 8), f[7] = (uint8_t)crc;
	}
}

// ---- host: GF(2) operators of the CRC-32 register -----------------------------------------
struct Op {
	uint32_t c[32];
};
uint32_t op_host_apply(const Op& m, uint32_t v) {
	uint32_t r = 0;
	for (int i = 0; i < 32; i++)
		if ((v >> i) & 1u) r ^= m.c[i];
	return r;
}
Op op_mul(const Op& a, const Op& b) {  // a after b
	Op r;
	for (int i = 0; i < 32; i++) r.c[i] = op_host_apply(a, b.c[i]);
	return r;
}
Op op_zero_byte() {
	Op r;
	for (int i = 0; i < 32; i++) {
		uint32_t c = 1u << i;
		for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
		r.c[i] = c;
	}
	return r;
}
Op op_identity() {
	Op r;
	for (int i = 0; i < 32; i++) r.c[i] = 1u << i;
	return r;
}
Op op_zeros(uint64_t n) {  // Z_n
	Op r = op_identity(), p = op_zero_byte();
	for (; n; n >>= 1, p = op_mul(p, p))
		if (n & 1u) r = op_mul(p, r);
	return r;
}
Op op_inverse(const Op& m) {  // Gauss-Jordan over GF(2); Z_n is invertible (x is a unit mod P)
	uint64_t rows[32];        // row i: [63:32] = row i of m, [31:0] = row i of the identity
	for (int i = 0; i < 32; i++) {
		uint32_t row = 0;
		for (int j = 0; j < 32; j++) row |= ((m.c[j] >> i) & 1u) << j;
		rows[i] = ((uint64_t)row << 32) | (1u << i);
	}
	for (int col = 0; col < 32; col++) {
		int piv = col;
		while (piv < 32 && !((rows[piv] >> (32 + col)) & 1u)) piv++;
		if (piv == 32) return op_identity();  // not reached for Z_n
		std::swap(rows[col], rows[piv]);
		for (int i = 0; i < 32; i++)
			if (i != col && ((rows[i] >> (32 + col)) & 1u)) rows[i] ^= rows[col];
	}
	Op r;
	for (int j = 0; j < 32; j++) {
		uint32_t cj = 0;
		for (int i = 0; i < 32; i++) cj |= (uint32_t)((rows[i] >> j) & 1u) << i;
		r.c[j] = cj;
	}
	return r;
}

void be32(uint8_t* p, uint32_t v) {
	p[0] = (uint8_t)(v >> 24), p[1] = (uint8_t)(v >> 16), p[2] = (uint8_t)(v >> 8), p[3] = (uint8_t)v;
}
uint32_t crc32_host(const uint8_t* p, size_t n) {
	uint32_t c = 0xFFFFFFFFu;
	for (size_t i = 0; i < n; i++) {
		c ^= p[i];
		for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
	}
	return ~c;
}

struct PngOps {
	uint32_t ops[10][32];
	uint32_t init;
};
// operators depend only on (number of spans, zlib end); cached (frames of one size share them)
std::mutex g_ops_mu;
std::map<std::pair<uint32_t, uint32_t>, PngOps> g_ops;

PngOps png_ops(uint32_t G, uint32_t zend) {
	std::lock_guard<std::mutex> lk(g_ops_mu);
	auto it = g_ops.find({G, zend});
	if (it != g_ops.end()) return it->second;
	PngOps o;
	const uint32_t m = (G + kFinThreads - 1u) / kFinThreads;
	Op zs = op_zeros(kSpan);
	memcpy(o.ops[0], zs.c, 128);
	Op zl = op_zeros((uint64_t)kSpan * m);
	for (int l = 0; l < kFinLevels; l++) {
		memcpy(o.ops[1 + l], zl.c, 128);
		zl = op_mul(zl, zl);
	}
	Op unpad = op_inverse(op_zeros((uint64_t)G * kSpan - zend));
	memcpy(o.ops[9], unpad.c, 128);
	o.init = op_host_apply(op_zeros(zend - kCrcStart), 0xFFFFFFFFu);
	if (g_ops.size() > 256) g_ops.clear();
	g_ops[{G, zend}] = o;
	return o;
}

// the 48 KB constant tables, per device, built once
std::mutex g_tab_mu;
uint32_t* g_tab_dev[64];

hipError_t tables_dev(uint32_t** out) {
	int dev = 0;
	hipError_t e = hipGetDevice(&dev);
	if (e != hipSuccess) return e;
	if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
	std::lock_guard<std::mutex> lk(g_tab_mu);
	if (!g_tab_dev[dev]) {
		std::vector<uint32_t> t(kTabWords);
		for (uint32_t b = 0; b < 256; b++) {
			uint32_t c = b;
			for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
			t[b] = c;
		}
		for (int s = 1; s < kSlice; s++)
			for (uint32_t b = 0; b < 256; b++) t[256 * s + b] = (t[256 * (s - 1) + b] >> 8) ^ t[t[256 * (s - 1) + b] & 255u];
		auto put = [&](int base, const Op& z) {
			for (int j = 0; j < 8; j++)
				for (uint32_t v = 0; v < 16; v++) t[base + j * 16 + v] = op_host_apply(z, v << (4 * j));
		};
		for (int l = 0; l < 64; l++) put(kLaneOps + 128 * l, op_zeros((uint64_t)(63 - l) * kPerThread));
		for (int w = 0; w < kWaves; w++) put(kWaveOps + 128 * w, op_zeros((uint64_t)(kWaves - 1 - w) * 64u * kPerThread));
		uint32_t* p = nullptr;
		e = hipMalloc((void**)&p, kTabWords * 4);
		if (e != hipSuccess) return e;
		e = hipMemcpy(p, t.data(), kTabWords * 4, hipMemcpyHostToDevice);
		if (e != hipSuccess) {
			(void)hipFree(p);
			return e;
		}
		g_tab_dev[dev] = p;
	}
	*out = g_tab_dev[dev];
	return hipSuccess;
}

uint64_t file_size(uint32_t format, uint32_t w, uint32_t h, uint32_t* prefix_len, uint32_t* row_bytes, uint64_t* raw) {
	if (w == 0 || h == 0 || w > 65535 || h > 65535) return 0;
	char hdr[64];
	switch (format) {
		case VP8G_ENC_RGB:
			*prefix_len = 0, *row_bytes = 3u * w, *raw = (uint64_t)h * 3u * w;
			return *raw;
		case VP8G_ENC_PPM:
			*prefix_len = (uint32_t)snprintf(hdr, sizeof(hdr), "P6\n%u %u\n255\n", w, h);
			*row_bytes = 3u * w, *raw = (uint64_t)h * 3u * w;
			return *prefix_len + *raw;
		case VP8G_ENC_PNG: {
			*prefix_len = kPngPrefix, *row_bytes = 1u + 3u * w, *raw = (uint64_t)h * (1u + 3u * w);
			const uint64_t blocks = (*raw + kBlk - 1u) / kBlk;
			return kPngPrefix + *raw + 5u * blocks + 4u + 4u + 12u;
		}
		default: return 0;
	}
}


}  // namespace

VP8G_API uint64_t vp8g_encoded_size(uint32_t format, uint32_t width, uint32_t height) {
	uint32_t pl, rb;
	uint64_t raw;
	return file_size(format, width, height, &pl, &rb, &raw);
}

VP8G_API uint64_t vp8g_encode_workspace_size(uint32_t total_spans) { return 16ull * (total_spans ? total_spans : 1u); }

VP8G_API uint32_t vp8g_make_enc_desc(uint32_t width, uint32_t height, uint32_t format, uint64_t src_y, uint64_t src_u,
                                     uint64_t src_v, uint32_t stride_y, uint32_t stride_uv, uint64_t out_offset,
                                     uint32_t span0, Vp8gEncDesc* d) {
	uint32_t pl = 0, rb = 0;
	uint64_t raw = 0;
	const uint64_t flen = d ? file_size(format, width, height, &pl, &rb, &raw) : 0;
	if (!flen || (out_offset & 15u) || stride_y < width || stride_uv < (width + 1u) / 2u) {
		errno = EINVAL;
		return 0;
	}
	if (raw > 0x7FFFFFFFu || flen > 0xFFFFFFFFull - 2 * kSpan) {  // the reference's EFBIG bound (yuv2rgb_png.c:241)
		errno = EFBIG;
		return 0;
	}
	memset(d, 0, sizeof(*d));
	d->width = width, d->height = height, d->stride_y = stride_y, d->stride_uv = stride_uv;
	d->src_y = src_y, d->src_u = src_u, d->src_v = src_v;
	d->out = out_offset, d->file_len = flen;
	d->format = format, d->prefix_len = pl, d->row_bytes = rb, d->raw_len = (uint32_t)raw;
	d->span0 = span0;
	d->nspans = (uint32_t)((flen + kSpan - 1u) / kSpan);
	if (format == VP8G_ENC_PPM) {
		snprintf((char*)d->prefix, sizeof(d->prefix), "P6\n%u %u\n255\n", width, height);
	} else if (format == VP8G_ENC_PNG) {
		static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
		uint8_t* o = d->prefix;
		memcpy(o, sig, 8);
		be32(o + 8, 13), memcpy(o + 12, "IHDR", 4);
		be32(o + 16, width), be32(o + 20, height);
		o[24] = 8, o[25] = 2, o[26] = 0, o[27] = 0, o[28] = 0;  // 8-bit truecolour, no interlace
		be32(o + 29, crc32_host(o + 12, 17));
		const uint64_t zlen = flen - 57u;  // zlib stream: header 2 + blocks + Adler 4 (file: + 41 before, + 16 after)
		be32(o + 33, (uint32_t)zlen), memcpy(o + 37, "IDAT", 4);
		o[41] = 0x78, o[42] = 0x01;
		d->zend = (uint32_t)(flen - 16u);
		const PngOps ops = png_ops(d->nspans, d->zend);
		memcpy(d->crc_ops, ops.ops, sizeof(ops.ops));
		d->crc_init = ops.init;
	}
	return d->nspans;
}

VP8G_API int vp8g_encode_batch_device(const Vp8gEncDesc* h, const Vp8gEncDesc* d_descs, uint32_t n, const uint8_t* d_src,
                                      uint8_t* d_out, uint8_t* d_work, void* stream) {
	if (!h || !d_descs || !d_src || !d_out || !d_work || n == 0) {
		errno = EINVAL;
		return -1;
	}
	uint32_t total = 0;
	bool any_png = false;
	for (uint32_t i = 0; i < n; i++) {
		if (h[i].span0 != total || h[i].nspans == 0) {  // tasks must be numbered image by image
			errno = EINVAL;
			return -1;
		}
		total += h[i].nspans;
		any_png |= h[i].format == VP8G_ENC_PNG;
	}
	uint32_t* tab = nullptr;
	const int cus = vp8g::device_cus();
	hipError_t e = any_png ? tables_dev(&tab) : hipSuccess;
	vp8g::GateScope gate((hipStream_t)stream);  // (vp8g_device.h: no cross-workgroup launch beside these)
	if (e == hipSuccess) e = gate.status();
	if (e == hipSuccess) {
		const uint32_t grid = min(total, (uint32_t)(cus > 0 ? cus : 256) * 16u);
		hipLaunchKernelGGL(enc_write_kernel, dim3(grid), dim3(kPlainThreads), 0, (hipStream_t)stream, d_descs, n, total, d_src,
		                   d_out);
		e = hipGetLastError();
	}
	if (e == hipSuccess && any_png) {
		const uint32_t grid = min(total, (uint32_t)(cus > 0 ? cus : 256) * 4u);
		hipLaunchKernelGGL(crc_kernel, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_descs, n, total, d_out,
		                   (uint32_t*)d_work, tab);
		e = hipGetLastError();
	}
	if (e == hipSuccess && any_png) {
		hipLaunchKernelGGL(png_finish_kernel, dim3(n), dim3(kFinThreads), 0, (hipStream_t)stream, d_descs, (const uint32_t*)d_work,
		                   d_out, tab);
		e = hipGetLastError();
	}
	if (e == hipSuccess) e = gate.done(false);
	if (e != hipSuccess) {
		vp8g::set_error_text("encode launch", e);
		errno = EIO;
		return -1;
	}
	return 0;
}

// ---- the reference's writers: host image -> device -> file bytes -> fd ---------------------
namespace {
struct EncDev {
	std::mutex mu;
	hipStream_t stream = nullptr;
	uint8_t* buf = nullptr;  // source planes | descriptor | workspace | output file
	size_t cap = 0;
	uint8_t* host = nullptr;  // pinned staging for the file bytes
	size_t host_cap = 0;
};
EncDev g_enc;

int write_all(int fd, const uint8_t* p, size_t n) {
	while (n) {
		const ssize_t w = write(fd, p, n);
		if (w < 0) {
			if (errno == EINTR) continue;
			return -1;
		}
		p += w;
		n -= (size_t)w;
	}
	return 0;
}

int write_image(int fd, const Yuv420Image* img, uint32_t format) {
	if (fd < 0 || !img || !img->y || !img->u || !img->v || img->width == 0 || img->height == 0 ||
	    img->stride_y < img->width || img->stride_uv < (img->width + 1u) / 2u) {
		errno = EINVAL;
		return -1;
	}
	const uint32_t w = img->width, h = img->height, cw = (w + 1u) / 2u, ch = (h + 1u) / 2u;
	const uint64_t ysz = (uint64_t)w * h, csz = (uint64_t)cw * ch;
	const uint64_t o_desc = (ysz + 2 * csz + 255u) & ~255ull;
	Vp8gEncDesc desc;
	const uint32_t spans = vp8g_make_enc_desc(w, h, format, 0, ysz, ysz + csz, w, cw, 0, 0, &desc);
	if (!spans) return -1;
	const uint64_t o_work = o_desc + ((sizeof(Vp8gEncDesc) + 255u) & ~255ull);
	const uint64_t o_out = (o_work + vp8g_encode_workspace_size(spans) + 255u) & ~255ull;
	const uint64_t flen = desc.file_len, need = o_out + ((flen + 15u) & ~15ull);
	std::lock_guard<std::mutex> lk(g_enc.mu);
	auto fail = [&](const char* where, hipError_t e) {
		vp8g::set_error_text(where, e);
		errno = EIO;
		return -1;
	};
	hipError_t e = hipSuccess;
	if (!g_enc.stream && (e = hipStreamCreateWithFlags(&g_enc.stream, hipStreamNonBlocking)) != hipSuccess)
		return fail("stream", e);
	if (need > g_enc.cap) {
		if (g_enc.buf) (void)hipFree(g_enc.buf);
		g_enc.buf = nullptr, g_enc.cap = 0;
		if ((e = hipMalloc((void**)&g_enc.buf, need + need / 4)) != hipSuccess) return fail("hipMalloc", e);
		g_enc.cap = need + need / 4;
	}
	if (flen > g_enc.host_cap) {
		if (g_enc.host) (void)hipHostFree(g_enc.host);
		g_enc.host = nullptr, g_enc.host_cap = 0;
		if ((e = hipHostMalloc((void**)&g_enc.host, flen, hipHostMallocDefault)) != hipSuccess) return fail("hipHostMalloc", e);
		g_enc.host_cap = flen;
	}
	hipStream_t s = g_enc.stream;
	uint8_t* b = g_enc.buf;
	desc.out = o_out;  // (the source offsets are relative to b, and so is the output)
	if ((e = hipMemcpy2DAsync(b, w, img->y, img->stride_y, w, h, hipMemcpyHostToDevice, s)) != hipSuccess ||
	    (e = hipMemcpy2DAsync(b + ysz, cw, img->u, img->stride_uv, cw, ch, hipMemcpyHostToDevice, s)) != hipSuccess ||
	    (e = hipMemcpy2DAsync(b + ysz + csz, cw, img->v, img->stride_uv, cw, ch, hipMemcpyHostToDevice, s)) != hipSuccess ||
	    (e = hipMemcpyAsync(b + o_desc, &desc, sizeof(desc), hipMemcpyHostToDevice, s)) != hipSuccess)
		return fail("H2D", e);
	if (vp8g_encode_batch_device(&desc, (const Vp8gEncDesc*)(b + o_desc), 1, b, b, b + o_work, s) != 0) return -1;
	if ((e = hipMemcpyAsync(g_enc.host, b + o_out, flen, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail("D2H", e);
	if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail("sync", e);
	return write_all(fd, g_enc.host, flen);
}
}  // namespace

VP8G_API int yuv420_write_ppm_fd(int fd, const Yuv420Image* img) { return write_image(fd, img, VP8G_ENC_PPM); }

VP8G_API int yuv420_write_png_fd(int fd, const Yuv420Image* img) { return write_image(fd, img, VP8G_ENC_PNG); }
