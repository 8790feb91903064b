/*
 * vp8_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path (src/m06_recon/vp8_recon.c + src/m07_loopfilter/
 * vp8_loopfilter.c) and of the next stage, m08/m09 (YUV->RGB, PPM/PNG writers), used as the parity checker by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  The product path (libvp8g.so) never links or calls it.
 *
 * Pinned by: tests/golden/manifest.json (sha256 of the reference decoder's own -yuv/-yuvf output
 * on every corpus file, generated from the reference compiled here, cross-checked with libwebp
 * 1.2.2) and tests/golden/synth_kat.json (reference m06/m07 output hashes on seeded synthetic
 * frames) -- see tests/test_oracle.py.
 */
#ifndef VP8_ORACLE_H
#define VP8_ORACLE_H

#include "../include/vp8g.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Padded (macroblock-aligned) reconstruction, optionally loop-filtered, into caller planes of
 * size (mb_cols*16) x (mb_rows*16) and (mb_cols*8) x (mb_rows*8). */
int oracle_recon_padded(const Vp8DecodedFrame* d, uint8_t* y, uint8_t* u, uint8_t* v, int filtered);

/* m07 alone, in place on a padded image (stride = width). */
int oracle_loopfilter(uint8_t* y, uint8_t* u, uint8_t* v, const Vp8DecodedFrame* d);

/* Full m06(+m07) with crop into a malloc()ed cropped I420 image (free with oracle_image_free). */
int oracle_reconstruct(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, Yuv420Image* out, int filtered);
void oracle_image_free(Yuv420Image* img);

/* Cropped I420 bytes written back to back (Y, U, V), as `decoder -yuv/-yuvf` writes them.
 * buf must hold w*h + 2*ceil(w/2)*ceil(h/2) bytes. */
int oracle_reconstruct_i420(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, uint8_t* buf, int filtered);

/* CPU baseline: reconstruct `n` frames (frames[i % nframes]) with `threads` pthreads, one frame
 * per task; returns elapsed seconds (wall), or < 0 on error. */
double oracle_time_batch(const Vp8KeyFrameHeader* const* kfs, const Vp8DecodedFrame* const* frames, int nframes, int n,
                         int threads, int filtered);

/* m08 / m09 (reference src/m08_yuv2rgb_ppm/yuv2rgb_ppm.c, src/m09_png/yuv2rgb_png.c): one RGB24
 * row of the fancy-upsampled conversion, and the complete PPM / PNG files the reference's
 * yuv420_write_ppm_fd / yuv420_write_png_fd emit, written to memory (byte count, or -1). */
void oracle_rgb_row(const Yuv420Image* img, uint32_t y, uint8_t* dst);
size_t oracle_ppm_size(uint32_t w, uint32_t h);
size_t oracle_png_size(uint32_t w, uint32_t h);
long oracle_ppm(const Yuv420Image* img, uint8_t* out, size_t cap);
long oracle_png(const Yuv420Image* img, uint8_t* out, size_t cap);

#ifdef __cplusplus
}
#endif

#endif
