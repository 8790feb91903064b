/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin C entry points around the REFERENCE decoder's own modules, compiled (by oracle/Makefile)
 * together with the reference sources where they lie under /root/reference into
 * oracle/_ref/libref.so.  Nothing from the reference is copied into this repository; this file
 * only calls the reference's public functions:
 *   webp_parse_simple_lossy (src/m01_container/webp_container.c:19)
 *   vp8_parse_keyframe_header (src/m02_vp8_header/vp8_header.c:13)
 *   vp8_decode_decoded_frame / vp8_decoded_frame_free (src/m05_tokens/vp8_tokens.c:673, :658)
 *   vp8_reconstruct_keyframe_yuv[_filtered] (src/m06_recon/vp8_recon.c:714, :718)
 *   vp8_loopfilter_apply_keyframe (src/m07_loopfilter/vp8_loopfilter.c:201)
 * Used to (1) generate the golden manifests, (2) pin the oracle and the host front end, and
 * (3) serve as the "reference" CPU baseline in bench.py.
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "m01_container/webp_container.h"
#include "m02_vp8_header/vp8_header.h"
#include "m05_tokens/vp8_tokens.h"
#include "m06_recon/vp8_recon.h"
#include "m07_loopfilter/vp8_loopfilter.h"

static uint8_t* slurp(const char* path, size_t* n) {
	FILE* fp = fopen(path, "rb");
	if (!fp) return NULL;
	fseek(fp, 0, SEEK_END);
	long sz = ftell(fp);
	fseek(fp, 0, SEEK_SET);
	uint8_t* buf = (uint8_t*)malloc(sz > 0 ? (size_t)sz : 1);
	if (buf && sz > 0 && fread(buf, 1, (size_t)sz, fp) != (size_t)sz) {
		free(buf);
		buf = NULL;
	}
	fclose(fp);
	*n = sz > 0 ? (size_t)sz : 0;
	return buf;
}

/* Decode a .webp with the reference front end.  Returns 0 or a stage code 1..4 on failure. */
int ref_decode_frame(const char* path, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* d) {
	size_t n = 0;
	uint8_t* buf = slurp(path, &n);
	if (!buf) return 1;
	ByteSpan file = {buf, n};
	WebPContainer c;
	int rc = 0;
	if (webp_parse_simple_lossy(file, &c) != 0) rc = 2;
	else {
		ByteSpan p = {buf + c.vp8_chunk_offset, c.vp8_chunk_size};
		if (vp8_parse_keyframe_header(p, kf) != 0 || !kf->is_key_frame) rc = 3;
		else if (vp8_decode_decoded_frame(p, d) != 0) rc = 4;
	}
	free(buf);
	return rc;
}

void ref_free_frame(Vp8DecodedFrame* d) { vp8_decoded_frame_free(d); }

static size_t i420_size(uint32_t w, uint32_t h) { return (size_t)w * h + 2 * (size_t)((w + 1) / 2) * ((h + 1) / 2); }

static void write_i420(const Yuv420Image* img, uint8_t* out) {
	size_t ysz = (size_t)img->stride_y * img->height, uvsz = (size_t)img->stride_uv * ((img->height + 1) / 2);
	memcpy(out, img->y, ysz);
	memcpy(out + ysz, img->u, uvsz);
	memcpy(out + ysz + uvsz, img->v, uvsz);
}

/* Reference m06(+m07) on a caller-provided decoded frame; cropped I420 into buf. */
int ref_recon_i420(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* d, uint8_t* buf, int filtered) {
	Yuv420Image img;
	int rc = filtered ? vp8_reconstruct_keyframe_yuv_filtered(kf, d, &img) : vp8_reconstruct_keyframe_yuv(kf, d, &img);
	if (rc != 0) return -1;
	write_i420(&img, buf);
	yuv420_free(&img);
	return 0;
}

/* Reference m07 alone on a padded frame held as three planes (stride = width). */
int ref_loopfilter_padded(uint8_t* y, uint8_t* u, uint8_t* v, uint32_t w, uint32_t h, const Vp8DecodedFrame* d) {
	Yuv420Image img = {w, h, w, (w + 1) / 2, y, u, v};
	return vp8_loopfilter_apply_keyframe(&img, d);
}

/* Whole reference decoder path for a file: what `decoder -yuv[f] in out` writes.  Returns the
 * number of bytes written, or -stage on failure.  buf may be NULL to query the size. */
long ref_decode_i420(const char* path, uint8_t* buf, size_t cap, int filtered) {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame d;
	int st = ref_decode_frame(path, &kf, &d);
	if (st) return -st;
	size_t need = i420_size(kf.width, kf.height);
	long rc = (long)need;
	if (buf) {
		if (cap < need || ref_recon_i420(&kf, &d, buf, filtered) != 0) rc = -5;
	}
	vp8_decoded_frame_free(&d);
	return rc;
}

uint64_t ref_coeff_hash(const char* path) {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame d;
	if (ref_decode_frame(path, &kf, &d)) return 0;
	uint64_t h = d.stats.coeff_hash_fnv1a64;
	vp8_decoded_frame_free(&d);
	return h;
}

/* ---- CPU baseline: reference m06+m07 on pre-decoded frames, one frame per task ---- */
typedef struct {
	const Vp8KeyFrameHeader* const* kfs;
	const Vp8DecodedFrame* const* frames;
	int nframes, n, filtered, next, err;
	pthread_mutex_t mu;
} RefJob;

static void* ref_worker(void* arg) {
	RefJob* j = (RefJob*)arg;
	for (;;) {
		pthread_mutex_lock(&j->mu);
		int i = j->next++;
		pthread_mutex_unlock(&j->mu);
		if (i >= j->n) break;
		Yuv420Image img;
		const Vp8KeyFrameHeader* kf = j->kfs[i % j->nframes];
		const Vp8DecodedFrame* d = j->frames[i % j->nframes];
		int rc = j->filtered ? vp8_reconstruct_keyframe_yuv_filtered(kf, d, &img) : vp8_reconstruct_keyframe_yuv(kf, d, &img);
		if (rc != 0) j->err = 1;
		else yuv420_free(&img);
	}
	return NULL;
}

double ref_time_batch(const Vp8KeyFrameHeader* const* kfs, const Vp8DecodedFrame* const* frames, int nframes, int n,
                      int threads, int filtered) {
	if (!kfs || !frames || nframes <= 0 || n <= 0 || threads <= 0 || threads > 1024) return -1.0;
	RefJob j = {kfs, frames, nframes, n, filtered, 0, 0, PTHREAD_MUTEX_INITIALIZER};
	pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
	if (!th) return -1.0;
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	int started = 0;
	for (int i = 0; i < threads; i++)
		if (pthread_create(&th[i], NULL, ref_worker, &j) == 0) started++;
	for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	free(th);
	if (j.err || !started) return -1.0;
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
