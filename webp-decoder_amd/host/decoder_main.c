/*
 * decoder_main.c -- the `decoder` CLI (C11 host), drop-in for the reference's -yuv / -yuvf
 * subcommands (reference src/main.c:556-628, :630-702, argv dispatch :1021-1071):
 *
 *   decoder -info <file.webp>
 *   decoder -yuv  <file.webp> <out.i420>    recon only            (m06 on the GPU)
 *   decoder -yuvf <file.webp> <out.i420>    recon + loop filter   (m06 + m07 on the GPU)
 *   decoder -ppm  <file.webp> <out.ppm>     recon + loop filter + RGB (m08 writer, on the GPU)
 *   decoder -png  <file.webp> <out.png>     recon + loop filter + RGB (m09 writer, on the GPU)
 *   decoder -diff_mb <file.webp> <oracle.i420>   per-macroblock SAD of our -yuv vs a file
 *
 * Output (-yuv/-yuvf): raw I420, Y (w*h) then U then V (each ceil(w/2)*ceil(h/2)), no header;
 * -ppm / -png: the files of yuv420_write_ppm_fd / yuv420_write_png_fd (reference src/main.c:706-844).
 * Exit codes: 0 ok, 1 failure (message on stderr), 2 usage.
 * The host front end (container, header, token decode) runs on the CPU; reconstruction goes
 * through libvp8g.so's reference entry points (vp8_reconstruct_keyframe_yuv[_filtered]).
 */
#include <errno.h>
#include <fcntl.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "vp8_front.h"

static void usage(void) {
	fputs("Usage:\n", stderr);
	fputs("  decoder -info <file.webp>\n", stderr);
	fputs("  decoder -yuv <file.webp> <out.i420>\n", stderr);
	fputs("  decoder -yuvf <file.webp> <out.i420>\n", stderr);
	fputs("  decoder -ppm <file.webp> <out.ppm>\n", stderr);
	fputs("  decoder -png <file.webp> <out.png>\n", stderr);
	fputs("  decoder -diff_mb <file.webp> <oracle.i420>\n", stderr);
}

static int write_all(int fd, const uint8_t* p, size_t n) {
	while (n) {
		ssize_t w = write(fd, p, n);
		if (w < 0) {
			if (errno == EINTR) continue;
			return -1;
		}
		p += w;
		n -= (size_t)w;
	}
	return 0;
}

static int front(const char* path, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* d) {
	int stage = 0;
	if (vp8f_decode_file(path, kf, d, &stage) == 0) return 0;
	switch (stage) {
		case 1: fputs("error: cannot open/map file\n", stderr); break;
		case 2: fputs("error: not a supported simple lossy WebP (RIFF/WEBP + single VP8 chunk)\n", stderr); break;
		case 3: fputs("error: VP8 key-frame header parse failed\n", stderr); break;
		default: fputs("error: VP8 macroblock/token decode failed\n", stderr); break;
	}
	return -1;
}

static int cmd_yuv(const char* in, const char* out_path, int filtered) {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame d;
	if (front(in, &kf, &d) != 0) return 1;
	Yuv420Image img;
	int rc = filtered ? vp8_reconstruct_keyframe_yuv_filtered(&kf, &d, &img) : vp8_reconstruct_keyframe_yuv(&kf, &d, &img);
	vp8_decoded_frame_free(&d);
	if (rc != 0) {
		fputs(filtered ? "error: VP8 reconstruction/loopfilter failed\n" : "error: VP8 reconstruction failed\n", stderr);
		const char* he = vp8g_last_error();
		if (he && *he) fprintf(stderr, "  (%s)\n", he);
		return 1;
	}
	int fd = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
	if (fd < 0) {
		fputs("error: cannot open output file\n", stderr);
		yuv420_free(&img);
		return 1;
	}
	const size_t ysz = (size_t)img.stride_y * img.height;
	const size_t uvsz = (size_t)img.stride_uv * ((img.height + 1u) / 2u);
	int w = write_all(fd, img.y, ysz) | write_all(fd, img.u, uvsz) | write_all(fd, img.v, uvsz);
	close(fd);
	yuv420_free(&img);
	if (w != 0) {
		fputs("error: write failed\n", stderr);
		return 1;
	}
	return 0;
}

/* reference src/main.c:706-773 (-ppm) and :775-844 (-png): filtered reconstruction, then the
 * m08 / m09 writer into the output file */
static int cmd_rgb(const char* in, const char* out_path, int png) {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame d;
	if (front(in, &kf, &d) != 0) return 1;
	Yuv420Image img;
	int rc = vp8_reconstruct_keyframe_yuv_filtered(&kf, &d, &img);
	vp8_decoded_frame_free(&d);
	if (rc != 0) {
		fputs("error: VP8 reconstruction/loopfilter failed\n", stderr);
		const char* he = vp8g_last_error();
		if (he && *he) fprintf(stderr, "  (%s)\n", he);
		return 1;
	}
	int fd = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
	if (fd < 0) {
		fputs("error: cannot open output file\n", stderr);
		yuv420_free(&img);
		return 1;
	}
	int wrc = png ? yuv420_write_png_fd(fd, &img) : yuv420_write_ppm_fd(fd, &img);
	close(fd);
	yuv420_free(&img);
	if (wrc != 0) {
		fputs(png ? "error: PNG write failed\n" : "error: PPM write failed\n", stderr);
		return 1;
	}
	return 0;
}

static int cmd_info(const char* in) {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame d;
	if (front(in, &kf, &d) != 0) return 1;
	const Vp8CoeffStats* s = &d.stats;
	printf("Frame: %ux%u  MBs: %ux%u\n", kf.width, kf.height, d.mb_cols, d.mb_rows);
	printf("  Quant: q_index=%u  Segmentation: %s%s\n", d.q_index, d.segmentation_enabled ? "on" : "off",
	       d.segmentation_enabled ? (d.segmentation_abs ? " (abs)" : " (delta)") : "");
	printf("  Loop filter: %s level=%u sharpness=%u deltas=%s\n", d.lf_use_simple ? "simple" : "normal", d.lf_level,
	       d.lf_sharpness, d.lf_delta_enabled ? "on" : "off");
	printf("  Modes: DC=%u V=%u H=%u TM=%u B=%u\n", s->ymode_counts[0], s->ymode_counts[1], s->ymode_counts[2],
	       s->ymode_counts[3], s->ymode_counts[4]);
	printf("  Nonzero coeffs: %u  abs max: %u\n", s->coeff_nonzero_total, s->coeff_abs_max);
	printf("  Coeff hash:       0x%016" PRIx64 "\n", s->coeff_hash_fnv1a64);
	vp8_decoded_frame_free(&d);
	return 0;
}

/* per-MB SAD of our unfiltered recon against an I420 file (reference src/main.c:846-1017) */
static int cmd_diff_mb(const char* in, const char* oracle_path) {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame d;
	if (front(in, &kf, &d) != 0) return 1;
	Yuv420Image img;
	if (vp8_reconstruct_keyframe_yuv(&kf, &d, &img) != 0) {
		fputs("error: VP8 reconstruction failed\n", stderr);
		vp8_decoded_frame_free(&d);
		return 1;
	}
	FILE* fp = fopen(oracle_path, "rb");
	const size_t ysz = (size_t)img.stride_y * img.height, uvsz = (size_t)img.stride_uv * ((img.height + 1u) / 2u);
	uint8_t* o = (uint8_t*)malloc(ysz + 2 * uvsz + 1);
	size_t got = (fp && o) ? fread(o, 1, ysz + 2 * uvsz + 1, fp) : 0;
	if (fp) fclose(fp);
	if (got != ysz + 2 * uvsz) {
		fputs("error: oracle size mismatch\n", stderr);
		free(o);
		yuv420_free(&img);
		vp8_decoded_frame_free(&d);
		return 1;
	}
	uint32_t bad = 0;
	for (uint32_t r = 0; r < d.mb_rows; r++) {
		for (uint32_t c = 0; c < d.mb_cols; c++) {
			uint64_t sad[3] = {0, 0, 0};
			for (uint32_t yy = r * 16; yy < r * 16 + 16 && yy < img.height; yy++)
				for (uint32_t xx = c * 16; xx < c * 16 + 16 && xx < img.width; xx++)
					sad[0] += (uint64_t)abs((int)img.y[yy * img.stride_y + xx] - (int)o[yy * img.stride_y + xx]);
			for (uint32_t yy = r * 8; yy < r * 8 + 8 && yy < (img.height + 1) / 2; yy++)
				for (uint32_t xx = c * 8; xx < c * 8 + 8 && xx < img.stride_uv; xx++) {
					size_t k = (size_t)yy * img.stride_uv + xx;
					sad[1] += (uint64_t)abs((int)img.u[k] - (int)o[ysz + k]);
					sad[2] += (uint64_t)abs((int)img.v[k] - (int)o[ysz + uvsz + k]);
				}
			if (sad[0] | sad[1] | sad[2]) {
				uint32_t mb = r * d.mb_cols + c;
				if (bad < 20)
					printf("MB %u (r=%u c=%u) ymode=%u uv=%u seg=%u  SAD Y=%" PRIu64 " U=%" PRIu64 " V=%" PRIu64 "\n", mb, r, c,
					       d.ymode[mb], d.uv_mode[mb], d.segment_id[mb], sad[0], sad[1], sad[2]);
				bad++;
			}
		}
	}
	printf("mismatching macroblocks: %u of %u\n", bad, d.mb_total);
	free(o);
	yuv420_free(&img);
	vp8_decoded_frame_free(&d);
	return bad ? 1 : 0;
}

int main(int argc, char** argv) {
	if (argc < 3) {
		usage();
		return 2;
	}
	const char* cmd = argv[1];
	if (!strcmp(cmd, "-info")) {
		if (argc != 3) {
			usage();
			return 2;
		}
		return cmd_info(argv[2]);
	}
	if (!strcmp(cmd, "-yuv") || !strcmp(cmd, "-yuvf")) {
		if (argc != 4) {
			usage();
			return 2;
		}
		return cmd_yuv(argv[2], argv[3], cmd[4] == 'f');
	}
	if (!strcmp(cmd, "-ppm") || !strcmp(cmd, "-png")) {
		if (argc != 4) {
			usage();
			return 2;
		}
		return cmd_rgb(argv[2], argv[3], cmd[2] == 'n');
	}
	if (!strcmp(cmd, "-diff_mb")) {
		if (argc != 4) {
			usage();
			return 2;
		}
		return cmd_diff_mb(argv[2], argv[3]);
	}
	usage();
	return 2;
}
