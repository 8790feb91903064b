/*
 * libwebp_probe.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The reference's own gates compare against libwebp's `dwebp -yuv [-nofilter]`
 * (reference scripts/m6_compare_yuv_with_dwebp.sh:56, scripts/m7_compare_yuv_filtered_with_oracle.sh:54).
 * The dwebp binary is absent from this image but the system libwebp (1.2.2) library is present,
 * so this probe reproduces `dwebp -quiet -yuv [-nofilter] in -o out` with the library API:
 * MODE_YUV output, bypass_filtering for -nofilter, rows cropped to w and ceil(w/2).
 * `-rgb` instead writes libwebp's RGB24 rows (MODE_RGB, default fancy upsampling): the payload
 * of `dwebp -ppm` (reference scripts/m8_compare_ppm_with_dwebp.sh compares -ppm files byte for byte).
 * Used only by tests/golden/make_manifest.py to cross-check the golden manifest.
 *
 *   libwebp_probe [-nofilter | -rgb] in.webp out
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <webp/decode.h>

int main(int argc, char** argv) {
	int nofilter = 0, rgb = 0, a = 1;
	if (argc > 1 && !strcmp(argv[1], "-nofilter")) nofilter = 1, a = 2;
	if (argc > 1 && !strcmp(argv[1], "-rgb")) rgb = 1, a = 2;
	if (argc - a != 2) {
		fprintf(stderr, "usage: libwebp_probe [-nofilter | -rgb] in.webp out\n");
		return 2;
	}
	FILE* fp = fopen(argv[a], "rb");
	if (!fp) return 1;
	fseek(fp, 0, SEEK_END);
	long n = ftell(fp);
	fseek(fp, 0, SEEK_SET);
	uint8_t* data = (uint8_t*)malloc((size_t)n);
	if (!data || fread(data, 1, (size_t)n, fp) != (size_t)n) return 1;
	fclose(fp);
	WebPDecoderConfig cfg;
	if (!WebPInitDecoderConfig(&cfg)) return 1;
	cfg.output.colorspace = rgb ? MODE_RGB : MODE_YUV;
	cfg.options.bypass_filtering = nofilter;
	if (WebPDecode(data, (size_t)n, &cfg) != VP8_STATUS_OK) return 1;
	if (rgb) {
		const WebPRGBABuffer* c = &cfg.output.u.RGBA;
		FILE* out = fopen(argv[a + 1], "wb");
		if (!out) return 1;
		for (int y = 0; y < cfg.output.height; y++) fwrite(c->rgba + (size_t)y * c->stride, 1, (size_t)cfg.output.width * 3, out);
		fclose(out);
		WebPFreeDecBuffer(&cfg.output);
		free(data);
		return 0;
	}
	const WebPYUVABuffer* b = &cfg.output.u.YUVA;
	int w = cfg.output.width, h = cfg.output.height, cw = (w + 1) / 2, ch = (h + 1) / 2;
	FILE* out = fopen(argv[a + 1], "wb");
	if (!out) return 1;
	for (int y = 0; y < h; y++) fwrite(b->y + (size_t)y * b->y_stride, 1, (size_t)w, out);
	for (int y = 0; y < ch; y++) fwrite(b->u + (size_t)y * b->u_stride, 1, (size_t)cw, out);
	for (int y = 0; y < ch; y++) fwrite(b->v + (size_t)y * b->v_stride, 1, (size_t)cw, out);
	fclose(out);
	WebPFreeDecBuffer(&cfg.output);
	free(data);
	return 0;
}
