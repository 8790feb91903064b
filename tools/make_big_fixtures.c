/*
 * make_big_fixtures.c -- generate the large lossy-WebP fixtures (tests/fixtures/big/) with the
 * system libwebp 1.2.2 encoder.  The reference corpus has no frame above 960x1162, only the
 * normal filter, sharpness 0 and no filter deltas, so these fill those gaps:
 * 1920x1080 and 3840x2160 frames, simple and normal filter, sharpness 0..7, 1 or 4 segments.
 *
 * Picture content: natural-image statistics taken from the reference's own penguin photo
 * (images/commons/penguin-q80.webp, decoded with libwebp), mirrored/tiled to the target size
 * with a per-variant offset, plus a smooth gradient overlay so variants differ.
 *
 *   make_big_fixtures <penguin.webp> <out_dir> [name,name,...]   (only the named variants)
 * Build: gcc -O2 -I/opt/conda/include tools/make_big_fixtures.c /usr/lib/x86_64-linux-gnu/libwebp.so.7
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <webp/decode.h>
#include <webp/encode.h>

typedef struct {
	const char* name;
	int w, h;
	int simple;    /* filter_type 0 = simple, 1 = normal ("strong") */
	int strength;  /* 0..100 */
	int sharpness; /* 0..7 */
	int segments;  /* 1..4 */
	float quality;
	int ox, oy; /* content offset */
	int partitions; /* log2 of the token partition count (libwebp WebPConfig.partitions, 0..3) */
} Variant;

static const Variant kVariants[] = {
    {"k128_normal", 128, 128, 0 + 0, 60, 0, 4, 75.f, 900, 1100},
    {"fhd_normal_sharp5", 1920, 1080, 0, 60, 5, 4, 75.f, 0, 0},
    {"fhd_simple_sharp3", 1920, 1080, 1, 50, 3, 4, 70.f, 200, 300},
    {"uhd_a_normal_seg4", 3840, 2160, 0, 60, 0, 4, 75.f, 0, 0},
    {"uhd_b_simple_sharp3", 3840, 2160, 1, 45, 3, 4, 75.f, 500, 700},
    {"uhd_c_normal_sharp6_seg1", 3840, 2160, 0, 80, 6, 1, 60.f, 1000, 200},
    {"uhd_d_normal_q90", 3840, 2160, 0, 30, 2, 4, 90.f, 1500, 1600},
    {"odd_1917x1083_normal", 1917, 1083, 0, 70, 1, 4, 50.f, 300, 900},
    /* round 2: two more 1080p frames for the 1080p batch (bench --workload fhd4) */
    {"fhd_c_normal_q85_seg4", 1920, 1080, 0, 40, 0, 4, 85.f, 700, 500},
    {"fhd_d_normal_sharp2_seg1", 1920, 1080, 0, 70, 2, 1, 60.f, 1300, 100},
    /* multi-partition token streams (2/4/8 partitions; the reference rejects them, ENOTSUP at
     * src/m05_tokens/vp8_tokens.c:357-360): tests/fixtures_mp/, pinned by libwebp's decode */
    {"mp2_fhd_normal", 1920, 1080, 0, 60, 0, 4, 75.f, 100, 200, 1},
    {"mp4_fhd_simple_sharp3", 1920, 1080, 1, 50, 3, 4, 70.f, 400, 50, 2},
    {"mp8_fhd_normal_seg1", 1920, 1080, 0, 55, 4, 1, 80.f, 900, 600, 3},
    {"mp2_uhd_normal_seg4", 3840, 2160, 0, 60, 0, 4, 75.f, 250, 350, 1},
    {"mp4_uhd_normal_q90", 3840, 2160, 0, 30, 2, 4, 90.f, 1200, 1400, 2},
    {"mp8_uhd_simple", 3840, 2160, 1, 45, 1, 4, 75.f, 600, 800, 3},
    {"mp8_odd_333x197_normal", 333, 197, 0, 70, 1, 4, 50.f, 30, 90, 3},
};

static int mirror(int v, int n) {
	int p = 2 * n;
	v %= p;
	if (v < 0) v += p;
	return v < n ? v : p - 1 - v;
}

int main(int argc, char** argv) {
	if (argc != 3 && argc != 4) {
		fprintf(stderr, "usage: make_big_fixtures <penguin.webp> <out_dir> [name,name,...]\n");
		return 2;
	}
	FILE* fp = fopen(argv[1], "rb");
	if (!fp) return 1;
	fseek(fp, 0, SEEK_END);
	long n = ftell(fp);
	fseek(fp, 0, SEEK_SET);
	uint8_t* data = malloc((size_t)n);
	if (fread(data, 1, (size_t)n, fp) != (size_t)n) return 1;
	fclose(fp);
	int sw = 0, sh = 0;
	uint8_t* src = WebPDecodeRGB(data, (size_t)n, &sw, &sh);
	if (!src) return 1;
	for (size_t vi = 0; vi < sizeof(kVariants) / sizeof(kVariants[0]); vi++) {
		const Variant* v = &kVariants[vi];
		if (argc == 4) { /* only the named variants */
			char want[1024];
			snprintf(want, sizeof(want), ",%s,", argv[3]);
			char key[128];
			snprintf(key, sizeof(key), ",%s,", v->name);
			if (!strstr(want, key)) continue;
		}
		uint8_t* rgb = malloc((size_t)v->w * v->h * 3);
		for (int y = 0; y < v->h; y++) {
			for (int x = 0; x < v->w; x++) {
				const uint8_t* s = src + ((size_t)mirror(y + v->oy, sh) * sw + mirror(x + v->ox, sw)) * 3;
				uint8_t* d = rgb + ((size_t)y * v->w + x) * 3;
				int g = (x * 37 / (v->w + 1) + y * 23 / (v->h + 1)) - 30;
				for (int c = 0; c < 3; c++) {
					int val = s[c] + g * (c + 1) / 3;
					d[c] = (uint8_t)(val < 0 ? 0 : val > 255 ? 255 : val);
				}
			}
		}
		WebPConfig cfg;
		WebPPicture pic;
		WebPMemoryWriter wr;
		if (!WebPConfigInit(&cfg) || !WebPPictureInit(&pic)) return 1;
		cfg.quality = v->quality;
		cfg.method = 4;
		cfg.filter_type = v->simple ? 0 : 1;
		cfg.filter_strength = v->strength;
		cfg.filter_sharpness = v->sharpness;
		cfg.segments = v->segments;
		cfg.partitions = v->partitions;
		/* libwebp 1.2.2 writes one partition whatever `partitions` says on its token-buffer path
		 * (method >= 3 without low_memory); low_memory selects the path that honours it */
		cfg.low_memory = v->partitions > 0;
		cfg.autofilter = 0;
		if (!WebPValidateConfig(&cfg)) return 1;
		pic.width = v->w;
		pic.height = v->h;
		if (!WebPPictureImportRGB(&pic, rgb, v->w * 3)) return 1;
		WebPMemoryWriterInit(&wr);
		pic.writer = WebPMemoryWrite;
		pic.custom_ptr = &wr;
		if (!WebPEncode(&cfg, &pic)) {
			fprintf(stderr, "encode failed %s\n", v->name);
			return 1;
		}
		char path[1024];
		snprintf(path, sizeof(path), "%s/%s.webp", argv[2], v->name);
		FILE* o = fopen(path, "wb");
		fwrite(wr.mem, 1, wr.size, o);
		fclose(o);
		printf("%s %dx%d %zu bytes\n", path, v->w, v->h, wr.size);
		WebPMemoryWriterClear(&wr);
		WebPPictureFree(&pic);
		free(rgb);
	}
	WebPFree(src);
	free(data);
	return 0;
}
