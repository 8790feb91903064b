/*
 * webp_riff.c -- RIFF/WEBP container (RFC 9649 simple lossy layout) and the VP8 frame tag /
 * key-frame header (RFC 6386 9.1), with the reference's acceptance rules:
 *   container: 'RIFF' <size> 'WEBP' then exactly one 'VP8 ' chunk, RIFF size + 8 == file size,
 *              nothing after the (even-padded) chunk  (reference src/m01_container/webp_container.c:19-89)
 *   header:    key frame, start code 9d 01 2a, 14-bit non-zero width/height, first partition
 *              fits in the payload  (reference src/m02_vp8_header/vp8_header.c:13-66)
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vp8_front.h"

static uint32_t rd_le32(const uint8_t* p) {
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

int webp_parse_simple_lossy(ByteSpan file, WebPContainer* out) {
	if (!out) return -1;
	memset(out, 0, sizeof(*out));
	out->actual_size = file.size;
	if (!file.data || file.size < 12 || memcmp(file.data, "RIFF", 4) != 0) {
		errno = EINVAL;
		return -1;
	}
	out->riff_size = rd_le32(file.data + 4);
	if (memcmp(file.data + 8, "WEBP", 4) != 0 || (size_t)out->riff_size + 8u != file.size || file.size < 20) {
		errno = EINVAL;
		return -1;
	}
	const uint8_t* chunk = file.data + 12;
	const uint32_t csize = rd_le32(chunk + 4);
	if (memcmp(chunk, "VP8 ", 4) != 0 || csize > file.size - 20) {
		errno = EINVAL;
		return -1;
	}
	size_t end = 20u + (size_t)csize;
	end += end & 1u; /* chunks are padded to even length */
	if (end != file.size) {
		errno = EINVAL;
		return -1;
	}
	out->vp8_chunk_offset = 20;
	out->vp8_chunk_size = csize;
	return 0;
}

int vp8_parse_keyframe_header(ByteSpan p, Vp8KeyFrameHeader* out) {
	if (!out) return -1;
	memset(out, 0, sizeof(*out));
	if (!p.data || p.size < 10) {
		errno = EINVAL;
		return -1;
	}
	const uint32_t tag = (uint32_t)p.data[0] | ((uint32_t)p.data[1] << 8) | ((uint32_t)p.data[2] << 16);
	out->is_key_frame = (tag & 1u) == 0;
	out->profile = (uint8_t)((tag >> 1) & 7u);
	out->show_frame = (int)((tag >> 4) & 1u);
	out->first_partition_len = tag >> 5;
	if (!out->is_key_frame) {
		errno = EINVAL;
		return -1;
	}
	out->start_code_ok = p.data[3] == 0x9d && p.data[4] == 0x01 && p.data[5] == 0x2a;
	if (!out->start_code_ok) {
		errno = EINVAL;
		return -1;
	}
	const uint16_t w = (uint16_t)(p.data[6] | (p.data[7] << 8));
	const uint16_t h = (uint16_t)(p.data[8] | (p.data[9] << 8));
	out->width = w & 0x3FFF;
	out->x_scale = (uint8_t)(w >> 14);
	out->height = h & 0x3FFF;
	out->y_scale = (uint8_t)(h >> 14);
	if (out->width == 0 || out->height == 0 || out->first_partition_len > p.size - 10) {
		errno = EINVAL;
		return -1;
	}
	return 0;
}

int vp8f_decode_memory(const uint8_t* data, size_t size, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* out, int* stage) {
	int st = 0;
	WebPContainer c;
	ByteSpan file = {data, size};
	int rc = -1;
	if (webp_parse_simple_lossy(file, &c) != 0) {
		st = 2;
		goto out;
	}
	ByteSpan payload = {data + c.vp8_chunk_offset, c.vp8_chunk_size};
	if (vp8_parse_keyframe_header(payload, kf) != 0 || !kf->is_key_frame) {
		st = 3;
		goto out;
	}
	if (vp8_decode_decoded_frame(payload, out) != 0) {
		st = 4;
		goto out;
	}
	rc = 0;
out:
	if (stage) *stage = st;
	return rc;
}

int vp8f_decode_packed_memory(const uint8_t* data, size_t size, Vp8gPackedFrame* out, int* stage, unsigned flags) {
	int st = 0, rc = -1;
	WebPContainer c;
	ByteSpan file = {data, size};
	if (out) memset(out, 0, sizeof(*out));
	if (!out) {
		errno = EINVAL;
		st = 4;
	} else if (webp_parse_simple_lossy(file, &c) != 0) {
		st = 2;
	} else {
		ByteSpan payload = {data + c.vp8_chunk_offset, c.vp8_chunk_size};
		if (vp8_parse_keyframe_header(payload, &out->kf) != 0 || !out->kf.is_key_frame) st = 3;
		else if (vp8f_decode_packed(payload, out, flags) != 0) st = 4;
		else rc = 0;
	}
	if (stage) *stage = st;
	return rc;
}

int vp8f_token_header_memory(const uint8_t* data, size_t size, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* hdr,
                             Vp8gTokFrame* tf, uint64_t* payload_off, uint32_t* payload_size, int* stage,
                             unsigned flags) {
	int st = 0, rc = -1;
	WebPContainer c;
	ByteSpan file = {data, size};
	if (!kf || !hdr || !tf || !payload_off || !payload_size) {
		errno = EINVAL;
		st = 4;
	} else if (webp_parse_simple_lossy(file, &c) != 0) {
		st = 2;
	} else if (c.vp8_chunk_size > 0xFFFFFFF0u) {
		errno = EFBIG;
		st = 4;
	} else {
		ByteSpan payload = {data + c.vp8_chunk_offset, c.vp8_chunk_size};
		if (vp8_parse_keyframe_header(payload, kf) != 0 || !kf->is_key_frame) {
			errno = EINVAL;
			st = 3;
		} else if (vp8f_token_header(payload, kf, hdr, tf, flags) != 0) {
			st = 4;
		} else {
			*payload_off = c.vp8_chunk_offset;
			*payload_size = (uint32_t)c.vp8_chunk_size;
			rc = 0;
		}
	}
	if (stage) *stage = st;
	return rc;
}

int vp8f_decode_file(const char* path, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* out, int* stage) {
	FILE* fp = fopen(path, "rb");
	if (!fp) {
		if (stage) *stage = 1;
		return -1;
	}
	uint8_t* buf = NULL;
	size_t cap = 0, n = 0;
	for (;;) {
		if (n == cap) {
			cap = cap ? cap * 2 : (1u << 16);
			uint8_t* nb = (uint8_t*)realloc(buf, cap);
			if (!nb) {
				free(buf);
				fclose(fp);
				errno = ENOMEM;
				if (stage) *stage = 1;
				return -1;
			}
			buf = nb;
		}
		size_t got = fread(buf + n, 1, cap - n, fp);
		n += got;
		if (got == 0) break;
	}
	int err = ferror(fp);
	fclose(fp);
	if (err) {
		free(buf);
		errno = EIO;
		if (stage) *stage = 1;
		return -1;
	}
	int rc = vp8f_decode_memory(buf, n, kf, out, stage);
	int e = errno;
	free(buf);
	errno = e;
	return rc;
}
