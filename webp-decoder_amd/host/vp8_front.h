/*
 * vp8_front.h -- C11 host front end (container, frame header, bool decoder, modes, tokens).
 *
 * This is the producer of the hot path's input (Vp8DecodedFrame).  It is NOT on the GPU path
 * (serial entropy decode), but the CLI and the GPU-box tests need it,
 * so it is written here from RFC 6386 with the reference's exact output semantics and the same
 * public names as the reference modules it stands in for:
 *   webp_parse_simple_lossy    <- src/m01_container/webp_container.c:19
 *   vp8_parse_keyframe_header  <- src/m02_vp8_header/vp8_header.c:13
 *   vp8_decode_decoded_frame   <- src/m05_tokens/vp8_tokens.c:673
 *   vp8_decoded_frame_free     <- src/m05_tokens/vp8_tokens.c:658
 * Unlike the reference (global g_coeff_probs, vp8_tokens.c:625) the decoder keeps all state
 * on the stack, so frames can be decoded concurrently from several threads.
 */
#ifndef VP8_FRONT_H
#define VP8_FRONT_H

#include "../../include/vp8g.h"

#ifdef __cplusplus
extern "C" {
#endif

/* reference: src/m01_container/webp_container.h:8-15 */
typedef struct {
	uint32_t riff_size;
	size_t actual_size;
	size_t vp8_chunk_offset;
	uint32_t vp8_chunk_size;
} WebPContainer;

int webp_parse_simple_lossy(ByteSpan file, WebPContainer* out);
int vp8_parse_keyframe_header(ByteSpan vp8_payload, Vp8KeyFrameHeader* out);
int vp8_decode_decoded_frame(ByteSpan vp8_payload, Vp8DecodedFrame* out);
void vp8_decoded_frame_free(Vp8DecodedFrame* f);

/* Convenience for tools/tests: read a .webp file, parse container + key-frame header and
 * decode the macroblock data.  Returns 0, or -1 with errno and a stage code in *stage
 * (1 = open/read, 2 = container, 3 = key-frame header, 4 = macroblock/token decode). */
int vp8f_decode_file(const char* path, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* out, int* stage);

/* Same for an in-memory file image. */
int vp8f_decode_memory(const uint8_t* data, size_t size, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* out, int* stage);

/* m05 into the packed wire format (Vp8gPackedFrame, include/vp8g.h): same
 * decode, side arrays and stats as vp8_decode_decoded_frame, but each 4x4 block leaves only its
 * non-zero mask and values (no dense coefficient arrays).  The FNV coefficient hash is computed
 * only with VP8F_PACK_HASH (stats.coeff_hash_fnv1a64 = 0 otherwise).  Reentrant. */
#define VP8F_PACK_HASH 1u
/* also accept 2/4/8 token partitions (RFC 6386 9.5), which the reference rejects with ENOTSUP
 * (vp8_tokens.c:357-360); SURVEY §8(f4) */
#define VP8F_MULTI_PARTITION 2u
int vp8f_decode_packed(ByteSpan vp8_payload, Vp8gPackedFrame* out, unsigned flags);
/* container + key-frame header + vp8f_decode_packed; stage codes as vp8f_decode_file */
int vp8f_decode_packed_memory(const uint8_t* data, size_t size, Vp8gPackedFrame* out, int* stage, unsigned flags);
void vp8f_packed_free(Vp8gPackedFrame* p);
/* RFC 6386 9.5 token partition bounds [off[p], end[p]) within the VP8 payload (off / end may be
 * NULL to validate only).  0, or -1 + EINVAL when the size table or a partition overruns. */
int vp8f_partition_table(ByteSpan vp8_payload, uint32_t first_partition_len, unsigned nparts, uint32_t* off,
                         uint32_t* end);

/* Host half of the device m05 (Vp8gTokFrame, include/vp8g.h): key-frame header + the first
 * partition's frame-level fields; hdr receives those fields (no arrays), tf the device job
 * (data / mb_offset left 0 for the caller).  flags: VP8F_MULTI_PARTITION accepts 2/4/8 token
 * partitions.  0, or -1 + errno (EINVAL, ENOTSUP). */
int vp8f_token_header(ByteSpan vp8_payload, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* hdr, Vp8gTokFrame* tf,
                      unsigned flags);
/* container + vp8f_token_header; *payload_off / *payload_size locate the VP8 payload in data.
 * Stage codes as vp8f_decode_file (2 container, 3 not a key frame / bad frame header, 4 first
 * partition or unsupported partitioning). */
int vp8f_token_header_memory(const uint8_t* data, size_t size, Vp8KeyFrameHeader* kf, Vp8DecodedFrame* hdr,
                             Vp8gTokFrame* tf, uint64_t* payload_off, uint32_t* payload_size, int* stage,
                             unsigned flags);

/* Seeded synthetic Vp8DecodedFrame (build-defined generator, see vp8_synth.c header for the
 * exact distribution).  profile 0 = "measured-like" statistics, 1 = stress (full-range coeffs,
 * all modes uniformly, random LF/segment parameters).  kf receives width/height. */
int vp8f_synth_frame(uint32_t width, uint32_t height, uint64_t seed, int profile, Vp8KeyFrameHeader* kf,
                     Vp8DecodedFrame* out);

/* FNV-1a 64 over a byte buffer (same constants as reference vp8_tokens.c:15-27). */
uint64_t vp8f_fnv1a64(const void* data, size_t n, uint64_t h);

#ifdef __cplusplus
}
#endif

#endif
