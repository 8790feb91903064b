/*
 * vp8g.h -- C ABI of the MI355X-native VP8 keyframe reconstruction + loop-filter path.
 *
 * This header is the drop-in boundary.  The first half re-declares, layout-identically, the
 * reference decoder's types and the five entry points of its m06/m07 hot path, so the
 * reference's own callers (src/main.c:591, :665, :742, :811, :881; src/main_ultra.c:43)
 * link against libvp8g.so unchanged.  The second half is an additive batch API used by the
 * batch/multi-GPU driver and the benchmark (device-resident frames, one launch per batch).
 *
 * Plain C: no HIP or torch types appear in any signature.  Streams are passed as void*.
 */
#ifndef VP8G_H
#define VP8G_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Reference types (layout-identical) ------------------------------------------------ */

/* reference: src/common/os.h:6-9 */
#ifndef VP8G_NO_BYTESPAN
typedef struct {
	const uint8_t* data;
	size_t size;
} ByteSpan;
#endif

/* reference: src/m02_vp8_header/vp8_header.h:7-18 (28 bytes; width @20, height @22) */
typedef struct {
	int is_key_frame;
	uint8_t profile;
	int show_frame;
	uint32_t first_partition_len;
	int start_code_ok;
	uint16_t width;
	uint16_t height;
	uint8_t x_scale;
	uint8_t y_scale;
} Vp8KeyFrameHeader;

/* reference: src/m05_tokens/vp8_tokens.h:7-50 (200 bytes) */
typedef struct {
	uint32_t mb_cols;
	uint32_t mb_rows;
	uint32_t mb_total;
	uint32_t part0_size_bytes;
	uint32_t part0_bytes_used;
	uint8_t part0_overread;
	uint32_t part0_overread_bytes;
	uint32_t token_part_size_bytes;
	uint32_t token_part_bytes_used;
	uint8_t token_overread;
	uint32_t token_overread_bytes;
	uint32_t token_overread_mb_index;
	uint32_t token_overread_plane;
	uint32_t token_overread_block_index;
	uint32_t token_overread_coeff_i;
	uint32_t token_overread_stage;
	uint32_t mb_skip_coeff;
	uint32_t mb_b_pred;
	uint32_t ymode_counts[5];
	uint32_t uv_mode_counts[4];
	uint32_t bmode_counts[10];
	uint32_t blocks_total_y2;
	uint32_t blocks_total_y;
	uint32_t blocks_total_u;
	uint32_t blocks_total_v;
	uint32_t blocks_nonzero_y2;
	uint32_t blocks_nonzero_y;
	uint32_t blocks_nonzero_u;
	uint32_t blocks_nonzero_v;
	uint32_t coeff_nonzero_total;
	uint32_t coeff_eob_tokens;
	uint32_t coeff_abs_max;
	uint64_t coeff_hash_fnv1a64;
} Vp8CoeffStats;

/* reference: src/m05_tokens/vp8_tokens.h:52-99 (320 bytes).  The hot path's input:
 * per-MB modes + dense int16 coefficients in natural (de-zigzagged) order. */
typedef struct {
	uint32_t mb_cols;
	uint32_t mb_rows;
	uint32_t mb_total;
	uint8_t q_index;
	int8_t y1_dc_delta_q;
	int8_t y2_dc_delta_q;
	int8_t y2_ac_delta_q;
	int8_t uv_dc_delta_q;
	int8_t uv_ac_delta_q;
	uint8_t segmentation_enabled;
	uint8_t segmentation_abs;
	int8_t seg_quant_idx[4];
	int8_t seg_lf_level[4];
	uint8_t lf_use_simple;
	uint8_t lf_level;
	uint8_t lf_sharpness;
	uint8_t lf_delta_enabled;
	int8_t lf_ref_delta[4];
	int8_t lf_mode_delta[4];
	uint8_t* segment_id; /* [mb_total] 0..3 */
	uint8_t* skip_coeff; /* [mb_total] */
	uint8_t* has_coeff;  /* [mb_total] (may be NULL: treated as all zero) */
	uint8_t* ymode;      /* [mb_total] 0..4 = DC,V,H,TM,B_PRED */
	uint8_t* uv_mode;    /* [mb_total] 0..3 */
	uint8_t* bmode;      /* [mb_total*16] 0..9 */
	int16_t* coeff_y2;   /* [mb_total*16] */
	int16_t* coeff_y;    /* [mb_total*256] */
	int16_t* coeff_u;    /* [mb_total*64] */
	int16_t* coeff_v;    /* [mb_total*64] */
	Vp8CoeffStats stats;
} Vp8DecodedFrame;

/* reference: src/m06_recon/vp8_recon.h:10-18 (40 bytes). Planes are malloc()ed host memory. */
typedef struct {
	uint32_t width;
	uint32_t height;
	uint32_t stride_y;
	uint32_t stride_uv;
	uint8_t* y;
	uint8_t* u;
	uint8_t* v;
} Yuv420Image;

/* ---- Reference entry points (exact signatures) ----------------------------------------- */

/* replaces src/m06_recon/vp8_recon.c:360 (decl vp8_recon.h:20).  Y zeroed, U/V = 128;
 * stride_y = width, stride_uv = (width+1)/2.  0 / -1 + errno (EINVAL, ENOMEM). */
int yuv420_alloc(Yuv420Image* img, uint32_t width, uint32_t height);

/* replaces src/m06_recon/vp8_recon.c:387 (decl vp8_recon.h:21).  Plain free() of the planes. */
void yuv420_free(Yuv420Image* img);

/* replaces src/m06_recon/vp8_recon.c:714 (decl vp8_recon.h:25): recon only (decoder -yuv). */
int vp8_reconstruct_keyframe_yuv(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* decoded, Yuv420Image* out);

/* replaces src/m06_recon/vp8_recon.c:718 (decl vp8_recon.h:28): recon + loop filter (-yuvf). */
int vp8_reconstruct_keyframe_yuv_filtered(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* decoded,
                                          Yuv420Image* out);

/* replaces src/m07_loopfilter/vp8_loopfilter.c:201 (decl vp8_loopfilter.h:14): in-place filter of a
 * macroblock-aligned frame (width == mb_cols*16, height == mb_rows*16, else EINVAL). */
int vp8_loopfilter_apply_keyframe(Yuv420Image* padded_img, const Vp8DecodedFrame* decoded);

/* ---- Batch API (build-only, additive) --------------------------------------------------- */

/* Per-frame launch descriptor (host computes it once per frame: geometry, output placement,
 * dequant factors per segment (RFC 6386 14.1, reference vp8_recon.c:57-76) and loop-filter
 * parameters per (segment, is_B_PRED) (reference vp8_loopfilter.c:166-199)). 176 bytes. */
typedef struct {
	uint32_t mb_cols, mb_rows;
	uint32_t width, height;       /* crop (visible) size written to the output */
	uint32_t stride_y, stride_uv; /* output strides in bytes */
	uint64_t mb_offset;           /* index of this frame's first MB in the batch SoA arrays */
	uint64_t out_y, out_u, out_v; /* byte offsets of the three planes in the output buffer */
	uint64_t src_y, src_u, src_v; /* (loop-filter-only mode) byte offsets of the padded input */
	uint32_t flags;               /* VP8G_F_* */
	uint32_t src_stride_y, src_stride_uv;
	uint32_t reserved;
	int16_t dq[4][6];  /* [segment][Y1dc, Y1ac, UVdc, UVac, Y2dc, Y2ac] */
	uint8_t lf[4][2][4]; /* [segment][is_bpred] = {level(E), interior I, hev T, 0}; level 0 = skip */
} Vp8gFrameDesc;

#define VP8G_F_LOOPFILTER 1u /* apply m07 (some MB has a non-zero level) */
#define VP8G_F_SIMPLE 2u     /* simple filter (luma only) instead of normal */
#define VP8G_F_LF_ONLY 4u    /* loop-filter-only: pixels come from src_* instead of recon */

/* Device pointers of a batch, concatenated over frames in the exact per-array layout of
 * Vp8DecodedFrame (so a frame uploads with nine plain memcpys).  MB index m of frame f is
 * desc.mb_offset + m. */
typedef struct {
	const int16_t* coeff_y;  /* [MB*256] */
	const int16_t* coeff_u;  /* [MB*64] */
	const int16_t* coeff_v;  /* [MB*64] */
	const int16_t* coeff_y2; /* [MB*16] */
	const uint8_t* ymode;    /* [MB] */
	const uint8_t* uv_mode;  /* [MB] */
	const uint8_t* segment_id; /* [MB] */
	const uint8_t* has_coeff;  /* [MB] */
	const uint8_t* bmode;      /* [MB*16] */
	const uint8_t* src;        /* LF-only mode input pixels (else NULL) */
	uint32_t* status;          /* device word: 0 ok, else VP8G_ERR_* (kernel-detected) */
} Vp8gBatchArrays;

#define VP8G_ERR_TIMEOUT 1u /* a wavefront dependency wait exceeded its bound */

/* Fill a descriptor for one frame.  kf may be NULL in LF-only mode.  Returns 0 / -1+errno. */
int vp8g_make_frame_desc(const Vp8KeyFrameHeader* kf, const Vp8DecodedFrame* decoded, int filtered,
                         uint64_t mb_offset, uint64_t out_offset, Vp8gFrameDesc* out);

/* Bytes of cropped I420 output for a w x h frame (Y + 2 * ceil(w/2)*ceil(h/2)). */
uint64_t vp8g_i420_size(uint32_t width, uint32_t height);

/* Launch the fused recon(+LF) kernel over n frames on `hip_stream` (NULL = default stream).
 * h_descs: host copy (launch geometry); d_descs: the same array in device memory.
 * All pointers in `arrays` and d_out are device pointers.  Asynchronous; returns 0 or -1+errno.
 * `waves_per_frame` 0 = default. */
int vp8g_decode_batch_device(const Vp8gFrameDesc* h_descs, const Vp8gFrameDesc* d_descs, uint32_t n_frames,
                             const Vp8gBatchArrays* arrays, uint8_t* d_out, void* hip_stream,
                             uint32_t waves_per_frame);

/* Per-frame 64-bit digests of a device-resident batch's outputs (parity without copying pixels
 * back): d_digests[i] = digest of frame i's cropped I420 bytes (Y, U, V at stride = row width, the
 * file the reference CLI writes): D = L*K + sum_i mix(w_i + (i+1)*K) mod 2^64 over the bytes as
 * little-endian u64 words w_i (last one zero-padded), K = 0x9E3779B97F4A7C15, mix = splitmix64's
 * finaliser.  Descriptors must have the contiguous layout vp8g_make_frame_desc
 * builds (else EINVAL).  Asynchronous on `hip_stream`; 0 or -1 + errno. */
int vp8g_frame_digests(const Vp8gFrameDesc* h_descs, const Vp8gFrameDesc* d_descs, uint32_t n_frames,
                       const uint8_t* d_out, uint64_t* d_digests, void* hip_stream);

/* Host-side batch: upload n decoded frames, run one launch, download into n freshly
 * yuv420_alloc()ed images.  Returns 0 / -1+errno (EIO on a HIP failure). */
int vp8g_reconstruct_batch(const Vp8KeyFrameHeader* const* kfs, const Vp8DecodedFrame* const* frames, uint32_t n,
                           int filtered, Yuv420Image* outs);

/* ---- End-to-end batch path: .webp bytes -> I420 (SURVEY §8(f1) step 1 + §8(f2)) ---------- */

/* Packed m05 output, the host -> device wire format.  Per MB the 25 blocks (Y 0..15, U 0..3,
 * V 0..3, Y2) each leave a 16-bit mask of the natural positions holding a non-zero coefficient;
 * the values follow block by block, natural order within a block.  A 4K frame of the bench
 * fixtures packs to ~2.5-5 MB instead of the 26.6 MB of dense int16 arrays. */
#define VP8G_PK_BLOCKS 25
typedef struct {
	Vp8KeyFrameHeader kf;
	Vp8DecodedFrame f;  /* header fields, side arrays and stats; coeff_* are NULL */
	uint16_t* masks;    /* [mb_total * 25] */
	uint32_t* mb_off;   /* [mb_total] index of the MB's first value in values[] */
	int16_t* values;    /* [n_values] */
	uint64_t n_values;
} Vp8gPackedFrame;

/* Device m05 job of one frame: the host parses the frame header and the
 * first partition's frame-level fields (RFC 6386 9.2-9.11, 13.4); the device decodes the
 * per-macroblock modes (partition 0, from the saved bool-decoder state) and the coefficient
 * tokens (the token partitions) into the batch SoA of Vp8gBatchArrays.  1296 bytes. */
typedef struct {
	uint64_t data;       /* byte offset of the VP8 payload in the device bitstream buffer (caller) */
	uint64_t mb_offset;  /* first MB of the frame in the batch arrays (caller) */
	uint64_t b_value;    /* partition-0 bool decoder at the first MB header: value window, */
	int32_t b_bits;      /*   bits below the 8-bit comparison window, */
	uint32_t b_range;    /*   range (128..255), */
	uint32_t b_next;     /*   payload offset of the next byte to load */
	uint32_t p0_end;     /* payload offset one past the first partition (bytes beyond read as 0) */
	uint32_t tok_off, tok_end; /* the (first) token partition [tok_off, tok_end) of the payload */
	uint32_t mb_cols, mb_rows;
	uint8_t seg_enabled, seg_map_update, use_skip, skip_prob;
	uint8_t seg_probs[3], reserved;
	uint8_t coeff_probs[4][8][3][12]; /* RFC 13.4 after this frame's updates; rows padded to 12 */
	uint32_t nparts;                  /* token partitions (1, 2, 4, 8; > 1 only with VP8F_MULTI_PARTITION) */
	uint32_t part_off[8], part_end[8]; /* partition p = [part_off[p], part_end[p]) (RFC 9.5); MB row r
	                                      reads partition r % nparts */
	uint32_t reserved2[3];
} Vp8gTokFrame;

/* Decode n .webp file images end to end: container/header/m05 on `threads` host threads (0 = the
 * CPUs this process may run on) into the packed format, chunks of frames uploaded packed,
 * expanded and reconstructed (+ loop filter when `filtered`) on the device while the next chunk
 * is being entropy-decoded, I420 downloaded into outs[i] (yuv420_alloc layout; the caller frees
 * each with yuv420_free).  status[i] (may be NULL) = 0 or the errno of frame i's failure (its
 * image is left zeroed).  Returns 0 when every frame decoded, else -1 + errno of the first
 * failing frame (EIO for a device failure, in which case no image is returned). */
int vp8g_decode_webp_batch(const ByteSpan* files, uint32_t n, int filtered, uint32_t threads, Yuv420Image* outs,
                           int* status);

/* vp8g_decode_webp_batch with options.  VP8G_BATCH_DEVICE_M05: the host threads only parse the
 * container and the frame headers; the compressed payloads are uploaded and m05 runs on the
 * device (vp8g_m05_batch_device), one wavefront per frame.  Same outputs and errors. */
#define VP8G_BATCH_DEVICE_M05 1u
/* also accept multi-partition token streams (which the reference rejects, ENOTSUP), in either
 * mode; on the device each partition gets its own wave */
#define VP8G_BATCH_MULTI_PARTITION 2u
int vp8g_decode_webp_batch_ex(const ByteSpan* files, uint32_t n, int filtered, uint32_t threads, uint32_t flags,
                              Yuv420Image* outs, int* status);

/* The schedule vp8g_decode_webp_batch_ex uses for `flags` (host code only, no device call; for
 * tests and tools): dev[i] = 1 if frame i's m05 runs on the device, 0 on the host threads;
 * order[] = the order the worker threads take the frames (device frames first).  In device-m05
 * mode the k heaviest payloads go to the host threads, k minimising max(host time, device
 * time) under the library's cost model (VP8G_HYBRID=0 in the environment keeps
 * every frame on the device).  0, or -1 + EINVAL. */
int vp8g_plan_batch(const ByteSpan* files, uint32_t n, uint32_t threads, uint32_t flags, uint8_t* dev, uint32_t* order);

/* Device m05 over n frames on `hip_stream`: h_jobs / d_jobs host and device copies of the jobs
 * (data = payload offset in d_bits, 4-aligned, with >= 512 readable bytes after the payload;
 * mb_offset = first MB in the arrays).  Writes ymode, uv_mode, segment_id, has_coeff, bmode and
 * the non-zero coefficients of `arrays` (the caller zeroes the four coefficient arrays first);
 * arrays->status (required) gets VP8G_ERR_TIMEOUT if the two waves of a frame lose each other.
 * Asynchronous; 0 or -1 + errno (EINVAL for an inconsistent job, EIO on a launch failure). */
int vp8g_m05_batch_device(const Vp8gTokFrame* h_jobs, const Vp8gTokFrame* d_jobs, uint32_t n, const uint8_t* d_bits,
                          const Vp8gBatchArrays* arrays, void* hip_stream);

/* ---- m08 / m09 boundary: I420 -> RGB24 ("fancy" 4:2:0 upsampling) and the file writers -- */

/* replaces src/m08_yuv2rgb_ppm/yuv2rgb_ppm.c:123 (decl yuv2rgb_ppm.h:10): binary PPM (P6) of img
 * to fd, full-range Rec.601 as libwebp's VP8YuvToRgb.  0, or -1 + errno (EINVAL bad arguments or
 * zero size, ENOMEM, EIO on a HIP failure, or write(2)'s errno). */
int yuv420_write_ppm_fd(int fd, const Yuv420Image* img);

/* replaces src/m09_png/yuv2rgb_png.c:208 (decl yuv2rgb_png.h:10): 8-bit RGB PNG, filter 0 on every
 * scanline, one IDAT holding a zlib stream of stored blocks (<= 65535 bytes each); EFBIG when the
 * raw scanline stream exceeds 2^31 - 1 bytes.  Same errors as yuv420_write_ppm_fd otherwise. */
int yuv420_write_png_fd(int fd, const Yuv420Image* img);

#define VP8G_ENC_RGB 0u /* RGB24 rows, no header: w*h*3 bytes */
#define VP8G_ENC_PPM 1u /* the file yuv420_write_ppm_fd writes */
#define VP8G_ENC_PNG 2u /* the file yuv420_write_png_fd writes */
#define VP8G_ENC_SPAN 32768u /* output bytes per workgroup task */

/* Per-image descriptor of the encoder kernels (built by vp8g_make_enc_desc).  1432 bytes. */
typedef struct {
	uint32_t width, height;
	uint32_t stride_y, stride_uv;  /* source plane strides */
	uint64_t src_y, src_u, src_v;  /* byte offsets of the source planes in the source buffer */
	uint64_t out;                  /* byte offset of the file in the output buffer (16-B aligned) */
	uint64_t file_len;             /* bytes of the file */
	uint32_t format;               /* VP8G_ENC_* */
	uint32_t prefix_len;           /* bytes before the first pixel byte (PNG: signature, IHDR, IDAT
	                                  header, zlib header = 43) */
	uint32_t row_bytes;            /* bytes per row of the pixel stream (3w; PNG 1 + 3w) */
	uint32_t raw_len;              /* pixel stream bytes (height * row_bytes) */
	uint32_t span0, nspans;        /* this image's VP8G_ENC_SPAN-byte tasks in the launch */
	uint32_t zend;                 /* PNG: file offset just past the zlib stream (Adler-32 ends here) */
	uint32_t crc_init;             /* PNG: CRC-32 correction for the 0xFFFFFFFF initial value */
	uint8_t prefix[48];
	uint32_t reserved[4];
	uint32_t crc_ops[10][32];      /* PNG: GF(2) operators (columns) of the checksum combine */
} Vp8gEncDesc;

/* Fill the descriptor of one w x h image whose planes sit at src_* (strides stride_*) in the
 * source buffer, encoded as `format` at out_offset (16-B aligned) of the output buffer; its tasks
 * start at span0.  Returns the image's task count (> 0), or 0 + errno (EINVAL, EFBIG). */
uint32_t vp8g_make_enc_desc(uint32_t width, uint32_t height, uint32_t format, uint64_t src_y, uint64_t src_u,
                            uint64_t src_v, uint32_t stride_y, uint32_t stride_uv, uint64_t out_offset,
                            uint32_t span0, Vp8gEncDesc* out);

/* Encoded file size (0 for a bad format / size). */
uint64_t vp8g_encoded_size(uint32_t format, uint32_t width, uint32_t height);

/* Device workspace bytes for a launch of `total_spans` tasks. */
uint64_t vp8g_encode_workspace_size(uint32_t total_spans);

/* Encode n images (device-resident source planes -> files in d_out) on `hip_stream`: one launch
 * over all tasks (pixels, layout, per-task checksum partials) plus, when some image is a PNG, one
 * that finishes the Adler-32 / CRC-32 fields.  h_descs / d_descs: host and device copies of the
 * descriptors; d_work: vp8g_encode_workspace_size() bytes.  Asynchronous; 0 or -1 + errno. */
int vp8g_encode_batch_device(const Vp8gEncDesc* h_descs, const Vp8gEncDesc* d_descs, uint32_t n, const uint8_t* d_src,
                             uint8_t* d_out, uint8_t* d_work, void* hip_stream);

/* Name of the last HIP error seen by this library in the calling thread ("" if none). */
const char* vp8g_last_error(void);

/* How the calling thread's last reconstruction launch through vp8g_decode_batch_device or the
 * reference entry points ran: VP8G_MODE_* bits, 0 = one workgroup per frame (also after a call that
 * failed before its launch).  The end-to-end batch path (vp8g_decode_webp_batch[_ex]) does not set
 * it.  Diagnostics and tests. */
#define VP8G_MODE_CHAIN 1u        /* one 16-wave workgroup per CU decodes a chain of frames */
#define VP8G_MODE_MIRROR_SPLIT 2u /* frames split between a workgroup and its mirror */
#define VP8G_MODE_INTERLEAVE 4u   /* two frames of a chain interleaved */
#define VP8G_MODE_QUAD 8u         /* the chain with four MB rows per wave (else two) */
#define VP8G_MODE_SPLIT_PARTS 16u /* each frame over several workgroups */
uint32_t vp8g_last_launch_mode(void);

/* ABI version of this header (bumped on any layout change). */
#define VP8G_ABI_VERSION 5
uint32_t vp8g_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* VP8G_H */
