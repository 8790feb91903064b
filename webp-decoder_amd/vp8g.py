"""vp8g -- Python mirror of the C ABI in include/vp8g.h (ctypes; no torch types cross it).

Loads the in-tree libraries built by the top-level Makefile:
  lib/libvp8host.so  C11 front end (reference m01-m05 equivalents) + synthetic frame generator
  lib/libvp8g.so     HIP gfx950 kernels behind the reference's m06/m07 entry points + batch API

The structures below are layout-identical to the reference's (reference src/m02_vp8_header/
vp8_header.h:7-18, src/m05_tokens/vp8_tokens.h:7-99, src/m06_recon/vp8_recon.h:10-18), so a
Vp8DecodedFrame produced by either front end can be handed to either reconstruction library.

Nothing here falls back to the CPU: if libvp8g.so (or a GPU) is missing, the GPU entry points
raise.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

PKG_DIR = pathlib.Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_DIR = PKG_DIR / "lib"


class ByteSpan(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("size", C.c_size_t)]


class Vp8KeyFrameHeader(C.Structure):
    _fields_ = [
        ("is_key_frame", C.c_int),
        ("profile", C.c_uint8),
        ("show_frame", C.c_int),
        ("first_partition_len", C.c_uint32),
        ("start_code_ok", C.c_int),
        ("width", C.c_uint16),
        ("height", C.c_uint16),
        ("x_scale", C.c_uint8),
        ("y_scale", C.c_uint8),
    ]


class Vp8CoeffStats(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "mb_cols", "mb_rows", "mb_total", "part0_size_bytes", "part0_bytes_used")] + [
        ("part0_overread", C.c_uint8), ("part0_overread_bytes", C.c_uint32),
        ("token_part_size_bytes", C.c_uint32), ("token_part_bytes_used", C.c_uint32),
        ("token_overread", C.c_uint8)] + [(n, C.c_uint32) for n in (
            "token_overread_bytes", "token_overread_mb_index", "token_overread_plane",
            "token_overread_block_index", "token_overread_coeff_i", "token_overread_stage",
            "mb_skip_coeff", "mb_b_pred")] + [
        ("ymode_counts", C.c_uint32 * 5), ("uv_mode_counts", C.c_uint32 * 4),
        ("bmode_counts", C.c_uint32 * 10)] + [(n, C.c_uint32) for n in (
            "blocks_total_y2", "blocks_total_y", "blocks_total_u", "blocks_total_v",
            "blocks_nonzero_y2", "blocks_nonzero_y", "blocks_nonzero_u", "blocks_nonzero_v",
            "coeff_nonzero_total", "coeff_eob_tokens", "coeff_abs_max")] + [
        ("coeff_hash_fnv1a64", C.c_uint64)]


class Vp8DecodedFrame(C.Structure):
    _fields_ = [
        ("mb_cols", C.c_uint32), ("mb_rows", C.c_uint32), ("mb_total", C.c_uint32),
        ("q_index", C.c_uint8), ("y1_dc_delta_q", C.c_int8), ("y2_dc_delta_q", C.c_int8),
        ("y2_ac_delta_q", C.c_int8), ("uv_dc_delta_q", C.c_int8), ("uv_ac_delta_q", C.c_int8),
        ("segmentation_enabled", C.c_uint8), ("segmentation_abs", C.c_uint8),
        ("seg_quant_idx", C.c_int8 * 4), ("seg_lf_level", C.c_int8 * 4),
        ("lf_use_simple", C.c_uint8), ("lf_level", C.c_uint8), ("lf_sharpness", C.c_uint8),
        ("lf_delta_enabled", C.c_uint8), ("lf_ref_delta", C.c_int8 * 4), ("lf_mode_delta", C.c_int8 * 4),
        ("segment_id", C.POINTER(C.c_uint8)), ("skip_coeff", C.POINTER(C.c_uint8)),
        ("has_coeff", C.POINTER(C.c_uint8)), ("ymode", C.POINTER(C.c_uint8)),
        ("uv_mode", C.POINTER(C.c_uint8)), ("bmode", C.POINTER(C.c_uint8)),
        ("coeff_y2", C.POINTER(C.c_int16)), ("coeff_y", C.POINTER(C.c_int16)),
        ("coeff_u", C.POINTER(C.c_int16)), ("coeff_v", C.POINTER(C.c_int16)),
        ("stats", Vp8CoeffStats),
    ]


class Yuv420Image(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("stride_y", C.c_uint32),
                ("stride_uv", C.c_uint32), ("y", C.POINTER(C.c_uint8)), ("u", C.POINTER(C.c_uint8)),
                ("v", C.POINTER(C.c_uint8))]


class Vp8gFrameDesc(C.Structure):
    _fields_ = [
        ("mb_cols", C.c_uint32), ("mb_rows", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
        ("stride_y", C.c_uint32), ("stride_uv", C.c_uint32), ("mb_offset", C.c_uint64),
        ("out_y", C.c_uint64), ("out_u", C.c_uint64), ("out_v", C.c_uint64),
        ("src_y", C.c_uint64), ("src_u", C.c_uint64), ("src_v", C.c_uint64),
        ("flags", C.c_uint32), ("src_stride_y", C.c_uint32), ("src_stride_uv", C.c_uint32),
        ("reserved", C.c_uint32), ("dq", (C.c_int16 * 6) * 4), ("lf", ((C.c_uint8 * 4) * 2) * 4),
    ]


class Vp8gBatchArrays(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "coeff_y", "coeff_u", "coeff_v", "coeff_y2", "ymode", "uv_mode", "segment_id", "has_coeff",
        "bmode", "src", "status")]


class Vp8gEncDesc(C.Structure):
    _fields_ = [
        ("width", C.c_uint32), ("height", C.c_uint32), ("stride_y", C.c_uint32), ("stride_uv", C.c_uint32),
        ("src_y", C.c_uint64), ("src_u", C.c_uint64), ("src_v", C.c_uint64), ("out", C.c_uint64),
        ("file_len", C.c_uint64), ("format", C.c_uint32), ("prefix_len", C.c_uint32), ("row_bytes", C.c_uint32),
        ("raw_len", C.c_uint32), ("span0", C.c_uint32), ("nspans", C.c_uint32), ("zend", C.c_uint32),
        ("crc_init", C.c_uint32), ("prefix", C.c_uint8 * 48), ("reserved", C.c_uint32 * 4),
        ("crc_ops", (C.c_uint32 * 32) * 10),
    ]


class Vp8gPackedFrame(C.Structure):
    """include/vp8g.h: packed m05 output (per block a non-zero mask, then the non-zero values)."""
    _fields_ = [("kf", Vp8KeyFrameHeader), ("f", Vp8DecodedFrame), ("masks", C.POINTER(C.c_uint16)),
                ("mb_off", C.POINTER(C.c_uint32)), ("values", C.POINTER(C.c_int16)), ("n_values", C.c_uint64)]


class Vp8gTokFrame(C.Structure):
    """include/vp8g.h: device m05 job of one frame (partition-0 bool state + token probabilities)."""
    _fields_ = [("data", C.c_uint64), ("mb_offset", C.c_uint64), ("b_value", C.c_uint64), ("b_bits", C.c_int32),
                ("b_range", C.c_uint32), ("b_next", C.c_uint32), ("p0_end", C.c_uint32), ("tok_off", C.c_uint32),
                ("tok_end", C.c_uint32), ("mb_cols", C.c_uint32), ("mb_rows", C.c_uint32),
                ("seg_enabled", C.c_uint8), ("seg_map_update", C.c_uint8), ("use_skip", C.c_uint8),
                ("skip_prob", C.c_uint8), ("seg_probs", C.c_uint8 * 3), ("reserved", C.c_uint8),
                ("coeff_probs", C.c_uint8 * (4 * 8 * 3 * 12)), ("nparts", C.c_uint32),
                ("part_off", C.c_uint32 * 8), ("part_end", C.c_uint32 * 8), ("reserved2", C.c_uint32 * 3)]


PK_BLOCKS = 25  # per MB: Y 0..15, U 0..3, V 0..3, Y2
VP8G_BATCH_DEVICE_M05 = 1
VP8G_BATCH_MULTI_PARTITION = 2
VP8F_PACK_HASH = 1
VP8F_MULTI_PARTITION = 2

ENC_FORMATS = {"rgb": 0, "ppm": 1, "png": 2}
ENC_SPAN = 32768

assert C.sizeof(Vp8gEncDesc) == 1432
assert C.sizeof(Vp8KeyFrameHeader) == 28
assert C.sizeof(Vp8CoeffStats) == 200
assert C.sizeof(Vp8DecodedFrame) == 320
assert C.sizeof(Yuv420Image) == 40
assert C.sizeof(Vp8gFrameDesc) == 176
assert C.sizeof(Vp8gTokFrame) == 1296

VP8G_F_LOOPFILTER = 1
VP8G_F_SIMPLE = 2
VP8G_F_LF_ONLY = 4

# Arrays of a decoded frame: (field, dtype, elements per MB)
FRAME_ARRAYS = [
    ("coeff_y", np.int16, 256), ("coeff_u", np.int16, 64), ("coeff_v", np.int16, 64),
    ("coeff_y2", np.int16, 16), ("ymode", np.uint8, 1), ("uv_mode", np.uint8, 1),
    ("segment_id", np.uint8, 1), ("has_coeff", np.uint8, 1), ("bmode", np.uint8, 16),
    ("skip_coeff", np.uint8, 1),
]
# Algorithmic bytes the hot path reads per macroblock: 800 B of dense int16
# coefficients + 20 B side info (ymode, uv_mode, segment_id, has_coeff, 16 x bmode).
BYTES_READ_PER_MB = 820


def i420_size(w: int, h: int) -> int:
    return w * h + 2 * ((w + 1) // 2) * ((h + 1) // 2)


_DIG_K = np.uint64(0x9E3779B97F4A7C15)


def digest64(buf) -> int:
    """Digest of a byte string as vp8g_frame_digests computes it on the device (include/vp8g.h):
    L*K + sum_i mix(w_i + (i+1)*K) mod 2^64 over little-endian u64 words (last zero-padded),
    mix = splitmix64's finaliser.  Returned as an unsigned Python int."""
    b = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf.view(np.uint8).reshape(-1)
    n = b.size
    pad = (-n) % 8
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    w = b.view("<u8")
    z = w + (np.arange(1, w.size + 1, dtype=np.uint64) * _DIG_K)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return (n * 0x9E3779B97F4A7C15 + int(z.sum(dtype=np.uint64))) & 0xFFFFFFFFFFFFFFFF


_libs: dict = {}


def _load(name: str, path: pathlib.Path):
    if name not in _libs:
        if not path.exists():
            raise OSError(f"{path} not built (run `make` at the repo root)")
        _libs[name] = C.CDLL(str(path), use_errno=True)
    return _libs[name]


def host_lib():
    lib = _load("host", LIB_DIR / "libvp8host.so")
    if not getattr(lib, "_typed", False):
        lib.vp8f_decode_file.argtypes = [C.c_char_p, C.POINTER(Vp8KeyFrameHeader), C.POINTER(Vp8DecodedFrame),
                                         C.POINTER(C.c_int)]
        lib.vp8f_decode_memory.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(Vp8KeyFrameHeader),
                                           C.POINTER(Vp8DecodedFrame), C.POINTER(C.c_int)]
        lib.vp8f_synth_frame.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.POINTER(Vp8KeyFrameHeader),
                                         C.POINTER(Vp8DecodedFrame)]
        lib.vp8_decoded_frame_free.argtypes = [C.POINTER(Vp8DecodedFrame)]
        lib.vp8_decoded_frame_free.restype = None
        lib.vp8f_fnv1a64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        lib.vp8f_fnv1a64.restype = C.c_uint64
        lib.vp8f_decode_packed_memory.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(Vp8gPackedFrame),
                                                  C.POINTER(C.c_int), C.c_uint]
        lib.vp8f_packed_free.argtypes = [C.POINTER(Vp8gPackedFrame)]
        lib.vp8f_token_header_memory.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(Vp8KeyFrameHeader),
                                                 C.POINTER(Vp8DecodedFrame), C.POINTER(Vp8gTokFrame),
                                                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_int),
                                                 C.c_uint]
        lib.vp8f_packed_free.restype = None
        lib._typed = True
    return lib


# vp8g_last_launch_mode bits (include/vp8g.h)
MODE_CHAIN, MODE_MIRROR_SPLIT, MODE_INTERLEAVE, MODE_QUAD, MODE_SPLIT_PARTS = 1, 2, 4, 8, 16


def gpu_lib():
    """libvp8g.so: the product path.  Raises if it is not built."""
    lib = _load("gpu", pathlib.Path(os.environ.get("VP8G_LIB", LIB_DIR / "libvp8g.so")))
    if not getattr(lib, "_typed", False):
        P = C.POINTER
        lib.vp8_reconstruct_keyframe_yuv.argtypes = [P(Vp8KeyFrameHeader), P(Vp8DecodedFrame), P(Yuv420Image)]
        lib.vp8_reconstruct_keyframe_yuv_filtered.argtypes = [P(Vp8KeyFrameHeader), P(Vp8DecodedFrame),
                                                              P(Yuv420Image)]
        lib.vp8_loopfilter_apply_keyframe.argtypes = [P(Yuv420Image), P(Vp8DecodedFrame)]
        lib.yuv420_alloc.argtypes = [P(Yuv420Image), C.c_uint32, C.c_uint32]
        lib.yuv420_free.argtypes = [P(Yuv420Image)]
        lib.yuv420_free.restype = None
        lib.vp8g_make_frame_desc.argtypes = [P(Vp8KeyFrameHeader), P(Vp8DecodedFrame), C.c_int, C.c_uint64,
                                             C.c_uint64, P(Vp8gFrameDesc)]
        lib.vp8g_i420_size.argtypes = [C.c_uint32, C.c_uint32]
        lib.vp8g_i420_size.restype = C.c_uint64
        lib.vp8g_decode_batch_device.argtypes = [P(Vp8gFrameDesc), C.c_void_p, C.c_uint32, P(Vp8gBatchArrays),
                                                 C.c_void_p, C.c_void_p, C.c_uint32]
        lib.vp8g_frame_digests.argtypes = [P(Vp8gFrameDesc), C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.c_void_p]
        lib.vp8g_reconstruct_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, P(Yuv420Image)]
        lib.vp8g_last_error.restype = C.c_char_p
        lib.vp8g_abi_version.restype = C.c_uint32
        if hasattr(lib, "vp8g_last_launch_mode"):  # (libraries built before round 5 lack it: A/B of old builds)
            lib.vp8g_last_launch_mode.restype = C.c_uint32
        lib.yuv420_write_ppm_fd.argtypes = [C.c_int, P(Yuv420Image)]
        lib.yuv420_write_png_fd.argtypes = [C.c_int, P(Yuv420Image)]
        lib.vp8g_encoded_size.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        lib.vp8g_encoded_size.restype = C.c_uint64
        lib.vp8g_encode_workspace_size.argtypes = [C.c_uint32]
        lib.vp8g_encode_workspace_size.restype = C.c_uint64
        lib.vp8g_make_enc_desc.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                                           C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, P(Vp8gEncDesc)]
        lib.vp8g_make_enc_desc.restype = C.c_uint32
        lib.vp8g_encode_batch_device.argtypes = [P(Vp8gEncDesc), C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                                 C.c_void_p, C.c_void_p]
        lib.vp8g_decode_webp_batch.argtypes = [P(ByteSpan), C.c_uint32, C.c_int, C.c_uint32, P(Yuv420Image),
                                               P(C.c_int)]
        lib.vp8g_decode_webp_batch_ex.argtypes = [P(ByteSpan), C.c_uint32, C.c_int, C.c_uint32, C.c_uint32,
                                                  P(Yuv420Image), P(C.c_int)]
        lib.vp8g_m05_batch_device.argtypes = [P(Vp8gTokFrame), C.c_void_p, C.c_uint32, C.c_void_p,
                                              P(Vp8gBatchArrays), C.c_void_p]
        lib._typed = True
    return lib


class Frame:
    """Owns one Vp8DecodedFrame (+ its key-frame header) allocated by libvp8host."""

    def __init__(self, kf: Vp8KeyFrameHeader, frame: Vp8DecodedFrame):
        self.kf = kf
        self.frame = frame
        self._alive = True

    @property
    def width(self) -> int:
        return int(self.kf.width)

    @property
    def height(self) -> int:
        return int(self.kf.height)

    @property
    def mb_total(self) -> int:
        return int(self.frame.mb_total)

    def array(self, name: str) -> np.ndarray:
        for n, dt, per in FRAME_ARRAYS:
            if n == name:
                ptr = getattr(self.frame, name)
                if not ptr:
                    return np.zeros(self.mb_total * per, dtype=dt)
                return np.ctypeslib.as_array(ptr, shape=(self.mb_total * per,)).view(dt)
        raise KeyError(name)

    def free(self):
        if self._alive:
            host_lib().vp8_decoded_frame_free(C.byref(self.frame))
            self._alive = False

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def decode_file(path) -> Frame:
    lib = host_lib()
    kf, fr, st = Vp8KeyFrameHeader(), Vp8DecodedFrame(), C.c_int(0)
    if lib.vp8f_decode_file(str(path).encode(), C.byref(kf), C.byref(fr), C.byref(st)) != 0:
        raise ValueError(f"decode failed at stage {st.value}: {path}")
    return Frame(kf, fr)


def synth_frame(width: int, height: int, seed: int, profile: int = 0) -> Frame:
    lib = host_lib()
    kf, fr = Vp8KeyFrameHeader(), Vp8DecodedFrame()
    if lib.vp8f_synth_frame(width, height, seed & 0xFFFFFFFFFFFFFFFF, profile, C.byref(kf), C.byref(fr)) != 0:
        raise ValueError("synth failed")
    return Frame(kf, fr)


class PackedFrame:
    """Owns one Vp8gPackedFrame decoded by libvp8host (vp8f_decode_packed_memory)."""

    def __init__(self, data: bytes, hash_coeffs: bool = False, multi_partition: bool = False):
        self.p = Vp8gPackedFrame()
        st = C.c_int(0)
        buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
        flags = (VP8F_PACK_HASH if hash_coeffs else 0) | (VP8F_MULTI_PARTITION if multi_partition else 0)
        if host_lib().vp8f_decode_packed_memory(buf, len(data), C.byref(self.p), C.byref(st), flags) != 0:
            raise ValueError(f"packed decode failed at stage {st.value}")
        self._alive = True

    def side(self, name: str) -> np.ndarray:
        per = 16 if name == "bmode" else 1
        return np.ctypeslib.as_array(getattr(self.p.f, name), shape=(int(self.p.f.mb_total) * per,)).copy()

    def masks(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.p.masks, shape=(int(self.p.f.mb_total), PK_BLOCKS)).copy()

    def mb_off(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.p.mb_off, shape=(int(self.p.f.mb_total),)).copy()

    def values(self) -> np.ndarray:
        n = int(self.p.n_values)
        return np.ctypeslib.as_array(self.p.values, shape=(n,)).copy() if n else np.zeros(0, np.int16)

    def free(self):
        if self._alive:
            host_lib().vp8f_packed_free(C.byref(self.p))
            self._alive = False

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def unpack_coeffs(pf: PackedFrame) -> dict:
    """Host restatement of the device expansion (expand_kernel): packed -> the four dense arrays
    (test infrastructure)."""
    masks, off, vals = pf.masks().astype(np.uint32), pf.mb_off().astype(np.int64), pf.values()
    nmb = masks.shape[0]
    dense = np.zeros((nmb, PK_BLOCKS, 16), np.int16)
    bits = ((masks[:, :, None] >> np.arange(16, dtype=np.uint32)) & 1).astype(bool)  # [mb, block, pos]
    flat = bits.reshape(nmb, -1)
    rank = np.cumsum(flat, axis=1) - 1  # index of each non-zero among the MB's values
    src = off[:, None] + rank
    dense.reshape(nmb, -1)[flat] = vals[src[flat]]
    return {"coeff_y": dense[:, :16].reshape(-1), "coeff_u": dense[:, 16:20].reshape(-1),
            "coeff_v": dense[:, 20:24].reshape(-1), "coeff_y2": dense[:, 24].reshape(-1)}


def token_header(data: bytes, multi_partition: bool = False):
    """vp8f_token_header_memory: (kf, hdr, Vp8gTokFrame, payload offset, payload size) or raises."""
    lib = host_lib()
    kf, hdr, tf = Vp8KeyFrameHeader(), Vp8DecodedFrame(), Vp8gTokFrame()
    off, size, st = C.c_uint64(0), C.c_uint32(0), C.c_int(0)
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    if lib.vp8f_token_header_memory(buf, len(data), C.byref(kf), C.byref(hdr), C.byref(tf), C.byref(off),
                                    C.byref(size), C.byref(st), VP8F_MULTI_PARTITION if multi_partition else 0) != 0:
        raise ValueError(f"vp8f_token_header_memory: stage {st.value}")
    return kf, hdr, tf, off.value, size.value


def gpu_m05(files: list[bytes], multi_partition: bool = False) -> list[dict]:
    """vp8g_m05_batch_device over .webp images (one launch): per frame the m05 arrays as numpy,
    named as FRAME_ARRAYS (skip_coeff excepted: the device does not keep it)."""
    import torch
    lib = gpu_lib()
    hdrs = [token_header(b, multi_partition) for b in files]
    n = len(files)
    jobs = (Vp8gTokFrame * n)()
    slots, mbs = [], []
    bo = mo = 0
    for i, (kf, hdr, tf, off, size) in enumerate(hdrs):
        jobs[i] = tf
        jobs[i].data, jobs[i].mb_offset = bo, mo
        slots.append((bo, off, size))
        mbs.append(hdr.mb_total)
        bo += (size + 512 + 15) & ~15  # >= 512 readable bytes after each payload
        mo += hdr.mb_total
    bits = np.zeros(max(bo, 16), np.uint8)
    for (b0, off, size), data in zip(slots, files):
        bits[b0:b0 + size] = np.frombuffer(data, np.uint8, size, off)
    dev = torch.device("cuda:0")
    d_bits = torch.from_numpy(bits).to(dev)
    d_jobs = torch.from_numpy(np.frombuffer(bytes(jobs), np.uint8).copy()).to(dev)
    per = {n_: (dt, k) for n_, dt, k in FRAME_ARRAYS}
    names = ["coeff_y", "coeff_u", "coeff_v", "coeff_y2", "ymode", "uv_mode", "segment_id", "has_coeff", "bmode"]
    tdt = {np.dtype(np.int16): torch.int16, np.dtype(np.uint8): torch.uint8}
    d = {k: torch.zeros(mo * per[k][1], dtype=tdt[np.dtype(per[k][0])], device=dev) for k in names}
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    arr = Vp8gBatchArrays(**{k: d[k].data_ptr() for k in names}, src=None, status=status.data_ptr())
    torch.cuda.synchronize()
    if lib.vp8g_m05_batch_device(jobs, d_jobs.data_ptr(), n, d_bits.data_ptr(), C.byref(arr), None) != 0:
        raise RuntimeError(f"vp8g_m05_batch_device failed: {lib.vp8g_last_error()!r}")
    torch.cuda.synchronize()
    if int(status.item()) != 0:
        raise RuntimeError(f"vp8g_m05_batch_device: device status {int(status.item())}")
    host = {k: v.cpu().numpy() for k, v in d.items()}
    out, m0 = [], 0
    for m in mbs:
        out.append({k: host[k][m0 * per[k][1]:(m0 + m) * per[k][1]] for k in names})
        m0 += m
    return out


def gpu_decode_webp_batch(files: list[bytes], filtered: bool = True, threads: int = 0, device_m05: bool = False,
                          multi_partition: bool = False):
    """vp8g_decode_webp_batch(_ex): .webp images -> (list of I420 bytes or None, list of errno).
    device_m05: m05 on the device (VP8G_BATCH_DEVICE_M05) instead of the host threads."""
    lib = gpu_lib()
    n = len(files)
    bufs = [(C.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0") for b in files]
    spans = (ByteSpan * n)(*[ByteSpan(C.cast(bufs[i], C.POINTER(C.c_uint8)), len(files[i])) for i in range(n)])
    imgs = (Yuv420Image * n)()
    st = (C.c_int * n)()
    import time
    t0 = time.perf_counter()
    rc = lib.vp8g_decode_webp_batch_ex(spans, n, int(filtered), threads,
                                       (VP8G_BATCH_DEVICE_M05 if device_m05 else 0)
                                       | (VP8G_BATCH_MULTI_PARTITION if multi_partition else 0), imgs, st)
    gpu_decode_webp_batch.seconds = time.perf_counter() - t0  # the C call alone (no Python copies)
    if rc != 0 and all(s == 5 for s in st):  # EIO: device failure, nothing returned
        raise RuntimeError(f"vp8g_decode_webp_batch failed: {lib.vp8g_last_error()!r}")
    out = []
    for i in range(n):
        out.append(_image_bytes(imgs[i]) if st[i] == 0 else None)
        lib.yuv420_free(C.byref(imgs[i]))
    return out, list(st)


def fnv1a64(buf: bytes | np.ndarray, h: int = 1469598103934665603) -> int:
    b = np.ascontiguousarray(np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else buf)
    return int(host_lib().vp8f_fnv1a64(b.ctypes.data, b.nbytes, h))


def _image_bytes(img: Yuv420Image) -> bytes:
    ysz = img.stride_y * img.height
    uvsz = img.stride_uv * ((img.height + 1) // 2)
    return C.string_at(img.y, ysz) + C.string_at(img.u, uvsz) + C.string_at(img.v, uvsz)


def gpu_reconstruct(f: Frame, filtered: bool) -> bytes:
    """Reference entry point vp8_reconstruct_keyframe_yuv[_filtered] through libvp8g.so."""
    lib = gpu_lib()
    img = Yuv420Image()
    fn = lib.vp8_reconstruct_keyframe_yuv_filtered if filtered else lib.vp8_reconstruct_keyframe_yuv
    if fn(C.byref(f.kf), C.byref(f.frame), C.byref(img)) != 0:
        raise RuntimeError(f"vp8g reconstruction failed: errno={C.get_errno()} {lib.vp8g_last_error()!r}")
    try:
        return _image_bytes(img)
    finally:
        lib.yuv420_free(C.byref(img))


def gpu_reconstruct_batch(frames: list[Frame], filtered: bool) -> list[bytes]:
    lib = gpu_lib()
    n = len(frames)
    kfs = (C.POINTER(Vp8KeyFrameHeader) * n)(*[C.pointer(f.kf) for f in frames])
    frs = (C.POINTER(Vp8DecodedFrame) * n)(*[C.pointer(f.frame) for f in frames])
    imgs = (Yuv420Image * n)()
    if lib.vp8g_reconstruct_batch(C.cast(kfs, C.c_void_p), C.cast(frs, C.c_void_p), n, int(filtered), imgs) != 0:
        raise RuntimeError(f"vp8g batch failed: {lib.vp8g_last_error()!r}")
    out = []
    for i in range(n):
        out.append(_image_bytes(imgs[i]))
        lib.yuv420_free(C.byref(imgs[i]))
    return out


def gpu_encode(i420: bytes, w: int, h: int, fmt: str) -> bytes:
    """The reference's m08/m09 writers (yuv420_write_ppm_fd / yuv420_write_png_fd) through
    libvp8g.so: the file they write for a cropped I420 image."""
    import tempfile
    lib = gpu_lib()
    img, keep = image_from_i420(i420, w, h)
    fn = lib.yuv420_write_ppm_fd if fmt == "ppm" else lib.yuv420_write_png_fd
    with tempfile.TemporaryFile() as t:
        if fn(t.fileno(), C.byref(img)) != 0:
            raise RuntimeError(f"vp8g {fmt} writer failed: errno={C.get_errno()} {lib.vp8g_last_error()!r}")
        t.seek(0)
        data = t.read()
    del keep
    return data


def make_enc_descs(sizes, fmt: str, src_offsets, out_align: int = 256):
    """Descriptors for images of the given (w, h) sizes whose planes sit at src_offsets[i] =
    (y, u, v) with tight strides, outputs packed at out_align-aligned offsets.  Returns
    (array of Vp8gEncDesc, output offsets, total output bytes, total tasks)."""
    lib = gpu_lib()
    n = len(sizes)
    descs = (Vp8gEncDesc * n)()
    outs, o, span0 = [], 0, 0
    for i, (w, h) in enumerate(sizes):
        y, u, v = src_offsets[i]
        k = lib.vp8g_make_enc_desc(w, h, ENC_FORMATS[fmt], y, u, v, w, (w + 1) // 2, o, span0, C.byref(descs[i]))
        if k == 0:
            raise ValueError(f"vp8g_make_enc_desc failed for {w}x{h} {fmt}")
        outs.append(o)
        o = (o + descs[i].file_len + out_align - 1) // out_align * out_align
        span0 += k
    return descs, outs, o, span0


def make_desc(f: Frame, filtered: bool, mb_offset: int, out_offset: int) -> Vp8gFrameDesc:
    d = Vp8gFrameDesc()
    if gpu_lib().vp8g_make_frame_desc(C.byref(f.kf), C.byref(f.frame), int(filtered), mb_offset, out_offset,
                                      C.byref(d)) != 0:
        raise ValueError("vp8g_make_frame_desc failed")
    return d


# ---- test/bench-only loaders (oracle/ is test infrastructure) ------------------------------

def oracle_lib():
    lib = _load("oracle", REPO_DIR / "oracle" / "liboracle.so")
    if not getattr(lib, "_typed", False):
        P = C.POINTER
        lib.oracle_reconstruct_i420.argtypes = [P(Vp8KeyFrameHeader), P(Vp8DecodedFrame), C.c_void_p, C.c_int]
        lib.oracle_recon_padded.argtypes = [P(Vp8DecodedFrame), C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        lib.oracle_loopfilter.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(Vp8DecodedFrame)]
        lib.oracle_time_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]
        lib.oracle_time_batch.restype = C.c_double
        lib.oracle_ppm_size.argtypes = [C.c_uint32, C.c_uint32]
        lib.oracle_ppm_size.restype = C.c_size_t
        lib.oracle_png_size.argtypes = [C.c_uint32, C.c_uint32]
        lib.oracle_png_size.restype = C.c_size_t
        lib.oracle_ppm.argtypes = [P(Yuv420Image), C.c_void_p, C.c_size_t]
        lib.oracle_ppm.restype = C.c_long
        lib.oracle_png.argtypes = [P(Yuv420Image), C.c_void_p, C.c_size_t]
        lib.oracle_png.restype = C.c_long
        lib._typed = True
    return lib


def image_from_i420(buf: bytes, w: int, h: int):
    """A Yuv420Image view of cropped I420 bytes (Y w*h, U, V each ceil(w/2)*ceil(h/2)); the
    returned numpy array keeps the memory alive."""
    a = np.frombuffer(buf, dtype=np.uint8).copy()
    cw, ch = (w + 1) // 2, (h + 1) // 2
    img = Yuv420Image(w, h, w, cw)
    base = a.ctypes.data
    img.y = C.cast(base, C.POINTER(C.c_uint8))
    img.u = C.cast(base + w * h, C.POINTER(C.c_uint8))
    img.v = C.cast(base + w * h + cw * ch, C.POINTER(C.c_uint8))
    return img, a


def oracle_encode(i420: bytes, w: int, h: int, fmt: str) -> bytes:
    """m08/m09 restatement: the PPM ("ppm") or PNG ("png") file of a cropped I420 image."""
    lib = oracle_lib()
    img, keep = image_from_i420(i420, w, h)
    n = (lib.oracle_ppm_size if fmt == "ppm" else lib.oracle_png_size)(w, h)
    out = np.empty(n, dtype=np.uint8)
    got = (lib.oracle_ppm if fmt == "ppm" else lib.oracle_png)(C.byref(img), out.ctypes.data, n)
    del keep
    if got != n:
        raise RuntimeError(f"oracle {fmt} failed ({got} of {n})")
    return out.tobytes()


def oracle_reconstruct(f: Frame, filtered: bool) -> bytes:
    buf = np.empty(i420_size(f.width, f.height), dtype=np.uint8)
    if oracle_lib().oracle_reconstruct_i420(C.byref(f.kf), C.byref(f.frame), buf.ctypes.data, int(filtered)) != 0:
        raise RuntimeError("oracle failed")
    return buf.tobytes()


def ref_lib():
    """oracle/_ref/libref.so: the reference's own m01-m07 compiled here (may be absent)."""
    lib = _load("ref", REPO_DIR / "oracle" / "_ref" / "libref.so")
    if not getattr(lib, "_typed", False):
        P = C.POINTER
        lib.ref_decode_i420.argtypes = [C.c_char_p, C.c_void_p, C.c_size_t, C.c_int]
        lib.ref_decode_i420.restype = C.c_long
        lib.ref_recon_i420.argtypes = [P(Vp8KeyFrameHeader), P(Vp8DecodedFrame), C.c_void_p, C.c_int]
        lib.ref_decode_frame.argtypes = [C.c_char_p, P(Vp8KeyFrameHeader), P(Vp8DecodedFrame)]
        lib.ref_free_frame.argtypes = [P(Vp8DecodedFrame)]
        lib.ref_free_frame.restype = None
        lib.ref_coeff_hash.argtypes = [C.c_char_p]
        lib.ref_coeff_hash.restype = C.c_uint64
        lib.ref_loopfilter_padded.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                              P(Vp8DecodedFrame)]
        lib.ref_time_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]
        lib.ref_time_batch.restype = C.c_double
        lib._typed = True
    return lib


def ref_available() -> bool:
    return (REPO_DIR / "oracle" / "_ref" / "libref.so").exists()


def ref_reconstruct(f: Frame, filtered: bool) -> bytes:
    buf = np.empty(i420_size(f.width, f.height), dtype=np.uint8)
    if ref_lib().ref_recon_i420(C.byref(f.kf), C.byref(f.frame), buf.ctypes.data, int(filtered)) != 0:
        raise RuntimeError("reference recon failed")
    return buf.tobytes()


def cpu_time_batch(frames: list[Frame], n: int, threads: int, filtered: bool, kind: str = "port") -> float:
    """Seconds for `n` frame reconstructions on `threads` host threads (oracle port or reference)."""
    lib = oracle_lib() if kind == "port" else ref_lib()
    fn = lib.oracle_time_batch if kind == "port" else lib.ref_time_batch
    k = len(frames)
    kfs = (C.POINTER(Vp8KeyFrameHeader) * k)(*[C.pointer(f.kf) for f in frames])
    frs = (C.POINTER(Vp8DecodedFrame) * k)(*[C.pointer(f.frame) for f in frames])
    return float(fn(C.cast(kfs, C.c_void_p), C.cast(frs, C.c_void_p), k, n, threads, int(filtered)))
