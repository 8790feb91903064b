"""vp8g_batch -- device-resident frame batches for the batch API (include/vp8g.h,
vp8g_decode_batch_device / vp8g_frame_digests), used by bench.py and the GPU tests.

A batch holds n frames of one geometry in HBM: the nine Vp8DecodedFrame arrays concatenated over
slots (Vp8gBatchArrays; the reference's per-frame layout, src/m05_tokens/vp8_tokens.h:52-99), one
Vp8gFrameDesc per slot, the cropped I420 outputs (256-B aligned per slot), the kernel status word
and one 64-bit digest per slot.  Torch is only the allocator / copy engine here; every compute
call goes through libvp8g.so.

Inputs of a slot come from either
  * `replicate(frames)`: slot i <- frames[(slot0 + i) % K] as separate HBM copies (decoded once on
    the host, copied on the device), or
  * `fill(i, frame)`: one host frame uploaded into slot i (synthetic batches, all frames distinct).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

import vp8g

ARRAY_NAMES = ("coeff_y", "coeff_u", "coeff_v", "coeff_y2", "ymode", "uv_mode", "segment_id", "has_coeff", "bmode")
_PER = {n: (dt, per) for n, dt, per in vp8g.FRAME_ARRAYS}


class DeviceBatch:
    def __init__(self, n: int, width: int, height: int, dev: torch.device):
        self.n, self.width, self.height, self.dev = n, width, height, dev
        self.mb_cols, self.mb_rows = (width + 15) // 16, (height + 15) // 16
        self.mb_per = self.mb_cols * self.mb_rows
        self.total_mb = n * self.mb_per
        self.arrays = {}
        for name in ARRAY_NAMES:
            dt, per = _PER[name]
            self.arrays[name] = torch.empty(self.total_mb * per, dtype=torch.int16 if dt == np.int16 else torch.uint8,
                                            device=dev)
        self.i420 = vp8g.i420_size(width, height)
        self.frame_bytes = (self.i420 + 255) // 256 * 256
        self.out = torch.empty(n * self.frame_bytes, dtype=torch.uint8, device=dev)
        self.status = torch.zeros(4, dtype=torch.int32, device=dev)
        self.digest_buf = torch.zeros(n, dtype=torch.int64, device=dev)
        self.h_descs = (vp8g.Vp8gFrameDesc * n)()
        self.d_descs = None
        a = vp8g.Vp8gBatchArrays()
        for name in ARRAY_NAMES:
            setattr(a, name, self.arrays[name].data_ptr())
        a.src = None
        a.status = self.status.data_ptr()
        self.c_arrays = a

    def _check(self, f: vp8g.Frame):
        if (f.width, f.height) != (self.width, self.height) or f.mb_total != self.mb_per:
            raise ValueError(f"frame {f.width}x{f.height} does not fit a {self.width}x{self.height} batch")

    def replicate(self, frames: list, filtered: bool, slot0: int = 0):
        """slot i <- frames[(slot0 + i) % K]; each distinct frame crosses PCIe once."""
        k = len(frames)
        for f in frames:
            self._check(f)
        for name in ARRAY_NAMES:
            per = _PER[name][1]
            view = self.arrays[name].view(self.n, self.mb_per * per)
            for j, f in enumerate(frames):
                first = (j - slot0) % k
                if first >= self.n:
                    continue
                src = torch.from_numpy(f.array(name).copy()).to(self.dev)
                view[first::k] = src
                del src
        for i in range(self.n):
            self.h_descs[i] = vp8g.make_desc(frames[(slot0 + i) % k], filtered, i * self.mb_per, i * self.frame_bytes)

    def fill(self, i: int, f: vp8g.Frame, filtered: bool):
        """Upload one host frame into slot i."""
        self._check(f)
        for name in ARRAY_NAMES:
            per = _PER[name][1]
            seg = self.arrays[name][i * self.mb_per * per:(i + 1) * self.mb_per * per]
            seg.copy_(torch.from_numpy(f.array(name)))
        self.h_descs[i] = vp8g.make_desc(f, filtered, i * self.mb_per, i * self.frame_bytes)

    def place(self, i: int, f: vp8g.Frame, filtered: bool):
        """Upload a frame no larger than the batch geometry into slot i (mixed-size batches: the
        frame's MBs and I420 output start at the slot's base; its descriptor carries its own size)."""
        if f.mb_total > self.mb_per or vp8g.i420_size(f.width, f.height) > self.frame_bytes:
            raise ValueError(f"frame {f.width}x{f.height} does not fit a {self.width}x{self.height} slot")
        for name in ARRAY_NAMES:
            per = _PER[name][1]
            o = i * self.mb_per * per
            self.arrays[name][o:o + f.mb_total * per].copy_(torch.from_numpy(f.array(name)))
        self.h_descs[i] = vp8g.make_desc(f, filtered, i * self.mb_per, i * self.frame_bytes)

    def commit(self):
        """Descriptors to the device (after every slot is filled)."""
        self.d_descs = torch.frombuffer(bytearray(bytes(self.h_descs)), dtype=torch.uint8).to(self.dev)
        return self.d_descs

    def launch(self, stream: int, waves: int = 0):
        """One launch of the fused recon(+LF) kernel over the batch (vp8g_decode_batch_device)."""
        rc = vp8g.gpu_lib().vp8g_decode_batch_device(self.h_descs, C.c_void_p(self.d_descs.data_ptr()), self.n,
                                                      C.byref(self.c_arrays), C.c_void_p(self.out.data_ptr()),
                                                      C.c_void_p(stream), waves)
        if rc != 0:
            raise RuntimeError(f"vp8g_decode_batch_device failed: {vp8g.gpu_lib().vp8g_last_error()!r}")

    def digests(self, stream: int) -> np.ndarray:
        """vp8g_frame_digests over every slot's output -> uint64[n] (synchronises the stream)."""
        lib = vp8g.gpu_lib()
        rc = lib.vp8g_frame_digests(self.h_descs, C.c_void_p(self.d_descs.data_ptr()), self.n,
                                    C.c_void_p(self.out.data_ptr()), C.c_void_p(self.digest_buf.data_ptr()),
                                    C.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"vp8g_frame_digests failed: {lib.vp8g_last_error()!r}")
        torch.cuda.synchronize(self.dev)
        return self.digest_buf.cpu().numpy().view(np.uint64).copy()

    def launch_mode(self) -> int:
        """VP8G_MODE_* bits of this thread's last launch (include/vp8g.h vp8g_last_launch_mode); -1 when
        the loaded library predates the symbol (an older build under VP8G_LIB)."""
        lib = vp8g.gpu_lib()
        if not hasattr(lib, "vp8g_last_launch_mode"):
            return -1
        return int(lib.vp8g_last_launch_mode())

    def status_word(self) -> int:
        return int(self.status[0].item())

    def frame_output(self, i: int) -> bytes:
        o = i * self.frame_bytes
        return self.out[o:o + self.i420].cpu().numpy().tobytes()
