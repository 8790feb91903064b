#!/usr/bin/env python3
"""Benchmark: megapixels/s of filtered I420 decode (m06 recon + m07 loop filter, `-yuvf`
semantics) on a batch of 512 independent 3840x2160 key frames per GPU (BASELINE.json configs[3];
configs[4] = the same per GPU, sharded over 8 GPUs).

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 it is launched by
torch.distributed.run, one rank per GPU.  A "step" = one launch of the fused kernel over the whole
per-GPU batch (512 frames), inputs already resident in HBM.  Timed region: barrier + sync, K
steps, sync + barrier; the max over ranks is taken; value = all frames of all ranks x 8.2944 MP /
that time.  Rank 0 prints one JSON line.

Inputs: the 4 distinct 4K libwebp-encoded fixtures (tests/fixtures/big/uhd_*.webp; normal and
simple filter, sharpness 0-6, 1 or 4 segments) are entropy-decoded once on the host by the C11
front end; slot i of the batch is a separate HBM copy of fixture i % 4 (512 x 26.6 MB >> the
256 MB Infinity Cache, so no cache inflation).  Correctness: after timing, 4 slots are copied
back and compared with the reference decoder's sha256 from tests/golden/manifest.json.

roofline: the kernel is HBM-bound (8-bit integer stencils, no MFMA).  Algorithmic bytes per
launch = MBs x 820 B (800 B int16 coefficients + 20 B side info); the achieved
rate uses the average kernel duration measured with HIP events on the launch stream.  `traffic`
(PMC HBM bytes) comes from the rocprofv3 FETCH_SIZE/WRITE_SIZE pass committed under profiles/
(see DESIGN.md §5), or null when that file is absent.

cpu_baseline (rank 0, N = 1 only): the reference's own m06+m07 (oracle/_ref/libref.so, compiled
from the reference sources) when present, else our C restatement (oracle/liboracle.so), timed on
a bounded sample of the same 4K frames with one frame per thread on 16 host threads.
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import pathlib
import sys
import time

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))
import vp8g  # noqa: E402
import vp8g_dist  # noqa: E402

FIXTURES = [
    "big/uhd_a_normal_seg4.webp",
    "big/uhd_b_simple_sharp3.webp",
    "big/uhd_c_normal_sharp6_seg1.webp",
    "big/uhd_d_normal_q90.webp",
]
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
TRAFFIC_FILE = ROOT / "profiles" / "traffic_4k_batch.json"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=512, help="frames per GPU (config 4: 512)")
    ap.add_argument("--unfiltered", action="store_true", help="-yuv semantics (m06 only)")
    ap.add_argument("--waves", type=int, default=0, help="waves per frame workgroup (0 = default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--e2e-frames", type=int, default=256,
                    help="frames of the end-to-end object (.webp bytes -> I420, vp8g_decode_webp_batch); 0 = off")
    ap.add_argument("--e2e-device-frames", type=int, default=1024,
                    help="frames of its device-m05 leg (VP8G_BATCH_DEVICE_M05: m05 on the device, one workgroup "
                         "per frame, so it wants a large batch); 0 = off")
    ap.add_argument("--encode", default="png", choices=["none", "rgb", "ppm", "png"],
                    help="also time the m08/m09 stage on the batch's output (secondary object 'encode')")
    return ap.parse_args()


class Batch:
    """Device-resident batch: the nine Vp8DecodedFrame arrays concatenated over frames."""

    def __init__(self, frames: list, n: int, filtered: bool, dev: torch.device):
        self.n = n
        mbs = [f.mb_total for f in frames]
        self.mb_per = mbs[0]
        assert all(m == self.mb_per for m in mbs)
        total = n * self.mb_per
        self.total_mb = total
        self.arrays = {}
        for name, dt, per in vp8g.FRAME_ARRAYS:
            if name == "skip_coeff":
                continue
            tdt = torch.int16 if dt == np.int16 else torch.uint8
            t = torch.empty(total * per, dtype=tdt, device=dev)
            view = t.view(n, self.mb_per * per)
            for k, f in enumerate(frames):
                src = torch.from_numpy(f.array(name).copy()).to(dev)
                view[k::len(frames)] = src  # slot i <- fixture i % K (separate HBM copies)
                del src
            self.arrays[name] = t
        self.frame_bytes = (vp8g.i420_size(frames[0].width, frames[0].height) + 255) // 256 * 256
        self.out = torch.empty(n * self.frame_bytes, dtype=torch.uint8, device=dev)
        self.status = torch.zeros(4, dtype=torch.int32, device=dev)
        descs = (vp8g.Vp8gFrameDesc * n)()
        for i in range(n):
            descs[i] = vp8g.make_desc(frames[i % len(frames)], filtered, i * self.mb_per, i * self.frame_bytes)
        self.h_descs = descs
        self.d_descs = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
        a = vp8g.Vp8gBatchArrays()
        for name in ("coeff_y", "coeff_u", "coeff_v", "coeff_y2", "ymode", "uv_mode", "segment_id", "has_coeff", "bmode"):
            setattr(a, name, self.arrays[name].data_ptr())
        a.src = None
        a.status = self.status.data_ptr()
        self.c_arrays = a

    def launch(self, stream, waves: int):
        rc = vp8g.gpu_lib().vp8g_decode_batch_device(self.h_descs, C.c_void_p(self.d_descs.data_ptr()), self.n,
                                                      C.byref(self.c_arrays), C.c_void_p(self.out.data_ptr()),
                                                      C.c_void_p(stream), waves)
        if rc != 0:
            raise RuntimeError(f"launch failed: {vp8g.gpu_lib().vp8g_last_error()!r}")

    def frame_output(self, i: int, w: int, h: int) -> bytes:
        o = i * self.frame_bytes
        return self.out[o:o + vp8g.i420_size(w, h)].cpu().numpy().tobytes()


class EncodeStage:
    """m08/m09 on the device: the batch's I420 outputs -> RGB / PPM / PNG files.
    Algorithmic bytes per frame: the I420 read once (w*h*1.5) + the file written."""

    def __init__(self, batch: "Batch", W: int, H: int, fmt: str, dev):
        cw, ch = (W + 1) // 2, (H + 1) // 2
        offs = [(i * batch.frame_bytes, i * batch.frame_bytes + W * H, i * batch.frame_bytes + W * H + cw * ch)
                for i in range(batch.n)]
        self.fmt = fmt
        self.descs, self.outs, total, spans = vp8g.make_enc_descs([(W, H)] * batch.n, fmt, offs)
        self.d_descs = torch.frombuffer(bytearray(bytes(self.descs)), dtype=torch.uint8).to(dev)
        self.out = torch.empty(total, dtype=torch.uint8, device=dev)
        self.work = torch.empty(vp8g.gpu_lib().vp8g_encode_workspace_size(spans), dtype=torch.uint8, device=dev)
        self.src = batch.out
        self.n = batch.n
        self.file_len = self.descs[0].file_len
        self.bytes = batch.n * (vp8g.i420_size(W, H) + self.file_len)

    def launch(self, stream):
        rc = vp8g.gpu_lib().vp8g_encode_batch_device(self.descs, C.c_void_p(self.d_descs.data_ptr()), self.n,
                                                      C.c_void_p(self.src.data_ptr()), C.c_void_p(self.out.data_ptr()),
                                                      C.c_void_p(self.work.data_ptr()), C.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"encode launch failed: {vp8g.gpu_lib().vp8g_last_error()!r}")

    def file(self, i: int) -> bytes:
        o = self.outs[i]
        return self.out[o:o + self.file_len].cpu().numpy().tobytes()


def end_to_end_device(manifest, n_frames, filtered, threads):
    """The same path with m05 on the device: host threads parse only the
    container and frame headers, the compressed payloads are uploaded, one workgroup per frame
    decodes modes + tokens, then the recon(+LF) kernel and D2H as before."""
    files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in FIXTURES]
    batch = [files[i % 4] for i in range(n_frames)]
    vp8g.gpu_decode_webp_batch(batch[:8], filtered, threads, device_m05=True)  # warm
    t = time.perf_counter()
    outs, st = vp8g.gpu_decode_webp_batch(batch, filtered, threads, device_m05=True)
    dt = vp8g.gpu_decode_webp_batch.seconds  # the C call: .webp bytes -> I420 images
    key = "yuvf_sha256" if filtered else "yuv_sha256"
    ok = all(s == 0 for s in st) and all(hashlib.sha256(outs[i]).hexdigest() == manifest["files"][FIXTURES[i % 4]][key]
                                         for i in range(n_frames))
    del outs
    return {"stage": "end to end with m05 on the device: .webp bytes in host memory -> I420 in host memory "
                     "(container + frame header on host threads; payload upload, m05 (one workgroup per frame), "
                     "recon+LF on the device; D2H)",
            "value": round(n_frames * 3840 * 2160 / 1e6 / dt, 1), "unit": "MP/s", "frames": n_frames,
            "threads": threads, "seconds": round(dt, 3),
            "parity": f"bit-exact vs reference ({n_frames} frames sha256)" if ok else "MISMATCH"}


def end_to_end(manifest, n_frames, filtered, threads):
    """SURVEY §8(f1) step 1 + §8(f2): whole decode from .webp bytes in host memory to I420 in host
    memory (vp8g_decode_webp_batch: threaded host m05 into the packed format, device expansion +
    recon(+LF), D2H), wall clock of one call; next to it the reference's own `decoder -yuvf`
    (oracle/_ref/decoder, one process per frame, `threads` at a time) on a sample of the same files."""
    files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in FIXTURES]
    batch = [files[i % 4] for i in range(n_frames)]
    vp8g.gpu_decode_webp_batch(batch[:8], filtered, threads)  # warm: device buffers, code objects
    t = time.perf_counter()
    outs, st = vp8g.gpu_decode_webp_batch(batch, filtered, threads)
    dt = vp8g.gpu_decode_webp_batch.seconds  # the C call: .webp bytes -> I420 images
    key = "yuvf_sha256" if filtered else "yuv_sha256"
    ok = all(s == 0 for s in st) and all(hashlib.sha256(outs[i]).hexdigest() == manifest["files"][FIXTURES[i % 4]][key]
                                         for i in range(min(8, n_frames)))
    mp = n_frames * 3840 * 2160 / 1e6
    obj = {"stage": "end to end: .webp bytes in host memory -> I420 in host memory (container, header, m05 on host "
                    "threads into the packed format; upload, expansion, recon+LF on the device; D2H)",
           "value": round(mp / dt, 1), "unit": "MP/s", "frames": n_frames, "threads": threads,
           "seconds": round(dt, 3), "parity": "bit-exact vs reference (8 frames sha256)" if ok else "MISMATCH",
           "reference_cli": None}
    dec = ROOT / "oracle" / "_ref" / "decoder"
    if dec.exists():
        import subprocess
        import tempfile
        from concurrent.futures import ThreadPoolExecutor
        n_ref = 8 * threads
        with tempfile.TemporaryDirectory() as td:
            src = [pathlib.Path(td) / f"f{i}.webp" for i in range(4)]
            for i in range(4):
                src[i].write_bytes(files[i])
            def one(i):
                r = subprocess.run([str(dec), "-yuvf" if filtered else "-yuv", str(src[i % 4]), str(pathlib.Path(td) / f"o{i}.yuv")],
                                   capture_output=True)
                (pathlib.Path(td) / f"o{i}.yuv").unlink(missing_ok=True)
                return r.returncode
            t = time.perf_counter()
            with ThreadPoolExecutor(threads) as ex:
                rcs = list(ex.map(one, range(n_ref)))
            rdt = time.perf_counter() - t
        if all(rc == 0 for rc in rcs):
            obj["reference_cli"] = {"value": round(n_ref * 3840 * 2160 / 1e6 / rdt, 1), "unit": "MP/s", "cores": threads,
                                    "sample": f"{n_ref} x `decoder -yuvf` (reference, one process per frame, {threads} at a "
                                              f"time), {rdt:.1f} s"}
    return obj


def cpu_baseline(frames, filtered, threads, seconds):
    kind = "reference" if vp8g.ref_available() else "port"
    # calibrate on one frame per thread, then size the sample for ~`seconds` of wall time
    t = vp8g.cpu_time_batch(frames, threads, threads, filtered, kind)
    if t <= 0:
        return None
    per = t / threads
    n = max(threads, int(seconds / per) // threads * threads)
    t = vp8g.cpu_time_batch(frames, n, threads, filtered, kind)
    if t <= 0:
        return None
    mp = n * frames[0].width * frames[0].height / 1e6
    return {"value": round(mp / t, 2), "unit": "MP/s", "cores": threads, "kind": kind,
            "sample": f"{n} x 3840x2160 frames (the 4 bench fixtures round-robin), one frame per thread, "
                      f"{'recon+LF (-yuvf)' if filtered else 'recon (-yuv)'} on pre-decoded input, {t:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    filtered = not args.unfiltered

    manifest = json.loads((ROOT / "tests" / "golden" / "manifest.json").read_text())
    frames = [vp8g.decode_file(ROOT / "tests" / "fixtures" / r) for r in FIXTURES]
    W, H = frames[0].width, frames[0].height
    batch = Batch(frames, args.frames, filtered, dev)
    # per-frame parameter blocks (dequant + loop-filter tables) are shared: rank 0's go to all
    vp8g_dist.share_frame_params(batch.d_descs, dist)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        batch.launch(stream.cuda_stream, args.waves)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    lib = vp8g.gpu_lib()
    stamps = hasattr(lib, "vp8g_debug_stamps")  # diagnostic build (VP8G_STAMPS) only
    if stamps:
        zero = (C.c_ulonglong * 16)()
        lib.vp8g_debug_stamps(zero, 1)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        evs[s][0].record(stream)
        batch.launch(stream.cuda_stream, args.waves)
        evs[s][1].record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    if int(batch.status[0].item()) != 0:
        raise RuntimeError("kernel reported a dependency-wait timeout")

    # parity spot check: 4 slots (one per fixture) vs the reference decoder's hashes; the
    # per-frame digests of all ranks are gathered (64 bits each, never pixels)
    key = "yuvf_sha256" if filtered else "yuv_sha256"
    outs = [batch.frame_output(i, W, H) for i in range(min(4, args.frames))]
    ok = all(hashlib.sha256(o).hexdigest() == manifest["files"][FIXTURES[i % 4]][key] for i, o in enumerate(outs))
    digests = torch.tensor([vp8g_dist.digest64(o) for o in outs], dtype=torch.int64, device=dev)
    all_digests = vp8g_dist.gather_frame_digests(digests, dist)
    ok = ok and bool((all_digests == all_digests[0]).all())  # every rank decoded the same fixtures alike
    elapsed, kern_ms, ok = vp8g_dist.reduce_timing(elapsed, kern_ms, ok, dist, dev)

    total_frames = args.frames * world
    mp = total_frames * W * H / 1e6
    value = mp * args.steps / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    bytes_read = batch.total_mb * vp8g.BYTES_READ_PER_MB
    bytes_written = args.frames * vp8g.i420_size(W, H)
    achieved = bytes_read / (kern_ms * 1e-3) / 1e9
    traffic = None
    if TRAFFIC_FILE.exists():
        tj = json.loads(TRAFFIC_FILE.read_text())
        if tj.get("frames") == args.frames and tj.get("filtered") == filtered:
            traffic = tj.get("hbm_bytes_per_launch")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(frames, filtered, args.cpu_threads, args.cpu_seconds)

    enc_obj = None
    if args.encode != "none" and filtered:
        enc = EncodeStage(batch, W, H, args.encode, dev)
        for _ in range(max(1, args.warmup)):
            enc.launch(stream.cuda_stream)
        torch.cuda.synchronize(dev)
        eevs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for s in range(args.steps):
            eevs[s][0].record(stream)
            enc.launch(stream.cuda_stream)
            eevs[s][1].record(stream)
        torch.cuda.synchronize(dev)
        enc_ms = sum(a.elapsed_time(b) for a, b in eevs) / args.steps
        fkey = {"ppm": "ppm_sha256", "png": "png_sha256"}.get(args.encode)
        if fkey:
            enc_ok = all(hashlib.sha256(enc.file(i)).hexdigest() == manifest["files"][FIXTURES[i % 4]][fkey]
                         for i in range(min(4, args.frames)))
        else:
            enc_ok = None
        enc_gbs = enc.bytes / (enc_ms * 1e-3) / 1e9
        enc_obj = {"stage": f"m08/m09 I420 -> {args.encode.upper()} files on the device (one launch over the batch"
                            + (" + checksum finish" if args.encode == "png" else "") + ")",
                   "kernel_ms_per_step": round(enc_ms, 3),
                   "value": round(args.frames * W * H / 1e6 / (enc_ms * 1e-3), 1), "unit": "MP/s",
                   "parity": None if enc_ok is None else ("bit-exact vs reference (4 slots sha256)" if enc_ok else "MISMATCH"),
                   "roofline": {"bound": "hbm", "achieved": round(enc_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                "frac": round(enc_gbs / PEAK_HBM_GBS, 4),
                                "algorithmic_bytes_per_launch": enc.bytes}}

    e2e = None
    if rank == 0 and world == 1 and args.e2e_frames > 0:
        e2e = end_to_end(manifest, args.e2e_frames, filtered, args.cpu_threads)
        if args.e2e_device_frames > 0:
            e2e["device_m05"] = end_to_end_device(manifest, args.e2e_device_frames, filtered, args.cpu_threads)

    stamp_shares = None
    if stamps:
        acc = (C.c_ulonglong * 16)()
        lib.vp8g_debug_stamps(acc, 1)
        tot = sum(acc[:8]) or 1
        names = ["residual+loads", "dep_wait", "borders", "recon", "save_ctx", "loopfilter", "store", "publish"]
        stamp_shares = {n: round(acc[i] / tot, 4) for i, n in enumerate(names)}
        stamp_shares["cycles_per_mb_per_wave"] = round(tot / (batch.total_mb * args.steps), 1)
    if rank == 0:
        line = {
            "metric": "megapixels/sec filtered I420 decode (4K keyframe batch)" if filtered else
                      "megapixels/sec unfiltered I420 decode (4K keyframe batch)",
            "value": round(value, 1),
            "unit": "MP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "4 libwebp-encoded 3840x2160 fixtures, host-entropy-decoded once, replicated to "
                    f"{args.frames} HBM slots per GPU (synthetic batch of real frames)",
            "config": {"workload": f"{args.frames} x 3840x2160 keyframes per GPU, recon+loop filter (-yuvf), "
                                   "inputs device-resident" if filtered else
                                   f"{args.frames} x 3840x2160 keyframes per GPU, recon only (-yuv)",
                       "frames_per_gpu": args.frames, "width": W, "height": H,
                       "parallelism": f"dp{world} (independent frames, no data-path collective)"},
            "parity": "bit-exact vs reference (4 slots sha256)" if ok else "MISMATCH",
            "kernel_ms_per_step": round(kern_ms, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                         "algorithmic_bytes_per_launch": bytes_read,
                         # SURVEY.md §8(d) secondary figure: read + written algorithmic bytes
                         "achieved_read_write": round((bytes_read + bytes_written) / (kern_ms * 1e-3) / 1e9, 1),
                         "binding_resource": "vector-instruction issue (VALU), see DESIGN.md §5"},
            "cpu_baseline": cpu,
        }
        if enc_obj:
            line["encode"] = enc_obj
        if e2e:
            line["end_to_end"] = e2e
        if stamp_shares:
            line["stamps"] = stamp_shares
        print(json.dumps(line), flush=True)
    for f in frames:
        f.free()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
