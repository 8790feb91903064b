#!/usr/bin/env python3
"""Benchmark: megapixels/s of filtered I420 decode (m06 recon + m07 loop filter, `-yuvf`
semantics) on batches of independent key frames, inputs resident in HBM (BASELINE.json
configs[3]: 512 x 3840x2160 per GPU; configs[4]: the same per GPU over 8 GPUs).

Contract (driver): `python bench.py --gpus N --steps K --warmup W`.  For N > 1 the driver launches
it under torch.distributed.run (one rank per GPU, RANK / LOCAL_RANK / WORLD_SIZE from the env);
started by hand with --gpus N > 1 and no WORLD_SIZE, bench.py starts torch.distributed.run itself
as a child before touching the GPU and exits with its code.  WORLD_SIZE != --gpus is an error.

A "step" = one launch of the fused kernel over the rank's whole batch.  Timed region: barrier +
sync, K steps, sync + barrier; the max over ranks is taken; value = all frames of all ranks x MP per
frame x K / that time.  Rank 0 prints one JSON line.

Workloads (--workload; the headline is uhd4, the other two are reported beside it at N = 1):
  uhd4   512 x 3840x2160 per GPU: the 4 libwebp-encoded 4K fixtures (tests/fixtures/big/uhd_*),
         entropy-decoded once on the host; global slot i <- fixture i % 4, each slot its own HBM copy
         (512 x 26.6 MB >> the 256 MB Infinity Cache: no cache inflation).
  fhd4   2048 x 1920x1080 per GPU: the 4 1080p fixtures (tests/fixtures/big/fhd_*), same scheme.
  synth  512 x 3840x2160 per GPU, all distinct: vp8_synth.c profile 0 ("measured-like"), seed
         0x5EED ^ global frame index (SURVEY.md §8(d) second mode).
  uhd4_yuv  the uhd4 batch with -yuv semantics (m06 reconstruction only, no loop filter).
Parity: after timing, vp8g_frame_digests digests every slot's output on the device; every rank's
digests are gathered and compared with tests/golden/digests.json (the digest of the reference
decoder's own I420 for that input) -- every frame of every rank, no pixel copies.

roofline: HBM-bound (8-bit integer stencils, no MFMA).  Algorithmic bytes per launch = MBs x 820 B
(800 B int16 coefficients + 20 B side info); the achieved rate uses the median
kernel duration from HIP events recorded on the launch stream.  `traffic` = the PMC HBM bytes per
launch measured by rocprofv3 (profiles/traffic_4k_batch.json).

cpu_baseline (rank 0, N = 1 only): the reference's own m06+m07 (oracle/_ref/libref.so, compiled from
the reference sources) when present, else our C restatement (oracle/liboracle.so), on a bounded
sample of the same frames, one frame per thread, at all host cores (the affinity mask, SURVEY.md
§8(d)) and at the per-GPU CPU share (OMP_NUM_THREADS, 16 on the GPU box); the faster is `value`,
`cores` = min(threads, cgroup CPU quota) of that run (more threads than the quota time-share it);
median of 5 runs each.
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import pathlib
import statistics
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "webp-decoder_amd"))

UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
       "big/uhd_d_normal_q90.webp"]
FHD = ["big/fhd_normal_sharp5.webp", "big/fhd_simple_sharp3.webp", "big/fhd_c_normal_q85_seg4.webp",
       "big/fhd_d_normal_sharp2_seg1.webp"]
WORKLOADS = {
    "uhd4": {"kind": "fixtures", "fixtures": UHD, "width": 3840, "height": 2160, "frames": 512},
    "fhd4": {"kind": "fixtures", "fixtures": FHD, "width": 1920, "height": 1080, "frames": 2048},
    "synth": {"kind": "synth", "width": 3840, "height": 2160, "frames": 512, "seed": 0x5EED, "profile": 0},
    # (diagnostics, not reported: synthetic 1280x720 frames, small enough for two chain workgroups per CU
    # with LDS context -- the occupancy experiment of DESIGN.md §5; outputs compared across builds)
    "synth720": {"kind": "synth", "width": 1280, "height": 720, "frames": 2048, "seed": 0x5EED, "profile": 0, "diagnostic": True},
    # BASELINE configs[1] semantics (-yuv, m06 only: no loop filter) on the uhd4 batch
    "uhd4_yuv": {"kind": "fixtures", "fixtures": UHD, "width": 3840, "height": 2160, "frames": 512, "unfiltered": True},
}
FIXTURES = UHD  # (back-compat name used by tools/)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
E2E_REPS = 3  # end-to-end legs: median of this many calls (host page-cache and allocator state vary call to call)
# measured HBM traffic per launch (rocprofv3 PMC passes, tools/profile_round.sh + traffic_summary.py)
TRAFFIC_FILES = {"uhd4": ROOT / "profiles" / "traffic_4k_batch.json", "synth": ROOT / "profiles" / "traffic_synth_batch.json"}
TRAFFIC_FILE = TRAFFIC_FILES["uhd4"]
# the committed PMC summary of the shipped kernel on uhd4 (tools/pmc_pass.sh + pmc_json.py): the
# instruction mix quoted in roofline.binding_resource comes from it, not from this run
PMC_FILE = ROOT / "profiles" / "r06fin_quad_kernel_pmc.json"


def binding_resource() -> str:
    """What limits the kernel, from the committed profiles (not from this run): the PMC instruction mix
    (PMC_FILE) and the HBM traffic ratio (TRAFFIC_FILE), each named with its source."""
    parts = ["latency-bound issue at 4 waves per SIMD (quad chain kernel)"]
    try:
        pj = json.loads(PMC_FILE.read_text())
        pm = pj["per_mb"]
        tot = pm["valu"] + pm["salu"] + pm["lds"] + pm["branch"] + pm["vmem_rd"] + pm["vmem_wr"]
        shares = pj.get("wave_time_shares", {})
        parts.append(f"{tot:.0f} instructions / {pm['valu']:.0f} VALU per MB, wave time {100 * shares.get('active_inst_any', 0):.0f} % "
                     f"issuing / {100 * shares.get('wait_inst_any', 0):.0f} % waiting on a result ({PMC_FILE.name})")
    except (OSError, KeyError, ValueError):
        pass
    try:
        tj = json.loads(TRAFFIC_FILE.read_text())
        pm = tj["per_mb"]
        ratio = (pm["read"] + pm["write"]) / (pm["algorithmic_read"] + pm["algorithmic_write"])
        parts.append(f"HBM traffic {ratio:.2f}x algorithmic read + write ({TRAFFIC_FILE.name}; FETCH_SIZE counted x2, "
                     "the gfx950 correction calibrated by tools/ubench/fetch_calib.hip, DESIGN.md §5)")
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        pass
    return "; ".join(parts) + "; DESIGN.md §3.1, §5"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="uhd4", choices=sorted(WORKLOADS))
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU (0 = the workload's: 512 / 2048 / 512)")
    ap.add_argument("--extra", default="auto", choices=["auto", "none"],
                    help="auto: at N = 1 also measure the other workloads (reported under 'workloads')")
    ap.add_argument("--unfiltered", action="store_true", help="-yuv semantics (m06 only)")
    ap.add_argument("--waves", type=int, default=0, help="waves per frame workgroup (0 = default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all host cores for the CPU baseline (and the per-GPU share beside it)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length (all repeats)")
    ap.add_argument("--e2e-frames", type=int, default=256,
                    help="frames of the end-to-end object (.webp bytes -> I420, vp8g_decode_webp_batch); 0 = off")
    ap.add_argument("--e2e-device-frames", type=int, default=1024,
                    help="frames of its device-m05 leg (VP8G_BATCH_DEVICE_M05); 0 = off")
    ap.add_argument("--encode", default="png", choices=["none", "rgb", "ppm", "png"],
                    help="also time the m08/m09 stage on the uhd4 batch's output (secondary object 'encode')")
    return ap.parse_args(argv)


def relaunch_if_needed(args) -> None:
    """--gpus N > 1 without a torch.distributed.run parent: become that parent (no GPU touched yet)."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), str(pathlib.Path(__file__).resolve())]
        cmd += sys.argv[1:]
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.run(cmd, env=env).returncode)
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")


def cpu_share() -> int:
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit() and int(n) > 0:
        return int(n)
    return len(os.sched_getaffinity(0))


def cpu_model() -> str:
    try:
        for line in pathlib.Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def sync(dev) -> None:
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


# ---- batches -------------------------------------------------------------------------------

def synth_frames(lo: int, hi: int, wl: dict, threads: int):
    """Host-generated synthetic frames for global indices [lo, hi), in order (thread pool; ctypes
    releases the GIL)."""
    import vp8g
    from concurrent.futures import ThreadPoolExecutor
    threads = max(1, threads)
    with ThreadPoolExecutor(threads) as ex:
        for c in range(lo, hi, 2 * threads):  # bounded: at most 2 x threads frames in host memory
            yield from ex.map(lambda i: vp8g.synth_frame(wl["width"], wl["height"], wl["seed"] ^ i, wl["profile"]),
                              range(c, min(hi, c + 2 * threads)))


class Rank:
    """One rank's view of a workload: its contiguous shard [lo, hi) of the global batch, the device
    batch, the expected digests (None where unpinned) and the frames for the CPU baseline."""

    def __init__(self, name, args, rank, world, dev, golden, dist):
        import vp8g
        import vp8g_batch
        import vp8g_dist
        self.name, self.wl = name, WORKLOADS[name]
        wl = self.wl
        self.filtered = not (args.unfiltered or wl.get("unfiltered", False))
        key = "yuvf" if self.filtered else "yuv"
        n = args.frames or wl["frames"]
        self.lo, self.hi = vp8g_dist.shard_range(n * world, rank, world)
        self.n = self.hi - self.lo
        self.batch = vp8g_batch.DeviceBatch(self.n, wl["width"], wl["height"], dev)
        self.cpu_frames = []
        if wl["kind"] == "fixtures":
            frames = [vp8g.decode_file(ROOT / "tests" / "fixtures" / r) for r in wl["fixtures"]]
            k = len(frames)
            self.batch.replicate(frames, self.filtered, slot0=self.lo % k)
            g = [golden["fixtures"].get(r, {}).get(key) for r in wl["fixtures"]]
            self.expected_for = lambda i: g[i % k]
            self.param_index = [(self.lo + i) % k for i in range(self.n)]
            self.cpu_frames = frames
        else:
            gs = golden.get("synth_uhd", {})
            same = (gs.get("width"), gs.get("height"), gs.get("profile")) == (wl["width"], wl["height"], wl["profile"])
            pinned = gs.get(key, []) if same else []
            self.expected_for = lambda i: pinned[i] if i < len(pinned) else None
            for i, f in enumerate(synth_frames(self.lo, self.hi, wl, cpu_share())):
                self.batch.fill(i, f, self.filtered)
                if i < 16:
                    self.cpu_frames.append(f)  # distinct frames for the CPU baseline sample
                else:
                    f.free()
            self.param_index = [0] * self.n  # profile 0: one parameter set for the whole batch
        self.share_params(dist)
        self.batch.commit()

    def share_params(self, dist):
        """RCCL broadcast of rank 0's frame-parameter blocks (dequant factors + loop-filter table +
        flags per distinct input); every rank applies them to its slots."""
        import torch
        import vp8g
        import vp8g_dist
        k = max(self.param_index) + 1
        firsts = [self.param_index.index(j) if j in self.param_index else None for j in range(k)]
        tmpl = (vp8g.Vp8gFrameDesc * k)()
        for j, i in enumerate(firsts):
            if i is not None:
                tmpl[j] = self.batch.h_descs[i]
        dev = self.batch.dev
        t = torch.frombuffer(bytearray(bytes(tmpl)), dtype=torch.uint8).to(dev)
        vp8g_dist.share_frame_params(t, dist)
        tmpl = (vp8g.Vp8gFrameDesc * k).from_buffer_copy(t.cpu().numpy().tobytes())
        self.params_agree = True
        for i, j in enumerate(self.param_index):
            d = self.batch.h_descs[i]
            src = tmpl[j]
            self.params_agree &= bytes(d.dq) == bytes(src.dq) and bytes(d.lf) == bytes(src.lf) and d.flags == src.flags
            d.dq, d.lf, d.flags = src.dq, src.lf, src.flags


def timed(launch, steps, warmup, dist, dev):
    """Warmup, then K launches bracketed by barrier + sync on both sides.  Returns (wall seconds,
    per-step kernel ms from HIP events on the launch stream)."""
    import torch
    for _ in range(warmup):
        launch()
    sync(dev)
    if dist is not None:
        dist.barrier()
    sync(dev)
    cuda = dev.type == "cuda"
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)] if cuda else []
    stream = torch.cuda.current_stream(dev) if cuda else None
    walls = []
    t0 = time.perf_counter()
    for s in range(steps):
        if cuda:
            evs[s][0].record(stream)
        else:
            walls.append(time.perf_counter())
        launch()
        if cuda:
            evs[s][1].record(stream)
        else:
            walls[-1] = (time.perf_counter() - walls[-1]) * 1e3
    sync(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = [a.elapsed_time(b) for a, b in evs] if cuda else walls
    return elapsed, kern


def all_cores() -> int:
    """Every CPU this process may run on (the CPU baseline uses all host cores)."""
    return len(os.sched_getaffinity(0))


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max), None if unlimited."""
    try:
        q, p = pathlib.Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def _cpu_rate(frames, filtered, threads, seconds, repeats, kind):
    """Median MP/s of `repeats` runs of the CPU path at `threads`, sized to ~seconds in total."""
    import vp8g
    t = vp8g.cpu_time_batch(frames, threads, threads, filtered, kind)  # calibration, one frame per thread
    if t <= 0:
        return None
    per = t / threads
    n = max(threads, int(seconds / repeats / per) // threads * threads)
    rates, tot = [], 0.0
    for _ in range(repeats):
        t = vp8g.cpu_time_batch(frames, n, threads, filtered, kind)
        if t <= 0:
            return None
        rates.append(n * frames[0].width * frames[0].height / 1e6 / t)
        tot += t
    return statistics.median(rates), n, tot


def cpu_baseline(frames, filtered, threads, seconds, repeats=5, share=None):
    """The reference's m06+m07 (or our restatement) on `frames` round-robin, one frame per thread;
    median MP/s of `repeats` runs sized to ~seconds in total, at `threads` (all host cores by default)
    and, when it differs, at `share` (the per-GPU CPU share the box grants, OMP_NUM_THREADS).  The
    faster of the two is `value`; `cores` = the cores that measurement could use, min(threads, the
    cgroup CPU quota) -- more threads than the quota only time-share it; the other rides in `other`."""
    import vp8g
    kind = "reference" if vp8g.ref_available() else "port"
    quota = cgroup_cpu_quota()
    counts = [threads] + ([share] if share and share != threads else [])
    runs = []
    for t in counts:
        r = _cpu_rate(frames, filtered, t, seconds, repeats, kind)
        if r is not None:
            runs.append((t,) + r)
    if not runs:
        return None
    w, h = frames[0].width, frames[0].height

    def eff(t):
        return int(min(t, quota)) if quota else t

    def sample(t, n, tot):
        return (f"{repeats} x {n} {w}x{h} frames ({len(frames)} distinct, round-robin), one frame per thread, "
                f"{t} threads, {'recon+LF (-yuvf)' if filtered else 'recon (-yuv)'} on pre-decoded input, "
                f"median of {repeats}, {tot:.1f} s")
    best = max(runs, key=lambda x: x[1])
    obj = {"value": round(best[1], 2), "unit": "MP/s", "cores": eff(best[0]), "threads": best[0], "kind": kind,
           "host_cpus": all_cores(), "cgroup_cpu_quota": quota, "cpu_model": cpu_model(),
           "sample": sample(best[0], best[2], best[3])}
    others = [x for x in runs if x is not best]
    if others:
        obj["other"] = [{"value": round(x[1], 2), "cores": eff(x[0]), "threads": x[0], "sample": sample(x[0], x[2], x[3])}
                        for x in others]
    return obj


def run_workload(name, args, rank, world, dist, dev, golden, rank_factory=Rank):
    """Build the rank's batch, time it, check every frame's digest, reduce over ranks.  Returns the
    measurement object (complete on rank 0)."""
    import numpy as np
    import torch
    import vp8g
    import vp8g_dist
    r = rank_factory(name, args, rank, world, dev, golden, dist)
    stream = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
    lib = vp8g.gpu_lib() if dev.type == "cuda" else None
    stamps = lib is not None and hasattr(lib, "vp8g_debug_stamps")  # diagnostic build (VP8G_STAMPS) only
    if stamps:
        for _ in range(args.warmup):
            r.batch.launch(stream, args.waves)
        sync(dev)
        lib.vp8g_debug_stamps((C.c_ulonglong * 16)(), 1)
    elapsed, kern = timed(lambda: r.batch.launch(stream, args.waves), args.steps, 0 if stamps else args.warmup, dist, dev)
    status = r.batch.status_word()
    dig = r.batch.digests(stream)
    # every rank's digests reach rank 0 (64 bits per frame, never pixels); rank 0 checks each one
    # against the reference's digest for that global frame (shards are contiguous and equal)
    allg = vp8g_dist.gather_frame_digests(torch.from_numpy(dig.view(np.int64).copy()).to(dev), dist)
    flat = allg.cpu().numpy().reshape(-1).view(np.uint64)
    exp = [r.expected_for(i) for i in range(flat.size)]
    match = sum(1 for d, e in zip(flat, exp) if e is not None and int(d) == int(e, 16))
    pinned = sum(1 for e in exp if e is not None)
    ok = status == 0 and r.params_agree
    kern_ms = statistics.median(kern)
    elapsed, kern_ms, ok = vp8g_dist.reduce_timing(elapsed, kern_ms, ok, dist, dev)
    ok = ok and match == pinned and pinned > 0
    total_frames = int(flat.size)
    counts = (match, pinned)
    wl = r.wl
    W, H = wl["width"], wl["height"]
    mb_per = r.batch.mb_per
    bytes_read = r.n * mb_per * vp8g.BYTES_READ_PER_MB
    bytes_written = r.n * vp8g.i420_size(W, H)
    achieved = bytes_read / (kern_ms * 1e-3) / 1e9
    obj = {
        "value": round(total_frames * W * H / 1e6 * args.steps / elapsed, 1),
        "unit": "MP/s",
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "kernel_ms_per_step": round(kern_ms, 3),
        "kernel_ms_steps": [round(x, 3) for x in kern],
        "frames_per_gpu": r.n, "frames_total": total_frames, "width": W, "height": H,
        "parity": (f"bit-exact vs reference ({counts[0]}/{counts[1]} frames, on-device digests)" if ok
                   else f"MISMATCH ({counts[0]}/{counts[1]} frames match; status {status})"),
        "parity_ok": bool(ok),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                     "algorithmic_bytes_per_launch": bytes_read,
                     "achieved_read_write": round((bytes_read + bytes_written) / (kern_ms * 1e-3) / 1e9, 1)},
        "cpu_baseline": None,
        "_rank": r,
    }
    if stamps:
        acc = (C.c_ulonglong * 16)()
        lib.vp8g_debug_stamps(acc, 1)
        slots = [13, 10, 11, 0, 1, 2, 12, 3, 4, 5, 6, 7]  # (8, 9: the launch clocks)
        tot = sum(acc[i] for i in slots) or 1
        names = ["prefetch_wait", "side_info", "residual_dequant_iwht", "residual_idct_park_prefetch", "dep_wait", "borders",
                 "whole_block_prediction", "b_pred", "save_ctx", "loopfilter", "store", "publish"]
        obj["stamps"] = {k: round(acc[i] / tot, 4) for i, k in zip(slots, names)}
        obj["stamps"]["cycles_per_mb_per_wave"] = round(tot / (r.batch.total_mb * args.steps), 1)
    tf = TRAFFIC_FILES.get(name)
    if tf is not None and tf.exists():
        tj = json.loads(tf.read_text())
        if tj.get("frames") == r.n and tj.get("filtered") == r.filtered and tj.get("workload", "uhd4") == name:
            obj["roofline"]["traffic"] = tj.get("hbm_bytes_per_launch")
            obj["roofline"]["traffic_source"] = f"{tf.relative_to(ROOT)} ({tj.get('tag', tj.get('source', ''))})"
    if rank == 0 and world == 1 and not args.no_cpu_baseline and r.cpu_frames:
        secs = args.cpu_seconds if name == args.workload else args.cpu_seconds / 2
        obj["cpu_baseline"] = cpu_baseline(r.cpu_frames, r.filtered, args.cpu_threads or all_cores(), secs,
                                           share=None if args.cpu_threads else cpu_share())
    return obj


# ---- secondary objects (N = 1) ----------------------------------------------------------------

class EncodeStage:
    """m08/m09 on the device: the batch's I420 outputs -> RGB / PPM / PNG files.
    Algorithmic bytes per frame: the I420 read once (w*h*1.5) + the file written."""

    def __init__(self, batch, W: int, H: int, fmt: str, dev):
        import torch
        import vp8g
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
        import vp8g
        rc = vp8g.gpu_lib().vp8g_encode_batch_device(self.descs, C.c_void_p(self.d_descs.data_ptr()), self.n,
                                                      C.c_void_p(self.src.data_ptr()), C.c_void_p(self.out.data_ptr()),
                                                      C.c_void_p(self.work.data_ptr()), C.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"encode launch failed: {vp8g.gpu_lib().vp8g_last_error()!r}")

    def file(self, i: int) -> bytes:
        o = self.outs[i]
        return self.out[o:o + self.file_len].cpu().numpy().tobytes()


def encode_object(r: Rank, args, manifest, dev):
    import torch
    W, H = r.wl["width"], r.wl["height"]
    enc = EncodeStage(r.batch, W, H, args.encode, dev)
    stream = torch.cuda.current_stream(dev)
    _, kern = timed(lambda: enc.launch(stream.cuda_stream), args.steps, max(1, args.warmup), None, dev)
    enc_ms = statistics.median(kern)
    fkey = {"ppm": "ppm_sha256", "png": "png_sha256"}.get(args.encode)
    fix = r.wl["fixtures"]
    enc_ok = None
    if fkey:
        enc_ok = all(hashlib.sha256(enc.file(i)).hexdigest() == manifest["files"][fix[(r.lo + i) % len(fix)]][fkey]
                     for i in range(min(4, r.n)))
    enc_gbs = enc.bytes / (enc_ms * 1e-3) / 1e9
    return {"stage": f"m08/m09 I420 -> {args.encode.upper()} files on the device (one launch over the batch"
                     + (" + checksum finish" if args.encode == "png" else "") + ")",
            "kernel_ms_per_step": round(enc_ms, 3),
            "value": round(r.n * W * H / 1e6 / (enc_ms * 1e-3), 1), "unit": "MP/s",
            "parity": None if enc_ok is None else ("bit-exact vs reference (4 files sha256)" if enc_ok else "MISMATCH"),
            "roofline": {"bound": "hbm", "achieved": round(enc_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(enc_gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_launch": enc.bytes}}


def end_to_end_device(manifest, n_frames, filtered, threads):
    """The same path with m05 on the device: host threads parse only the
    container and frame headers, the compressed payloads are uploaded, one workgroup per frame
    decodes modes + tokens, then the recon(+LF) kernel and D2H as before."""
    import vp8g
    files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in UHD]
    batch = [files[i % 4] for i in range(n_frames)]
    vp8g.gpu_decode_webp_batch(batch[:8], filtered, threads, device_m05=True)  # warm
    key = "yuvf_sha256" if filtered else "yuv_sha256"
    runs, ok = [], True
    for rep in range(E2E_REPS):  # median of E2E_REPS calls; every call's output checked
        outs, st = vp8g.gpu_decode_webp_batch(batch, filtered, threads, device_m05=True)
        runs.append(vp8g.gpu_decode_webp_batch.seconds)  # the C call: .webp bytes -> I420 images
        ok = ok and all(s == 0 for s in st) and all(
            hashlib.sha256(outs[i]).hexdigest() == manifest["files"][UHD[i % 4]][key]
            for i in range(0, n_frames, 1 if rep == 0 else 16))  # first call: every frame; repeats: 1 in 16
        del outs
    dt = statistics.median(runs)
    return {"stage": "end to end with m05 on the device: .webp bytes in host memory -> I420 in host memory "
                     "(container + frame header on host threads; payload upload, m05 (one workgroup per frame), "
                     "recon+LF on the device; D2H; the heaviest frames' m05 on the host threads instead when that "
                     "finishes sooner)",
            "value": round(n_frames * 3840 * 2160 / 1e6 / dt, 1), "unit": "MP/s", "frames": n_frames,
            "threads": threads, "seconds": round(dt, 3), "seconds_runs": [round(x, 3) for x in runs],
            "parity": f"bit-exact vs reference ({n_frames} frames sha256; repeats sampled 1 in 16)" if ok else "MISMATCH"}


def end_to_end(manifest, n_frames, filtered, threads):
    """SURVEY §8(f1) step 1 + §8(f2): whole decode from .webp bytes in host memory to I420 in host
    memory (vp8g_decode_webp_batch: threaded host m05 into the packed format, device expansion +
    recon(+LF), D2H), wall clock of one call; next to it the reference's own `decoder -yuvf`
    (oracle/_ref/decoder, one process per frame, `threads` at a time) on a sample of the same files."""
    import vp8g
    files = [(ROOT / "tests" / "fixtures" / r).read_bytes() for r in UHD]
    batch = [files[i % 4] for i in range(n_frames)]
    vp8g.gpu_decode_webp_batch(batch[:8], filtered, threads)  # warm: device buffers, code objects
    key = "yuvf_sha256" if filtered else "yuv_sha256"
    runs, ok = [], True
    for rep in range(E2E_REPS):  # median of E2E_REPS calls; every call's output checked
        outs, st = vp8g.gpu_decode_webp_batch(batch, filtered, threads)
        runs.append(vp8g.gpu_decode_webp_batch.seconds)  # the C call: .webp bytes -> I420 images
        ok = ok and all(s == 0 for s in st) and all(
            hashlib.sha256(outs[i]).hexdigest() == manifest["files"][UHD[i % 4]][key]
            for i in range(0, n_frames, 1 if rep == 0 else 16))  # first call: every frame; repeats: 1 in 16
        del outs
    dt = statistics.median(runs)
    mp = n_frames * 3840 * 2160 / 1e6
    obj = {"stage": "end to end: .webp bytes in host memory -> I420 in host memory (container, header, m05 on host "
                    "threads into the packed format; upload, expansion, recon+LF on the device; D2H)",
           "value": round(mp / dt, 1), "unit": "MP/s", "frames": n_frames, "threads": threads,
           "seconds": round(dt, 3), "seconds_runs": [round(x, 3) for x in runs],
           "parity": f"bit-exact vs reference ({n_frames} frames sha256; repeats sampled 1 in 16)" if ok else "MISMATCH",
           "reference_cli": None}
    dec = ROOT / "oracle" / "_ref" / "decoder"
    if dec.exists():
        # the reference's own CLI, one process per frame: at the per-GPU share and on all host cores
        obj["reference_cli"] = reference_cli(dec, files, filtered, threads, 8)
        if all_cores() != threads:
            obj["reference_cli_all_cores"] = reference_cli(dec, files, filtered, all_cores(), 2)
    return obj


def reference_cli(dec, files, filtered, threads, per_thread):
    """`decoder -yuvf` of the reference (oracle/_ref/decoder), one process per 4K frame, `threads` at a
    time, `per_thread` frames per thread (bounded sample); MP/s over the wall clock."""
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    n_ref = per_thread * threads
    with tempfile.TemporaryDirectory() as td:
        src = [pathlib.Path(td) / f"f{i}.webp" for i in range(len(files))]
        for p, b in zip(src, files):
            p.write_bytes(b)

        def one(i):
            o = pathlib.Path(td) / f"o{i}.yuv"
            rc = subprocess.run([str(dec), "-yuvf" if filtered else "-yuv", str(src[i % len(src)]), str(o)],
                                capture_output=True).returncode
            o.unlink(missing_ok=True)
            return rc
        t = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            rcs = list(ex.map(one, range(n_ref)))
        rdt = time.perf_counter() - t
    if not all(rc == 0 for rc in rcs):
        return None
    return {"value": round(n_ref * 3840 * 2160 / 1e6 / rdt, 1), "unit": "MP/s", "cores": threads,
            "cgroup_cpu_quota": cgroup_cpu_quota(),
            "sample": f"{n_ref} x `decoder -{'yuvf' if filtered else 'yuv'}` (reference, one process per frame, "
                      f"{threads} at a time), {rdt:.1f} s"}


def public(obj: dict) -> dict:
    return {k: v for k, v in obj.items() if not k.startswith("_")}


def main(argv=None):
    args = parse(argv)
    relaunch_if_needed(args)
    import torch
    import vp8g_dist  # noqa: F401
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    manifest = json.loads((ROOT / "tests" / "golden" / "manifest.json").read_text())
    golden = json.loads((ROOT / "tests" / "golden" / "digests.json").read_text())

    head = run_workload(args.workload, args, rank, world, dist, dev, golden)
    r = head["_rank"]
    extra = {}
    enc_obj = e2e = None
    if world == 1:
        if args.encode != "none" and r.filtered and r.wl["kind"] == "fixtures":
            enc_obj = encode_object(r, args, manifest, dev)
        threads = args.cpu_threads or cpu_share()
        if args.e2e_frames > 0:
            e2e = end_to_end(manifest, args.e2e_frames, r.filtered, threads)
            if args.e2e_device_frames > 0:
                # device-m05 mode (hybrid: the heaviest frames on the host threads) at the host leg's
                # batch size and at a full device chunk
                e2e["device_m05"] = end_to_end_device(manifest, args.e2e_frames, r.filtered, threads)
                if args.e2e_device_frames != args.e2e_frames:
                    e2e["device_m05_large"] = end_to_end_device(manifest, args.e2e_device_frames, r.filtered, threads)
    del head["_rank"], r
    torch.cuda.empty_cache()
    if world == 1 and args.extra == "auto":
        for name in WORKLOADS:
            if name != args.workload and not WORKLOADS[name].get("diagnostic"):
                o = run_workload(name, args, rank, world, dist, dev, golden)
                del o["_rank"]
                torch.cuda.empty_cache()
                extra[name] = public(o)
    if rank == 0:
        wl = WORKLOADS[args.workload]
        W, H = wl["width"], wl["height"]
        filtered = not args.unfiltered
        ok = head["parity_ok"] and all(o["parity_ok"] for o in extra.values())
        if wl["kind"] == "fixtures":
            data = (f"{len(wl['fixtures'])} libwebp-encoded {W}x{H} fixtures, host-entropy-decoded once, replicated to "
                    f"{head['frames_per_gpu']} HBM slots per GPU (synthetic batch of real frames)")
        else:
            data = f"{head['frames_per_gpu']} distinct synthetic {W}x{H} frames per GPU (vp8_synth.c profile 0)"
        line = {
            "metric": ("megapixels/sec filtered I420 decode (4K keyframe batch)" if filtered else
                       "megapixels/sec unfiltered I420 decode (4K keyframe batch)") if W == 3840 else
                      f"megapixels/sec {'filtered' if filtered else 'unfiltered'} I420 decode ({H}p keyframe batch)",
            "value": head["value"],
            "unit": "MP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": data,
            "config": {"workload": f"{args.workload}: {head['frames_per_gpu']} x {W}x{H} keyframes per GPU, "
                                   + ("recon+loop filter (-yuvf)" if filtered else "recon only (-yuv)")
                                   + ", inputs device-resident",
                       "frames_per_gpu": head["frames_per_gpu"], "width": W, "height": H,
                       "parallelism": f"dp{world} (independent frames, contiguous shards, no data-path collective)"},
            "parity": head["parity"],
            "kernel_ms_per_step": head["kernel_ms_per_step"],
            "kernel_ms_steps": head["kernel_ms_steps"],
            "roofline": dict(head["roofline"], binding_resource=binding_resource()),
            "cpu_baseline": head["cpu_baseline"],
        }
        if extra:
            line["workloads"] = extra
        if enc_obj:
            line["encode"] = enc_obj
        if e2e:
            line["end_to_end"] = e2e
        if "stamps" in head:
            line["stamps"] = head["stamps"]
        if not ok:
            line["parity_failure"] = True
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
