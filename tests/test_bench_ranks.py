"""bench.py's multi-rank logic on CPU (gloo, world size 2) with the GPU launch stubbed: contiguous
equal shards of the global batch, the broadcast of rank 0's frame-parameter blocks, the all-gather of
every frame's digest and rank 0's check of each one against the golden digest of its global index,
the max-over-ranks timing and the whole-job value (BASELINE configs[4])."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def expected_digest(i):
    return "0x%016x" % ((i * 0x9E3779B97F4A7C15 + 11) & ((1 << 64) - 1))


class StubBatch:
    def __init__(self, n, mb_per, lo, bad, dev):
        import vp8g
        self.n, self.mb_per, self.lo, self.bad, self.dev = n, mb_per, lo, bad, dev
        self.h_descs = (vp8g.Vp8gFrameDesc * n)()
        self.launches = 0

    def launch(self, stream, waves):
        self.launches += 1

    def status_word(self):
        return 0

    def digests(self, stream):
        d = np.array([int(expected_digest(self.lo + i), 16) for i in range(self.n)], dtype=np.uint64)
        if self.bad:
            d[3] ^= np.uint64(1)
        return d


class StubRank:
    """What bench.Rank provides, without a GPU: frames of param set (global index % 3)."""

    def __init__(self, name, args, rank, world, dev, golden, dist):
        import vp8g_dist
        self.name, self.wl, self.filtered = name, bench.WORKLOADS[name], True
        n = args.frames or self.wl["frames"]
        self.lo, self.hi = vp8g_dist.shard_range(n * world, rank, world)
        self.n = self.hi - self.lo
        self.batch = StubBatch(self.n, 32400, self.lo, rank == 1 and os.environ.get("STUB_BAD") == "1", dev)
        self.param_index = [(self.lo + i) % 3 for i in range(self.n)]
        for i, j in enumerate(self.param_index):
            d = self.batch.h_descs[i]
            garbage = rank == 1 and os.environ.get("STUB_BAD") == "1"  # the broadcast overwrites it
            d.dq[0][0] = 7 if garbage else 100 + j
            d.lf[1][0][1] = 9 if garbage else 50 + j
        bench.Rank.share_params(self, dist)
        self.expected_for = expected_digest
        self.cpu_frames = []


def _worker(rank, world, port, bad, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), STUB_BAD="1" if bad else "0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        args = bench.parse(["--gpus", "2", "--steps", "3", "--warmup", "1", "--frames", "8", "--no-cpu-baseline"])
        obj = bench.run_workload("uhd4", args, rank, world, dist, torch.device("cpu"), {}, rank_factory=StubRank)
        r = obj.pop("_rank")
        q.put((rank, r.lo, r.hi, r.batch.launches, r.params_agree,
               [(int(d.dq[0][0]), int(d.lf[1][0][1])) for d in r.batch.h_descs], bench.public(obj)))
    finally:
        dist.destroy_process_group()


def _run(bad):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_ranks_shard_broadcast_gather_reduce():
    (r0, lo0, hi0, n0, agree0, p0, o0), (r1, lo1, hi1, n1, agree1, p1, o1) = _run(bad=False)
    assert (lo0, hi0, lo1, hi1) == (0, 8, 8, 16)  # contiguous, equal shards of 2 x 8 frames
    assert n0 == n1 == 4  # warmup 1 + 3 timed launches per rank
    # rank 0's parameter block for each global frame reached rank 1
    assert p0 == [(100 + i % 3, 50 + i % 3) for i in range(8)]
    assert p1 == [(100 + i % 3, 50 + i % 3) for i in range(8, 16)]
    assert agree0 and agree1
    assert o0["frames_total"] == 16 and o0["frames_per_gpu"] == 8
    assert o0["parity"].startswith("bit-exact") and "16/16" in o0["parity"] and o0["parity_ok"]
    exp_value = 16 * 3840 * 2160 / 1e6 * 3 / (o0["ms_per_step"] * 3 / 1e3)
    assert o0["value"] == pytest.approx(exp_value, rel=2e-2)  # (ms_per_step is rounded)


def test_ranks_detect_bad_digest_and_disagreeing_params():
    res = _run(bad=True)
    (r0, lo0, hi0, n0, agree0, p0, o0), (r1, lo1, hi1, n1, agree1, p1, o1) = res
    assert agree0 and not agree1  # rank 1's own parameter blocks differed from rank 0's ...
    assert p1 == [(100 + i % 3, 50 + i % 3) for i in range(8, 16)]  # ... and were replaced by them
    assert "15/16" in o0["parity"] and o0["parity_ok"] is False


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit):
        bench.relaunch_if_needed(bench.parse(["--gpus", "1"]))
    monkeypatch.setenv("WORLD_SIZE", "1")
    bench.relaunch_if_needed(bench.parse(["--gpus", "1"]))  # consistent: returns


def test_gpus_n_without_launcher_starts_torchrun(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, env):
        seen["cmd"] = cmd
        return R()
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    with pytest.raises(SystemExit) as e:
        bench.relaunch_if_needed(bench.parse(["--gpus", "4", "--steps", "2"]))
    assert e.value.code == 0
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert "127.0.0.1" in cmd and cmd[-3:] == ["--gpus", "4", "--steps", "2"][-3:]
