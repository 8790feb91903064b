"""Multi-rank logic of the batch decoder on CPU (gloo, world_size 2): sharding covers every frame
exactly once, rank 0's frame parameters reach every rank, digests are gathered in rank order and
timings reduce to the max (the contract bench.py relies on for N > 1)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import vp8g_dist as vd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_total = 1031
        lo, hi = vd.shard_range(n_total, rank, world)
        # parameter blocks: rank-dependent garbage before the broadcast
        desc = torch.full((4 * 176,), rank + 7, dtype=torch.uint8)
        vd.share_frame_params(desc, dist)
        dig = torch.tensor([vd.digest64(bytes([rank, i])) for i in range(3)], dtype=torch.int64)
        allg = vd.gather_frame_digests(dig, dist)
        t = vd.reduce_timing(1.0 + rank, 10.0 * (rank + 1), rank != 1, dist, "cpu")
        q.put((rank, lo, hi, int(desc.min()), int(desc.max()), allg.tolist(), t))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 512, 4096, 4097):
        for world in (1, 2, 3, 8):
            spans = [vd.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        vd.shard_range(8, 2, 2)


def test_single_process_passthrough():
    d = torch.arange(5, dtype=torch.int64)
    assert vd.gather_frame_digests(d, None).shape == (1, 5)
    assert vd.reduce_timing(1.5, 2.5, True, None, "cpu") == (1.5, 2.5, True)


def test_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, mn0, mx0, g0, t0), (r1, lo1, hi1, mn1, mx1, g1, t1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 516, 516, 1031)
    assert mn0 == mx0 == mn1 == mx1 == 7  # rank 0's block everywhere
    expect = [[vd.digest64(bytes([r, i])) for i in range(3)] for r in range(world)]
    assert g0 == g1 == expect
    assert t0 == t1 == (2.0, 20.0, False)  # max time; rank 1 reported a parity failure
