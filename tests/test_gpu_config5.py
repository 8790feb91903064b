"""GPU: BASELINE configs[4] -- 4096 independent 3840x2160 keyframes sharded over 8 GPUs -- rehearsed
shard by shard on one GPU (verdict r04: "config 5 is not exercised").

Each of the eight ranks' shards is built by bench.py's own rank logic (`bench.Rank`, world size 8:
`vp8g_dist.shard_range`, the synthetic frames of global indices [lo, hi) seeded 0x5EED ^ i, the
parameter-block share with no process group), launched once through the timed entry point
(`vp8g_decode_batch_device`, the chain kernel bench.py times) and checked slot by slot against the
digests of the reference decoder's own output for all 4096 frames (tests/golden/digests.json,
tests/golden/make_digests.py).  What a node of eight MI355X adds on top -- one process per GPU,
the RCCL broadcast and the digest all-gather -- is covered with gloo (tests/test_dist.py,
tests/test_bench_ranks.py).  Reference path: src/m06_recon/vp8_recon.c:718 + m07 per frame.
"""
import json

import pytest
import torch

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def test_config5_all_eight_shards_every_frame():
    import sys
    sys.path.insert(0, str(ROOT))
    import bench
    golden = json.loads((GOLDEN / "digests.json").read_text())
    s = golden["synth_uhd"]
    assert len(s["yuvf"]) >= 4096
    args = bench.parse(["--workload", "synth", "--no-cpu-baseline"])
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    seen = []
    for rank in range(8):
        r = bench.Rank("synth", args, rank, 8, dev, golden, None)
        assert (r.lo, r.hi) == (512 * rank, 512 * (rank + 1))
        assert r.params_agree
        r.batch.status.zero_()
        r.batch.launch(stream)
        got = r.batch.digests(stream)
        assert r.batch.status_word() == 0
        bad = [r.lo + i for i in range(r.n) if "0x%016x" % int(got[i]) != r.expected_for(r.lo + i)]
        assert not bad, f"rank {rank}: {len(bad)} of {r.n} frames differ, e.g. {bad[:8]}"
        seen.append((r.lo, r.hi))
        for f in r.cpu_frames:
            f.free()
        del r
        torch.cuda.empty_cache()
    assert seen == [(512 * k, 512 * (k + 1)) for k in range(8)]
