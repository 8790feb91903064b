"""CPU: the end-to-end batch path's schedule (vp8g_plan_batch, host code only).

In device-m05 mode the heaviest payloads go to the host threads: the k heaviest, for the k that
minimises max(host time, device time) under the library's cost model; the worker threads take the
device frames first, then the host frames heaviest first.  Host-m05 mode keeps index order and
VP8G_HYBRID=0 keeps every frame on the device.  No device call is made.
"""
import ctypes as C

import pytest

from conftest import FIXTURES

UHD = ["big/uhd_a_normal_seg4.webp", "big/uhd_b_simple_sharp3.webp", "big/uhd_c_normal_sharp6_seg1.webp",
       "big/uhd_d_normal_q90.webp"]


def plan(vp8g, files, threads, flags):
    lib = C.CDLL(str(vp8g.LIB_DIR / "libvp8g.so"), use_errno=True)
    n = len(files)
    bufs = [(C.c_uint8 * len(b)).from_buffer_copy(b) for b in files]
    spans = (vp8g.ByteSpan * n)(*[vp8g.ByteSpan(C.cast(bufs[i], C.POINTER(C.c_uint8)), len(files[i])) for i in range(n)])
    dev = (C.c_uint8 * n)()
    order = (C.c_uint32 * n)()
    assert lib.vp8g_plan_batch(spans, n, threads, flags, dev, order) == 0
    return list(dev), list(order)


@pytest.fixture(scope="module")
def uhd():
    return [(FIXTURES / r).read_bytes() for r in UHD]


def check_invariants(files, dev, order):
    n = len(files)
    assert sorted(order) == list(range(n))  # a permutation
    nd = sum(dev)
    assert all(dev[i] for i in order[:nd]) and not any(dev[i] for i in order[nd:])  # device frames first
    assert order[:nd] == sorted(order[:nd])  # in index order
    host_sizes = [len(files[i]) for i in order[nd:]]
    assert host_sizes == sorted(host_sizes, reverse=True)  # heaviest first
    if nd and nd < n:  # every host frame is at least as heavy as every device frame
        assert min(host_sizes) >= max(len(files[i]) for i in order[:nd])


def test_host_mode_keeps_index_order(vp8g, uhd):
    files = [uhd[i % 4] for i in range(64)]
    dev, order = plan(vp8g, files, 16, 0)
    assert dev == [0] * 64 and order == list(range(64))


@pytest.mark.parametrize("n,all_host,none_host", [(1024, {3}, {0, 1, 2}), (256, {1, 3}, {0})])
def test_device_mode_sends_heaviest_to_host(vp8g, uhd, monkeypatch, n, all_host, none_host):
    """4 bench fixtures round-robin (uhd_d 1.9 MB > uhd_b 0.84 MB > uhd_c 0.579 MB > uhd_a 0.576 MB):
    1024 frames on 16 threads -> exactly the 256 uhd_d on the host; 256 frames -> every uhd_d and
    uhd_b and, as the device's download shrinks with each frame moved, some uhd_c."""
    monkeypatch.delenv("VP8G_HYBRID", raising=False)
    for k in ("VP8G_HOST_NS_PER_BYTE", "VP8G_DEV_NS_PER_BYTE", "VP8G_D2H_NS_PER_BYTE"):
        monkeypatch.delenv(k, raising=False)
    files = [uhd[i % 4] for i in range(n)]
    dev, order = plan(vp8g, files, 16, 1)
    check_invariants(files, dev, order)
    host = [i % 4 for i in range(n) if not dev[i]]
    for f in all_host:
        assert host.count(f) == n // 4
    assert not set(host) & none_host


def test_hybrid_off_and_cost_knobs(vp8g, uhd, monkeypatch):
    files = [uhd[i % 4] for i in range(128)]
    monkeypatch.setenv("VP8G_HYBRID", "0")
    dev, order = plan(vp8g, files, 16, 1)
    assert dev == [1] * 128 and order == list(range(128))
    monkeypatch.setenv("VP8G_HYBRID", "1")
    monkeypatch.setenv("VP8G_HOST_NS_PER_BYTE", "1e9")  # host threads hopelessly slow: all on the device
    dev, _ = plan(vp8g, files, 16, 1)
    assert dev == [1] * 128
    monkeypatch.setenv("VP8G_HOST_NS_PER_BYTE", "0.001")  # host threads free: all on the host
    dev, order = plan(vp8g, files, 16, 1)
    assert dev == [0] * 128
    check_invariants(files, dev, order)


def test_unparsable_frames_and_errors(vp8g, uhd):
    files = [uhd[3], b"not a webp file at all", uhd[0]]
    dev, order = plan(vp8g, files, 4, 1)
    check_invariants(files, dev, order)
    lib = C.CDLL(str(vp8g.LIB_DIR / "libvp8g.so"), use_errno=True)
    dev_b = (C.c_uint8 * 1)()
    order_b = (C.c_uint32 * 1)()
    C.set_errno(0)
    assert lib.vp8g_plan_batch(None, 1, 4, 1, dev_b, order_b) == -1 and C.get_errno() == 22
