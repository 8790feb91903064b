"""Multi-partition fixtures, made on the fly from the corpus by the test-only
generator oracle/librepart.so (oracle/vp8_repartition.c): the same key frame with its tokens
re-encoded over 2 / 4 / 8 partitions, so its decoded output must equal the original's."""
import ctypes as C

from conftest import ROOT

_lib = None


def repart_lib():
    global _lib
    if _lib is None:
        path = ROOT / "oracle" / "librepart.so"
        if not path.exists():
            raise RuntimeError("oracle/librepart.so missing: run make")
        _lib = C.CDLL(str(path), use_errno=True)
        _lib.vp8_repartition.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_size_t]
        _lib.vp8_repartition.restype = C.c_long
    return _lib


def repartition(data: bytes, log2k: int) -> bytes:
    out = (C.c_uint8 * (2 * len(data) + 4096))()
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    n = repart_lib().vp8_repartition(buf, len(data), log2k, out, len(out))
    if n <= 0:
        raise ValueError(f"vp8_repartition failed: errno {C.get_errno()}")
    return bytes(out[:n])
