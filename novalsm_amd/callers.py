"""Native caller threads for the per-SSTable paths (libnova_sst_callers.so,
novalsm_amd/csrc/sst_callers.cpp): T host threads, each checksumming its own
device-resident SSTable image back to back -- through the persistent engine
(nova_sst_queue_*), the coalescing queue, or direct calls with a stream sync --
optionally beside one thread of plain calls (block verify, log verify, CRC
batch).  Used by bench.py's sst_engine secondary, tools/concurrent_sst.py and
the mixed-caller GPU test.  Results are checked natively, as the
sst_callers.cpp header states exactly: every verify call's mismatch count and
flags, the trailers' final image, every plain call's result; the returned dict
says whether all were right.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Optional

from . import build as _build

PATHS = {"direct": 0, "engine": 1, "queue": 2}

_lib: Optional[ctypes.CDLL] = None


class Plain(ctypes.Structure):
    _fields_ = [
        ("v_img", ctypes.c_void_p), ("v_offs", ctypes.c_void_p), ("v_lens", ctypes.c_void_p),
        ("v_n", ctypes.c_uint64), ("v_expect_ok", ctypes.c_void_p), ("v_expect_bad", ctypes.c_uint32),
        ("l_img", ctypes.c_void_p), ("l_len", ctypes.c_uint64), ("l_offs", ctypes.c_void_p),
        ("l_n", ctypes.c_uint64), ("l_expect", ctypes.c_void_p), ("l_expect_bad", ctypes.c_uint32),
        ("b_img", ctypes.c_void_p), ("b_offs", ctypes.c_void_p), ("b_lens", ctypes.c_void_p),
        ("b_n", ctypes.c_uint64), ("b_expect", ctypes.c_void_p), ("gap_us", ctypes.c_double)]


class Cfg(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int), ("threads", ctypes.c_int), ("blocks", ctypes.c_uint64),
                ("warm_s", ctypes.c_double), ("secs", ctypes.c_double), ("path", ctypes.c_int),
                ("seed", ctypes.c_uint64), ("plain", ctypes.POINTER(Plain))]


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        from . import crc32c as C
        C.load()  # the product library first (the callers library links it)
        if not os.path.exists(_build.CALLERS_LIB):
            raise ImportError(f"{_build.CALLERS_LIB} is not built (novalsm_amd.build.build())")
        L = ctypes.CDLL(_build.CALLERS_LIB)
        L.nova_callers_run.restype = ctypes.c_int
        L.nova_callers_run.argtypes = [ctypes.POINTER(Cfg), ctypes.c_char_p, ctypes.c_size_t]
        _lib = L
    return _lib


def run(op: str, threads: int, blocks: int, secs: float, path: str = "engine", warm_s: float = 0.3,
        seed: int = 1, plain: Optional[Plain] = None) -> dict:
    """One measured window; returns the harness's JSON as a dict (raises on a
    library error code)."""
    cfg = Cfg(0 if op == "verify" else 1, int(threads), int(blocks), float(warm_s), float(secs), PATHS[path],
              int(seed), ctypes.pointer(plain) if plain is not None else None)
    buf = ctypes.create_string_buffer(1 << 16)
    rc = load().nova_callers_run(ctypes.byref(cfg), buf, len(buf))
    out = json.loads(buf.value.decode()) if buf.value else {}
    if rc != 0:
        raise RuntimeError(f"nova_callers_run rc={rc}: {out}")
    return out
