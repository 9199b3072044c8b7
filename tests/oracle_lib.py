"""Test-side loader for the CPU oracle (oracle/liboracle_crc32c.so).

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() use this:
the oracle is the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_crc32c.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libref_crc32c.so")

APPEND_TYPE, MASK_OUTPUT = 0x1, 0x2


def build_oracle() -> None:
    src = os.path.join(ORACLE_DIR, "crc32c_oracle.c")
    if (not os.path.exists(ORACLE_SO)) or os.path.getmtime(src) > os.path.getmtime(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "oracle"], check=True)


class Oracle:
    def __init__(self, lib: ctypes.CDLL):
        self.lib = lib
        u32, u64, sz, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
        lib.oracle_extend.restype = u32
        lib.oracle_extend.argtypes = [u32, ctypes.c_char_p, sz]
        lib.oracle_value.restype = u32
        lib.oracle_value.argtypes = [ctypes.c_char_p, sz]
        lib.oracle_mask.restype = u32
        lib.oracle_mask.argtypes = [u32]
        lib.oracle_unmask.restype = u32
        lib.oracle_unmask.argtypes = [u32]
        lib.oracle_batch.restype = None
        lib.oracle_batch.argtypes = [vp, vp, vp, vp, vp, sz, u32]
        lib.oracle_batch_strided.restype = None
        lib.oracle_batch_strided.argtypes = [vp, u64, u32, sz, vp, vp, u32]
        lib.oracle_batch_strided_mt.restype = ctypes.c_int
        lib.oracle_batch_strided_mt.argtypes = [vp, u64, u32, sz, vp, ctypes.c_int, ctypes.c_int]
        lib.oracle_trailer.restype = None
        lib.oracle_trailer.argtypes = [ctypes.c_char_p, sz, ctypes.c_uint8, ctypes.c_int, vp]
        lib.oracle_verify.restype = ctypes.c_int
        lib.oracle_verify.argtypes = [ctypes.c_char_p, sz]
        lib.oracle_fill_splitmix64.restype = None
        lib.oracle_fill_splitmix64.argtypes = [vp, sz, u64, u64]
        lib.oracle_log_write.restype = None
        lib.oracle_log_write.argtypes = [vp]
        lib.oracle_log_verify.restype = ctypes.c_int
        lib.oracle_log_verify.argtypes = [vp]
        lib.oracle_xor_parity.restype = None
        lib.oracle_xor_parity.argtypes = [vp, vp, sz, sz, vp]
        lib.oracle_tables.restype = None
        lib.oracle_tables.argtypes = [vp, vp]
        lib.oracle_batch_mt.restype = ctypes.c_int
        lib.oracle_batch_mt.argtypes = [vp, vp, vp, vp, vp, sz, u32, ctypes.c_int]
        lib.oracle_log_check.restype = ctypes.c_int
        lib.oracle_log_check.argtypes = [vp, u64, u64]
        lib.oracle_dbbench_crc32c.restype = u32
        lib.oracle_dbbench_crc32c.argtypes = [ctypes.c_int64]

    def batch_mt(self, buf: np.ndarray, offsets, lengths, init=None, flags: int = 0,
                 threads: int = 16) -> np.ndarray:
        """oracle_batch on `threads` host threads (full-size batches)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
        out = np.empty(len(off), dtype=np.uint32)
        self.lib.oracle_batch_mt(buf.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                 None if ini is None else ini.ctypes.data, out.ctypes.data,
                                 len(off), flags, threads)
        return out

    def log_check(self, buf: np.ndarray, rec_offsets, buf_len=None) -> np.ndarray:
        """db/log_reader.cc:196-262 per record: 1 ok, 0 checksum mismatch,
        2 bad record length, 3 zero record (skipped), 4 cut by end of file."""
        n = buf.size if buf_len is None else buf_len
        return np.array([self.lib.oracle_log_check(buf.ctypes.data, n, int(o))
                         for o in rec_offsets], dtype=np.uint8)

    def extend(self, init: int, data: bytes) -> int:
        return self.lib.oracle_extend(init & 0xFFFFFFFF, data, len(data))

    def value(self, data: bytes) -> int:
        return self.lib.oracle_value(data, len(data))

    def mask(self, c: int) -> int:
        return self.lib.oracle_mask(c)

    def unmask(self, c: int) -> int:
        return self.lib.oracle_unmask(c)

    def batch(self, buf: np.ndarray, offsets, lengths, init=None, flags: int = 0) -> np.ndarray:
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
        out = np.empty(len(off), dtype=np.uint32)
        self.lib.oracle_batch(buf.ctypes.data, off.ctypes.data, ln.ctypes.data,
                              None if ini is None else ini.ctypes.data, out.ctypes.data,
                              len(off), flags)
        return out

    def batch_strided(self, buf: np.ndarray, stride: int, length: int, n: int, init=None,
                      flags: int = 0) -> np.ndarray:
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
        out = np.empty(n, dtype=np.uint32)
        self.lib.oracle_batch_strided(buf.ctypes.data, stride, length, n,
                                      None if ini is None else ini.ctypes.data,
                                      out.ctypes.data, flags)
        return out

    def batch_strided_mt(self, buf: np.ndarray, stride: int, length: int, n: int,
                         threads: int, reps: int = 1) -> np.ndarray:
        out = np.empty(n, dtype=np.uint32)
        self.lib.oracle_batch_strided_mt(buf.ctypes.data, stride, length, n, out.ctypes.data,
                                         threads, reps)
        return out

    def trailer(self, block: bytes, type_byte: int, tb_quirk: bool) -> bytes:
        out = (ctypes.c_uint8 * 5)()
        self.lib.oracle_trailer(block, len(block), type_byte, 1 if tb_quirk else 0,
                                ctypes.addressof(out))
        return bytes(out)

    def verify(self, record: bytes) -> bool:
        return bool(self.lib.oracle_verify(record, len(record) - 5))

    def splitmix64(self, nbytes: int, seed: int, first_word: int = 0) -> np.ndarray:
        out = np.empty(nbytes, dtype=np.uint8)
        self.lib.oracle_fill_splitmix64(out.ctypes.data, nbytes, seed, first_word)
        return out

    def log_write(self, buf: np.ndarray, rec_offsets) -> None:
        for o in rec_offsets:
            self.lib.oracle_log_write(buf.ctypes.data + int(o))

    def log_verify(self, buf: np.ndarray, rec_offsets) -> np.ndarray:
        return np.array([self.lib.oracle_log_verify(buf.ctypes.data + int(o))
                         for o in rec_offsets], dtype=np.uint8)

    def xor_parity(self, buf: np.ndarray, frag_offsets, parity_len: int) -> np.ndarray:
        fo = np.ascontiguousarray(frag_offsets, dtype=np.uint64)
        out = np.empty(parity_len, dtype=np.uint8)
        self.lib.oracle_xor_parity(buf.ctypes.data, fo.ctypes.data, len(fo), parity_len,
                                   out.ctypes.data)
        return out

    def tables(self):
        bt = np.empty(256, dtype=np.uint32)
        st = np.empty((4, 256), dtype=np.uint32)
        self.lib.oracle_tables(bt.ctypes.data, st.ctypes.data)
        return bt, st


_cache = None


def load_oracle() -> Oracle:
    global _cache
    if _cache is None:
        build_oracle()
        _cache = Oracle(ctypes.CDLL(ORACLE_SO))
    return _cache


def log_reader_case(oracle, case):
    """A tests/golden/log_reader_cases.json case rebuilt with the ORACLE's CRC
    (oracle/gen_log_cases.py used the reference's): (image, offsets, expected
    statuses).  The image must hash to the fixture's SHA-256."""
    import hashlib
    from novalsm_amd.synth import big_string, log_case_image

    writes = []
    for w in case["writes"]:
        if w[0] == "lit":
            writes.append(w[1].encode())
        elif w[0] == "big":
            writes.append(big_string(w[1].encode(), w[2]))
        else:  # "numbers": NumberString(i), db/log_test.cc:29-33
            writes.extend(f"{i}.".encode() for i in range(w[1]))
    img, offs = log_case_image(writes, case["edits"],
                               lambda b: oracle.mask(oracle.value(b)))
    assert hashlib.sha256(img.tobytes()).hexdigest() == case["sha256"], case["name"]
    assert img.size == case["buf_len"], case["name"]
    offsets = [int(x) for x in offs] + [int(x) for x in case["probes"]]
    if case["offsets"] is not None:
        assert offsets == case["offsets"], case["name"]
    expect = case["expect"] if case["expect"] is not None else [case["expect_all"]] * len(offsets)
    assert len(expect) == case["n_records"] == len(offsets)
    return img, np.array(offsets, np.uint64), np.array(expect, np.uint8)
