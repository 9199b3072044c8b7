#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- generate tests/golden/crc32c_golden.json.

Every expected value in the fixture is produced by the REFERENCE's own
util/crc32c.cc, compiled unmodified into oracle/_ref/libref_crc32c.so
(``make -C oracle ref``; this container only -- /root/reference is absent on the
GPU box).  Inputs are small literals or splitmix64 streams (novalsm_amd/synth.py)
identified by (seed, byte offset, length), so the fixture holds data, not code.

Run:  make -C oracle && python oracle/gen_golden.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from novalsm_amd.synth import log_image, splitmix64_bytes  # noqa: E402

REF_SO = os.path.join(HERE, "_ref", "libref_crc32c.so")


def load_ref():
    lib = ctypes.CDLL(REF_SO)
    lib.ref_extend.restype = ctypes.c_uint32
    lib.ref_extend.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    lib.ref_value.restype = ctypes.c_uint32
    lib.ref_value.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    lib.ref_mask.restype = ctypes.c_uint32
    lib.ref_mask.argtypes = [ctypes.c_uint32]
    lib.ref_unmask.restype = ctypes.c_uint32
    lib.ref_unmask.argtypes = [ctypes.c_uint32]
    return lib


def main() -> None:
    ref = load_ref()

    def ext(init: int, b: bytes) -> int:
        return ref.ref_extend(init, b, len(b))

    out: dict = {"generator": "oracle/gen_golden.py via oracle/_ref/libref_crc32c.so "
                              "(reference util/crc32c.cc compiled unmodified, g++ -O2)"}

    # 1. util/crc32c_test.cc:14-46 RFC 3720 B.4 + self-test constant util/crc32c.cc:479-481
    iscsi = bytes([0x01, 0xc0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x14, 0, 0, 0, 0, 0,
                   0x04, 0, 0, 0, 0, 0x14, 0, 0, 0, 0x18, 0x28, 0, 0, 0, 0, 0, 0, 0, 0x02,
                   0, 0, 0, 0, 0, 0, 0])
    kat = [
        ("zeros32", bytes(32), 0x8a9136aa),
        ("ones32", b"\xff" * 32, 0x62a8ab43),
        ("inc32", bytes(range(32)), 0x46dd794e),
        ("dec32", bytes(range(31, -1, -1)), 0x113fdb5c),
        ("iscsi48", iscsi, 0xd9963a56),
        ("TestCRCBuffer", b"TestCRCBuffer", 0xdcbc59fa),
    ]
    out["known_answers"] = []
    for name, data, want in kat:
        got = ext(0, data)
        assert got == want, (name, hex(got), hex(want))
        out["known_answers"].append({"name": name, "hex": data.hex(), "crc": got})

    # 2. probe-derived goldens
    x4096 = b"x" * 4096
    v = ext(0, x4096)
    v_t = ext(v, b"\x00")
    m = ref.ref_mask(v_t)
    out["extra"] = {
        "check_123456789": ext(0, b"123456789"),
        "hello_world": ext(0, b"hello world"),
        "extend_hello_world": ext(ext(0, b"hello "), b"world"),
        "a": ext(0, b"a"),
        "foo": ext(0, b"foo"),
        "x4096_value": v,
        "x4096_type0": v_t,
        "x4096_mask": m,
    }
    assert out["extra"]["check_123456789"] == 0xe3069283
    assert out["extra"]["hello_world"] == out["extra"]["extend_hello_world"] == 0xc99465aa

    # 3. byte table pin: kByteExtensionTable[b] = Extend(~0, {b}, 1) ^ ~0
    out["byte_table"] = [ext(0xFFFFFFFF, bytes([b])) ^ 0xFFFFFFFF for b in range(256)]

    # 4. mask / unmask
    rng = np.random.default_rng(7)
    vals = [0, 1, 0xFFFFFFFF, 0x80000000, 0xa282ead8] + [int(x) for x in rng.integers(0, 2**32, 27)]
    out["mask"] = [{"crc": x, "mask": ref.ref_mask(x), "unmask": ref.ref_unmask(x)} for x in vals]

    # 5. single-buffer cases: every length 0..160 and edge lengths, at every
    # start misalignment 0..15, with zero and random init (Extend semantics).
    cases = []
    lengths = list(range(0, 161)) + [255, 256, 257, 1023, 1024, 1025, 4095, 4096, 4097, 4101,
                                     8191, 16384, 16389, 65536, 65536 + 63]
    seed = 11
    for li, n in enumerate(lengths):
        for off in ([0, 1, 3, 13] if n <= 160 else list(range(16))):
            init = 0 if (li + off) % 3 else int(rng.integers(0, 2**32))
            data = splitmix64_bytes(seed, n, off).tobytes()
            cases.append({"seed": seed, "offset": off, "length": n, "init": init,
                          "crc": ext(init, data)})
    out["cases"] = cases

    # 6. an SSTable-like packed buffer: blocks back-to-back with 5-byte trailers,
    # sizes jittered around LevelDB block_size classes (BASELINE config 3 shape).
    seed = 3
    sizes = []
    r = np.random.default_rng(3)
    for i in range(97):
        cls = [4096, 16384, 65536][int(r.integers(0, 3))] if i % 7 else int(r.integers(1, 600))
        sizes.append(cls + int(r.integers(0, 64)) + 1 if i % 7 else cls)
    offs, pos = [], 0
    for s in sizes:
        offs.append(pos)
        pos += s + 5
    total = pos
    buf = bytearray(splitmix64_bytes(seed, total).tobytes())
    crcs, tb, stoc = [], [], []
    for o, s in zip(offs, sizes):
        blk = bytes(buf[o:o + s])
        c = ext(0, blk)
        crcs.append(c)
        ct = ext(c, b"\x00")
        mm = ref.ref_mask(ct)
        enc = bytes([mm & 0xff, (mm >> 8) & 0xff, (mm >> 16) & 0xff, (mm >> 24) & 0xff])
        tb.append((b"\x00" + enc[:3] + b"!").hex())       # table/table_builder.cc:202-206
        stoc.append((b"\x00" + enc).hex())                # ltc/stoc_file_client_impl.cpp:714-719
    out["packed"] = {"seed": seed, "total": total, "offsets": offs, "sizes": sizes,
                     "crc": crcs, "tb_trailer_hex": tb, "stoc_trailer_hex": stoc}

    # 7. a write-ahead/MANIFEST log image as log::Writer::AddRecord lays it out
    # (db/log_writer.cc:53-97, novalsm_amd/synth.log_layout): 300 logical
    # records (a few longer than a 32 KiB block, so FIRST/MIDDLE/LAST
    # fragments and zero block trailers occur), each physical record's crc is
    # db/log_writer.cc:105-111: Mask(Extend(type_crc[t], payload, len)),
    # type_crc[t] = Value(&t, 1) (:16-21).
    r = np.random.default_rng(4)
    plens = []
    for i in range(300):
        if i % 11 == 0:
            plens.append(int(r.integers(0, 4)))
        elif i % 97 == 5:
            plens.append(int(r.integers(33000, 70000)))
        else:
            plens.append(int(r.integers(0, 3000)))
    logbuf, loffs, llens, ltypes = log_image(6, plens)
    log_crc = []
    for o, ln, t in zip(loffs.tolist(), llens.tolist(), ltypes.tolist()):
        c = ref.ref_mask(ext(ext(0, bytes([t])), logbuf[o + 7:o + 7 + ln].tobytes()))
        log_crc.append(c)
    out["log"] = {"seed": 6, "payload_lens": plens, "total": int(logbuf.size),
                  "records": [[o, ln, t] for o, ln, t in zip(loffs.tolist(), llens.tolist(),
                                                             ltypes.tolist())],
                  "header_crc": log_crc}

    # 8. BASELINE config 1 sample: 1024 x 4 KiB blocks, splitmix64 seed 1
    data = splitmix64_bytes(1, 1024 * 4096).tobytes()
    c1 = [ext(0, data[i * 4096:(i + 1) * 4096]) for i in range(1024)]
    out["config1"] = {"seed": 1, "n": 1024, "len": 4096, "crc": c1}

    path = os.path.join(ROOT, "tests", "golden", "crc32c_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {path}: {len(cases)} cases, {len(sizes)} packed blocks")


if __name__ == "__main__":
    main()
