#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- generate tests/golden/log_reader_cases.json.

The reference's own log reader tests (db/log_test.cc) as golden data for the
per-record statuses of nova_log_verify_records.  Each case
is the file a test writes with log::Writer (db/log_writer.cc:53-114), the edits
it makes to it (IncrementByte / SetByte / ShrinkSize / FixChecksum,
db/log_test.cc:76-97) and the physical records a reader's walk visits.  Its
expected statuses restate what that test asserts about ReadRecord's results,
the dropped bytes and the reported error (cited per case):

  OK (1)                 the record is returned (checksum good);
  CHECKSUM_MISMATCH (0)  "checksum mismatch" reported (db/log_reader.cc:251-260);
  BAD_LENGTH (2)         "bad record length" reported (:230-235);
  TRUNCATED (4)          the read ends at the end of the file without a report
                         (:204-211, :236-239);
  BLOCK_TRAILER (5)      fewer than 7 bytes left in a full block: skipped
                         silently (:198-203).
n_bad counts the reported ones.  Physical checks only: a record whose type a
test then rejects at the logical layer ("unknown record type", "missing
start") has a good checksum, status OK -- ReadRecord's fragment assembly is the
host walk's job.

The file bytes are pinned, not stored: each header CRC is computed by the
REFERENCE's util/crc32c.cc (oracle/_ref, compiled unmodified), and the fixture
keeps the SHA-256 of the final image; tests rebuild the image with the oracle's
CRC and must reproduce that hash.  The script also checks every expected status
against the oracle's ReadPhysicalRecord restatement (oracle_log_check).

Run:  make -C oracle oracle ref && python oracle/gen_log_cases.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from novalsm_amd.synth import LOG_BLOCK, LOG_HEADER, big_string, log_case_image  # noqa: E402
from oracle.gen_golden import load_ref  # noqa: E402

OK, MISMATCH, BAD_LENGTH, ZERO, TRUNCATED, TRAILER = 1, 0, 2, 3, 4, 5
kB, kH = LOG_BLOCK, LOG_HEADER


def payloads(spec):
    """Writes of a case: ["lit", s], ["big", partial, n] (BigString), ["numbers", count]
    (NumberString(i) for i < count, db/log_test.cc:29-33)."""
    out = []
    for w in spec:
        if w[0] == "lit":
            out.append(w[1].encode())
        elif w[0] == "big":
            out.append(big_string(w[1].encode(), w[2]))
        elif w[0] == "numbers":
            out.extend(f"{i}.".encode() for i in range(w[1]))
        else:
            raise ValueError(w)
    return out


# (name, db/log_test.cc lines, writes, edits, extra probe offsets, expected statuses
#  over the writer's records followed by the probes, n_bad)
CASES = [
    ("ReadWrite", "283-294", [["lit", "foo"], ["lit", "bar"], ["lit", ""], ["lit", "xxxx"]], [], [],
     [OK, OK, OK, OK], 0),
    ("ManyBlocks", "296-304", [["numbers", 100000]], [], [], None, 0),
    ("Fragmentation", "306-314", [["lit", "small"], ["big", "medium", 50000], ["big", "large", 100000]], [],
     [], None, 0),
    # an empty record fills the last 7 bytes of block 0 exactly
    ("MarginalTrailer", "316-327", [["big", "foo", kB - 2 * kH], ["lit", ""], ["lit", "bar"]], [], [],
     [OK, OK, OK], 0),
    # "bar" starts as a zero-length FIRST fragment in those 7 bytes
    ("MarginalTrailer2", "329-340", [["big", "foo", kB - 2 * kH], ["lit", "bar"]], [], [],
     [OK, OK, OK], 0),
    # 3 bytes left: the writer pads them; a walk that probes them finds the trailer
    ("ShortTrailer", "342-352", [["big", "foo", kB - 2 * kH + 4], ["lit", ""], ["lit", "bar"]], [],
     [kB - 3], [OK, OK, OK, TRAILER], 0),
    # the file ends 3 bytes short of the block: a probe there is the end of the file
    ("AlignedEof", "354-360", [["big", "foo", kB - 2 * kH + 4]], [], [kB - 3], [OK, TRUNCATED], 0),
    # physical checksum good; ReadRecord rejects the type ("unknown record type")
    ("BadRecordType", "394-402", [["lit", "foo"]], [["inc", 6, 100], ["fixcrc", 0, 3]], [], [OK], 0),
    ("TruncatedTrailingRecordIsIgnored", "404-411", [["lit", "foo"]], [["shrink", 4]], [], [TRUNCATED], 0),
    ("BadLength", "413-422", [["big", "bar", kB - kH], ["lit", "foo"]], [["inc", 4, 1]], [],
     [BAD_LENGTH, OK], 1),
    ("BadLengthAtEndIsIgnored", "424-430", [["lit", "foo"]], [["shrink", 1]], [], [TRUNCATED], 0),
    ("ChecksumMismatch", "432-438", [["lit", "foo"]], [["inc", 0, 10]], [], [MISMATCH], 1),
    # physical checksum good; ReadRecord reports "missing start"
    ("UnexpectedMiddleType", "440-447", [["lit", "foo"]], [["set", 6, 3], ["fixcrc", 0, 3]], [], [OK], 0),
    # the LAST fragment (7 + 7 bytes) is cut off entirely: its offset is the file's end
    ("MissingLastIsIgnored", "480-487", [["big", "bar", kB]], [["shrink", 14]], [], [OK, TRUNCATED], 0),
    # the LAST fragment's payload runs one byte past the end of the file
    ("PartialLastIsIgnored", "489-496", [["big", "bar", kB]], [["shrink", 1]], [], [OK, TRUNCATED], 0),
]


def main() -> None:
    ref = load_ref()
    from tests.oracle_lib import load_oracle
    orc = load_oracle()

    def crc_of(b: bytes) -> int:  # Mask(Value(type || payload)), db/log_writer.cc:105-111
        return ref.ref_mask(ref.ref_value(b, len(b)))

    out = {"generator": "oracle/gen_log_cases.py; header CRCs by the reference util/crc32c.cc "
                        "(oracle/_ref/libref_crc32c.so, compiled unmodified)",
           "statuses": {"CHECKSUM_MISMATCH": MISMATCH, "OK": OK, "BAD_LENGTH": BAD_LENGTH,
                        "ZERO_RECORD": ZERO, "TRUNCATED": TRUNCATED, "BLOCK_TRAILER": TRAILER},
           "cases": []}
    for name, lines, writes, edits, probes, expect, n_bad in CASES:
        img, offs = log_case_image(payloads(writes), edits, crc_of)
        offsets = [int(x) for x in offs] + [int(x) for x in probes]
        if expect is None:  # every record read back
            expect = [OK] * len(offsets)
        assert len(expect) == len(offsets), name
        got = orc.log_check(img, np.array(offsets, np.uint64), buf_len=int(img.size))
        assert list(int(x) for x in got) == expect, (name, list(got), expect)
        assert sum(1 for x in expect if x in (MISMATCH, BAD_LENGTH)) == n_bad, name
        out["cases"].append({"name": name, "ref": f"db/log_test.cc:{lines}", "writes": writes,
                             "edits": edits, "probes": probes, "buf_len": int(img.size),
                             "sha256": hashlib.sha256(img.tobytes()).hexdigest(),
                             "n_records": len(offsets),
                             "offsets": offsets if len(offsets) <= 64 else None,
                             "expect": expect if len(expect) <= 64 else None,
                             "expect_all": None if len(expect) <= 64 else OK, "n_bad": n_bad})
    path = os.path.join(ROOT, "tests", "golden", "log_reader_cases.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {path}: {len(out['cases'])} cases")


if __name__ == "__main__":
    main()
