"""Host-side drop-in API and C-ABI surface (CPU only, no compute on a GPU).

* leveldb::crc32c::{Extend,Value,Mask,Unmask} mirror (util/crc32c.h) on the
  host scalar path, against the reference-generated golden fixture.
* libnova_crc32c.so loads and exports every symbol include/nova_crc32c.h
  declares.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from novalsm_amd import crc32c as C
from novalsm_amd.synth import splitmix64_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def lib():
    return C.load(build_if_missing=True)


def declared_symbols():
    with open(os.path.join(ROOT, "include", "nova_crc32c.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nova_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported(lib):
    syms = declared_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), s


def test_abi_version(lib):
    assert lib.nova_crc32c_abi_version() == 1


def test_standard_results():
    # util/crc32c_test.cc:14-46
    assert C.Value(bytes(32)) == 0x8A9136AA
    assert C.Value(b"\xff" * 32) == 0x62A8AB43
    assert C.Value(bytes(range(32))) == 0x46DD794E
    assert C.Value(bytes(range(31, -1, -1))) == 0x113FDB5C


def test_values_extend_mask():
    # util/crc32c_test.cc:48-61
    assert C.Value(b"a") != C.Value(b"foo")
    assert C.Value(b"hello world") == C.Extend(C.Value(b"hello "), b"world")
    crc = C.Value(b"foo")
    assert crc != C.Mask(crc)
    assert crc != C.Mask(C.Mask(crc))
    assert crc == C.Unmask(C.Mask(crc))
    assert crc == C.Unmask(C.Unmask(C.Mask(C.Mask(crc))))
    assert C.kMaskDelta == 0xA282EAD8


def test_golden_cases_host(golden):
    for k in golden["known_answers"]:
        assert C.Value(bytes.fromhex(k["hex"])) == k["crc"]
    for c in golden["cases"]:
        data = splitmix64_bytes(c["seed"], c["length"], c["offset"]).tobytes()
        assert C.Extend(c["init"], data) == c["crc"], c
    for m in golden["mask"]:
        assert C.Mask(m["crc"]) == m["mask"]
        assert C.Unmask(m["crc"]) == m["unmask"]


def test_combine(golden, oracle):
    rng = np.random.default_rng(1)
    for _ in range(50):
        na, nb = (int(x) for x in rng.integers(0, 3000, 2))
        a = splitmix64_bytes(int(rng.integers(1, 99)), na).tobytes()
        b = splitmix64_bytes(int(rng.integers(1, 99)), nb).tobytes()
        assert C.Combine(C.Value(a), C.Value(b), nb) == oracle.value(a + b)


def test_hook_without_gpu_reports_cannot_accelerate():
    # port::AcceleratedCRC32C contract: 0 means "cannot accelerate"
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu suite")
    assert C.AcceleratedCRC32C(0, b"TestCRCBuffer") == 0


def test_batch_refuses_cpu_tensors():
    import torch
    t = torch.zeros(64, dtype=torch.uint8)
    with pytest.raises(C.NovaError):
        C.batch_strided(t, 16, 16, 4)


def test_device_init_fails_loudly_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert lib.nova_device_init() != 0
    out = ctypes.c_uint32(0)
    rc = lib.nova_crc32c_batch_strided(ctypes.c_void_p(16), 16, 16, 1, None,
                                       ctypes.addressof(out), 0, None)
    assert rc != 0  # no silent CPU fallback


@pytest.mark.parametrize("n,lanes,chunk", [
    (1, 16, 4), (6144, 16, 4), (6145, 8, 8), (98303, 8, 8), (98304, 8, 16),
    (196607, 8, 16), (196608, 8, 32), (1 << 20, 8, 32)])
def test_rounds_plan_sized_to_the_batch(n, lanes, chunk):
    """Host-side dispatch (no device call): variable SSTable batches go to the
    rounds kernel with 16-lane groups and 4-block chunks while they fit two
    chunks per wave slot (256 CUs x 12 waves), then 8-lane groups with 8/16/32-
    block chunks; the large-blocks hint picks the units kernel."""
    d = C.describe(n, 0, 0, variable=True)
    assert d["kernel"].startswith("crc32c_rounds_kernel")
    assert (d["lanes_per_block"], d["chunk_blocks"]) == (lanes, chunk)
    assert C.describe(n, 0, 0, variable=True, large=True)["kernel"].startswith("crc32c_units_kernel")
