"""GPU parity: the HIP kernels (through the C-ABI) against the CPU oracle and the
reference-generated golden fixture.  Integer work -> bit-exact everywhere.

Run on a real MI355X:  python -m pytest tests -m gpu
"""
import numpy as np
import pytest

from novalsm_amd import crc32c as C
from novalsm_amd.synth import splitmix64_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    C.load(build_if_missing=True)
    assert C.load().nova_device_init() == 0
    return torch


@pytest.fixture(autouse=True)
def _reset_tuning():
    # product-library tuning (per thread); the diagnostics library's knobs are
    # reset when a test's C.diagnostics() block exits
    yield
    C.set_tuning(0, 0)


def dev(torch, arr, dtype=None):
    t = torch.from_numpy(np.array(arr, order="C"))  # writable copy
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def pack_cases(cases, pad=16):
    """Place every case's bytes so that its start keeps the fixture's misalignment."""
    pos, offs, chunks = 0, [], []
    for c in cases:
        pos = (pos + 15) & ~15
        start = pos + c["offset"]
        data = splitmix64_bytes(c["seed"], c["length"], c["offset"])
        chunks.append((start, data))
        offs.append(start)
        pos = start + c["length"] + 1
    buf = np.zeros(pos + pad, dtype=np.uint8)
    for s, d in chunks:
        buf[s:s + len(d)] = d
    return buf, np.array(offs, dtype=np.uint64)


def test_known_answers_device(torch_gpu, golden):
    torch = torch_gpu
    cases = [bytes.fromhex(k["hex"]) for k in golden["known_answers"]]
    pos, offs, buf = 0, [], bytearray()
    for c in cases:
        offs.append(len(buf))
        buf += c + b"\x00" * 3
    b = dev(torch, np.frombuffer(bytes(buf) + bytes(16), dtype=np.uint8))
    out = C.batch(b, dev(torch, np.array(offs, np.uint64), torch.int64),
                  dev(torch, np.array([len(c) for c in cases], np.uint32), torch.int32))
    assert [int(x) for x in u32(out)] == [k["crc"] for k in golden["known_answers"]]


@pytest.mark.parametrize("lanes", [0, 1, 2, 4, 8, 16])
def test_golden_cases_device(torch_gpu, golden, lanes):
    torch = torch_gpu
    C.set_tuning(lanes, 0)
    cases = golden["cases"]
    buf, offs = pack_cases(cases)
    lens = np.array([c["length"] for c in cases], np.uint32)
    init = np.array([c["init"] for c in cases], np.uint32)
    out = C.batch(dev(torch, buf), dev(torch, offs, torch.int64), dev(torch, lens, torch.int32),
                  init=dev(torch, init.view(np.int32)))
    got = u32(out)
    want = np.array([c["crc"] for c in cases], np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(cases[i], hex(got[i])) for i in bad[:5]]


def test_golden_cases_split_path(torch_gpu, golden):
    """The reference-generated golden cases (every misalignment 0..15, lengths
    0..160 and edge lengths up to 64 KiB+63, random inits) through the
    split-and-combine path (forced): 16 KiB pieces in 128 slots per block,
    folded, then finished by the finish kernel."""
    torch = torch_gpu
    cases = golden["cases"]
    buf, offs = pack_cases(cases)
    lens = np.array([c["length"] for c in cases], np.uint32)
    init = np.array([c["init"] for c in cases], np.uint32)
    with C.diagnostics() as D:
        D.nova_diag_set_split(1)
        out = C.batch(dev(torch, buf), dev(torch, offs, torch.int64), dev(torch, lens, torch.int32),
                      init=dev(torch, init.view(np.int32)))
    got = u32(out)
    want = np.array([c["crc"] for c in cases], np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(cases[i], hex(got[i])) for i in bad[:5]]


def test_config1_fixture_strided(torch_gpu, golden):
    torch = torch_gpu
    c1 = golden["config1"]
    buf = dev(torch, splitmix64_bytes(c1["seed"], c1["n"] * c1["len"]))
    out = C.batch_strided(buf, c1["len"], c1["len"], c1["n"])
    assert [int(x) for x in u32(out)] == c1["crc"]


def test_packed_sstable_and_trailers(torch_gpu, golden, oracle):
    torch = torch_gpu
    pk = golden["packed"]
    host = splitmix64_bytes(pk["seed"], pk["total"])
    buf = dev(torch, host)
    offs = dev(torch, np.array(pk["offsets"], np.uint64), torch.int64)
    sizes = dev(torch, np.array(pk["sizes"], np.uint32), torch.int32)
    out = C.batch(buf, offs, sizes)
    assert [int(x) for x in u32(out)] == pk["crc"]
    # table/table_builder.cc:192-212 trailers (with the '!' quirk)
    C.write_trailers(buf, offs, sizes, 0, tb_quirk=True)
    h = buf.cpu().numpy()
    for o, s, tb in zip(pk["offsets"], pk["sizes"], pk["tb_trailer_hex"]):
        assert h[o + s:o + s + 5].tobytes().hex() == tb
    # ltc/stoc_file_client_impl.cpp:704-723 trailers (correct masked CRC)
    C.write_trailers(buf, offs, sizes, 0, tb_quirk=False)
    h = buf.cpu().numpy()
    for o, s, st in zip(pk["offsets"], pk["sizes"], pk["stoc_trailer_hex"]):
        assert h[o + s:o + s + 5].tobytes().hex() == st
    # table/table.cc:434-440 verify: all StoC-trailed blocks pass
    ok, bad = C.verify_blocks(buf, offs, sizes)
    assert ok.cpu().numpy().all() and int(bad.item()) == 0
    # corrupt a byte in 5 blocks -> exactly those fail
    victims = [0, 7, 13, 50, 96]
    for v in victims:
        o = pk["offsets"][v] + pk["sizes"][v] // 2
        buf[o] ^= 0x40
    ok, bad = C.verify_blocks(buf, offs, sizes)
    okh = ok.cpu().numpy()
    assert sorted(np.nonzero(okh == 0)[0].tolist()) == victims
    assert int(bad.item()) == len(victims)
    for i in range(len(pk["sizes"])):
        o, s = pk["offsets"][i], pk["sizes"][i]
        assert bool(okh[i]) == oracle.verify(buf[o:o + s + 5].cpu().numpy().tobytes())


@pytest.mark.parametrize("length", [0, 1, 2, 3, 4, 5, 7, 15, 16, 17, 31, 63, 64, 65, 100, 255,
                                    1000, 4095, 4096, 4097, 16384, 16389, 65536, 65599])
def test_strided_vs_oracle(torch_gpu, oracle, length):
    torch = torch_gpu
    rng = np.random.default_rng(length)
    stride = length + int(rng.integers(0, 40))
    n = max(1, min(300, (8 << 20) // max(stride, 1)))
    base = int(rng.integers(0, 16))
    host = splitmix64_bytes(length + 17, base + n * stride + 16)
    buf = dev(torch, host)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for flags, ini in [(0, None), (0, init), (C.APPEND_TYPE | C.TYPE(1) | C.MASK_OUTPUT, init),
                       (C.MASK_OUTPUT, None)]:
        out = C.batch_strided(buf, stride, length, n, init=None if ini is None else
                              dev(torch, ini.view(np.int32)), flags=flags, base_offset=base)
        want = oracle.batch_strided(host[base:], stride, length, n, init=ini, flags=flags)
        assert np.array_equal(u32(out), want), (flags, length)


@pytest.mark.parametrize("lanes,seg,chunk,steal", [
    (0, 0, 0, -1), (1, 0, 0, -1), (2, 0, 0, -1), (4, 0, 0, -1), (8, 0, 0, -1), (16, 0, 0, -1),
    (4, 16, 0, -1), (4, 64, 0, -1), (4, 1024, 0, -1), (1, 4096, 0, -1), (16, 256, 0, -1),
    (8, 65536, 0, -1), (16, 16384, 1, 0), (16, 16384, 3, 1), (8, 8192, 16, 255),
    (4, 4096, 5, 8)])
@pytest.mark.parametrize("waves,var", [(0, 0), (7, 2)])
def test_variable_batch_vs_oracle(torch_gpu, oracle, lanes, seg, chunk, steal, waves, var):
    """Variable-length batch through the units kernel, across unit sizes and
    the claim scheduler's chunk size / steal bound."""
    torch = torch_gpu
    with C.diagnostics() as L:
        C.set_tuning(lanes, seg)
        L.nova_diag_set_chunk_blocks(chunk)
        L.nova_diag_set_static_pct(steal)
        L.nova_diag_set_stream_waves(waves)
        L.nova_diag_set_variant(var)
        _variable_batch_checks(torch, oracle, lanes, seg)


@pytest.mark.parametrize("lanes", [2, 4, 8, 16])
def test_rounds_tiny_and_mixed_blocks(torch_gpu, oracle, lanes):
    """Rounds kernel at every group width on blocks that hold no full 16-B
    piece (the tail path alone: 5 B at several alignments) and on rounds that
    mix long and tiny blocks.  Round 3's continuous-rounds experiment (DESIGN.md
    3.5a) failed exactly these shapes at G = 2 and 4 before it was fixed; the
    test stays as a guard for any change to the rounds' line bookkeeping."""
    torch = torch_gpu
    host = splitmix64_bytes(99, 64 * 70000 + 256)
    buf = dev(torch, host)
    cases = []
    for L in (5, 17, 129, 4099):
        for align in (0, 1, 7, 13):
            n = 256
            stride = ((L + 64 + 15) // 16) * 16
            cases.append((np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(align),
                          np.full(n, L, np.uint32)))
    for a, b in ((4096, 17), (500, 5), (129, 3), (300, 40), (16384, 1)):
        n = 384
        lens = np.where(np.arange(n) % 3 == 0, a, b).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        pos = 3
        for i in range(n):
            offs[i] = pos
            pos += int(lens[i]) + 5
        cases.append((offs, lens))
    try:
        C.set_tuning(lanes, 0)
        for offs, lens in cases:
            want = oracle.batch(host, offs, lens, np.full(len(offs), 0xFFFFFFFF, np.uint32)) ^ np.uint32(
                0xFFFFFFFF)
            out = C.batch(buf, dev(torch, offs, torch.int64), dev(torch, lens, torch.int32), flags=C.RAW)
            bad = np.nonzero(u32(out) != want)[0]
            assert bad.size == 0, (lanes, int(lens[0]), int(offs[0]) % 16, bad[:8].tolist())
    finally:
        C.set_tuning(0, 0)


def _variable_batch_checks(torch, oracle, lanes, seg):
    rng = np.random.default_rng(lanes * 1000 + seg)
    n = 1500
    cls = rng.choice([1, 3, 4, 17, 600, 4096, 16384, 65536], n, p=[.03, .03, .04, .1, .1, .4,
                                                                     .2, .1])
    lens = (cls + rng.integers(0, 64, n) * (cls > 4)).astype(np.uint32)
    gaps = rng.integers(0, 24, n)
    offs = np.zeros(n, np.uint64)
    pos = 3
    for i in range(n):
        offs[i] = pos
        pos += int(lens[i]) + int(gaps[i])
    perm = rng.permutation(n)          # descriptors need not be in address order
    offs, lens = offs[perm], lens[perm]
    host = splitmix64_bytes(99, pos + 64)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    buf = dev(torch, host)
    want = oracle.batch(host, offs, lens, init)
    do, dl, di = (dev(torch, offs, torch.int64), dev(torch, lens, torch.int32),
                  dev(torch, init.view(np.int32)))
    for _ in range(3):  # the schedule is dynamic: several launches, sentinel-filled outputs
        out = torch.full((n,), -559038737, dtype=torch.int32, device="cuda")  # 0xDEADBEEF
        C.batch(buf, do, dl, init=di, out=out)
        bad = np.nonzero(u32(out) != want)[0]
        assert bad.size == 0, [(int(offs[i]), int(lens[i])) for i in bad[:5]]
    # RAW flag: linear part only; Extend(c, D) = ~(M_n(~c) ^ raw(D)) <=> raw == Extend(~0..)
    out_raw = C.batch(buf, dev(torch, offs, torch.int64), dev(torch, lens, torch.int32),
                      flags=C.RAW)
    # raw(D) = Extend(0xFFFFFFFF, D) ^ 0xFFFFFFFF (register starts at 0)
    want_raw = oracle.batch(host, offs, lens, np.full(n, 0xFFFFFFFF, np.uint32)) ^ np.uint32(
        0xFFFFFFFF)
    assert np.array_equal(u32(out_raw), want_raw)


def test_extend_chaining_property(torch_gpu, oracle):
    # util/crc32c_test.cc:50-53 generalised: Extend(Value(A), B) == Value(A||B)
    torch = torch_gpu
    n, la, lb = 512, 3000, 5001
    host = splitmix64_bytes(21, n * (la + lb) + 16)
    buf = dev(torch, host)
    stride = la + lb
    whole = C.batch_strided(buf, stride, la + lb, n)
    first = C.batch_strided(buf, stride, la, n)
    chained = C.batch_strided(buf, stride, lb, n, init=first, base_offset=la)
    assert torch.equal(whole, chained)


def test_zero_and_tiny_lengths(torch_gpu, oracle):
    torch = torch_gpu
    host = splitmix64_bytes(4, 256)
    buf = dev(torch, host)
    offs = np.array([0, 5, 9, 100, 101, 102, 200], np.uint64)
    lens = np.array([0, 1, 2, 3, 0, 4, 5], np.uint32)
    init = np.array([0x12345678, 0, 7, 0xFFFFFFFF, 0xDEADBEEF, 1, 2], np.uint32)
    out = C.batch(buf, dev(torch, offs, torch.int64), dev(torch, lens, torch.int32),
                  init=dev(torch, init.view(np.int32)))
    want = oracle.batch(host, offs, lens, init)
    assert np.array_equal(u32(out), want)
    assert u32(out)[0] == 0x12345678 and u32(out)[4] == 0xDEADBEEF  # n=0 returns init


def test_device_splitmix64_matches_host(torch_gpu):
    torch = torch_gpu
    for n, seed, w in [(1 << 20, 2, 0), (4097, 3, 11)]:
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(t, seed, w)
        assert np.array_equal(t.cpu().numpy(), splitmix64_bytes(seed, n, 8 * w))


def test_stream_host_matches_device(torch_gpu, oracle):
    torch = torch_gpu
    n, L = 20000, 16384
    host = torch.empty(n * L, dtype=torch.uint8).pin_memory()
    host.copy_(torch.from_numpy(splitmix64_bytes(5, n * L)))
    got = C.stream_host(host, L, L, n, chunk_blocks=1024, n_streams=3)
    hn = host.numpy()
    idx = np.arange(0, n, 37)
    want = np.array([oracle.value(hn[i * L:(i + 1) * L].tobytes()) for i in idx], np.uint32)
    assert np.array_equal(got[idx], want)
    dv = C.batch_strided(host.cuda(), L, L, n)
    assert np.array_equal(u32(dv), got)
    # pageable input is registered on the fly
    pg = hn[: 300 * L].copy()
    got2 = C.stream_host(pg, L, L, 300, chunk_blocks=64, n_streams=2)
    assert np.array_equal(got2, got[:300])


def test_pageable_adjacent_subpage_ranges_two_threads(torch_gpu, oracle):
    """hipHostRegister pins whole pages, so two callers on
    disjoint byte ranges of one pageable slab that share a page must not see
    each other's registration as caller-pinned memory (HostReg rounds ranges
    out to pages and counts references, crc32c_stream.cpp).  Two threads
    checksum adjacent sub-page ranges back to back; every result is checked."""
    import threading
    L, n = 256, 8  # 2 KiB per range
    slab = splitmix64_bytes(21, 5 * 4096)
    a0 = (-slab.ctypes.data) % 4096 + 512  # 512 B into the slab's first whole page
    ranges = [slab[a0:a0 + L * n], slab[a0 + L * n:a0 + 2 * L * n]]  # that page | it and the next
    want = [np.array([oracle.value(r[i * L:(i + 1) * L].tobytes()) for i in range(n)], np.uint32)
            for r in ranges]
    errors = []
    start = threading.Barrier(2)

    def work(k):
        try:
            start.wait()
            for it in range(150):
                got = C.stream_host(ranges[k], L, L, n, chunk_blocks=4, n_streams=2)
                if not np.array_equal(got, want[k]):
                    errors.append((k, it, got, want[k]))
                    return
        except Exception as e:  # pragma: no cover
            errors.append((k, e))
    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:2]


def test_lane_xor(torch_gpu):
    """the kernels' lane_xor<K> (DPP for K <= 8, the gfx950
    v_permlane16/32_swap for 16 and 32) equals __shfl_xor on every lane of a
    wave64 for every K, on distinct lane values; wave_max (the swaps without a
    lane select) gives every lane the wave's maximum."""
    torch = torch_gpu
    rng = np.random.default_rng(5)
    vals = rng.permutation(2**31)[:64].astype(np.uint32)
    inp = dev(torch, vals.view(np.int32))
    out = torch.zeros(7 * 64, dtype=torch.int32, device="cuda")
    ref = torch.zeros(6 * 64, dtype=torch.int32, device="cuda")
    D = C.load_diag()
    assert D.nova_diag_lane_xor_probe(inp.data_ptr(), out.data_ptr(), ref.data_ptr(), None) == 0
    torch.cuda.synchronize()
    o, r = u32(out).reshape(7, 64), u32(ref).reshape(6, 64)
    lanes = np.arange(64)
    for k in range(6):
        assert np.array_equal(r[k], vals[lanes ^ (1 << k)]), k  # the reference itself
        assert np.array_equal(o[k], r[k]), (1 << k, np.nonzero(o[k] != r[k])[0][:8])
    assert np.all(o[6] == vals.max())


def test_accelerated_hook(torch_gpu, oracle):
    """port::AcceleratedCRC32C self-test (util/crc32c.cc:477-485), then sizes on
    both sides of NOVA_HOOK_MIN_BYTES (8 MiB): the 1-byte type-byte Extend of
    table/table_builder.cc:203 and a 4 KiB block never launch a kernel; large
    buffers run on the GPU."""
    assert C.AcceleratedCRC32C(0, b"TestCRCBuffer") == 0xDCBC59FA
    s0 = C.port_stats()
    for n, init in [(1, 0), (4096, 5), (4097, 0xFFFFFFFF)]:
        d = splitmix64_bytes(n, n).tobytes()
        assert C.AcceleratedCRC32C(init, d) == oracle.extend(init, d)
    s1 = C.port_stats()
    assert s1["device"] == s0["device"] and s1["host"] - s0["host"] == 3
    for n, init in [(8 << 20, 0x1234), (9 << 20 | 77, 9)]:
        d = splitmix64_bytes(n, n).tobytes()
        assert C.AcceleratedCRC32C(init, d) == oracle.extend(init, d)
    s2 = C.port_stats()
    assert s2["device"] - s1["device"] == 2 and s2["fallback"] == s1["fallback"]


def test_accelerated_hook_device_failure_falls_back(torch_gpu, oracle, tmp_path):
    """A device-side failure (here: a staging cap below the buffer size, set
    before the process's first hook call) gives Extend's value, not 0."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from novalsm_amd import crc32c as C\n"
            "from novalsm_amd.synth import splitmix64_bytes\n"
            "d = splitmix64_bytes(3, 9 << 20).tobytes()\n"
            "print(C.AcceleratedCRC32C(7, d), C.port_stats()['fallback'], C.port_stats()['device'])\n"
            ) % (str(__import__('pathlib').Path(__file__).resolve().parents[1]),)
    env = dict(__import__('os').environ, NOVA_HOOK_MAX_STAGING=str(1 << 20))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    crc, fb, devc = (int(x) for x in r.stdout.split()[-3:])
    d = splitmix64_bytes(3, 9 << 20).tobytes()
    assert crc == oracle.extend(7, d) and fb == 1 and devc == 0


@pytest.mark.timeout(300)
def test_no_device_memory_growth(torch_gpu, oracle):
    """the hook and the host-streamed paths reuse pooled streams,
    so thousands of calls from several threads leave the claim-counter slot
    count and free device memory flat; nova_stream_release frees a caller
    stream's slot."""
    torch = torch_gpu
    import threading
    d = splitmix64_bytes(4, (8 << 20) + 5).tobytes()  # above NOVA_HOOK_MIN_BYTES: the device path
    want = oracle.extend(0, d)
    host = torch.from_numpy(splitmix64_bytes(6, 64 * 4096)).pin_memory()
    C.AcceleratedCRC32C(0, d)
    C.stream_host(host, 4096, 4096, 64, chunk_blocks=16, n_streams=3)
    torch.cuda.synchronize()
    slots0, free0 = C.stream_slots(), torch.cuda.mem_get_info()[0]
    errors = []

    def work():
        try:
            for _ in range(150):
                assert C.AcceleratedCRC32C(0, d) == want
            for _ in range(20):
                C.stream_host(host, 4096, 4096, 64, chunk_blocks=16, n_streams=3)
        except Exception as e:  # pragma: no cover
            errors.append(e)
    th = [threading.Thread(target=work) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    torch.cuda.synchronize()
    # 4 threads: at most 4 hook streams + 3 x 4 stream_host streams in the pool
    assert C.stream_slots() <= slots0 + 16
    s = torch.cuda.Stream()  # a batch above the burst size: the stream kernel takes a slot
    C.batch_strided(dev(torch, splitmix64_bytes(1, 4096 * 16384)), 4096, 4096, 16384, stream=s)
    s.synchronize()
    n1 = C.stream_slots()
    C.stream_release(s)
    assert C.stream_slots() == n1 - 1
    for _ in range(300):  # more hook calls on the warm pool: no growth at all
        C.AcceleratedCRC32C(0, d)
    torch.cuda.synchronize()
    assert C.stream_slots() == n1 - 1
    assert torch.cuda.mem_get_info()[0] >= free0 - (64 << 20)


def test_shared_stream_trailer_threads(torch_gpu, oracle):
    """several host threads writing trailers of large batches (the
    rounds kernel, > 12288 blocks; blocks of 1..599 B, so the byte-store form) on
    the SAME stream (the default one) each get their own layout-flag scratch:
    every trailer matches the oracle."""
    torch = torch_gpu
    import threading
    n = 13000
    imgs, descs = [], []
    for t in range(4):
        rng = np.random.default_rng(300 + t)
        lens = rng.integers(1, 600, n).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
        host = splitmix64_bytes(40 + t, int(offs[-1]) + int(lens[-1]) + 5 + 16)
        imgs.append((host, dev(torch, host)))
        descs.append((offs, lens, dev(torch, offs, torch.int64), dev(torch, lens, torch.int32)))
    torch.cuda.synchronize()
    errors = []

    def work(t):
        try:
            for _ in range(5):
                C.write_trailers(imgs[t][1], descs[t][2], descs[t][3], 0, True,
                                 stream=torch.cuda.default_stream())
        except Exception as e:  # pragma: no cover
            errors.append(e)
    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    torch.cuda.synchronize()
    for t in range(4):
        host, dbuf = imgs[t]
        offs, lens = descs[t][0], descs[t][1]
        got = dbuf.cpu().numpy()
        for i in range(0, n, 7):
            o, ln = int(offs[i]), int(lens[i])
            assert oracle.trailer(host[o:o + ln].tobytes(), 0, True) == got[o + ln:o + ln + 5].tobytes()


@pytest.mark.parametrize("form", [0, 2, 3, 8])
@pytest.mark.parametrize("layout", ["packed", "gaps", "tiny", "small", "permuted", "aligned"])
@pytest.mark.parametrize("quirk,ctype", [(True, 0), (False, 1)])
def test_trailer_store_forms(torch_gpu, oracle, layout, quirk, ctype, form):
    """Large trailer batches (the rounds kernel, > 12288 blocks) in every store
    form: 0 the product's byte stores from the CRC kernel; diagnostics 2 (CRC
    array + scatter pass) and 3 (whole 64-B pieces around each trailer where
    trailer_layout_kernel allows: blocks ascending and disjoint, no neighbour's
    trailer in the piece -- "tiny" and "small" mix both forms, "permuted" falls
    back to byte stores), 8 (CRC array, then a second pass that reads,
    patches and stores those whole pieces).  The WHOLE image must equal the input with each
    block's trailer (table/table_builder.cc:202-206,
    ltc/stoc_file_client_impl.cpp:713-719) in place: no byte outside the
    trailers changes, including gap bytes, the bytes before the first block and
    after the last one."""
    torch = torch_gpu
    n = 13000
    layouts = ["packed", "gaps", "tiny", "small", "permuted", "aligned"]
    rng = np.random.default_rng(layouts.index(layout) * 2 + quirk)
    lens = rng.integers(32, 3000, n).astype(np.uint32)
    if layout == "tiny":
        lens[rng.choice(n, 400, replace=False)] = rng.integers(0, 32, 400).astype(np.uint32)
    if layout == "small":
        lens = rng.integers(0, 100, n).astype(np.uint32)
    if layout == "aligned":
        lens = (lens + 63) & ~np.uint32(63)  # lengths a multiple of 64
    gaps = rng.integers(0, 80, n).astype(np.uint64) if layout == "gaps" else np.zeros(n, np.uint64)
    lead = 48 if layout != "aligned" else 0  # first block starts inside a piece
    offs = np.zeros(n, np.uint64)
    offs[0] = lead
    offs[1:] = lead + np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5) + gaps[:-1])
    total = int(offs[-1]) + int(lens[-1]) + 5 + 64
    host = splitmix64_bytes(77, total)  # trailer bytes start as noise
    want = host.copy()
    for i in range(n):
        o, ln = int(offs[i]), int(lens[i])
        want[o + ln:o + ln + 5] = np.frombuffer(oracle.trailer(host[o:o + ln].tobytes(), ctype, quirk),
                                                dtype=np.uint8)
    order = rng.permutation(n) if layout == "permuted" else np.arange(n)
    buf = dev(torch, host)
    do, dl = dev(torch, offs[order], torch.int64), dev(torch, lens[order], torch.int32)
    if form:
        with C.diagnostics() as D:
            D.nova_diag_set_trailer_single_pass(form)
            C.write_trailers(buf, do, dl, ctype, quirk)
    else:
        C.write_trailers(buf, do, dl, ctype, quirk)
    got = buf.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
    if not quirk:  # StoC order: every block verifies
        ok, nbad = C.verify_blocks(buf, dev(torch, offs, torch.int64), dev(torch, lens, torch.int32))
        assert ok.cpu().numpy().all() and int(nbad.item()) == 0


@pytest.mark.parametrize("shape", ["sst4k", "large"])
@pytest.mark.parametrize("pinned", [True, False])
def test_host_resident_sstable_paths(torch_gpu, oracle, pinned, shape):
    """an SSTable image in host memory (the Format() buffer /
    ReadAll() slab, ltc/stoc_file_client_impl.cpp:183-377, :843-882) -- CRCs,
    trailers and verify through H2D -> kernel -> D2H chunks, equal to the
    device paths and the oracle; descriptors partly out of address order.
    "large": 16 KiB - 3 MiB blocks, whose chunks the host path sends with the
    large-blocks hint (units kernel, or the split path for a few blocks)."""
    torch = torch_gpu
    rng = np.random.default_rng(11)
    if shape == "sst4k":
        n = 5000
        lens = (4096 + rng.integers(0, 256, n)).astype(np.uint32)
        lens[rng.integers(0, n, 50)] = rng.integers(0, 40, 50)
        rev, victims = slice(100, 200), [3, 150, 4999]
    else:
        n = 60
        lens = (rng.choice([16384, 65536, 3 << 20], n) + rng.integers(0, 50, n)).astype(np.uint32)
        lens[5] = 7
        rev, victims = slice(10, 20), [3, 15, 59]
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
    total = int(offs[-1]) + int(lens[-1]) + 5
    img0 = splitmix64_bytes(12, total)
    perm = np.arange(n)
    perm[rev] = perm[rev][::-1]  # a reversed run: spans still bounded
    po, pl = offs[perm], lens[perm]
    img = torch.from_numpy(img0.copy())
    if pinned:
        img = img.pin_memory()
    got = C.batch_host(img, po, pl, chunk_bytes=3 << 20, n_streams=3)
    assert np.array_equal(got, oracle.batch(img0, po, pl, None))
    C.write_trailers_host(img, po, pl, 0, True, chunk_bytes=3 << 20)
    want = img0.copy()
    for i in range(n):
        o, ln = int(offs[i]), int(lens[i])
        want[o + ln:o + ln + 5] = np.frombuffer(oracle.trailer(img0[o:o + ln].tobytes(), 0, True),
                                                np.uint8)
    assert np.array_equal(img.numpy(), want)
    C.write_trailers_host(img, po, pl, 0, False, chunk_bytes=1 << 20, n_streams=2)
    ok, nbad = C.verify_blocks_host(img, po, pl, chunk_bytes=2 << 20)
    assert ok.all() and nbad == 0
    for v in victims:
        img[int(offs[perm[v]])] ^= 1 if lens[perm[v]] else 0
        if not lens[perm[v]]:
            img[int(offs[perm[v]]) + 1] ^= 1
    ok, nbad = C.verify_blocks_host(img, po, pl)
    assert sorted(np.nonzero(ok == 0)[0].tolist()) == victims and nbad == len(victims)
    dok, _ = C.verify_blocks(img.cuda(), dev(torch, po, torch.int64), dev(torch, pl, torch.int32))
    assert np.array_equal(dok.cpu().numpy(), ok)


def test_device_batches_validate_arguments(torch_gpu):
    """wrong descriptor dtypes, non-contiguous views and CPU tensors
    are refused before the C-ABI (the kernels would read them as raw u64/u32)."""
    torch = torch_gpu
    data = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(4, dtype=torch.int64, device="cuda")
    lens = torch.full((4,), 16, dtype=torch.int32, device="cuda")
    C.batch(data, offs, lens)  # the good case
    for args in [(data, offs.to(torch.int32), lens), (data, offs, lens.to(torch.int64)),
                 (data.view(torch.int32), offs, lens),
                 (data, torch.zeros(8, dtype=torch.int64, device="cuda")[::2], lens),
                 (data, offs.cpu(), lens)]:
        with pytest.raises(C.NovaError):
            C.batch(*args)
    with pytest.raises(C.NovaError):
        C.batch(data, offs, lens, out=torch.empty(4, dtype=torch.int64, device="cuda"))
    with pytest.raises(C.NovaError):
        C.verify_blocks(data, offs, lens, ok=torch.empty(4, dtype=torch.int32, device="cuda"))
    with pytest.raises(C.NovaError):
        C.log_write_crcs(data, offs.to(torch.int32))


def test_determinism(torch_gpu):
    torch = torch_gpu
    buf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 8)
    a = C.batch_strided(buf, 4096, 4096, (64 << 20) // 4096)
    for _ in range(3):
        assert torch.equal(a, C.batch_strided(buf, 4096, 4096, (64 << 20) // 4096))


def test_baseline_config2_full(torch_gpu, oracle):
    """BASELINE config 2 at full size: 1M x 4 KiB = 4 GiB, every block checked."""
    torch = torch_gpu
    n, L = 1 << 20, 4096
    buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 2)
    out = u32(C.batch_strided(buf, L, L, n))
    host = buf.cpu().numpy()
    want = oracle.batch_strided_mt(host, L, L, n, threads=16)
    assert np.array_equal(out, want)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("hint", ["large_blocks", "default"])
def test_baseline_config3_full(torch_gpu, oracle, hint):
    """BASELINE config 3 at full size: 1M blocks of {4,16,64} KiB + U[1,64] bytes
    packed back to back (unaligned, ~28 GiB), EVERY block checked against the
    multithreaded oracle -- on the path bench.py times (HINT_LARGE_BLOCKS:
    crc32c_units_kernel<16> with 32 KiB segments) and on the default dispatch
    (crc32c_rounds_kernel)."""
    torch = torch_gpu
    from bench import config3_layout
    offs, lens, total = config3_layout(1 << 20, seed=3)
    buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 3)
    flags = C.HINT_LARGE_BLOCKS if hint == "large_blocks" else 0
    d = C.describe(1 << 20, 0, 0, variable=True, large=bool(flags))
    assert d["kernel"].startswith("crc32c_units_kernel<16" if flags else "crc32c_rounds_kernel"), d
    out = u32(C.batch(buf, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), flags=flags))
    host = buf.cpu().numpy()
    del buf
    torch.cuda.empty_cache()
    want = oracle.batch_mt(host, offs, lens, threads=16)
    bad = np.flatnonzero(out != want)
    assert bad.size == 0, (bad.size, bad[:10])


@pytest.mark.timeout(600)
def test_baseline_config4_shard_full(torch_gpu, oracle):
    """BASELINE config 4's per-GPU shard at full size: 1M x 16 KiB = 16 GiB through
    crc32c_stream_kernel<16>, EVERY block checked; the shard of rank 7 of 8
    (splitmix64 words offset as bench.py's ranks)."""
    torch = torch_gpu
    n, L = 1 << 20, 16384
    d = C.describe(n, L, L)
    assert d["kernel"].startswith("crc32c_stream_kernel<16"), d
    buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 4, first_word=7 * (n * L // 8))
    out = u32(C.batch_strided(buf, L, L, n))
    host = buf.cpu().numpy()
    del buf
    torch.cuda.empty_cache()
    want = oracle.batch_strided_mt(host, L, L, n, threads=16)
    bad = np.flatnonzero(out != want)
    assert bad.size == 0, (bad.size, bad[:10])


@pytest.mark.parametrize("length", [256, 1024, 2048, 4096, 8192, 16384, 65536])
@pytest.mark.parametrize("n", [1, 7, 100, 4099])
@pytest.mark.parametrize("kernel", ["auto", "stream"])
def test_stream_kernel_shapes(torch_gpu, oracle, length, n, kernel):
    """Aligned uniform batches: crc32c_stream_kernel (forced by a lane count;
    ragged tail rounds, batches smaller than one round) and the dispatcher's
    choice for these SSTable-sized batches (the burst kernel); init arrays and
    flags."""
    torch = torch_gpu
    if kernel == "stream":
        C.set_tuning(16 if length >= 16384 else 8, 0)
    d = C.describe(n, length, length)
    assert d["kernel"].startswith("crc32c_stream_kernel" if kernel == "stream"
                                  else "crc32c_burst_kernel"), d
    host = splitmix64_bytes(length + n, n * length)
    buf = dev(torch, host)
    rng = np.random.default_rng(n)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for flags, ini in [(0, None), (0, init), (C.APPEND_TYPE | C.TYPE(0) | C.MASK_OUTPUT, init),
                       (C.RAW, None)]:
        out = C.batch_strided(buf, length, length, n, flags=flags,
                              init=None if ini is None else dev(torch, ini.view(np.int32)))
        if flags & C.RAW:
            want = oracle.batch_strided(host, length, length, n,
                                        init=np.full(n, 0xFFFFFFFF, np.uint32)) ^ np.uint32(
                0xFFFFFFFF)
        else:
            want = oracle.batch_strided(host, length, length, n, init=ini, flags=flags)
        assert np.array_equal(u32(out), want), (flags, length, n)


@pytest.mark.parametrize("mode", ["store", "trailers", "verify"])
@pytest.mark.parametrize("lanes", [0, 16, 65])
def test_burst_kernel(torch_gpu, oracle, mode, lanes):
    """The one-SSTable latency path (crc32c_burst_kernel): one
    wave per block on the compact tables (the dispatcher's choice), and the
    measured-slower variants of the diagnostics build (16 lanes per block on
    the replicated M_256 image; a 16-way replicated M_1024); every alignment
    and length from 0 B to 300 KiB (many passes), per-block inits and all
    flags, every mode, against the oracle."""
    torch = torch_gpu
    if lanes == 0:
        assert C.describe(3000, 0, 0, variable=True)["kernel"].startswith("crc32c_burst_kernel<64")
        _burst_checks(torch, oracle, mode)
        return
    with C.diagnostics() as L:
        L.nova_diag_set_burst_lanes(lanes)
        _burst_checks(torch, oracle, mode)


def _burst_checks(torch, oracle, mode):
    rng = np.random.default_rng(61)
    n = 3000
    lens = rng.choice([0, 1, 2, 3, 4, 5, 15, 16, 17, 1000, 1023, 1024, 1025, 4096, 4200, 8191,
                       8192, 8193, 16384, 65599, 300000], n).astype(np.uint32)
    lens += (rng.integers(0, 16, n) * (lens > 20)).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5) +
                         rng.integers(0, 3, n - 1).astype(np.uint64))
    offs += np.uint64(3)
    perm = rng.permutation(n)
    offs, lens = offs[perm], lens[perm]
    total = int((offs + lens).max()) + 5 + 64
    host = splitmix64_bytes(62, total).copy()
    do, dl = dev(torch, offs, torch.int64), dev(torch, lens, torch.int32)
    assert C.describe(n, 0, 0, variable=True)["kernel"].startswith("crc32c_burst_kernel")
    if mode == "store":
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        buf = dev(torch, host)
        for flags, ini in [(0, None), (0, init), (C.APPEND_TYPE | C.TYPE(1) | C.MASK_OUTPUT, init)]:
            out = C.batch(buf, do, dl, flags=flags,
                          init=None if ini is None else dev(torch, ini.view(np.int32)))
            want = oracle.batch(host, offs, lens, ini, flags=flags)
            bad = np.flatnonzero(u32(out) != want)
            assert bad.size == 0, (flags, [(int(offs[i]), int(lens[i])) for i in bad[:5]])
        out = C.batch(buf, do, dl, flags=C.RAW)
        want = oracle.batch(host, offs, lens, np.full(n, 0xFFFFFFFF, np.uint32)) ^ np.uint32(0xFFFFFFFF)
        assert np.array_equal(u32(out), want)
    elif mode == "trailers":
        buf = dev(torch, host)
        C.write_trailers(buf, do, dl, 3, True)
        got = buf.cpu().numpy()
        for i in range(n):
            o, ln = int(offs[i]), int(lens[i])
            assert oracle.trailer(host[o:o + ln].tobytes(), 3, True) == got[o + ln:o + ln + 5].tobytes(), i
    else:
        buf = dev(torch, host)
        C.write_trailers(buf, do, dl, 0, False)
        victims = rng.choice(n, 11, replace=False)
        for v in victims:
            buf[int(offs[v]) + int(lens[v]) // 2] ^= 0x20
        ok, bad = C.verify_blocks(buf, do, dl)
        assert sorted(np.flatnonzero(ok.cpu().numpy() == 0).tolist()) == sorted(victims.tolist())
        assert int(bad.item()) == len(victims)


@pytest.mark.parametrize("lanes,bpg,steal,waves,var", [
    (1, 1, 0, 0, 0), (2, 3, 1, 0, 0), (4, 2, 8, 0, 0), (8, 1, 8, 0, 0), (8, 4, 0, 0, 0),
    (16, 2, 255, 0, 0), (16, 1, 8, 0, 0), (8, 2, 8, 1, 0), (8, 2, 8, 5, 2), (16, 1, 8, 12, 0),
    (8, 2, 8, 16, 2)])
def test_stream_kernel_tuning_variants(torch_gpu, oracle, lanes, bpg, steal, waves, var):
    torch = torch_gpu
    with C.diagnostics() as L:
        C.set_tuning(lanes, 0)
        L.nova_diag_set_blocks_per_group(bpg)
        L.nova_diag_set_static_pct(steal)
        L.nova_diag_set_stream_waves(waves)
        L.nova_diag_set_variant(var)  # 2 = default-policy loads instead of nt
        n, length = 30011, 4096
        buf = torch.empty(n * length, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 77)
        out = u32(C.batch_strided(buf, length, length, n))
        want = oracle.batch_strided_mt(buf.cpu().numpy(), length, length, n, threads=8)
        assert np.array_equal(out, want)


def test_pinned_host_zero_copy(torch_gpu, oracle, golden):
    """Kernels read (and the trailer writer writes) pinned host memory directly:
    the RDMA-registered backing_mem_ integration of INTEGRATION.md 3a."""
    torch = torch_gpu
    n, length = 2000, 4096
    host = torch.empty(n * length, dtype=torch.uint8).pin_memory()
    host.copy_(torch.from_numpy(splitmix64_bytes(9, n * length)))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    rc = C.load().nova_crc32c_batch_strided(host.data_ptr(), length, length, n, None,
                                            out.data_ptr(), 0, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert np.array_equal(u32(out), oracle.batch_strided(host.numpy(), length, length, n))
    # trailers written in place into pinned host memory
    pk = golden["packed"]
    img = torch.from_numpy(splitmix64_bytes(pk["seed"], pk["total"])).pin_memory()
    offs = dev(torch, np.array(pk["offsets"], np.uint64), torch.int64)
    sizes = dev(torch, np.array(pk["sizes"], np.uint32), torch.int32)
    rc = C.load().nova_sstable_write_trailers(img.data_ptr(), offs.data_ptr(), sizes.data_ptr(),
                                              len(pk["sizes"]), C.TYPE(0) | C.TB_QUIRK, None)
    assert rc == 0
    torch.cuda.synchronize()
    h = img.numpy()
    for o, s, tb in zip(pk["offsets"], pk["sizes"], pk["tb_trailer_hex"]):
        assert h[o + s:o + s + 5].tobytes().hex() == tb


def test_concurrent_host_threads(torch_gpu, oracle):
    """Reentrancy (SURVEY 8(b) Threading): several host threads, each on its own
    HIP stream, checksum different batches at the same time."""
    torch = torch_gpu
    import threading
    n, length = 20000, 4096
    bufs = []
    for t in range(6):
        b = torch.empty(n * length, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(b, 100 + t)
        bufs.append(b)
    torch.cuda.synchronize()
    results = [None] * 6
    errors = []

    def work(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                outs = []
                for _ in range(5):
                    outs.append(C.batch_strided(bufs[t], length, length, n, stream=s))
                    outs.append(C.batch(bufs[t], torch.arange(0, n * length, length,
                                                              device="cuda", dtype=torch.int64),
                                        torch.full((n,), length, device="cuda",
                                                   dtype=torch.int32), stream=s))
            s.synchronize()
            results[t] = [u32(o) for o in outs]
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in range(6):
        want = oracle.batch_strided_mt(bufs[t].cpu().numpy(), length, length, n, threads=8)
        for r in results[t]:
            assert np.array_equal(r, want)


def test_concurrent_split_path(torch_gpu, oracle):
    """The split-and-combine path from several host threads at once, each on its
    own stream and on the shared default stream: every call owns its
    stream-ordered scratch, so results never mix."""
    torch = torch_gpu
    import threading
    n, length = 3, (3 << 20) + 5  # 3 blocks of 3 MiB: fixed stride > 64 KiB -> split
    bufs = []
    for t in range(4):
        b = torch.empty(n * length, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(b, 300 + t)
        bufs.append(b)
    torch.cuda.synchronize()
    assert C.describe(n, length, length)["kernel"] == "split"
    results = [None] * 8
    errors = []

    def work(i):
        try:
            t = i % 4
            s = torch.cuda.Stream() if i < 4 else None
            outs = []
            for _ in range(6):
                outs.append(C.batch_strided(bufs[t], length, length, n, stream=s))
            if s is not None:
                s.synchronize()
            else:
                torch.cuda.synchronize()
            results[i] = [u32(o) for o in outs]
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for i in range(8):
        t = i % 4
        want = oracle.batch_strided(bufs[t].cpu().numpy(), length, length, n)
        for r in results[i]:
            assert np.array_equal(r, want), i


@pytest.fixture
def sst_backend(request):
    """Route the nova_sst_queue_* calls to the persistent engine (1) or the
    round-3 coalescing queue (0) for one test."""
    C.engine_set_enabled(request.param)
    yield request.param
    C.engine_set_enabled(-1)


@pytest.mark.parametrize("sst_backend", [1, 0], indirect=True, ids=["engine", "queue"])
def test_sst_queue_concurrent(torch_gpu, oracle, sst_backend):
    """nova_sst_queue_* (DESIGN.md 3.5d, 3.5g): 12 host threads,
    each on its own stream with its own SSTable image (ragged layouts, 0 to 3000
    blocks, gaps between blocks, three trailer types, one with the TableBuilder
    quirk), write trailers then verify with corrupted blocks, many calls each.
    The image is filled asynchronously on the caller's stream right before the
    first call (the request must wait for it).  Every trailer equals the oracle's
    and every verify flags exactly the corrupted blocks.  Engine: every call ran
    on it (no fallback).  Queue: the calls shared launches (batches < requests)."""
    torch = torch_gpu
    import threading
    T, R = 12, 12
    rng = np.random.default_rng(77)
    sizes_n = [0, 1, 7, 64, 500, 3000, 1, 33, 1200, 2048, 250, 9]
    tabs = []
    for t in range(T):
        n = sizes_n[t]
        sz = rng.integers(1, 8193, n).astype(np.uint32)
        gap = rng.integers(0, 4, n).astype(np.uint64)
        offs = np.zeros(n, np.uint64)
        if n:
            offs[1:] = np.cumsum(sz[:-1].astype(np.uint64) + 5 + gap[:-1])
        total = int(offs[-1] + sz[-1] + 5) if n else 16
        bad = rng.choice(n, size=min(n, 1 + t % 4), replace=False) if n else np.zeros(0, np.int64)
        tabs.append(dict(n=n, sz=sz, offs=offs, total=total, bad=np.sort(bad), type=t % 3,
                         quirk=(t == 5)))
    before = C.queue_stats()
    ebefore = C.engine_stats()
    results, errors = [None] * T, []
    # One batch in flight: while it runs, the other threads' calls queue up
    # behind it and the next leader takes them together.  (With 4 slots a fast
    # box can serve Python-paced callers one by one, so "batches < requests"
    # depended on timing.)
    C.queue_set_slots(1)

    def work(t):
        try:
            tb = tabs[t]
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                img = torch.empty(tb["total"] + 64, dtype=torch.uint8, device="cuda")
                offs = torch.from_numpy(tb["offs"].view(np.int64)).to("cuda", non_blocking=False)
                szs = torch.from_numpy(tb["sz"].view(np.int32)).to("cuda", non_blocking=False)
                C.fill_splitmix64(img, 500 + t, stream=s)  # in flight when the queue is called
                for _ in range(R):
                    C.queue_write_trailers(img, offs, szs, tb["type"], tb["quirk"], stream=s)
                good = img.cpu().numpy().copy()
                for j in tb["bad"]:  # corrupt one byte of each chosen block, on s
                    img[int(tb["offs"][j])] ^= 0x5A
                oks, bads = [], []
                for _ in range(R):
                    ok = torch.full((max(tb["n"], 1),), 7, dtype=torch.uint8, device="cuda")
                    nb = torch.zeros(1, dtype=torch.int32, device="cuda")
                    C.queue_verify_blocks(img, offs, szs, ok, nb, stream=s)
                    oks.append(ok.cpu().numpy()[:tb["n"]])
                    bads.append(int(nb.item()))
            s.synchronize()
            results[t] = (good, oks, bads)
        except Exception as e:  # pragma: no cover
            errors.append((t, e))

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    try:
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        C.queue_set_slots(0)
    assert not errors, errors
    calls = 0
    for t in range(T):
        tb, (good, oks, bads) = tabs[t], results[t]
        n = tb["n"]
        calls += 2 * R if n else 0
        if n:
            want = oracle.batch(good, tb["offs"], tb["sz"], None,
                                flags=C.APPEND_TYPE | C.MASK_OUTPUT | C.TYPE(tb["type"]))
            for j in range(n):
                o = int(tb["offs"][j] + tb["sz"][j])
                tr = good[o:o + 5]
                assert tr[0] == tb["type"], (t, j)
                word = int(want[j]).to_bytes(4, "little")
                if tb["quirk"]:
                    word = word[:3] + b"!"
                assert tr[1:].tobytes() == word, (t, j)
        expect = np.ones(n, np.uint8)
        if tb["quirk"] and n:  # TableBuilder's '!' trailer (table/table_builder.cc:206)
            expect[:] = (want >> 24) == 0x21  # verifies only where the CRC's top byte is '!'
        expect[tb["bad"]] = 0
        for ok, nb in zip(oks, bads):
            assert np.array_equal(ok, expect), (t, np.nonzero(ok != expect)[0][:8])
            assert nb == int((expect == 0).sum()), (t, nb)
    if sst_backend:
        eafter = C.engine_stats()
        assert eafter["requests"] - ebefore["requests"] == calls, (ebefore, eafter, calls)
        assert eafter["fallbacks"] == ebefore["fallbacks"], (ebefore, eafter)
        return
    after = C.queue_stats()
    served = after["requests"] - before["requests"]
    assert served == calls, (served, calls)
    assert after["batches"] - before["batches"] < served, (before, after)


@pytest.mark.parametrize("sst_backend", [1, 0], indirect=True, ids=["engine", "queue"])
@pytest.mark.parametrize("threads", [2, 4, 16])
def test_sst_queue_stress(torch_gpu, oracle, threads, sst_backend):
    """nova_sst_queue_* under back-to-back calls (tools/concurrent_sst.py's
    shape): `threads` callers, each verifying its own 1024-block SSTable image
    (4096+U[0,255] B blocks) 60 times with no pause, every third call on a
    copy with one corrupted block; every call's flags and count are checked."""
    torch = torch_gpu
    import threading
    n, R = 1024, 60
    from bench import sst4k_layout
    offs_np, lens_np = sst4k_layout(n, 5)[:2]
    total = int(offs_np[-1]) + int(lens_np[-1]) + 5
    offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
    lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
    imgs, bads = [], []
    for t in range(threads):
        img = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(img, 900 + t)
        C.write_trailers(img, offs, lens)
        bad_img = img.clone()
        j = (37 * t + 11) % n
        bad_img[int(offs_np[j]) + 100] ^= 1
        imgs.append((img, bad_img, j))
    torch.cuda.synchronize()
    errors = []

    def work(t):
        try:
            img, bad_img, j = imgs[t]
            s = torch.cuda.Stream()
            ok = torch.empty(n, dtype=torch.uint8, device="cuda")
            nb = torch.zeros(1, dtype=torch.int32, device="cuda")
            for r in range(R):
                corrupt = r % 3 == 2
                with torch.cuda.stream(s):
                    nb.zero_()
                    C.queue_verify_blocks(bad_img if corrupt else img, offs, lens, ok, nb, stream=s)
                    got, cnt = ok.cpu().numpy(), int(nb.item())
                want = np.ones(n, np.uint8)
                if corrupt:
                    want[j] = 0
                if not np.array_equal(got, want) or cnt != int(corrupt):
                    errors.append((t, r, cnt, np.nonzero(got != want)[0][:4]))
                    return
        except Exception as e:  # pragma: no cover
            errors.append((t, e))

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:4]


def _sst_tables(torch, oracle, ns, seed):
    """SSTable images (4096+U[0,255] B blocks, 5-B trailers) with their oracle
    trailer CRCs (type 0, TableBuilder ordering without the quirk)."""
    from bench import sst4k_layout
    out = []
    for k, n in enumerate(ns):
        offs_np, lens_np, total = sst4k_layout(n, seed + k)
        img = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(img, seed * 131 + k)
        out.append(dict(n=n, offs_np=offs_np, lens_np=lens_np, img=img,
                        offs=torch.from_numpy(offs_np.view(np.int64)).cuda(),
                        lens=torch.from_numpy(lens_np.view(np.int32)).cuda()))
    torch.cuda.synchronize()
    return out


def _trailer_words(oracle, host, offs_np, lens_np):
    return oracle.batch(host, offs_np, lens_np, None, flags=C.APPEND_TYPE | C.MASK_OUTPUT | C.TYPE(0))


def _check_trailers(host, offs_np, lens_np, want):
    ends = offs_np.astype(np.int64) + lens_np.astype(np.int64)
    got = np.stack([host[ends + i] for i in range(5)], axis=1)
    assert np.all(got[:, 0] == 0)
    words = got[:, 1].astype(np.uint32) | (got[:, 2].astype(np.uint32) << 8) | \
        (got[:, 3].astype(np.uint32) << 16) | (got[:, 4].astype(np.uint32) << 24)
    bad = np.nonzero(words != want)[0]
    assert bad.size == 0, bad[:8]


def test_engine_start_stop_restart(torch_gpu, oracle):
    """The persistent engine through its whole life: started
    explicitly, trailers then verify (with one corrupted block) on tables of
    1, 5, 4096 and 20000 blocks, stopped, restarted by the next call, stopped
    again; every result bit-exact, no request fell back to the plain call."""
    torch = torch_gpu
    C.engine_set_enabled(1)
    try:
        C.engine_stop()
        s0 = C.engine_stats()
        C.engine_start()
        assert C.engine_stats()["running"]
        tabs = _sst_tables(torch, oracle, [1, 5, 4096, 20000], 41)
        for cycle in range(2):
            for tb in tabs:
                C.queue_write_trailers(tb["img"], tb["offs"], tb["lens"])
                host = tb["img"].cpu().numpy()
                want = _trailer_words(oracle, host, tb["offs_np"], tb["lens_np"])
                _check_trailers(host, tb["offs_np"], tb["lens_np"], want)
                j = (7 * tb["n"]) // 11
                tb["img"][int(tb["offs_np"][j]) + 3] ^= 0x10
                ok = torch.full((tb["n"],), 9, dtype=torch.uint8, device="cuda")
                nb = torch.zeros(1, dtype=torch.int32, device="cuda")
                C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb)
                exp = np.ones(tb["n"], np.uint8)
                exp[j] = 0
                assert np.array_equal(ok.cpu().numpy(), exp), (cycle, tb["n"])
                assert int(nb.item()) == 1
                tb["img"][int(tb["offs_np"][j]) + 3] ^= 0x10
            C.engine_stop()
            assert not C.engine_stats()["running"]
        s1 = C.engine_stats()
        assert s1["launches"] - s0["launches"] >= 2, (s0, s1)
        assert s1["fallbacks"] == s0["fallbacks"], (s0, s1)
        assert s1["requests"] - s0["requests"] == 16, (s0, s1)
    finally:
        C.engine_set_enabled(-1)


_ENGINE_WRAP_CHILD = r"""
import sys, threading
sys.path.insert(0, %r)
import numpy as np, torch
from novalsm_amd import crc32c as C
from tests.oracle_lib import load_oracle
orc = load_oracle()
C.engine_set_enabled(1)

def table(n, seed, lo, hi):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
    total = int(offs[-1]) + int(lens[-1]) + 5
    img = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(img, seed)
    torch.cuda.synchronize()
    return dict(n=n, img=img, offs_np=offs, lens_np=lens,
                offs=torch.from_numpy(offs.view(np.int64)).cuda(),
                lens=torch.from_numpy(lens.view(np.int32)).cuda())

def check(tb, errs, tag):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        C.queue_write_trailers(tb["img"], tb["offs"], tb["lens"], stream=s)
        host = tb["img"].cpu().numpy()
        want = orc.batch(host, tb["offs_np"], tb["lens_np"], None,
                         flags=C.APPEND_TYPE | C.MASK_OUTPUT | C.TYPE(0))
        ends = tb["offs_np"].astype(np.int64) + tb["lens_np"].astype(np.int64)
        w = sum(host[ends + 1 + i].astype(np.uint32) << (8 * i) for i in range(4))
        if not (np.array_equal(w, want) and (host[ends] == 0).all()):
            errs.append((tag, "trailers", int(np.count_nonzero(w != want))))
            return
        vic = [tb["n"] // 3, tb["n"] - 1]
        for v in vic:
            tb["img"][int(tb["offs_np"][v])] ^= 0x40
        ok = torch.full((tb["n"],), 9, dtype=torch.uint8, device="cuda")
        nb = torch.zeros(1, dtype=torch.int32, device="cuda")
        C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb, stream=s)
        okh = ok.cpu().numpy()
        if sorted(np.nonzero(okh != 1)[0].tolist()) != vic or int(nb.item()) != 2:
            errs.append((tag, "verify", np.nonzero(okh != 1)[0][:4].tolist(), int(nb.item())))
        for v in vic:
            tb["img"][int(tb["offs_np"][v])] ^= 0x40

big = [table(1 << 20, 71 + k, 8, 72) for k in range(2)]   # 1M blocks: 2^18 tickets at 4 per chunk
small = [table(n, 90 + n, 4000, 4300) for n in (3, 700, 4096)]
errs = []
def big_caller():
    for it in range(3):
        for k, tb in enumerate(big):
            check(tb, errs, ("big", it, k))
def small_caller():
    for it in range(40):
        check(small[it %% 3], errs, ("small", it))
th = [threading.Thread(target=big_caller), threading.Thread(target=small_caller)]
for t in th: t.start()
for t in th: t.join()
st = C.engine_stats()
print("ERRS", errs[:4], "FALLBACKS", st["fallbacks"], "REQUESTS", st["requests"])
sys.exit(1 if errs or st["fallbacks"] else 0)
"""


def test_engine_ticket_pages_wrap(torch_gpu):
    """The engine maps ticket pages (16 tickets) to requests as hints, in a
    table of 2^18 tickets -- exactly one 1M-block request at 4 blocks per
    chunk (NOVA_SST_ENGINE_CB=4, read once per process: a child process).
    With a second caller's small tables in flight, later requests' pages
    overwrite a running request's pages, so its waves read hints past their
    own request and must fall back to their cursor (crc32c_engine.hip).  Both
    callers' trailers and verify results (two corrupted blocks per call) are
    checked against the oracle; no request may fall back to the plain call."""
    import os
    import subprocess
    import sys
    root = str(__import__("pathlib").Path(__file__).resolve().parents[1])
    env = dict(os.environ, NOVA_SST_ENGINE_CB="4")
    r = subprocess.run([sys.executable, "-c", _ENGINE_WRAP_CHILD % root], env=env, capture_output=True,
                       text=True, timeout=240, cwd=root)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])


def test_engine_idle_exit_and_buffer_rewrite(torch_gpu, oracle):
    """Between requests the engine stays resident (or exits when idle and is
    relaunched by the next call: both happen here, with a 300 us idle time).
    A caller that rewrites its image and descriptors in place between calls --
    new bytes, new block layout, on its own stream -- must get results for the
    new contents: the engine's loads of caller memory bypass L1
    (kVarEngine), so no line cached from an earlier request is used.  Two
    threads keep the device unevenly loaded while the checked caller runs."""
    torch = torch_gpu
    import threading
    import time
    from bench import sst4k_layout
    C.engine_set_enabled(1)
    C.engine_stop()
    C.engine_set_idle_us(300)
    fb0 = C.engine_stats()["fallbacks"]
    stop = threading.Event()
    errors = []
    noise = _sst_tables(torch, oracle, [3000, 700], 77)

    def load(tb):
        try:
            s = torch.cuda.Stream()
            ok = torch.empty(tb["n"], dtype=torch.uint8, device="cuda")
            with torch.cuda.stream(s):
                C.queue_write_trailers(tb["img"], tb["offs"], tb["lens"], stream=s)
                while not stop.is_set():
                    C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, stream=s)
                    if not bool((ok == 1).all()):
                        errors.append("noise verify")
                        return
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=load, args=(tb,)) for tb in noise]
    try:
        for x in th:
            x.start()
        n = 2048
        cap = n * (4096 + 255 + 5) + 64
        img = torch.empty(cap, dtype=torch.uint8, device="cuda")
        offs = torch.empty(n, dtype=torch.int64, device="cuda")
        lens = torch.empty(n, dtype=torch.int32, device="cuda")
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        for it in range(12):
            offs_np, lens_np, total = sst4k_layout(n, 300 + it)
            with torch.cuda.stream(s):
                C.fill_splitmix64(img, 1000 + it, stream=s)
                offs.copy_(torch.from_numpy(offs_np.view(np.int64)), non_blocking=False)
                lens.copy_(torch.from_numpy(lens_np.view(np.int32)), non_blocking=False)
                C.queue_write_trailers(img, offs, lens, stream=s)
                host = img.cpu().numpy()
            want = _trailer_words(oracle, host, offs_np, lens_np)
            _check_trailers(host, offs_np, lens_np, want)
            with torch.cuda.stream(s):
                C.queue_verify_blocks(img, offs, lens, ok, stream=s)
                got = ok.cpu().numpy()
            assert np.all(got == 1), (it, np.nonzero(got != 1)[0][:8])
            if it % 4 == 3:
                stop.set()  # let the engine go idle and exit
                for x in th:
                    x.join()
                time.sleep(0.01)
                assert not C.engine_stats()["running"]
                stop.clear()
                th = [threading.Thread(target=load, args=(tb,)) for tb in noise]
                for x in th:
                    x.start()
    finally:
        stop.set()
        for x in th:
            x.join()
        C.engine_set_idle_us(0)
        C.engine_stop()
        C.engine_set_enabled(-1)
    assert not errors, errors[:4]
    assert C.engine_stats()["fallbacks"] == fb0


@pytest.mark.parametrize("size", ["one_pass", "two_pass"])
def test_queue_batched_trailers_adjacent_tables(torch_gpu, oracle, size):
    """the coalescing queue's batched trailer writer on four tables
    that are adjacent, unpadded slices of one buffer: above 12288 blocks the
    rounds kernel, and from 2^18 blocks (kTrailerTwoPassMin) the whole-piece
    second pass.  Every trailer equals the oracle's, and no byte outside the
    tables' trailers changes -- in particular not the next table's first
    bytes, which the last block's 64-B trailer piece reaches when it is
    rewritten whole."""
    torch = torch_gpu
    import threading
    import time
    from bench import sst4k_layout
    ns = [5000, 4500, 5100, 4900] if size == "one_pass" else [70000, 66000, 68000, 65000]
    lays = [sst4k_layout(n, 60 + k) for k, n in enumerate(ns)]
    # table k starts where table k-1's last trailer ends, plus 0..40 bytes
    starts, pos = [], 0
    for k, (o, ln, total) in enumerate(lays):
        starts.append(pos)
        pos += total + (7 * k) % 41
    buf = torch.empty(pos + 64, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 4242)
    torch.cuda.synchronize()
    before = buf.cpu().numpy().copy()
    C.engine_set_enabled(0)
    C.queue_set_slots(1)
    views = []
    for k, (o, ln, total) in enumerate(lays):
        views.append((buf[starts[k]:starts[k] + total],
                      torch.from_numpy(o.view(np.int64)).cuda(), torch.from_numpy(ln.view(np.int32)).cuda()))
    errors = []

    def work(k):
        try:
            v, o, ln = views[k]
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                C.queue_write_trailers(v, o, ln, stream=s)
            s.synchronize()
        except Exception as e:  # pragma: no cover
            errors.append(e)

    # the queue is held (test hook) until all four callers
    # are enqueued, then released: the front one leads and takes all four in
    # ONE batch -- deterministic, no timing window, no retries.
    try:
        qb = C.queue_stats()
        assert C.queue_hold(1) == 0
        th = [threading.Thread(target=work, args=(k,)) for k in range(len(ns))]
        for x in th:
            x.start()
        deadline = time.perf_counter() + 30.0
        while C.queue_hold(-1) < len(ns) and time.perf_counter() < deadline and not errors:
            time.sleep(0.001)
        queued = C.queue_hold(0)
        for x in th:
            x.join()
        qa = C.queue_stats()
    finally:
        C.queue_hold(0)
        C.queue_set_slots(0)
        C.engine_set_enabled(-1)
    assert queued == len(ns), queued
    assert qa["requests"] - qb["requests"] == len(ns), (qb, qa)
    assert not errors, errors
    assert qa["batches"] - qb["batches"] == 1, (qb, qa)  # one batch of all four tables
    after = buf.cpu().numpy()
    expect = before.copy()
    for k, (o, ln, total) in enumerate(lays):
        base = starts[k]
        want = _trailer_words(oracle, before[base:base + total], o, ln)
        ends = base + o.astype(np.int64) + ln.astype(np.int64)
        expect[ends] = 0
        for b in range(4):
            expect[ends + 1 + b] = ((want >> np.uint32(8 * b)) & np.uint32(0xFF)).astype(np.uint8)
    diff = np.nonzero(after != expect)[0]
    assert diff.size == 0, diff[:8]


@pytest.mark.parametrize("kernel", ["default", "logstream"])
def test_log_records_write_verify(torch_gpu, golden, oracle, kernel):
    """MANIFEST/WAL record CRCs (db/log_writer.cc:99-114,
    db/log_reader.cc:196-262) against the reference-generated log fixture (a
    log::Writer layout with FULL/FIRST/MIDDLE/LAST fragments over ~20 blocks),
    then the reader's per-record statuses against the oracle.  "logstream"
    forces the whole-image log-stream experiment (diagnostics build only,
    DESIGN.md 3.5e; the product always runs the rounds kernel)."""
    if kernel == "logstream":
        with C.diagnostics() as L:
            L.nova_diag_set_variable_kernel(4)
            _golden_log_checks(torch_gpu, golden, oracle)
    else:
        _golden_log_checks(torch_gpu, golden, oracle)


def _golden_log_checks(torch, golden, oracle):
    from tests.test_oracle_golden import golden_log_image
    host, offs = golden_log_image(golden)
    buf = dev(torch, host)
    doffs = dev(torch, offs, torch.int64)
    C.log_write_crcs(buf, doffs)
    h = buf.cpu().numpy()
    for o, c in zip(offs, golden["log"]["header_crc"]):
        assert int.from_bytes(h[int(o):int(o) + 4].tobytes(), "little") == c
    ok, bad = C.log_verify_records(buf, doffs)
    assert (ok.cpu().numpy() == C.LOG_OK).all() and int(bad.item()) == 0
    victims = [3, 50, 299]
    for v in victims:
        o = int(offs[v]) + 6  # corrupt the type byte (covered by the crc)
        buf[o] ^= 0x01
    ok, bad = C.log_verify_records(buf, doffs)
    assert sorted(np.nonzero(ok.cpu().numpy() == C.LOG_CHECKSUM_MISMATCH)[0].tolist()) == victims
    assert int(bad.item()) == 3
    assert np.array_equal(ok.cpu().numpy(), oracle.log_check(buf.cpu().numpy(), offs))


def _log_reader_cases():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "log_reader_cases.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("kernel", ["default", "units"])
@pytest.mark.parametrize("case", _log_reader_cases(), ids=lambda c: c["name"])
def test_log_reader_cases_device(torch_gpu, oracle, case, kernel):
    """nova_log_verify_records on the files the reference's
    own reader tests write and edit (db/log_test.cc, tests/golden/
    log_reader_cases.json; MarginalTrailer, ShortTrailer, AlignedEof,
    TruncatedTrailingRecordIsIgnored, BadLength, BadLengthAtEndIsIgnored,
    ChecksumMismatch, MissingLast/PartialLastIsIgnored, ...): every record's
    status and n_bad equal what that test asserts.  The buffer extends past
    buf_len (the bytes there must not matter); "units" forces the units
    kernel's log path."""
    torch = torch_gpu
    from tests.oracle_lib import log_reader_case
    host, offs, expect = log_reader_case(oracle, case)
    buf = dev(torch, np.concatenate([host, np.full(512, 0x5A, np.uint8)]))
    doffs = dev(torch, offs, torch.int64)
    ctx = C.diagnostics() if kernel != "default" else None
    if ctx:
        ctx.__enter__()
        C.set_tuning(16, 4096)  # forced segments: the units kernel's log path
    try:
        st, bad = C.log_verify_records(buf, doffs, buf_len=case["buf_len"])
        got = st.cpu().numpy()
        assert np.array_equal(got, expect), (case["name"], np.nonzero(got != expect)[0][:8])
        assert int(bad.item()) == case["n_bad"]
    finally:
        if ctx:
            ctx.__exit__(None, None, None)


@pytest.mark.parametrize("kernel", ["default", "units", "logstream"])
def test_log_record_bounds(torch_gpu, golden, oracle, kernel):
    """ADVICE r01 / db/log_reader.cc:196-247: a record whose length field runs
    past its 32 KiB block or the image is never read (bad length, counted; or
    EOF if the image ends inside that block), a type-0 length-0 record is
    skipped, a header past buf_len is not read; write skips them all.  Status
    per record equals the oracle's ReadPhysicalRecord restatement."""
    from tests.test_oracle_golden import golden_log_image
    torch = torch_gpu
    host, offs = golden_log_image(golden)
    oracle.log_write(host, offs)
    n = len(offs)
    rng = np.random.default_rng(9)
    vic = rng.choice(n - 1, 30, replace=False)
    for k, v in enumerate(vic):
        o = int(offs[v])
        if k % 3 == 0:
            host[o + 5] = 0xFF  # length >= 65280: past any block
        elif k % 3 == 1:
            host[o + 4:o + 7] = 0  # zero record
        else:
            host[o + 8] ^= 0x80  # payload / CRC mismatch (or a 1-byte record's crc field)
    want_img = host.copy()
    cut = host.size - 3  # the image ends inside the last record: EOF for it
    # plus descriptors past the image (EOF) and in the last 1-6 bytes of the
    # full block 0 (its trailer: skipped, not reported -- ADVICE r02)
    from novalsm_amd.synth import LOG_BLOCK
    assert cut > LOG_BLOCK
    offs_x = np.concatenate([offs, np.array([cut - 2, cut + 100], np.uint64),
                             np.array([LOG_BLOCK - k for k in range(1, 7)], np.uint64)])
    buf = dev(torch, np.concatenate([host, np.zeros(256, np.uint8)]))
    doffs = dev(torch, offs_x, torch.int64)
    ctx = C.diagnostics() if kernel != "default" else None
    if ctx:
        L = ctx.__enter__()
        if kernel == "units":
            C.set_tuning(16, 4096)  # forced segments: the units kernel's log path
        else:
            L.nova_diag_set_variable_kernel(4)
    try:
        st, bad = C.log_verify_records(buf, doffs, buf_len=cut)
        want = oracle.log_check(host, offs_x, buf_len=cut)
        assert np.array_equal(st.cpu().numpy(), want)
        assert int(bad.item()) == int(((want == 0) | (want == 2)).sum())
        assert {0, 1, 2, 3, 4, 5} <= set(want.tolist())
        assert (want[-6:] == C.LOG_BLOCK_TRAILER).all()
        # an image of whole blocks: past its end is EOF, a full block's last
        # bytes are its trailer
        st2, bad2 = C.log_verify_records(buf, doffs[-6:], buf_len=LOG_BLOCK)
        assert (st2.cpu().numpy() == C.LOG_BLOCK_TRAILER).all() and int(bad2.item()) == 0
        d3 = dev(torch, np.array([LOG_BLOCK, LOG_BLOCK + 5], np.uint64), torch.int64)
        st3, bad3 = C.log_verify_records(buf, d3, buf_len=LOG_BLOCK)
        assert (st3.cpu().numpy() == C.LOG_TRUNCATED).all() and int(bad3.item()) == 0
        # write: recompute every readable record; the rest are left untouched
        before = buf.cpu().numpy().copy()
        C.log_write_crcs(buf, doffs, buf_len=cut)
        got = buf.cpu().numpy()
        for i, o in enumerate(offs_x.tolist()):
            o = int(o)
            if want[i] in (0, 1, 3):  # readable: crc field = Mask(Value(type + payload))
                ln = int(host[o + 4]) | (int(host[o + 5]) << 8)
                c = oracle.mask(oracle.value(want_img[o + 6:o + 7 + ln].tobytes()))
                assert int.from_bytes(got[o:o + 4].tobytes(), "little") == c, i
            elif o + 4 <= got.size:
                assert np.array_equal(got[o:o + 4], before[o:o + 4]), i
    finally:
        if ctx:
            ctx.__exit__(None, None, None)


@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("plen", [1, 15, 16, 17, 4096, 16389, 100003, (1 << 20) + 3])
@pytest.mark.parametrize("k", [1, 3, 8])
def test_xor_parity(torch_gpu, oracle, align, plen, k):
    """XOR parity block (ltc/stoc_file_client_impl.cpp:334-349).
    The last fragment's parity region ends exactly at the end of the buffer."""
    torch = torch_gpu
    rng = np.random.default_rng(plen * 10 + k)
    offs = np.array([f * (plen + 64) + (0 if align else int(rng.integers(0, 16)))
                     for f in range(k)], np.uint64)
    total = int(offs[-1]) + plen
    host = splitmix64_bytes(plen + k, total)
    out = C.xor_parity(dev(torch, host), dev(torch, offs, torch.int64), plen)
    assert np.array_equal(out.cpu().numpy(), oracle.xor_parity(host, offs, plen))


@pytest.mark.parametrize("align", [True, False])
def test_xor_parity_variants(torch_gpu, oracle, align):
    """Every instantiated (chunks per lane, fragments per load group) form of
    xor_parity_kernel, on a capped grid-stride walk and on the product's
    one-pass grid, equals the oracle (diagnostics knob; the default is 8 x 1,
    one pass)."""
    torch = torch_gpu
    k, plen = 8, (1 << 20) + 3
    rng = np.random.default_rng(41)
    offs = np.array([f * (plen + 64) + (0 if align else int(rng.integers(0, 16)))
                     for f in range(k)], np.uint64)
    host = splitmix64_bytes(77, int(offs[-1]) + plen)
    want = oracle.xor_parity(host, offs, plen)
    d, do = dev(torch, host), dev(torch, offs, torch.int64)
    with C.diagnostics() as L:
        for u, fu in [(1, 1), (2, 1), (4, 1), (4, 2), (4, 4), (2, 4), (2, 2), (8, 1), (8, 2),
                      (1, 8), (2, 8), (1, 4), (1, 2), (16, 1)]:
            for cap in (8, 0xff):
                L.nova_diag_set_parity_variant(u | fu << 5 | cap << 9)
                out = C.xor_parity(d, do, plen)
                assert np.array_equal(out.cpu().numpy(), want), (u, fu, cap)
        L.nova_diag_set_parity_variant(0)


def test_claim_counters_reset_between_launches(torch_gpu, oracle):
    """Each launch leaves its stream's claim counters zeroed for the next one
    (no per-launch memset).  Launches of varying grid size back to back on one
    stream, then on a second stream, alternating the stream and units kernels:
    a stale counter would skip rounds and leave sentinel outputs behind."""
    torch = torch_gpu
    length = 4096
    nmax = 60000
    host = splitmix64_bytes(123, nmax * length + 64)
    buf = dev(torch, host)
    want_all = oracle.batch_strided_mt(host, length, length, nmax, threads=8)
    rng = np.random.default_rng(5)
    s2 = torch.cuda.Stream()
    for it in range(40):
        n = int(rng.choice([1, 7, 300, 5000, 20011, nmax]))
        stream = s2 if it % 3 == 2 else None
        out = torch.full((n,), -559038737, dtype=torch.int32, device="cuda")  # 0xDEADBEEF
        if it % 4 == 1:  # offsets/lengths -> variable-length units kernel
            lens = torch.full((n,), length, dtype=torch.int32, device="cuda")
            offs = torch.arange(n, dtype=torch.int64, device="cuda") * length
            C.batch(buf, offs, lens, out=out, stream=stream)
        else:
            C.batch_strided(buf, length, length, n, out=out, stream=stream)
        if stream is not None:
            stream.synchronize()
        assert np.array_equal(u32(out), want_all[:n]), (it, n)


@pytest.mark.parametrize("kernel,lanes,chunk,waves", [
    (2, 0, 0, 0), (2, 2, 0, 0), (2, 4, 0, 0), (2, 8, 0, 0), (2, 16, 0, 0), (2, 16, 9, 0),
    (2, 16, 64, 0), (2, 8, 0, 3), (2, 4, 40, 5), (2, 16, 0, 1), (2, 16, 0, 12), (2, 8, 0, 10),
    (3, 0, 3, 0), (3, 2, 3, 0), (3, 4, 3, 0), (3, 8, 3, 0), (3, 16, 3, 0), (3, 16, 3, 1),
    (3, 8, 3, 5), (3, 4, 3, 12), (3, 16, 0, 0), (3, 8, 0, 7), (3, 16, 1, 0), (3, 4, 1, 0),
    (3, 16, 4 * 4 + 3, 0), (3, 16, 64 * 4 + 2, 3), (3, 8, 8 * 4 + 3, 0), (3, 2, 32 * 4 + 3, 0)])
def test_flat_many_blocks(torch_gpu, oracle, kernel, lanes, chunk, waves):
    """Flat (2) and rounds (3) kernels with enough blocks for every wave to
    switch descriptor banks and claim chunks many times, including the
    stealing tail: mixed tiny/empty/long blocks at random offsets (descriptors
    not in address order), random inits, for every lane count, chunk size,
    wave count, sorted and unsorted rounds."""
    torch = torch_gpu
    with C.diagnostics() as L:
        C.set_tuning(lanes, 0)
        L.nova_diag_set_variable_kernel(kernel)
        if kernel == 3:  # rounds kernel: "chunk" = chunk blocks * 4 + sort mode (3: per chunk)
            L.nova_diag_set_rounds_sort(2 if (chunk & 3) == 3 else (chunk & 3))
            L.nova_diag_set_chunk_blocks(chunk >> 2)
        else:
            L.nova_diag_set_chunk_blocks(chunk)
        L.nova_diag_set_stream_waves(waves)
        _many_blocks_checks(torch, oracle, lanes, chunk, waves)


def _many_blocks_checks(torch, oracle, lanes, chunk, waves):
    rng = np.random.default_rng(1000 + lanes * 7 + chunk + waves)
    n = 120000
    lens = rng.choice([0, 1, 2, 3, 4, 5, 17, 100, 600, 1500, 4096, 9000], n,
                      p=[.02, .02, .02, .02, .02, .05, .1, .25, .2, .1, .15, .05]).astype(np.uint32)
    lens += (rng.integers(0, 64, n) * (lens > 5)).astype(np.uint32)
    pos = np.cumsum(lens.astype(np.uint64) + rng.integers(0, 9, n).astype(np.uint64))
    offs = (pos - lens.astype(np.uint64)).astype(np.uint64)
    perm = rng.permutation(n)
    offs, lens = offs[perm], lens[perm]
    host = splitmix64_bytes(lanes + 3, int(pos[-1]) + 64)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    buf = dev(torch, host)
    want = oracle.batch(host, offs, lens, init)
    do, dl, di = (dev(torch, offs, torch.int64), dev(torch, lens, torch.int32),
                  dev(torch, init.view(np.int32)))
    for _ in range(3):  # the schedule is dynamic: several launches, sentinel-filled outputs
        out = torch.full((n,), -559038737, dtype=torch.int32, device="cuda")  # 0xDEADBEEF
        C.batch(buf, do, dl, init=di, out=out)
        bad = np.nonzero(u32(out) != want)[0]
        assert bad.size == 0, [(int(offs[i]), int(lens[i])) for i in bad[:5]]


@pytest.mark.parametrize("kernel,lanes,chunk", [
    (0, 0, 0), (1, 4, 0), (1, 16, 0), (2, 0, 0), (2, 2, 0), (2, 4, 0), (2, 8, 0), (2, 16, 0),
    (2, 8, 16), (2, 4, 17), (2, 16, 64), (3, 0, 0), (3, 2, 0), (3, 4, 0), (3, 16, 0),
    (3, 8, 16), (3, 8, 32), (3, 16, 16), (3, 8, 8), (4, 0, 0)])
def test_log_many_records(torch_gpu, oracle, kernel, lanes, chunk):
    """Log record CRC write + verify over a log::Writer image (db/log_writer.cc:
    53-114) with enough records to exercise every kernel's header pipeline
    (db/log_reader.cc:249-262), every lane count and chunk size; kernel 0 is
    the product dispatch, 1-3 force units / flat / rounds, 4 the log-stream
    kernel (diagnostics build).  ~90 records per 32 KiB block: the log-stream
    kernel reloads its 64-record windows and folds mid-swath."""
    torch = torch_gpu
    if kernel == 0:
        _log_many_checks(torch, oracle, lanes, chunk)
        return
    with C.diagnostics() as L:
        C.set_tuning(lanes, 0)
        L.nova_diag_set_chunk_blocks(chunk)
        L.nova_diag_set_variable_kernel(kernel)
        _log_many_checks(torch, oracle, lanes, chunk)


def _log_many_checks(torch, oracle, lanes, chunk):
    from novalsm_amd.synth import log_image
    rng = np.random.default_rng(77 + lanes + chunk)
    n = 60000
    plen = rng.integers(0, 700, n)
    plen[rng.integers(0, n, 200)] = rng.integers(0, 3, 200)  # empty / tiny payloads
    plen[rng.integers(0, n, 20)] = rng.integers(30000, 70000, 20)  # fragmented records
    host, offs, _, _ = log_image(lanes + 11, plen)
    buf = dev(torch, host)
    doffs = dev(torch, offs, torch.int64)
    C.log_write_crcs(buf, doffs)
    want = host.copy()
    oracle.log_write(want, offs)
    got = buf.cpu().numpy()
    assert np.array_equal(got, want)
    ok, bad = C.log_verify_records(buf, doffs)
    assert (ok.cpu().numpy() == C.LOG_OK).all() and int(bad.item()) == 0
    victims = rng.choice(len(offs), 25, replace=False)
    for v in victims:
        buf[int(offs[v]) + 6] ^= 0x02  # type byte: a FULL/FIRST... record stays readable
    ok, bad = C.log_verify_records(buf, doffs)
    okh = ok.cpu().numpy()
    assert sorted(np.nonzero(okh == C.LOG_CHECKSUM_MISMATCH)[0].tolist()) == sorted(victims.tolist())
    assert int(bad.item()) == len(victims)


@pytest.mark.parametrize("case", ["clean", "corrupt", "permuted"])
def test_log_write_store_forms(torch_gpu, oracle, case):
    """The diagnostics build's whole-64-B-piece form of large log writes
    (>= 32768 records; log_window_kernel decides per record) against the
    product's byte stores.  Over a big log::Writer image with bad-length and
    zero records, an image cut inside a record (buf_len), descriptors past the
    image and (case "permuted") descriptors out of file order, the WHOLE images
    must be equal, and on the clean image equal to what the oracle's
    log::Writer restatement writes (db/log_writer.cc:99-114)."""
    from novalsm_amd.synth import log_image
    torch = torch_gpu
    rng = np.random.default_rng(["clean", "corrupt", "permuted"].index(case) + 5)
    n = 40000
    plen = rng.integers(0, 300, n)
    plen[rng.integers(0, n, 300)] = rng.integers(0, 3, 300)
    host, offs, _, _ = log_image(3, plen)
    offs = np.asarray(offs, np.uint64)
    buf_len = host.size
    if case != "clean":
        for k, v in enumerate(rng.choice(len(offs) - 1, 200, replace=False)):
            o = int(offs[v])
            if k % 2 == 0:
                host[o + 5] = 0xFF  # bad length: not read, not written
            else:
                host[o + 4:o + 7] = 0  # zero record
        buf_len = host.size - 3  # the last record is cut (EOF)
        offs = np.concatenate([offs, np.array([buf_len - 2, buf_len + 100], np.uint64)])
    if case == "permuted":
        offs = offs[rng.permutation(len(offs))]
    img = np.concatenate([host, np.zeros(256, np.uint8)])
    doffs = dev(torch, offs, torch.int64)
    a = dev(torch, img)
    C.log_write_crcs(a, doffs, buf_len=buf_len)
    b = dev(torch, img)
    with C.diagnostics() as L:
        L.nova_diag_set_trailer_single_pass(3)  # whole-piece stores
        C.log_write_crcs(b, doffs, buf_len=buf_len)
    ga, gb = a.cpu().numpy(), b.cpu().numpy()
    diff = np.nonzero(ga != gb)[0]
    assert diff.size == 0, (diff[:10], ga[diff[:10]], gb[diff[:10]])
    if case == "clean":
        want = img.copy()
        oracle.log_write(want, offs)
        assert np.array_equal(ga, want)


@pytest.mark.parametrize("mode", ["store", "trailers", "verify"])
def test_large_blocks_hint_same_results(torch_gpu, oracle, mode):
    """NOVA_CRC32C_HINT_LARGE_BLOCKS only changes the schedule (units kernel with
    32 KiB segments instead of whole-block rounds): results are identical and
    equal to the oracle on an SSTable image of mixed 100 B - 200 KiB blocks."""
    torch = torch_gpu
    rng = np.random.default_rng(4242)
    n = 3000
    lens = rng.choice([100, 4096, 16384, 65536, 200000], n, p=[.2, .3, .2, .2, .1])
    lens = (lens + rng.integers(0, 64, n)).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
    host = splitmix64_bytes(99, int(offs[-1]) + int(lens[-1]) + 5 + 64).copy()
    do, dl = dev(torch, offs, torch.int64), dev(torch, lens, torch.int32)
    if mode == "store":
        want = oracle.batch(host, offs, lens, None)
        for hint in (0, C.HINT_LARGE_BLOCKS):
            out = torch.full((n,), -559038737, dtype=torch.int32, device="cuda")
            C.batch(dev(torch, host), do, dl, flags=hint, out=out)
            assert np.array_equal(u32(out), want), hint
    elif mode == "trailers":
        bufs = []
        for hint in (False, True):
            buf = dev(torch, host)
            C.write_trailers(buf, do, dl, 0, True, hint_large=hint)
            bufs.append(buf.cpu().numpy())
        with C.diagnostics() as L:  # the two-pass A/B (CRC array + scatter)
            L.nova_diag_set_trailer_single_pass(2)
            buf = dev(torch, host)
            C.write_trailers(buf, do, dl, 0, True)
            bufs.append(buf.cpu().numpy())
        assert np.array_equal(bufs[0], bufs[1]) and np.array_equal(bufs[0], bufs[2])
        for i in np.linspace(0, n - 1, 40).astype(np.int64):
            o, ln = int(offs[i]), int(lens[i])
            assert oracle.trailer(host[o:o + ln].tobytes(), 0, True) == bufs[0][o + ln:o + ln + 5].tobytes()
    else:
        buf = dev(torch, host)
        C.write_trailers(buf, do, dl, 0, False)
        victims = rng.choice(n, 7, replace=False)
        for v in victims:
            buf[int(offs[v]) + 1] ^= 0x10
        for tune in ((0, 0), (16, 32768)):  # default rounds; forced units with segments
            C.set_tuning(*tune)
            ok, bad = C.verify_blocks(buf, do, dl)
            assert sorted(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == sorted(victims.tolist())
            assert int(bad.item()) == len(victims)
        C.set_tuning(0, 0)
        ok, bad = C.verify_blocks(buf, do, dl, hint_large=True)  # units kernel via the hint
        assert sorted(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == sorted(victims.tolist())
        assert int(bad.item()) == len(victims)


@pytest.mark.parametrize("n", [1, 5, 12288, 12289, 49152, 98303, 98304, 196608])
def test_batch_size_dispatch_thresholds(torch_gpu, oracle, n):
    """The burst kernel up to 4 blocks per wave slot (12288 on 256 CUs x 12
    waves), then plan() sizes the rounds kernel to the batch (8-, 16- and
    32-block chunks at 16x / 32x two blocks per slot).  Every side of each threshold,
    on ragged unaligned blocks, through store, trailers and verify, matches the
    oracle; describe() names the chunk the dispatcher picked."""
    torch = torch_gpu
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 300, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
    host = splitmix64_bytes(n + 17, int(offs[-1]) + int(lens[-1]) + 5 + 64).copy()
    do, dl = dev(torch, offs, torch.int64), dev(torch, lens, torch.int32)
    out = C.batch(dev(torch, host), do, dl)
    assert np.array_equal(u32(out), oracle.batch(host, offs, lens, None))
    buf = dev(torch, host)
    C.write_trailers(buf, do, dl, 0, False)
    h = buf.cpu().numpy()
    for i in np.linspace(0, n - 1, min(n, 64)).astype(np.int64):
        o, ln = int(offs[i]), int(lens[i])
        assert oracle.trailer(host[o:o + ln].tobytes(), 0, False) == h[o + ln:o + ln + 5].tobytes()
    victims = rng.choice(n, min(n, 3), replace=False)
    for v in victims:
        if lens[v]:
            buf[int(offs[v])] ^= 0x01
        else:  # empty block: corrupt its stored CRC
            buf[int(offs[v]) + 1] ^= 0x01
    ok, bad = C.verify_blocks(buf, do, dl)
    assert sorted(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == sorted(victims.tolist())
    assert int(bad.item()) == len(victims)
    d = C.describe(n, 0, 0, variable=True)
    if n <= 12288:
        assert d["kernel"].startswith("crc32c_burst_kernel"), d
    else:
        want_chunk = 32 if n >= 196608 else 16 if n >= 98304 else 8
        assert d["chunk_blocks"] == want_chunk and d["lanes_per_block"] == 8


def _log_stream_image(torch, seed, plen, pad=256, shift=0):
    """A log::Writer image (novalsm_amd/synth.log_image) on the device, placed
    `shift` bytes into its allocation (the image start need not be aligned)."""
    from novalsm_amd.synth import log_image
    host, offs, _, _ = log_image(seed, plen)
    full = np.zeros(shift + host.size + pad, np.uint8)
    full[shift:shift + host.size] = host
    t = dev(torch, full)
    return host, offs, t[shift:shift + host.size]


@pytest.mark.parametrize("shape", ["u4096", "tiny", "fragments", "mixed"])
@pytest.mark.parametrize("shift", [0, 5, 64, 127])
def test_logstream_kernel(torch_gpu, oracle, shape, shift):
    """The log-stream kernel on log::Writer images of every
    record-size regime -- U[1,4096] B payloads (the bench shape), tiny records
    (payload 0..40 B: hundreds per block, several ending in one swath, window
    reloads), 30-70 KB logical records (every block one fragment) and a mix --
    at image starts 0/5/64/127 bytes into a 128-B line.  Write equals the
    oracle's log::Writer CRCs byte for byte over the whole image; verify
    reports every record OK, then exactly the corrupted ones."""
    torch = torch_gpu
    import zlib
    rng = np.random.default_rng(zlib.crc32(f"{shape}/{shift}".encode()))  # (hash() is salted per process)
    if shape == "u4096":
        plen = rng.integers(1, 4097, 3000)
    elif shape == "tiny":
        plen = rng.integers(0, 41, 40000)
    elif shape == "fragments":
        plen = rng.integers(30000, 70000, 60)
    else:
        plen = np.concatenate([rng.integers(0, 4, 2000), rng.integers(1, 4097, 2000),
                               rng.integers(30000, 70000, 10), rng.integers(0, 300, 3000)])
        rng.shuffle(plen)
    host, offs, buf = _log_stream_image(torch, 17 + shift, plen, shift=shift)
    doffs = dev(torch, offs, torch.int64)
    want = host.copy()
    oracle.log_write(want, offs)
    with C.diagnostics() as L:
        L.nova_diag_set_variable_kernel(4)
        for _ in range(2):  # dynamic schedule: two launches
            C.log_write_crcs(buf, doffs)
            got = buf.cpu().numpy()
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (bad[:8], np.searchsorted(offs.astype(np.int64), bad[:8], "right") - 1)
        ok, nbad = C.log_verify_records(buf, doffs)
        assert (ok.cpu().numpy() == C.LOG_OK).all() and int(nbad.item()) == 0
        # a zero-length FIRST fragment (a block with exactly a header's room
        # left) flipped to type 0 reads as a zero-type record, kBadRecord,
        # before its CRC is checked (db/log_reader.cc:243-249): not a victim
        o64 = offs.astype(np.int64)
        cand = np.flatnonzero(~((host[o64 + 6] == 2) & (host[o64 + 4] == 0) & (host[o64 + 5] == 0)))
        victims = rng.choice(cand, min(40, len(cand)), replace=False)
        for v in victims:
            buf[int(offs[v]) + 6] ^= 0x02  # type byte: covered by the CRC, record stays readable
        ok, nbad = C.log_verify_records(buf, doffs)
        okh = ok.cpu().numpy()
        assert np.array_equal(okh, oracle.log_check(buf.cpu().numpy(), offs))
        assert sorted(np.nonzero(okh == C.LOG_CHECKSUM_MISMATCH)[0].tolist()) == sorted(victims.tolist())
        assert int(nbad.item()) == len(victims)


@pytest.mark.parametrize("case", ["unsorted", "overlap", "subset", "gaps"])
def test_logstream_preconditions(torch_gpu, oracle, case):
    """The log-stream kernel's preconditions and their gated fallback: offsets
    out of file order (pre-pass flag) or a read record starting inside the
    previous one (in-kernel flag) rerun the batch on the rounds kernel -- the
    statuses and the mismatch count equal the oracle's and are counted once.
    A sparse subset of records ("subset") and every other record ("gaps") stay
    on the log-stream kernel: the skipped records are masked out like block
    trailers, and write touches only the selected headers."""
    torch = torch_gpu
    rng = np.random.default_rng(31)
    plen = rng.integers(1, 2000, 4000)
    host, offs, buf = _log_stream_image(torch, 5, plen)
    blank = host.copy()  # CRC fields not yet written
    oracle.log_write(host, offs)
    n = len(offs)
    for v in rng.choice(n, 30, replace=False):
        host[int(offs[v]) + 9] ^= 0x10  # payload byte (or the next header): mismatches
    buf.copy_(torch.from_numpy(host))
    o = offs.copy()
    if case == "unsorted":
        o = o[rng.permutation(n)]
    elif case == "overlap":
        o = np.sort(np.concatenate([o, o[rng.choice(n, 5, replace=False)] + 3])).astype(np.uint64)
    elif case == "subset":
        o = np.sort(o[rng.choice(n, n // 7, replace=False)]).astype(np.uint64)
    else:
        o = o[::2].copy()
    want = oracle.log_check(host, o)
    with C.diagnostics() as L:
        L.nova_diag_set_variable_kernel(4)
        ok, nbad = C.log_verify_records(buf, dev(torch, o, torch.int64))
    assert np.array_equal(ok.cpu().numpy(), want)
    assert int(nbad.item()) == int(((want == 0) | (want == 2)).sum())
    if case in ("subset", "gaps"):  # write: the selected records only
        fresh = dev(torch, blank)
        exp = blank.copy()
        oracle.log_write(exp, o)
        with C.diagnostics() as L:
            L.nova_diag_set_variable_kernel(4)
            C.log_write_crcs(fresh, dev(torch, o, torch.int64))
        assert np.array_equal(fresh.cpu().numpy(), exp)


@pytest.mark.parametrize("order", ["file", "file_g8", "shuffled", "windows_only", "in_place", "unsorted",
                                   "window_1024", "window_64"])
def test_log_sorted_windows(torch_gpu, oracle, order):
    """Log verify of >= 64K records runs in the order of the windowed
    step-count sort (log_sort_kernel), keyed from the offsets
    alone, with results by position moved back by log_unperm_kernel.  The
    results are the oracle's whatever the key says: offsets in file order,
    shuffled (the keys are then garbage), the window sort without the
    per-chunk sort (diagnostics; log write sorted too, by position), results
    stored in place (window 128), no sort at all, and the widest and narrowest
    windows the adaptive choice takes (1024; 64 with log write sorted too);
    write is bit-exact over the image, verify finds exactly the corrupted
    records.  These records average ~0.7 KiB, so the default plan ("file")
    runs 4-lane groups without the sort; every other case forces the 8-lane
    groups the sort runs with."""
    from novalsm_amd.synth import log_image
    torch = torch_gpu
    rng = np.random.default_rng(91)
    n = 150000
    plen = rng.integers(0, 1400, n)
    plen[rng.integers(0, n, 300)] = rng.integers(0, 3, 300)
    plen[rng.integers(0, n, 30)] = rng.integers(20000, 70000, 30)
    host, offs, _, _ = log_image(29, plen)
    assert len(offs) >= 1 << 16
    if order == "shuffled":
        offs = offs[rng.permutation(len(offs))]
    buf = dev(torch, host)
    doffs = dev(torch, offs, torch.int64)
    want = host.copy()
    oracle.log_write(want, offs)

    def run():
        C.log_write_crcs(buf, doffs)
        assert np.array_equal(buf.cpu().numpy(), want)
        ok, bad = C.log_verify_records(buf, doffs)
        assert (ok.cpu().numpy() == C.LOG_OK).all() and int(bad.item()) == 0
        victims = rng.choice(len(offs), 40, replace=False)
        for v in victims:
            buf[int(offs[v]) + 6] ^= 0x02
        ok, bad = C.log_verify_records(buf, doffs)
        okh = ok.cpu().numpy()
        assert sorted(np.nonzero(okh == C.LOG_CHECKSUM_MISMATCH)[0].tolist()) == sorted(victims.tolist())
        assert int(bad.item()) == len(victims)
        for v in victims:
            buf[int(offs[v]) + 6] ^= 0x02

    if order != "file":
        C.set_tuning(8, 0)  # (reset by the autouse fixture)
    if order in ("windows_only", "in_place", "unsorted", "window_1024", "window_64"):
        with C.diagnostics() as L:
            C.set_tuning(8, 0)  # the diagnostics library's own knob (reset on exit)
            L.nova_diag_set_rounds_sort({"windows_only": 3, "in_place": 5, "unsorted": 0}.get(order, 2))
            L.nova_diag_set_log_window({"windows_only": -512, "in_place": -128, "unsorted": 0,
                                        "window_1024": 1024, "window_64": -64}[order])
            run()
    else:
        run()


@pytest.mark.parametrize("pmax", [64, 600, 800, 1500, 2400, 3000])
def test_log_plan_by_record_size(torch_gpu, oracle, pmax):
    """The default log plan picks its group width from the mean record span
    (buf_len / n): 2-lane groups for write below 350 B and for verify below
    420 B, 4-lane groups below 1280 B, 8-lane groups (verify: with the windowed
    pre-sort) above.  Each side of every threshold: write is
    bit-exact over the image, verify is clean, and finds exactly the records
    whose payload was corrupted."""
    from novalsm_amd.synth import log_image
    torch = torch_gpu
    rng = np.random.default_rng(pmax)
    n = max(70000, (48 << 20) // (pmax // 2 + 7))
    n = min(n, 300000)
    plen = rng.integers(1, pmax + 1, n)
    host, offs, _, _ = log_image(31, plen)
    assert len(offs) >= 1 << 16
    span = host.size // len(offs)
    for verify, pair in ((False, 350), (True, 420)):
        g = 2 if span < pair else 4 if span < 1280 else 8
        k = C.describe(len(offs) + 1, host.size // (len(offs) + 1), 0, log=True, log_verify=verify)["kernel"]
        assert k.startswith(f"crc32c_rounds_kernel<{g}, "), (span, verify, k)
    # plus a probe at the end of the file: TRUNCATED, so nothing may be stored
    # for it (its header bytes read as a length past the block)
    offs = np.append(offs, np.uint64(host.size))
    buf = dev(torch, np.append(host, np.full(64, 0xA5, np.uint8)))
    doffs = dev(torch, offs, torch.int64)
    want = host.copy()
    oracle.log_write(want, offs[:-1])  # (the oracle writes at every offset it is given)
    C.log_write_crcs(buf, doffs)
    got = buf.cpu().numpy()
    assert np.array_equal(got[:host.size], want) and (got[host.size:] == 0xA5).all()
    ok, bad = C.log_verify_records(buf[:host.size], doffs)
    okh = ok.cpu().numpy()
    assert (okh[:-1] == C.LOG_OK).all() and okh[-1] == C.LOG_TRUNCATED and int(bad.item()) == 0
    victims = rng.choice(len(offs) - 1, 50, replace=False)
    for v in victims:
        buf[int(offs[v]) + 6] ^= 0x02  # the type byte is CRC input
    ok, bad = C.log_verify_records(buf[:host.size], doffs)
    okh = ok.cpu().numpy()
    assert sorted(np.nonzero(okh == C.LOG_CHECKSUM_MISMATCH)[0].tolist()) == sorted(victims.tolist())
    assert int(bad.item()) == len(victims)


@pytest.mark.parametrize("kernel", ["default", "logstream"])
def test_log_96mib(torch_gpu, oracle, kernel):
    """A 96 MiB log::Writer image with U[1,4096] B payloads (the bench_ops log
    shape): write is bit-exact over the whole image vs the oracle, verify is
    clean, and after 64 type bytes are flipped the statuses and the count
    equal the oracle's -- through the product dispatch and through the
    log-stream experiment (diagnostics build)."""
    if kernel == "logstream":
        with C.diagnostics() as L:
            L.nova_diag_set_variable_kernel(4)
            _log_96mib_checks(torch_gpu, oracle)
    else:
        _log_96mib_checks(torch_gpu, oracle)


def _log_96mib_checks(torch_gpu, oracle):
    torch = torch_gpu
    rng = np.random.default_rng(8)
    plen = rng.integers(1, 4097, (96 << 20) // 2055)
    host, offs, buf = _log_stream_image(torch, 23, plen)
    assert host.size >= 64 << 20
    doffs = dev(torch, offs, torch.int64)
    want = host.copy()
    oracle.log_write(want, offs)
    C.log_write_crcs(buf, doffs)
    assert np.array_equal(buf.cpu().numpy(), want)
    ok, nbad = C.log_verify_records(buf, doffs)
    assert (ok.cpu().numpy() == C.LOG_OK).all() and int(nbad.item()) == 0
    victims = rng.choice(len(offs), 64, replace=False)
    for v in victims:
        buf[int(offs[v]) + 6] ^= 0x02  # type byte (covered by the CRC)
    ok, nbad = C.log_verify_records(buf, doffs)
    want_st = oracle.log_check(buf.cpu().numpy(), offs)
    assert np.array_equal(ok.cpu().numpy(), want_st)
    assert int(nbad.item()) == int(((want_st == 0) | (want_st == 2)).sum()) >= 60


@pytest.mark.parametrize("flags", [0, C.MASK_OUTPUT | C.APPEND_TYPE | C.TYPE(1), C.RAW])
def test_split_few_large_blocks(torch_gpu, oracle, flags):
    """Few large blocks take the split-and-combine path (pieces over the whole
    device, linear parts folded with M_{16 m} shifts, then Extend's init and the
    mode epilogue): fixed-stride blocks over 64 KiB in small batches, and
    variable batches of <= 1024 blocks with HINT_LARGE_BLOCKS.  Equal to the
    oracle's util/crc32c.cc restatement for odd lengths, odd offsets, per-block
    init values and every flag; the same batches with the split path turned
    off (diagnostics) give the same words."""
    torch = torch_gpu
    rng = np.random.default_rng(314)
    # fixed stride: 1 x (5 MiB + 13) at offset 3; 7 x (300 KiB + 5), stride + 11 (both
    # > 64 piece slots per block: finish kernel); 2000 x (96 KiB + 16): 32 slots, the
    # fold finishes each block itself
    for n, L, pad, base in ((1, (5 << 20) + 13, 0, 3), (7, (300 << 10) + 5, 11, 1),
                            (2000, (96 << 10) + 16, 0, 0)):
        stride = L + pad
        host = splitmix64_bytes(n + 40, base + n * stride + 16).copy()
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        assert C.describe(n, L, stride)["kernel"] == "split"
        buf = dev(torch, host)
        if flags & C.RAW:  # raw(D) = Extend(0xFFFFFFFF, D) ^ 0xFFFFFFFF; init is ignored
            want = oracle.batch_strided(host[base:], stride, L, n,
                                        np.full(n, 0xFFFFFFFF, np.uint32)) ^ np.uint32(0xFFFFFFFF)
        else:
            want = oracle.batch_strided(host[base:], stride, L, n, init, flags)
        for split in (0, -1):
            out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            with C.diagnostics() as D:
                D.nova_diag_set_split(split)
                C.batch_strided(buf, stride, L, n, init=dev(torch, init.view(np.int32)), flags=flags,
                                out=out, base_offset=base)
            assert np.array_equal(u32(out), want), (n, L, split)
    # variable with the hint: lengths 0 .. 33 MiB, out of address order
    lens = np.array([1, (70 << 10) + 3, (2 << 20) + 7, 0, (33 << 20) + 1, 5000, 65536, 17],
                    dtype=np.uint32)
    n = len(lens)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(9))
    offs += 5
    perm = rng.permutation(n)
    offs, lens = offs[perm], lens[perm]
    host = splitmix64_bytes(77, int(offs.max() + lens.max()) + 64).copy()
    if flags & C.RAW:
        want = oracle.batch(host, offs, lens, np.full(n, 0xFFFFFFFF, np.uint32)) ^ np.uint32(
            0xFFFFFFFF)
    else:
        want = oracle.batch(host, offs, lens, None, flags)
    assert C.describe(n, 0, 0, variable=True, large=True)["kernel"] == "split"
    out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    C.batch(dev(torch, host), dev(torch, offs, torch.int64), dev(torch, lens, torch.int32),
            flags=flags | C.HINT_LARGE_BLOCKS, out=out)
    assert np.array_equal(u32(out), want)


@pytest.mark.parametrize("n", [1, 3, 64, 1024])
def test_split_trailers_and_verify(torch_gpu, oracle, n):
    """Trailers (HINT_LARGE_BLOCKS, <= 1024 blocks: the split path) written
    byte-for-byte as table/table_builder.cc:202-206 with the quirk, nothing
    else in the image touched; read-verify through the split path (the hint via
    nova_sstable_verify_blocks_ex, and forced) flags exactly the corrupted
    blocks."""
    torch = torch_gpu
    rng = np.random.default_rng(n)
    lens = rng.choice([3, 4096, 70000, 300000, 1 << 20], n).astype(np.uint32)
    lens = (lens + rng.integers(0, 50, n)).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
    total = int(offs[-1]) + int(lens[-1]) + 5 + 64
    host = splitmix64_bytes(n + 3, total).copy()
    want = host.copy()
    for i in range(n):
        o, ln = int(offs[i]), int(lens[i])
        want[o + ln:o + ln + 5] = np.frombuffer(oracle.trailer(host[o:o + ln].tobytes(), 0, True),
                                                dtype=np.uint8)
    do, dl = dev(torch, offs, torch.int64), dev(torch, lens, torch.int32)
    buf = dev(torch, host)
    C.write_trailers(buf, do, dl, 0, True, hint_large=True)
    assert np.array_equal(buf.cpu().numpy(), want)
    # StoC order (verifiable), then corrupt a few blocks
    buf = dev(torch, host)
    C.write_trailers(buf, do, dl, 0, False, hint_large=True)
    victims = rng.choice(n, min(n, 3), replace=False)
    for v in victims:
        buf[int(offs[v]) + int(lens[v]) // 2] ^= 0x40
    ok, bad = C.verify_blocks(buf, do, dl, hint_large=True)
    assert sorted(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == sorted(victims.tolist())
    assert int(bad.item()) == len(victims)
    with C.diagnostics() as D:
        D.nova_diag_set_split(1)
        ok, bad = C.verify_blocks(buf, do, dl)
    assert sorted(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == sorted(victims.tolist())
    assert int(bad.item()) == len(victims)
