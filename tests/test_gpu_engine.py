"""The persistent per-SSTable engine sharing the GPU (round 5):
yields to other launches of the library, takes failed requests back before any
plain call, keeps its results exact under mixed callers, and survives a waiter
that starts late by more than a whole ring turn.

Run on a real MI355X:  python -m pytest tests -m gpu
"""
import json
import threading
import time

import numpy as np
import pytest

from novalsm_amd import crc32c as C

pytestmark = pytest.mark.gpu

RING = 1024  # crc32c_engine.hip kRing


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    C.load(build_if_missing=True)
    assert C.load().nova_device_init() == 0
    return torch


@pytest.fixture
def engine_on():
    C.engine_set_enabled(1)
    C.engine_reset()
    yield
    C.engine_set_timeout_ms(0)
    C.engine_set_idle_us(0)
    C.engine_set_slice_us(0)
    C.engine_reset()
    C.engine_set_enabled(-1)


def _sst_table(torch, oracle, n, seed, victims=()):
    """An SSTable image (4096+U[0,255] B blocks, StoC trailers) with some blocks
    corrupted; the oracle's expected flags."""
    from bench import sst4k_layout
    offs_np, lens_np, total = sst4k_layout(n, seed)
    img = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(img, 1000 + seed)
    offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
    lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
    C.write_trailers(img, offs, lens)
    torch.cuda.synchronize()
    host = img.cpu().numpy()
    want = np.array([oracle.verify(host[int(o):int(o) + int(ln) + 5].tobytes())
                     for o, ln in zip(offs_np, lens_np)], np.uint8)
    assert want.all()
    for v in victims:
        img[int(offs_np[v]) + 11] ^= 0x08
        want[v] = 0
    torch.cuda.synchronize()
    return dict(n=n, img=img, offs=offs, lens=lens, offs_np=offs_np, lens_np=lens_np, want=want)


def _plain_inputs(torch, oracle):
    """The plain thread's three calls, with expected results from the oracle:
    an SSTable verify (2 corrupted blocks), a log verify (3 corrupted records)
    and a CRC batch of mixed block sizes."""
    from novalsm_amd.callers import Plain
    from novalsm_amd.synth import log_image
    keep = []
    v = _sst_table(torch, oracle, 2048, 71, victims=(5, 1500))
    rng = np.random.default_rng(5)
    plen = rng.integers(0, 700, 20000)
    host, loffs, _, _ = log_image(13, plen)
    oracle.log_write(host, loffs)
    vic = rng.choice(len(loffs), 3, replace=False)
    for r in vic:
        host[int(loffs[r]) + 6] ^= 0x02
    lbuf = torch.from_numpy(host.copy()).cuda()
    ldoffs = torch.from_numpy(np.asarray(loffs, np.int64)).cuda()
    lwant = oracle.log_check(host, loffs).astype(np.uint8)
    lbad = int((lwant == C.LOG_CHECKSUM_MISMATCH).sum())
    assert lbad == 3
    bl = rng.choice([4096, 16384, 65536], 600).astype(np.uint32) + rng.integers(1, 64, 600).astype(np.uint32)
    bo = np.zeros(600, np.uint64)
    bo[1:] = np.cumsum(bl[:-1].astype(np.uint64))
    bhost = np.frombuffer(np.random.default_rng(9).bytes(int(bo[-1] + bl[-1]) + 64), np.uint8).copy()
    bwant = oracle.batch(bhost, bo, bl, None).astype(np.uint32)
    bbuf = torch.from_numpy(bhost).cuda()
    bdo = torch.from_numpy(bo.view(np.int64)).cuda()
    bdl = torch.from_numpy(bl.view(np.int32)).cuda()
    vwant = np.ascontiguousarray(v["want"])
    keep += [v, lbuf, ldoffs, lwant, bbuf, bdo, bdl, bwant, vwant]
    p = Plain(v_img=v["img"].data_ptr(), v_offs=v["offs"].data_ptr(), v_lens=v["lens"].data_ptr(), v_n=v["n"],
              v_expect_ok=vwant.ctypes.data, v_expect_bad=2,
              l_img=lbuf.data_ptr(), l_len=len(host), l_offs=ldoffs.data_ptr(), l_n=len(loffs),
              l_expect=lwant.ctypes.data, l_expect_bad=lbad,
              b_img=bbuf.data_ptr(), b_offs=bdo.data_ptr(), b_lens=bdl.data_ptr(), b_n=600,
              b_expect=bwant.ctypes.data, gap_us=0.0)
    torch.cuda.synchronize()
    return p, keep


@pytest.mark.parametrize("op", ["verify", "trailers"])
def test_engine_mixed_callers(torch_gpu, oracle, engine_on, op):
    """8 native threads hammer nova_sst_queue_* on their
    own 4096-block tables for 1 s while a 9th thread issues plain
    nova_sstable_verify_blocks, nova_log_verify_records and nova_crc32c_batch
    calls on its own stream, one every 0.5 ms (below the yield-storm rate; back
    to back: test_engine_yield_storm_goes_plain).  Every engine call's result and every
    plain call's result is exact (sst_callers.cpp checks them natively against
    expectations taken from the oracle), nothing falls back or times out, the
    engine yields to the plain calls (its instances exit for them), and the
    plain calls' largest latency is bounded: 2 ms, the yield's whole budget
    (the requests the engine had taken, its exit, and the plain call itself)."""
    from novalsm_amd import callers
    plain, keep = _plain_inputs(torch_gpu, oracle)
    plain.gap_us = 500.0
    r = callers.run(op, 8, 4096, 1.0, "engine", warm_s=0.3, seed=3, plain=plain)
    print(json.dumps(r))
    assert r["verified"] and r["wrong_results"] == 0 and r["rc"] == 0, r
    e, pl = r["engine"], r["plain"]
    assert e["fallbacks"] == 0 and e["timeouts"] == 0 and e["errors"] == 0 and e["unsafe"] == 0, e
    assert e["exits_yield"] >= 1 and e["storm_declined"] == 0, e
    for name, s in pl.items():
        assert s["wrong"] == 0, (name, s)
        assert s["calls"] >= 10, (name, s)
        assert s["max_us"] <= 2000.0, (name, s)
    assert r["calls_in_window"] >= 1000, r  # the engine callers kept going
    del keep


def test_engine_yield_storm_goes_plain(torch_gpu, oracle, engine_on):
    """Plain calls back to back (~7900 instance exits for yields a second) made
    every engine instance exit after a few requests: 8 engine callers fell to ~1.2 TB/s,
    half of what their direct calls reach.  In such a storm the engine
    declines requests for 20 ms at a time and the callers run the plain call
    (storm_declined counts them; they are not fallbacks).  Every result exact,
    nothing failed, the plain calls' latency bounded as with yields."""
    from novalsm_amd import callers
    plain, keep = _plain_inputs(torch_gpu, oracle)
    plain.gap_us = 0.0
    r = callers.run("verify", 8, 4096, 1.0, "engine", warm_s=0.3, seed=4, plain=plain)
    print(json.dumps(r))
    assert r["verified"] and r["wrong_results"] == 0 and r["rc"] == 0, r
    e, pl = r["engine"], r["plain"]
    assert e["fallbacks"] == 0 and e["timeouts"] == 0 and e["errors"] == 0 and e["unsafe"] == 0, e
    assert e["storm_declined"] >= 1, e
    for name, s in pl.items():
        assert s["wrong"] == 0 and s["calls"] >= 10 and s["max_us"] <= 2000.0, (name, s)
    assert r["calls_in_window"] >= 1000, r
    del keep
    # the storm is over once the plain calls stop: the next requests run on the engine
    time.sleep(0.05)
    c0 = C.engine_counters()
    tb = _sst_table(torch_gpu, oracle, 256, 91, victims=(17,))
    ok = torch_gpu.empty(tb["n"], dtype=torch_gpu.uint8, device="cuda")
    nb = torch_gpu.zeros(1, dtype=torch_gpu.int32, device="cuda")
    torch_gpu.cuda.synchronize()
    for _ in range(3):
        C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb)
    c1 = C.engine_counters()
    assert np.array_equal(ok.cpu().numpy(), tb["want"])
    assert c1["requests"] - c0["requests"] >= 1 and c1["fallbacks"] == c0["fallbacks"], (c0, c1)


def test_engine_yields_to_a_plain_call(torch_gpu, oracle, engine_on):
    """A resident engine with a long idle time (500 ms) holds every CU's LDS;
    a plain verify on another stream must not wait for its idle exit: the
    plain call makes it yield (exits_yield counts it), finishes in well under
    the idle time, and the next queue call relaunches the engine."""
    torch = torch_gpu
    C.engine_stop()
    C.engine_set_idle_us(500000)
    C.engine_set_slice_us(None)  # no time slice: only the yield can end the instance early
    tb = _sst_table(torch, oracle, 1024, 33, victims=(7,))
    ok = torch.empty(tb["n"], dtype=torch.uint8, device="cuda")
    nb = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    ok2 = torch.empty(tb["n"], dtype=torch.uint8, device="cuda")
    nb2 = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # (a device-wide sync waits for a resident instance: not below)
    C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb)
    assert np.array_equal(ok.cpu().numpy(), tb["want"]) and int(nb.item()) == 1
    assert C.engine_counters()["running"] == 1
    c0 = C.engine_counters()
    t0 = time.perf_counter()
    C.verify_blocks(tb["img"], tb["offs"], tb["lens"], stream=s, ok=ok2, bad=nb2)
    s.synchronize()
    dt = time.perf_counter() - t0
    assert np.array_equal(ok2.cpu().numpy(), tb["want"]) and int(nb2.item()) == 1
    c1 = C.engine_counters()
    assert dt < 0.1, dt  # not the 500 ms idle exit
    time.sleep(0.01)
    nb.zero_()
    C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb)
    assert np.array_equal(ok.cpu().numpy(), tb["want"]) and int(nb.item()) == 1
    c2 = C.engine_counters()
    assert c2["exits_yield"] - c0["exits_yield"] >= 1, (c0, c1, c2)
    assert c2["launches"] - c0["launches"] >= 1 and c2["fallbacks"] == c0["fallbacks"], (c0, c2)
    C.engine_set_slice_us(0)
    C.engine_stop()


def test_engine_waiter_past_ring_turn(torch_gpu, oracle, engine_on):
    """VERDICT r04 item 5, the round-4 hang: one caller's waiter starts 400 ms
    late (nova_sst_engine_set_wait_delay_us), while four other threads complete
    more than a whole ring turn (1024) of requests, so the caller's ring slot
    and completion word are reused before it looks.  It must still see its
    request done (the word only grows: a >= test), with the right flags, no
    timeout, no fallback and no relaunch storm."""
    torch = torch_gpu
    C.engine_set_slice_us(None)  # no time slice: every relaunch below would be a storm
    C.engine_stop()
    late = _sst_table(torch, oracle, 4096, 21, victims=(100, 4000))
    small = [_sst_table(torch, oracle, 1, 50 + k) for k in range(4)]
    c0 = C.engine_counters()
    res, errors, ends = {}, [], []
    started = threading.Event()

    def late_caller():
        try:
            C.engine_set_wait_delay_us(400000)
            ok = torch.empty(late["n"], dtype=torch.uint8, device="cuda")
            nb = torch.zeros(1, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            started.set()
            t0 = time.perf_counter()
            C.queue_verify_blocks(late["img"], late["offs"], late["lens"], ok, nb)
            res["span"] = (t0, time.perf_counter())
            res["ok"], res["bad"] = ok.cpu().numpy(), int(nb.item())
        except Exception as e:  # pragma: no cover
            errors.append(e)
        finally:
            C.engine_set_wait_delay_us(0)

    def filler(tb):
        try:
            ok = torch.empty(1, dtype=torch.uint8, device="cuda")
            s = torch.cuda.Stream()
            started.wait()
            deadline = time.perf_counter() + 0.38
            while time.perf_counter() < deadline:
                C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, stream=s)
                ends.append(time.perf_counter())
            if int(ok.cpu()[0]) != 1:
                errors.append("filler flags")
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=late_caller)] + [threading.Thread(target=filler, args=(tb,)) for tb in small]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    t0, t1 = res["span"]
    inside = sum(1 for t in ends if t0 < t < t1)
    assert inside > RING, (inside, len(ends))  # more than a ring turn completed while it slept
    assert np.array_equal(res["ok"], late["want"]) and res["bad"] == 2
    c1 = C.engine_counters()
    assert c1["fallbacks"] == c0["fallbacks"] and c1["timeouts"] == c0["timeouts"], (c0, c1)
    assert c1["errors"] == c0["errors"] and c1["taken_back"] == c0["taken_back"], (c0, c1)
    assert c1["launches"] - c0["launches"] <= 3, (c0, c1)


def test_engine_take_back_when_held_off(torch_gpu, oracle, engine_on):
    """a request whose engine cannot run -- here a foreign
    kernel (nova_diag_hold_cus, another library's, so no yield) holds every
    CU's LDS for 400 ms -- times out (30 ms) and is taken back before the plain
    call computes it: results exact, one timeout, one take-back, one fallback.
    When the held engine instance finally starts it must skip the request:
    sentinels written into the outputs after the call returned stay untouched.
    After the backoff the engine serves requests again."""
    torch = torch_gpu
    D = C.load_diag()
    C.engine_stop()
    tb = _sst_table(torch, oracle, 4096, 44, victims=(9, 3000))
    ok = torch.empty(tb["n"], dtype=torch.uint8, device="cuda")
    nb = torch.zeros(1, dtype=torch.int32, device="cuda")
    C.engine_set_timeout_ms(30)
    hold = torch.cuda.Stream()
    torch.cuda.synchronize()
    assert D.nova_diag_hold_cus(400000, hold.cuda_stream) == 0
    time.sleep(0.02)  # the hold occupies every CU
    c0 = C.engine_counters()
    t0 = time.perf_counter()
    C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb)
    dt = time.perf_counter() - t0
    c1 = C.engine_counters()
    assert np.array_equal(ok.cpu().numpy(), tb["want"]) and int(nb.item()) == 2
    assert c1["timeouts"] - c0["timeouts"] == 1 and c1["taken_back"] - c0["taken_back"] == 1, (c0, c1)
    assert c1["fallbacks"] - c0["fallbacks"] == 1 and c1["unsafe"] == c0["unsafe"], (c0, c1)
    assert not c1["broken"], c1  # (the 100 ms backoff ran out while the plain call waited for the hold)
    assert dt > 0.2, dt  # the plain call itself waited for the hold
    ok.fill_(0xEE)
    nb.fill_(12345)
    torch.cuda.synchronize()
    hold.synchronize()
    time.sleep(0.3)  # the held instance has started and skipped the request
    torch.cuda.synchronize()
    assert (ok.cpu().numpy() == 0xEE).all() and int(nb.item()) == 12345
    C.engine_set_timeout_ms(0)
    C.engine_reset()
    nb.zero_()
    C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb)
    assert np.array_equal(ok.cpu().numpy(), tb["want"]) and int(nb.item()) == 2
    c2 = C.engine_counters()
    assert c2["fallbacks"] == c1["fallbacks"] and c2["requests"] - c1["requests"] == 1, (c1, c2)
    C.engine_stop()


def test_engine_lost_request_frees_its_slot(torch_gpu, oracle, engine_on):
    """an instance that took a request and ended without
    finishing it (here a "lost" exit: test hooks make the workers run no chunk
    and cut the give-up and idle times to 1 us, so the dispatcher gives up on
    the table ~1 us after taking it, whatever the engine's speed) left
    that request's completion words unwritten; no later instance revisits it,
    so its ring slot never freed and the request reaching that slot a ring
    turn later waited 1 s and fell back.  Now the take-back writes them once
    the instance has ended (host_marked_done): the failed call's results are
    exact (plain call), and more than a ring turn of engine calls after it
    all run on the engine -- no fallback, no 1-s stall."""
    torch = torch_gpu
    C.engine_stop()
    big = _sst_table(torch, oracle, 131072, 81, victims=(3, 120000))
    small = _sst_table(torch, oracle, 1, 82)
    ok = torch.empty(big["n"], dtype=torch.uint8, device="cuda")
    nb = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    c0 = C.engine_counters()
    try:
        C.engine_set_give_up_us(1)
        C.engine_set_idle_us(1)
        C.engine_set_drop_chunks(True)
        C.queue_verify_blocks(big["img"], big["offs"], big["lens"], ok, nb)
    finally:
        C.engine_set_give_up_us(0)
        C.engine_set_idle_us(0)
        C.engine_set_drop_chunks(False)
    assert np.array_equal(ok.cpu().numpy(), big["want"]) and int(nb.item()) == 2
    c1 = C.engine_counters()
    assert c1["exits_lost"] - c0["exits_lost"] >= 1 or c1["errors"] - c0["errors"] >= 1, (c0, c1)
    assert c1["fallbacks"] - c0["fallbacks"] == 1 and c1["taken_back"] - c0["taken_back"] == 1, (c0, c1)
    assert c1["host_marked_done"] - c0["host_marked_done"] == 1 and not c1["broken"], (c0, c1)
    C.engine_reset()  # end the backoff
    ok1 = torch.empty(1, dtype=torch.uint8, device="cuda")
    worst = 0.0
    for _ in range(RING + 64):
        t0 = time.perf_counter()
        C.queue_verify_blocks(small["img"], small["offs"], small["lens"], ok1)
        worst = max(worst, time.perf_counter() - t0)
    assert int(ok1.cpu()[0]) == 1
    c2 = C.engine_counters()
    assert c2["fallbacks"] == c1["fallbacks"] and c2["requests"] - c1["requests"] == RING + 64, (c1, c2)
    assert worst < 0.5, worst  # no ring-full wait (kRingWaitMs = 1 s)
    C.engine_stop()


def test_engine_stop_under_traffic(torch_gpu, oracle, engine_on):
    """nova_sst_engine_stop while four threads keep calling: the stop takes
    effect (the dispatcher stops taking requests even though new ones keep
    arriving), returns, and the callers' next requests relaunch the engine;
    every result exact, nothing falls back."""
    torch = torch_gpu
    tabs = [_sst_table(torch, oracle, 512, 60 + k, victims=(k,)) for k in range(4)]
    stop = threading.Event()
    errors, counts = [], [0] * 4
    c0 = C.engine_counters()

    def caller(k):
        try:
            tb = tabs[k]
            s = torch.cuda.Stream()
            ok = torch.empty(tb["n"], dtype=torch.uint8, device="cuda")
            nb = torch.zeros(1, dtype=torch.int32, device="cuda")
            while not stop.is_set():
                with torch.cuda.stream(s):
                    nb.zero_()
                    C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb, stream=s)
                    if not np.array_equal(ok.cpu().numpy(), tb["want"]) or int(nb.item()) != 1:
                        errors.append(k)
                        return
                counts[k] += 1
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=caller, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for _ in range(5):
        time.sleep(0.05)
        C.engine_stop()
    time.sleep(0.05)
    stop.set()
    for x in th:
        x.join()
    assert not errors, errors
    c1 = C.engine_counters()
    assert c1["exits_stop"] - c0["exits_stop"] >= 3, (c0, c1)
    assert c1["fallbacks"] == c0["fallbacks"] and c1["timeouts"] == c0["timeouts"], (c0, c1)
    assert min(counts) > 0, counts


def test_engine_leaves_other_streams_alone(torch_gpu, engine_on):
    """HIP maps streams onto a few shared hardware queues whose packets run in
    order, so a resident kernel on a shared queue blocks every stream mapped to
    it for as long as requests arrive (round 5: a torch op waited 1.6 s,
    tools/queue_probe.py).  The engine is launched as a cooperative kernel,
    which runs on a queue of its own, from a non-blocking stream: while two
    native threads keep it busy, a small torch op on each of 16 fresh streams
    and on the null stream finishes in milliseconds, and a device-wide sync
    returns once the running instance ends its 20 ms time slice."""
    torch = torch_gpu
    from novalsm_amd import callers
    res, errors = {}, []

    def bg():
        try:
            res["bg"] = callers.run("verify", 2, 4096, 1.5, "engine", warm_s=0.1, seed=8)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    t = threading.Thread(target=bg)
    t.start()
    time.sleep(0.4)
    x = torch.empty(1 << 20, device="cuda")
    lat = []
    for _ in range(16):
        s = torch.cuda.Stream()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            x.zero_()
        s.synchronize()
        lat.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    float(x.sum().item())  # the null stream
    null = time.perf_counter() - t0
    t0 = time.perf_counter()
    torch.cuda.synchronize()  # device-wide: waits for the running instance, one time slice (20 ms)
    dsync = time.perf_counter() - t0
    busy = C.engine_counters()["running"]
    t.join()
    assert not errors, errors
    assert res["bg"]["verified"], res["bg"]
    assert busy == 1  # the engine was resident throughout
    assert max(lat) < 0.1 and null < 0.1 and dsync < 0.05, (lat, null, dsync)


@pytest.mark.parametrize("env", [{"NOVA_SST_ENGINE_RING": "host"}, {"NOVA_SST_ENGINE_PAGE_POLL": "0"}],
                         ids=["host_ring", "no_page_poll"])
def test_engine_alternate_paths(torch_gpu, env):
    """The request ring in pinned host memory (the path of a device without a
    large BAR) and workers that wait for the end word only (no page polls):
    8 native callers for 0.5 s in a child process (the settings are read when
    the engine starts), every result exact, nothing falls back."""
    import os
    import subprocess
    import sys
    code = ("import json, sys; sys.path.insert(0, %r); from novalsm_amd import callers; "
            "print(json.dumps(callers.run('verify', 8, 4096, 0.5, 'engine', warm_s=0.1, seed=11)))"
            % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True,
                       text=True, timeout=100)
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and line, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    r = json.loads(line[-1])
    assert r["verified"] and r["wrong_results"] == 0 and r["rc"] == 0, r
    e = r["engine"]
    assert e["fallbacks"] == 0 and e["timeouts"] == 0 and e["errors"] == 0, e
    assert e["ring_device"] == (0 if "NOVA_SST_ENGINE_RING" in env else e["ring_device"]), e
    assert r["calls_in_window"] >= 100, r


def test_engine_mixed_request_sizes(torch_gpu, oracle, engine_on):
    """Tiny and large requests in flight together: 6 threads, each with tables
    of 1, 2, 7, 64, 65, 300, 1024 and 5000 blocks, alternating verify (one
    corrupted block) and trailer writes (trailer bytes scrubbed first) 6 times
    over.  Small requests leave most ticket groups without tickets (their
    completion words are written at publication), share ticket pages with
    their neighbours and count in either completion bank; every result equals
    the plain path's (trailers) or the expectation (verify)."""
    import threading
    from bench import sst4k_layout
    torch = torch_gpu
    sizes = [1, 2, 7, 64, 65, 300, 1024, 5000]
    tabs = []
    for k, n in enumerate(sizes):
        offs_np, lens_np, total = sst4k_layout(n, 70 + k)
        img = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(img, 7000 + k)
        offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
        lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
        C.write_trailers(img, offs, lens)  # the plain path: the reference image
        torch.cuda.synchronize()
        ends = torch.from_numpy((offs_np.astype(np.int64) + lens_np.astype(np.int64))).cuda()
        tabs.append(dict(n=n, offs=offs, lens=lens, want=img.clone(), ends=ends,
                         j=(5 * n) // 7, cut=int(offs_np[(5 * n) // 7]) + 2))
    want0 = tabs[0]["want"].cpu().numpy()
    assert oracle.verify(want0[int(tabs[0]["offs"][0]):int(tabs[0]["ends"][0]) + 5].tobytes())
    errors = []

    def work(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                mine = [dict(tb, img=tb["want"].clone()) for tb in tabs]
                s.synchronize()
                for rep in range(6):
                    for k in range((t + rep) % len(sizes), (t + rep) % len(sizes) + len(sizes)):
                        tb = mine[k % len(sizes)]
                        if (rep + k) % 2:
                            for b in range(5):  # scrub the trailers, then write them
                                tb["img"][tb["ends"] + b] = 0xEE
                            C.queue_write_trailers(tb["img"], tb["offs"], tb["lens"], stream=s)
                            if not torch.equal(tb["img"], tb["want"]):
                                errors.append((t, rep, tb["n"], "trailers"))
                                return
                        else:
                            tb["img"][tb["cut"]] ^= 0x40
                            ok = torch.full((tb["n"],), 7, dtype=torch.uint8, device="cuda")
                            nb = torch.zeros(1, dtype=torch.int32, device="cuda")
                            C.queue_verify_blocks(tb["img"], tb["offs"], tb["lens"], ok, nb, stream=s)
                            okh = ok.cpu().numpy()
                            exp = np.ones(tb["n"], np.uint8)
                            exp[tb["j"]] = 0
                            if not np.array_equal(okh, exp) or int(nb.item()) != 1:
                                errors.append((t, rep, tb["n"], "verify", np.nonzero(okh != exp)[0][:4]))
                                return
                            tb["img"][tb["cut"]] ^= 0x40
        except Exception as e:  # pragma: no cover
            errors.append((t, repr(e)))

    c0 = C.engine_counters()
    th = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    c1 = C.engine_counters()
    assert not errors, errors[:4]
    assert c1["requests"] - c0["requests"] >= 6 * 6 * len(sizes), (c0, c1)
    assert c1["fallbacks"] == c0["fallbacks"] and c1["timeouts"] == c0["timeouts"], (c0, c1)


def test_engine_empty_and_single_block_requests(torch_gpu, oracle, engine_on):
    """Edge sizes through the engine: an empty table returns at once without a
    request (the counter is left alone), a one-block table and a block of 0
    bytes (its CRC covers the type byte only) verify and write exactly."""
    torch = torch_gpu
    img = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    ok = torch.empty(0, dtype=torch.uint8, device="cuda")
    nb = torch.full((1,), 5, dtype=torch.int32, device="cuda")
    r0 = C.engine_counters()["requests"]
    C.queue_verify_blocks(img, e, e.to(torch.int32), ok, nb)
    C.queue_write_trailers(img, e, e.to(torch.int32))
    assert C.engine_counters()["requests"] == r0 and int(nb.item()) == 5
    C.fill_splitmix64(img, 99)
    for lens in ([1000], [0], [0, 17, 0]):
        offs_np = np.cumsum([0] + [ln + 5 for ln in lens[:-1]]).astype(np.int64)
        offs = torch.from_numpy(offs_np).cuda()
        ln_t = torch.tensor(lens, dtype=torch.int32, device="cuda")
        C.queue_write_trailers(img, offs, ln_t)
        host = img.cpu().numpy()
        for o, ln in zip(offs_np, lens):
            blk = host[int(o):int(o) + ln + 5].tobytes()
            assert oracle.trailer(blk[:ln], 0, False) == blk[ln:], (lens, ln)
        okv = torch.full((len(lens),), 9, dtype=torch.uint8, device="cuda")
        nb.zero_()
        C.queue_verify_blocks(img, offs, ln_t, okv, nb)
        assert okv.cpu().numpy().tolist() == [1] * len(lens) and int(nb.item()) == 0, lens


def test_engine_one_pass_build_in_child():
    """The default engine is the 12-wave build (a block's loads in two passes,
    DESIGN.md 3.5g "Round 6"); NOVA_SST_ENGINE_WAVES <= 8 selects the round-5
    one-pass build.  A child process (the variable is read once per process)
    runs both ops at 1 and 4 callers on that build through the native caller
    harness, which checks every call's flags and the final trailers against
    the oracle: all verified, nothing fell back, launched at 8 waves."""
    import os
    import subprocess
    import sys
    code = (
        "import json\n"
        "from novalsm_amd import callers\n"
        "out = []\n"
        "for op in ('verify', 'trailers'):\n"
        "    for t in (1, 4):\n"
        "        r = callers.run(op, t, 1024, 0.2, 'engine', warm_s=0.05, seed=21 + t)\n"
        "        out.append({'op': op, 't': t, 'verified': r['verified'], 'calls': r['calls'],\n"
        "                    'fallbacks': r['engine']['fallbacks'], 'launches': r['engine']['launches'],\n"
        "                    'waves': r['engine']['waves']})\n"
        "print(json.dumps(out))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NOVA_SST_ENGINE_WAVES="8", PYTHONPATH=root)
    p = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                       timeout=100)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    for r in res:
        assert r["verified"] and r["fallbacks"] == 0 and r["calls"] > 0 and r["launches"] >= 1, r
        assert r["waves"] == 8, r
    assert C.engine_counters()["waves"] in (0, 12)  # this process: the default build
