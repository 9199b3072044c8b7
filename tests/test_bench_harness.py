"""bench.py's multi-GPU launcher on CPU: `python bench.py --gpus 2` (no torchrun
around it) must start 2 ranks itself, and the ranks' collective must see a
world of 2 (gloo here; RCCL on the GPU node).  --harness-check runs only the
launcher and the collective plumbing -- no GPU, no measurement."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


@pytest.mark.timeout(300)
def test_launcher_starts_two_ranks():
    r, lines = _run(["--gpus", "2", "--harness-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout  # rank 0 only prints
    res = json.loads(lines[0])
    assert res["harness_check"] is True
    assert res["n_gpus"] == 2
    assert res["max_rank"] == 1  # the all_reduce(MAX) crossed both ranks
    assert res["crc"] == f"0x{_value(bytes(range(256)) * 16):08x}"


@pytest.mark.timeout(600)
def test_launcher_starts_eight_ranks():
    """the driver's 8-GPU launch shape, rehearsed on the
    CPU -- `bench.py --gpus 8` starts 8 ranks (gloo here), every rank takes its
    own LOCAL_RANK, the collectives span all 8, and every child exits cleanly
    (torch.distributed.run returns nonzero if any rank fails)."""
    r, lines = _run(["--gpus", "8", "--harness-check"], timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 8
    assert res["max_rank"] == 7
    assert res["ranks"] == list(range(8))
    assert res["local_ranks"] == list(range(8))


def test_hbm_preflight_fails_loudly(monkeypatch, capsys):
    """bench.py checks each rank's free HBM against the workload before it
    allocates: a GPU that cannot hold it ends the run
    with an error line, not a late failure inside a launch."""
    sys.path.insert(0, ROOT)
    import types
    import bench
    fake_torch = types.SimpleNamespace(cuda=types.SimpleNamespace(
        mem_get_info=lambda dev: (8 << 30, 288 << 30)))
    monkeypatch.setitem(sys.modules, "torch", fake_torch)
    ctx = types.SimpleNamespace(dev="cuda:0", rank=3)
    bench.hbm_preflight(2, bench.workload(2), ctx)  # 4 GiB fits in 8 GiB free
    with pytest.raises(SystemExit) as e:
        bench.hbm_preflight(4, bench.workload(4), ctx)  # 16 GiB does not
    assert e.value.code == 4
    err = json.loads(capsys.readouterr().err.strip().splitlines()[-1])
    assert err["error"] == "HBM preflight" and err["rank"] == 3 and err["config"] == 4
    for cfg in (3, 5, "sst4k_verify", "log512_verify", "parity"):
        assert bench.hbm_need(bench.workload(cfg)) > 0


@pytest.mark.timeout(120)
def test_single_process_when_one_gpu():
    r, lines = _run(["--gpus", "1", "--harness-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(lines[0])["n_gpus"] == 1


def test_host_cpus_reports_share():
    sys.path.insert(0, ROOT)
    import bench
    n, info = bench.host_cpus()
    assert n >= 1
    assert info["affinity_cpus"] >= n


def _value(b: bytes) -> int:
    from tests.oracle_lib import load_oracle
    return load_oracle().value(b)
