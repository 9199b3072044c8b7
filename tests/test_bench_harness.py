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


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=240)
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
