"""N>1 path on CPU: world_size-2 gloo ranks shard a batch exactly as bench.py does
on RCCL, checksum their shards (oracle as the stand-in compute on CPU), and
the gathered result equals the single-process batch; max-over-ranks timing."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from novalsm_amd.shard import shard_blocks, shard_by_bytes


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from novalsm_amd.shard import gather_crcs, max_over_ranks
    from novalsm_amd.synth import splitmix64_bytes
    from tests.oracle_lib import load_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = load_oracle()
        rng = np.random.default_rng(5)
        lens = (rng.choice([4096, 16384, 65536], 200) + rng.integers(1, 65, 200)).astype(np.uint32)
        offs = np.concatenate(([0], np.cumsum(lens[:-1].astype(np.uint64)))).astype(np.uint64)
        data = splitmix64_bytes(3, int(offs[-1]) + int(lens[-1]))
        lo, hi = shard_by_bytes(lens, world, rank)
        local = orc.batch(data, offs[lo:hi], lens[lo:hi])
        counts = [0] * world
        for r in range(world):
            a, b = shard_by_bytes(lens, world, r)
            counts[r] = b - a
        full = gather_crcs(local, counts)
        t = max_over_ranks(float(rank + 1))
        dist.barrier()
        if rank == 0:
            q.put((full.tolist(), orc.batch(data, offs, lens).tolist(), t))
    finally:
        dist.destroy_process_group()


def test_shard_ranges_cover_batch():
    for n in (0, 1, 7, 1 << 20, 8 << 20):
        for w in (1, 2, 4, 8):
            rs = [shard_blocks(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    lens = np.random.default_rng(0).integers(1, 70000, 1001)
    for w in (2, 3, 8):
        rs = [shard_by_bytes(lens, w, r) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == lens.size
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        sizes = [lens[a:b].sum() for a, b in rs]
        assert max(sizes) - min(sizes) <= 2 * lens.max()


@pytest.mark.timeout(300)
def test_gloo_world2_sharded_equals_single():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, single, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert full == single
    assert tmax == 2.0


def _gpu_worker(rank, world, port, q):
    """One rank of the sharded batch on the GPU: the HIP kernel computes the
    rank's byte-balanced shard; gloo carries the gather and the max-over-ranks
    time (both ranks share the box's single GPU)."""
    import torch
    import torch.distributed as dist
    from novalsm_amd import crc32c as C
    from novalsm_amd.shard import gather_crcs, max_over_ranks
    from novalsm_amd.synth import splitmix64_bytes
    from tests.oracle_lib import load_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        assert C.load().nova_device_init() == 0
        rng = np.random.default_rng(9)
        n = 3000
        lens = (rng.choice([4096, 16384, 65536], n) + rng.integers(1, 65, n)).astype(np.uint32)
        offs = np.concatenate(([0], np.cumsum(lens[:-1].astype(np.uint64)))).astype(np.uint64)
        data = splitmix64_bytes(4, int(offs[-1]) + int(lens[-1]))
        lo, hi = shard_by_bytes(lens, world, rank)
        buf = torch.from_numpy(data).cuda()
        d_offs = torch.from_numpy(offs[lo:hi].view(np.int64).copy()).cuda()
        d_lens = torch.from_numpy(lens[lo:hi].view(np.int32).copy()).cuda()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        out = C.batch(buf, d_offs, d_lens)
        t1.record()
        torch.cuda.synchronize()
        local = out.cpu().numpy().view(np.uint32)
        counts = [b - a for a, b in (shard_by_bytes(lens, world, r) for r in range(world))]
        full = gather_crcs(local, counts)
        tmax = max_over_ranks(t0.elapsed_time(t1))
        dist.barrier()
        if rank == 0:
            want = load_oracle().batch(data, offs, lens)
            q.put((bool(np.array_equal(full, want)), tmax > 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_world2_sharded_on_gpu_equals_oracle():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    equal, timed = q.get(timeout=360)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert equal and timed
