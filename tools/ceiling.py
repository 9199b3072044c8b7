#!/usr/bin/env python3
"""Read-ceiling probe: how fast can this chip stream-read a config-2/4 sized
buffer at all, by loads in flight per lane, cache policy, workgroup size and
grid size -- next to the CRC streaming kernel under the same clock (default
and nt load policy).  One process, interleaved rounds, median.
Writes gpurun_out/ceiling.json.

--only parity: the XOR parity kernel (nova_xor_parity, k = 8 fragments x
512 MiB, bench_ops.py's parity workload) next to copy ceilings of the same
traffic shape (crc32c_diag.hip copy_ceiling_kernel): 8 reads + 1 write with
nothing else, the 8 reads alone, a 1:1 copy, the write alone -- by chunks per
lane, load/store policy and grid.  --one NAME runs one of them 20 times
(a PMC pass: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, tools/pmc_parity.sh).
Writes gpurun_out/parity_ceiling.json.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--gib", type=int, default=4)
    ap.add_argument("--only", default="read,crc", help="comma list of kinds to run")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ceiling.json"))
    ap.add_argument("--one", default="", help="parity mode: run one variant 20x (PMC pass)")
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    if "parity" in args.only.split(","):
        return parity_ceiling(args, torch, C)

    L = C.enable_diagnostics()
    L.nova_diag_read_ceiling.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.nova_diag_read_ceiling.restype = ctypes.c_int
    assert L.nova_device_init() == 0
    nbytes = args.gib << 30
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 2)
    sink = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
    out = torch.empty(nbytes // 4096, dtype=torch.int32, device="cuda")

    def timeit(fn):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.iters)]
        fn()
        torch.cuda.synchronize()
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) for a, b in ev) / 1e3

    variants = {}
    for u in (4, 8, 16):
        for nt in (0, 1):
            for t1024 in (0, 1):
                for wgs in (256, 512, 1024, 2048):
                    if t1024 and wgs > 512:
                        continue
                    v = u | (0x100 * nt) | (0x200 * t1024)

                    def f(v=v, wgs=wgs):
                        rc = L.nova_diag_read_ceiling(buf.data_ptr(), nbytes, sink.data_ptr(),
                                                      wgs, v, None)
                        assert rc == 0, rc
                    variants[("read", u, nt, 1024 if t1024 else 256, wgs)] = f
    # crc variants: (block bytes, variant 0 = nt / 2 = default policy, BPG, waves per WG)
    for Lb in (4096, 16384):
        for var in (0, 2):
            for bpg in (0, 1, 2, 4):
                for w in (4, 8, 16):
                    if var == 2 and w != 16:
                        continue
                    def f(Lb=Lb, var=var, bpg=bpg, w=w):
                        L.nova_diag_set_variant(var)
                        L.nova_diag_set_blocks_per_group(bpg)
                        L.nova_diag_set_stream_waves(w)
                        C.batch_strided(buf, Lb, Lb, nbytes // Lb, out=out[: nbytes // Lb])
                    variants[("crc", Lb, var, bpg, w)] = f
    kinds = set(args.only.split(","))
    variants = {k: f for k, f in variants.items() if k[0] in kinds}
    times: dict = {}
    for _ in range(args.rounds):
        for k, f in variants.items():
            times.setdefault(k, []).append(timeit(f))
    L.nova_diag_set_variant(0)
    L.nova_diag_set_blocks_per_group(0)
    L.nova_diag_set_stream_waves(0)
    # correctness of every production-policy crc variant
    for Lb in (4096, 16384):
        n = nbytes // Lb
        ref = C.batch_strided(buf, Lb, Lb, n).clone()
        for k, f in variants.items():
            if k[0] == "crc" and k[1] == Lb:
                f()
                torch.cuda.synchronize()
                assert torch.equal(out[:n], ref), ("mismatch", k)
        L.nova_diag_set_variant(0)
        L.nova_diag_set_blocks_per_group(0)
        L.nova_diag_set_stream_waves(0)
    res = []
    for k, ts in times.items():
        t = statistics.median(ts)
        row = {"kind": k[0], "params": list(k[1:]), "sec": t, "GBps": nbytes / t / 1e9,
               "frac_8TBs": nbytes / t / 8e12}
        res.append(row)
        print(f"{k[0]:5s} {str(k[1:]):24s} {t * 1e3:8.3f} ms {nbytes / t / 1e9:8.1f} GB/s "
              f"{100 * nbytes / t / 8e12:5.1f}%", flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fo:
        json.dump(res, fo, indent=1)


def parity_ceiling(args, torch, C):
    L = C.enable_diagnostics()
    assert L.nova_device_init() == 0
    k, plen = 8, 512 << 20
    buf = torch.empty(k * plen, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 21)
    fo = torch.arange(0, k * plen, plen, dtype=torch.int64, device="cuda")
    out = torch.empty(plen, dtype=torch.uint8, device="cuda")
    sink = torch.empty(256, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    bytes_of = {0: (k + 1) * plen, 1: k * plen, 2: 2 * plen, 3: plen}
    variants = {"product": (lambda: C.xor_parity(buf, fo, plen, out=out, stream=stream), (k + 1) * plen)}
    for kind in (0, 1, 2, 3):
        for u in (1, 2, 4, 8):
            for ntl in (0, 1):
                for nts in (0, 1):
                    if (kind == 1 and nts) or (kind == 3 and ntl):
                        continue
                    for wgs in (0, 4096, 16384):
                        v = u | ntl << 4 | nts << 5 | kind << 8

                        def f(v=v, wgs=wgs):
                            rc = L.nova_diag_copy_ceiling(buf.data_ptr(), fo.data_ptr(), plen, out.data_ptr(),
                                                          sink.data_ptr(), wgs, v, stream.cuda_stream)
                            assert rc == 0, rc
                        name = f"k{kind}_u{u}_l{ntl}_s{nts}_g{wgs}"
                        variants[name] = (f, bytes_of[kind])
    if args.one:
        f, _ = variants[args.one]
        for _ in range(20):
            f()
        torch.cuda.synchronize()
        print(json.dumps({"ran": args.one, "launches": 20}))
        return 0
    # correctness: the product and every 8R+1W variant give the same parity
    ref = buf.view(k, plen)[0].clone()
    for i in range(1, k):
        ref ^= buf.view(k, plen)[i]
    for name, (f, _) in variants.items():
        if name == "product" or name.startswith("k0_"):
            out.zero_()
            f()
            torch.cuda.synchronize()
            assert torch.equal(out, ref), name

    def timeit(fn):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.iters)]
        fn()
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) for a, b in ev) / 1e3

    times: dict = {}
    for _ in range(args.rounds):
        for name, (f, _) in variants.items():
            times.setdefault(name, []).append(timeit(f))
    res = []
    for name, (f, nb) in variants.items():
        t = statistics.median(times[name])
        res.append({"name": name, "bytes": nb, "ms": round(t * 1e3, 4), "GBps": round(nb / t / 1e9, 1),
                    "frac_8TBs": round(nb / t / 8e12, 4)})
    best = {}
    for r in res:
        kind = r["name"].split("_")[0]
        if kind not in best or r["GBps"] > best[kind]["GBps"]:
            best[kind] = r
    prod = res[0]
    summary = {"product": prod, "best": best,
               "product_vs_8r1w_ceiling": round(prod["GBps"] / best["k0"]["GBps"], 4)}
    for r in res:
        print(json.dumps(r), flush=True)
    print(json.dumps(summary), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(os.path.join(os.path.dirname(args.out), "parity_ceiling.json"), "w") as fo_:
        json.dump({"rows": res, "summary": summary}, fo_, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
