#!/usr/bin/env python3
"""Throughput of the SURVEY 8(f) composites on one MI355X, same clock as bench.py
(HIP events on the launch stream, warmup past the launch transient), each
against the HBM roofline with its own algorithmic bytes:

  trailers    nova_sstable_write_trailers over a config-3 SSTable image
              (blocks + 5-B trailer gaps): reads sum(len), writes 5 B/block
  verify      nova_sstable_verify_blocks over the same image with trailers:
              reads sum(len + 5), writes 1 B/block
  log_write   nova_log_write_crcs over a 4 GiB log image of records with
              U[1,4096] B payloads: reads sum(1 + len) (type + payload) plus the
              3-B length/type header, writes 4 B/record
  log_verify  nova_log_verify_records over the same image: reads sum(7 + len)
  parity      nova_xor_parity of k=8 fragments x 512 MiB: reads 8 x 512 MiB,
              writes 512 MiB

One JSON line per op (rank 0 only, single GPU).  Sample-verified against the
oracle outside the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def timed(torch, fn, steps, warmup, stream):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    return sum(ms) / len(ms) / 1e3


def log_layout(total_target: int, seed: int, pmax: int = 4096, pmin: int = 1):
    """A log file of ~total_target bytes as log::Writer lays it out
    (db/log_writer.cc:53-97, novalsm_amd/synth.log_layout): logical records of
    U[pmin,pmax] B payload from splitmix64(seed), fragmented at 32 KiB blocks.
    Returns the physical records' (offsets, payload lengths, types, total)."""
    from novalsm_amd.synth import splitmix64_words, log_layout as writer_layout
    n = total_target // (7 + (pmax + pmin) // 2)
    r = splitmix64_words(seed, 0, n)
    plens = ((r % np.uint64(pmax - pmin + 1)) + np.uint64(pmin)).astype(np.int64)
    offs, lens, types, _, total = writer_layout(plens)
    return offs, lens.astype(np.uint64), types, total


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="trailers,verify,log_write,log_verify,parity")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--n", type=int, default=1 << 20, help="blocks for trailers/verify")
    ap.add_argument("--images", default="sst4k,cfg3",
                    help="SSTable images for trailers/verify: sst4k (4096+U[0,255] B blocks), cfg3")
    ap.add_argument("--parity-sweep", default="",
                    help="comma list of nova_diag_set_parity_variant values (tuning)")
    ap.add_argument("--lanes-sweep", action="store_true",
                    help="also time each CRC op at 4/8/16 lanes per unit (tuning)")
    ap.add_argument("--sort-sweep", default="",
                    help="log ops: comma list of nova_diag_set_rounds_sort values (0 in order, "
                         "2 windows + chunks, 3 windows only)")
    ap.add_argument("--log-seed", type=int, default=6, help="log image: payload-length seed")
    ap.add_argument("--log-payload-max", type=int, default=4096, help="log image: payloads U[min,max] B")
    ap.add_argument("--log-payload-min", type=int, default=1, help="log image: payloads U[min,max] B")
    ap.add_argument("--chunk-sweep", default="",
                    help="comma list of rounds-kernel chunk sizes (nova_diag_set_chunk_blocks), log ops")
    ap.add_argument("--no-ablations", action="store_true", help="skip the diagnostics ablations")
    ap.add_argument("--lanes", type=int, default=0, help="force lanes per block/record (nova_crc32c_set_tuning)")
    ap.add_argument("--var-ab", default="",
                    help="comma list of rounds-kernel variants to A/B against the product (8192 16 waves, 2 cached)")
    ap.add_argument("--waves-sweep", default="",
                    help="comma list of waves per workgroup for the variable kernels (diagnostics)")
    ap.add_argument("--decode-ablations", action="store_true",
                    help="log ops: time the decode stage without its tail-line / header loads "
                         "(timing ablations, WRONG results; nova_diag_set_trailer_single_pass 8/9/10)")
    ap.add_argument("--log-bound", action="store_true",
                    help="log write: time its composite bound (no-store pass + isolated CRC-field stores)")
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    from tests.oracle_lib import load_oracle
    import bench

    assert C.load().nova_device_init() == 0
    if args.lanes:
        C.set_tuning(args.lanes, 0)
    orc = load_oracle()
    stream = torch.cuda.current_stream()
    ops = args.ops.split(",")
    rows = []

    def sort_sweep(op, fn, alg_bytes, check=None, reset=None):
        # entries "sort", "sort:window", "sort:window:key" or "sort:window:key:ablation"
        # (nova_diag_set_rounds_sort / _log_window / _log_key / _trailer_single_pass)
        for v in [x for x in args.sort_sweep.split(",") if x]:
            so, win, key, abl = (v.split(":") + ["0", "0", "0"])[:4]
            if reset is not None:
                reset()
            with C.diagnostics() as D:
                if args.lanes:  # (the diagnostics library keeps its own tuning)
                    D.nova_crc32c_set_tuning(args.lanes, 0)
                D.nova_diag_set_rounds_sort(int(so))
                D.nova_diag_set_log_window(int(win or 0))
                D.nova_diag_set_log_key(int(key or 0))
                D.nova_diag_set_trailer_single_pass(int(abl or 0))
                sec = timed(torch, fn, args.steps, args.warmup, stream)
                D.nova_diag_set_rounds_sort(2)
                D.nova_diag_set_log_window(0)
                D.nova_diag_set_log_key(0)
                D.nova_diag_set_trailer_single_pass(0)
            extra = {} if check is None else {"results_ok": bool(check())}
            print(json.dumps({"sweep": op, "rounds_sort": int(so), "log_window": int(win or 0),
                              "log_key": int(key or 0), "ablation": int(abl or 0), **extra,
                              "GBps": round(alg_bytes / sec / 1e9, 1),
                              "frac": round(alg_bytes / sec / 1e9 / HBM_PEAK_GBS, 4)}), flush=True)

    def decode_ablations(op, fn, alg_bytes):
        """The rounds kernel's decode stage reads each record's header and tail
        line a whole chunk before its data pass reads the same lines; timed
        without them (WRONG results, written as usual): 8 no tail line, 9 no
        header (lengths from the next offset), 10 neither.  The step work, the
        same way: 12 no head masking, 13 no group fold at a round's end."""
        if not args.decode_ablations:
            return
        for tk, name in ((8, "no_tail_line"), (9, "no_header"), (10, "no_tail_no_header"),
                         (12, "no_head_masking"), (13, "no_group_fold")):
            with C.diagnostics() as D:
                if args.lanes:
                    D.nova_crc32c_set_tuning(args.lanes, 0)
                D.nova_diag_set_trailer_single_pass(tk)
                sec = timed(torch, fn, args.steps, args.warmup, stream)
                D.nova_diag_set_trailer_single_pass(0)
            print(json.dumps({"sweep": op, "decode_ablation": name, "GBps": round(alg_bytes / sec / 1e9, 1),
                              "frac": round(alg_bytes / sec / 1e9 / HBM_PEAK_GBS, 4)}), flush=True)

    def waves_sweep(op, fn, alg_bytes):
        """Waves per workgroup of the rounds kernel (nova_diag_set_stream_waves;
        the product runs 12), alternated with the product twice."""
        ws = [int(x) for x in args.waves_sweep.split(",") if x]
        for rep in range(2 if ws else 0):
            for w in [0] + ws:
                with C.diagnostics() as D:
                    if args.lanes:
                        D.nova_crc32c_set_tuning(args.lanes, 0)
                    D.nova_diag_set_stream_waves(w)
                    sec = timed(torch, fn, args.steps, args.warmup, stream)
                    D.nova_diag_set_stream_waves(0)
                print(json.dumps({"sweep": op, "waves": w, "rep": rep, "GBps": round(alg_bytes / sec / 1e9, 1),
                                  "frac": round(alg_bytes / sec / 1e9 / HBM_PEAK_GBS, 4)}), flush=True)

    def chunk_sweep(op, fn, alg_bytes):
        for c in [int(x) for x in args.chunk_sweep.split(",") if x]:
            with C.diagnostics() as D:
                D.nova_diag_set_chunk_blocks(c)
                sec = timed(torch, fn, args.steps, args.warmup, stream)
            print(json.dumps({"sweep": op, "chunk": c, "GBps": round(alg_bytes / sec / 1e9, 1),
                              "frac": round(alg_bytes / sec / 1e9 / HBM_PEAK_GBS, 4)}), flush=True)

    def sweep(op, fn, alg_bytes):
        if not args.lanes_sweep:
            return
        for g in (2, 4, 8, 16):
            C.set_tuning(g, 0)  # default segment size
            sec = timed(torch, fn, args.steps, args.warmup, stream)
            print(json.dumps({"sweep": op, "lanes": g, "GBps": round(alg_bytes / sec / 1e9, 1),
                              "frac": round(alg_bytes / sec / 1e9 / HBM_PEAK_GBS, 4)}),
                  flush=True)
        C.set_tuning(0, 0)

    def var_ab(op, fn, alg_bytes):
        """Rounds-kernel A/Bs against the product, alternated: 8192 = 16 waves
        per workgroup (128 VGPRs, a few spilled dwords),
        2 = default-policy data loads instead of non-temporal ones."""
        vs = [int(x) for x in args.var_ab.split(",") if x]
        if not vs:
            return
        for rep in range(2):
            for var in [0] + vs:
                with C.diagnostics() as D:
                    D.nova_diag_set_variant(var)
                    sec = timed(torch, fn, args.steps, args.warmup, stream)
                    D.nova_diag_set_variant(0)
                print(json.dumps({"sweep": op, "variant": var, "rep": rep,
                                  "GBps": round(alg_bytes / sec / 1e9, 1),
                                  "frac": round(alg_bytes / sec / 1e9 / HBM_PEAK_GBS, 4)}), flush=True)

    def log_write_bound(buf, o, n, total, sum_rec, sec_product):
        """log write's composite bound, all in this run --
        the same launch without its result stores (diagnostics ablation 6) plus
        the CRC-field stores alone (one unaligned 4-B store per record at its
        header, nova_diag_log_field_scatter), each timed right after a read of
        the whole image so they find the image out of the caches, as the
        product's stores do."""
        with C.diagnostics() as D:
            D.nova_diag_set_trailer_single_pass(6)
            t_ns = timed(torch, lambda: C.log_write_crcs(buf, o, stream=stream), args.steps, args.warmup, stream)
            D.nova_diag_set_trailer_single_pass(0)
        D = C.load_diag()
        wgs = 4096
        sink = torch.zeros(wgs * 256, dtype=torch.int32, device="cuda")  # read_stream: one word per thread
        sp = stream.cuda_stream
        ms = []
        for it in range(args.warmup + args.steps):
            assert D.nova_diag_read_stream(buf.data_ptr(), total, sink.data_ptr(), wgs, sp) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            assert D.nova_diag_log_field_scatter(buf.data_ptr(), o.data_ptr(), n, sp) == 0
            e1.record(stream)
            e1.synchronize()
            if it >= args.warmup:
                ms.append(e0.elapsed_time(e1))
        ms.sort()
        t_sc = ms[len(ms) // 2] / 1e3
        C.log_write_crcs(buf, o, stream=stream)  # the CRC fields again
        torch.cuda.synchronize()
        bound = t_ns + t_sc
        print(json.dumps({"sweep": "log_write_bound", "records": n, "no_store_ms": round(t_ns * 1e3, 4),
                          "field_scatter_ms": round(t_sc * 1e3, 4), "bound_ms": round(bound * 1e3, 4),
                          "product_ms": round(sec_product * 1e3, 4),
                          "bound_frac": round(sum_rec / bound / 1e9 / HBM_PEAK_GBS, 4),
                          "product_over_bound": round(sec_product / bound, 4)}), flush=True)

    def emit(op, workload, alg_bytes, sec, ok, extra=None):
        gbs = alg_bytes / sec / 1e9
        row = {"op": op, "workload": workload, "algorithmic_bytes": int(alg_bytes),
               "ms_per_launch": round(sec * 1e3, 4), "GBps": round(gbs, 1),
               "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)},
               "verified_sample": bool(ok)}
        if extra:
            row.update(extra)
        rows.append(row)
        print(json.dumps(row), flush=True)

    for image in (args.images.split(",") if ("trailers" in ops or "verify" in ops) else []):
        n = args.n
        if image == "cfg3":
            _, lens_np, _ = bench.config3_layout(n, 3)
            wl = f"config3 SSTable image: {n} blocks {{4,16,64}} KiB+U[1,64], 5-B trailers"
            large = True  # the caller's block_size is >= 16 KiB: scheduling hint
        else:
            from novalsm_amd.synth import splitmix64_words
            r = splitmix64_words(5, 0, n)
            lens_np = (np.uint64(4096) + (r % np.uint64(256))).astype(np.uint32)
            wl = f"SSTable image: {n} blocks of 4096+U[0,255] B, 5-B trailers"
            large = False
        offs_np = np.zeros(n, np.uint64)
        offs_np[1:] = np.cumsum(lens_np[:-1].astype(np.uint64) + np.uint64(5))
        total = int(offs_np[-1]) + int(lens_np[-1]) + 5
        buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 31)
        offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
        lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
        sum_len = int(lens_np.astype(np.uint64).sum())
        sample = np.linspace(0, n - 1, 129).astype(np.int64)
        if "trailers" in ops:
            def tw():
                C.write_trailers(buf, offs, lens, 0, True, stream=stream, hint_large=large)
            sec = timed(torch, tw, args.steps, args.warmup, stream)
            ok = True
            for i in sample:
                o, ln = int(offs_np[i]), int(lens_np[i])
                blk = buf[o:o + ln + 5].cpu().numpy().tobytes()
                ok &= orc.trailer(blk[:ln], 0, True) == blk[ln:]
            emit("trailers", wl, sum_len + 5 * n, sec, ok, {"image": image})
            # store-form A/B (diagnostics build; the product stores the trailer
            # bytes from the CRC kernel): 2 = two passes (CRC array + scatter),
            # 8 = two passes, the second reading, patching and storing whole
            # 64-B pieces, 3 = whole 64-B pieces, 4 = the same non-temporal, 5 = pieces and
            # 6 = the product form without result writes (timing only)
            # (round 3: the product is 8, the CRC pass then whole-piece stores)
            for var, name in (() if args.no_ablations else (
                              (9, "trailers_one_pass"), (2, "trailers_two_pass"),
                              (3, "trailers_pieces"),
                              (4, "trailers_pieces_nt"), (5, "trailers_pieces_no_writes"),
                              (6, "trailers_crc_pass_only"), (7, "trailers_crc_pass_no_epilogue"))):
                with C.diagnostics() as D:
                    D.nova_diag_set_trailer_single_pass(var)
                    sec1 = timed(torch, tw, args.steps, args.warmup, stream)
                    D.nova_diag_set_trailer_single_pass(0)
                gbs1 = (sum_len + 5 * n) / sec1 / 1e9
                print(json.dumps({"sweep": name, "image": image, "GBps": round(gbs1, 1),
                                  "frac": round(gbs1 / HBM_PEAK_GBS, 4)}), flush=True)
            sweep("trailers", tw, sum_len + 5 * n)
        if "verify" in ops:
            C.write_trailers(buf, offs, lens, 0, False, stream=stream)  # StoC order: verifiable
            okb = torch.empty(n, dtype=torch.uint8, device="cuda")
            bad = torch.zeros(1, dtype=torch.int32, device="cuda")

            def vf():
                bad.zero_()
                C.verify_blocks(buf, offs, lens, stream=stream, ok=okb, bad=bad, hint_large=large)
            sec = timed(torch, vf, args.steps, args.warmup, stream)
            ok = int(bad.item()) == 0 and bool(okb.cpu().numpy().all())
            emit("verify", wl, sum_len + 6 * n, sec, ok, {"image": image})
            sweep("verify", vf, sum_len + 6 * n)
            var_ab("verify", vf, sum_len + 6 * n)
            for vv, name in (() if args.no_ablations else ((2048, "verify_round_epilogue"),)):
                with C.diagnostics() as D:  # A/B: the per-round epilogue (rounds 1-2)
                    D.nova_diag_set_variant(vv)
                    sec1 = timed(torch, vf, args.steps, args.warmup, stream)
                    D.nova_diag_set_variant(0)
                gbs1 = (sum_len + 6 * n) / sec1 / 1e9
                print(json.dumps({"sweep": name, "image": image, "GBps": round(gbs1, 1),
                                  "frac": round(gbs1 / HBM_PEAK_GBS, 4)}), flush=True)
            with C.diagnostics() as D:  # timing ablation: no ok/mismatch writes
                D.nova_diag_set_trailer_single_pass(6)
                sec1 = timed(torch, vf, args.steps, args.warmup, stream)
                D.nova_diag_set_trailer_single_pass(0)
            gbs1 = (sum_len + 6 * n) / sec1 / 1e9
            print(json.dumps({"sweep": "verify_no_writes", "image": image, "GBps": round(gbs1, 1),
                              "frac": round(gbs1 / HBM_PEAK_GBS, 4)}), flush=True)
            with C.diagnostics() as D:  # timing ablation: no tail-line loads, no writes (vs verify_no_writes)
                D.nova_diag_set_variant(256)
                D.nova_diag_set_trailer_single_pass(6)
                sec1 = timed(torch, vf, args.steps, args.warmup, stream)
                D.nova_diag_set_trailer_single_pass(0)
                D.nova_diag_set_variant(0)
            gbs1 = (sum_len + 6 * n) / sec1 / 1e9
            print(json.dumps({"sweep": "verify_no_tail_loads_no_writes", "image": image, "GBps": round(gbs1, 1),
                              "frac": round(gbs1 / HBM_PEAK_GBS, 4)}), flush=True)
        del buf
        torch.cuda.empty_cache()

    if "log_write" in ops or "log_verify" in ops:
        pmax = args.log_payload_max
        pmin = args.log_payload_min
        offs_np, lens_np, types_np, total = log_layout(4 << 30, args.log_seed, pmax, pmin)
        n = len(offs_np)
        buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 41)
        # headers: length (LE16) and type bytes, written with torch scatter
        o = torch.from_numpy(offs_np.view(np.int64)).cuda()
        ln = torch.from_numpy(lens_np.astype(np.int64)).cuda()
        buf[o + 4] = (ln & 0xFF).to(torch.uint8)
        buf[o + 5] = (ln >> 8).to(torch.uint8)
        buf[o + 6] = torch.from_numpy(types_np).cuda()
        sum_rec = int(lens_np.sum()) + 7 * n
        wl = f"log image: {n} records, payload U[{pmin},{pmax}] B, {total / 2**30:.2f} GiB"
        sample = np.linspace(0, n - 1, 129).astype(np.int64)
        if "log_write" in ops:
            sec = timed(torch, lambda: C.log_write_crcs(buf, o, stream=stream), args.steps,
                        args.warmup, stream)
            ok = True
            for i in sample:
                a, L = int(offs_np[i]), int(lens_np[i])
                rec = buf[a:a + 7 + L].cpu().numpy()  # (the type byte is the header's last)
                want = orc.mask(orc.extend(orc.value(rec[6:7].tobytes()), rec[7:].tobytes()))
                ok &= int.from_bytes(rec[:4].tobytes(), "little") == want
            emit("log_write", wl, sum_rec, sec, ok)

            def check_write():  # the sampled records' CRC fields against the oracle
                good = True
                for i in sample:
                    a, L = int(offs_np[i]), int(lens_np[i])
                    rec = buf[a:a + 7 + L].cpu().numpy()
                    want = orc.mask(orc.extend(orc.value(rec[6:7].tobytes()), rec[7:].tobytes()))
                    good &= int.from_bytes(rec[:4].tobytes(), "little") == want
                return good
            sweep("log_write", lambda: C.log_write_crcs(buf, o, stream=stream), sum_rec)
            # (each entry starts from CRC fields whose first byte is cleared: it must rewrite them)
            sort_sweep("log_write", lambda: C.log_write_crcs(buf, o, stream=stream), sum_rec, check_write,
                       lambda: buf.__setitem__(o, 0))
            chunk_sweep("log_write", lambda: C.log_write_crcs(buf, o, stream=stream), sum_rec)
            for var, name in (() if args.no_ablations else ((3, "log_write_pieces"), (4, "log_write_pieces_nt"),
                              (5, "log_write_pieces_no_writes"), (6, "log_write_no_writes"),
                              (7, "log_write_no_epilogue"))):
                with C.diagnostics() as D:
                    D.nova_diag_set_trailer_single_pass(var)
                    sec1 = timed(torch, lambda: C.log_write_crcs(buf, o, stream=stream), args.steps,
                                 args.warmup, stream)
                    D.nova_diag_set_trailer_single_pass(0)
                gbs1 = sum_rec / sec1 / 1e9
                print(json.dumps({"sweep": name, "GBps": round(gbs1, 1),
                                  "frac": round(gbs1 / HBM_PEAK_GBS, 4)}), flush=True)
            var_ab("log_write", lambda: C.log_write_crcs(buf, o, stream=stream), sum_rec)
            decode_ablations("log_write", lambda: C.log_write_crcs(buf, o, stream=stream), sum_rec)
            waves_sweep("log_write", lambda: C.log_write_crcs(buf, o, stream=stream), sum_rec)
            if args.log_bound:
                log_write_bound(buf, o, n, total, sum_rec, sec)
        if "log_verify" in ops:
            C.log_write_crcs(buf, o, stream=stream)
            okb = torch.empty(n, dtype=torch.uint8, device="cuda")
            bad = torch.zeros(1, dtype=torch.int32, device="cuda")

            def lv():
                bad.zero_()
                C.log_verify_records(buf, o, stream=stream, ok=okb, bad=bad)
            sec = timed(torch, lv, args.steps, args.warmup, stream)
            ok = int(bad.item()) == 0 and bool((okb.cpu().numpy() == C.LOG_OK).all())
            emit("log_verify", wl, sum_rec + n, sec, ok)
            sort_sweep("log_verify", lv, sum_rec + n,
                       lambda: int(bad.item()) == 0 and bool((okb.cpu().numpy() == C.LOG_OK).all()),
                       lambda: okb.fill_(0xEE))
            chunk_sweep("log_verify", lv, sum_rec + n)
            for var, name in (() if args.no_ablations else
                              ((0, "log_verify_no_writes"), (256, "log_verify_no_tail_loads_no_writes"))):
                with C.diagnostics() as D:  # timing ablations (no result writes; 256: WRONG CRCs)
                    D.nova_diag_set_variant(var)
                    D.nova_diag_set_trailer_single_pass(6)
                    sec1 = timed(torch, lv, args.steps, args.warmup, stream)
                    D.nova_diag_set_trailer_single_pass(0)
                    D.nova_diag_set_variant(0)
                gbs1 = (sum_rec + n) / sec1 / 1e9
                print(json.dumps({"sweep": name, "GBps": round(gbs1, 1),
                                  "frac": round(gbs1 / HBM_PEAK_GBS, 4)}), flush=True)
            var_ab("log_verify", lv, sum_rec + n)
            decode_ablations("log_verify", lv, sum_rec + n)
            waves_sweep("log_verify", lv, sum_rec + n)
            sweep("log_verify", lv, sum_rec + n)
        del buf
        torch.cuda.empty_cache()

    if "parity" in ops:
        k, plen = 8, 512 << 20
        buf = torch.empty(k * plen, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 51)
        fo = torch.arange(k, dtype=torch.int64, device="cuda") * plen
        out = torch.empty(plen, dtype=torch.uint8, device="cuda")
        sec = timed(torch, lambda: C.xor_parity(buf, fo, plen, out=out, stream=stream),
                    args.steps, args.warmup, stream)
        idx = np.linspace(0, plen - 4097, 33).astype(np.int64)
        ok = True
        for i in idx:
            want = np.zeros(4096, np.uint8)
            for f in range(k):
                want ^= buf[f * plen + i:f * plen + i + 4096].cpu().numpy()
            ok &= np.array_equal(out[i:i + 4096].cpu().numpy(), want)
        emit("parity", f"{k} fragments x {plen >> 20} MiB", (k + 1) * plen, sec, ok)
        if args.parity_sweep:
            with C.diagnostics() as L:
                for v in args.parity_sweep.split(","):
                    L.nova_diag_set_parity_variant(int(v, 0))
                    sec = timed(torch, lambda: C.xor_parity(buf, fo, plen, out=out, stream=stream),
                                args.steps, args.warmup, stream)
                    gbs = (k + 1) * plen / sec / 1e9
                    print(json.dumps({"sweep": "parity", "variant": v, "GBps": round(gbs, 1),
                                      "frac": round(gbs / HBM_PEAK_GBS, 4)}), flush=True)

    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_ops.json"), "w") as f:
        json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
