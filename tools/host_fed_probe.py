#!/usr/bin/env python3
"""Host-fed C2 throughput on one GPU across pool geometries (batch size,
slots in flight, feeder threads per GPU): the same 1M signatures from
page-locked host memory through fd_ed25519_hip_pool_run, verdicts checked.

    python tools/host_fed_probe.py [--reps 4] [--out gpurun_out/host_fed_probe.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, tile, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--out", default="gpurun_out/host_fed_probe.json")
    ap.add_argument("--stream-copies", type=int, default=4)
    ap.add_argument("--near", type=int, default=1, help="allocate host buffers on the GPU's NUMA node")
    ap.add_argument("--bench-leg", type=int, default=1, help="also run bench.py's host-fed leg")
    ap.add_argument("--only-bench-leg", type=int, default=0)
    args = ap.parse_args()
    cfg = workload.CONFIGS["C2"]
    eng = ed25519.Engine(0, max_chunk=1 << 20)
    wl = ed25519.DeviceWorkload(eng, cfg["n"], cfg["lo"], cfg["hi"], cfg["ppm"], seed=0x5EED)
    n = wl.n
    if args.near:
        near = tile.NearDevice(eng.info())
        near.__enter__()
    msgs = wl.msgs.download(np.uint8, wl.msg_bytes + 16)
    off = wl.off.download(np.uint64, n)
    sz = wl.sizes.astype(np.uint32)
    sigs = wl.sigs.download(np.uint8, 64 * n)
    pubs = wl.pubs.download(np.uint8, 32 * n)
    expect = wl.expect.download(np.int8, n)
    out = np.zeros(n, np.int8)
    # device-resident reference rate
    for _ in range(2):
        wl.verify()
    eng.sync()
    t = time.perf_counter()
    for _ in range(5):
        wl.verify()
    eng.sync()
    dev_rate = 5 * n / (time.perf_counter() - t)
    res = {"device_resident": dev_rate, "h2d_GBps": tile.h2d_gbps(0, 256 << 20, 8), "runs": []}
    print(json.dumps(res), flush=True)
    with tile.HostRegistration(msgs, off, sz, sigs, pubs, out):
        for feeders, batch, slots in [] if args.only_bench_leg else [(1, 131072, 4), (1, 65536, 4), (1, 262144, 3), (1, 131072, 2), (2, 131072, 3),
                                      (2, 65536, 4), (4, 65536, 2)]:
            pool = tile.Pool([0] * feeders, batch, slots, tile.max_span(off, sz, batch))
            pool.run(msgs, off, sz, sigs, pubs, out)
            t = time.perf_counter()
            for _ in range(args.reps):
                _, _, st = pool.run(msgs, off, sz, sigs, pubs, out)
            dt = time.perf_counter() - t
            pool.close()
            r = {"feeders": feeders, "batch": batch, "slots": slots, "verifies_per_s": args.reps * n / dt,
                 "h2d_GBps": args.reps * st["h2d_bytes"] / dt / 1e9, "ok": bool(np.array_equal(out, expect)),
                 "direct": st["direct_batches"]}
            res["runs"].append(r)
            print(json.dumps(r), flush=True)
        # a longer stream: the same set 4 times back to back in one run
        # (pipeline fill and drain once per 4M instead of once per 1M)
        k = args.stream_copies if not args.only_bench_leg else 1
        if k > 1:
            msgs4 = np.concatenate([msgs[:wl.msg_bytes]] * k + [np.zeros(16, np.uint8)])
            off4 = np.concatenate([off + np.uint64(c * wl.msg_bytes) for c in range(k)])
            sz4, sigs4, pubs4 = np.tile(sz, k), np.tile(sigs, k), np.tile(pubs, k)
            out4 = np.zeros(k * n, np.int8)
            with tile.HostRegistration(msgs4, off4, sz4, sigs4, pubs4, out4):
                for feeders, batch, slots in [(1, 65536, 4), (1, 131072, 4), (2, 65536, 4)]:
                    pool = tile.Pool([0] * feeders, batch, slots, tile.max_span(off4, sz4, batch))
                    pool.run(msgs4, off4, sz4, sigs4, pubs4, out4)
                    t = time.perf_counter()
                    _, _, st = pool.run(msgs4, off4, sz4, sigs4, pubs4, out4)
                    dt = time.perf_counter() - t
                    pool.close()
                    r = {"stream": k * n, "feeders": feeders, "batch": batch, "slots": slots,
                         "verifies_per_s": k * n / dt, "h2d_GBps": st["h2d_bytes"] / dt / 1e9,
                         "ok": bool(np.array_equal(out4, np.tile(expect, k)))}
                    res["runs"].append(r)
                    print(json.dumps(r), flush=True)
        # host memory kinds for the same 4M stream: numpy (default pages),
        # mmap + MADV_HUGEPAGE, hipHostMalloc (driver pinned)
        if k > 1:
            try:
                res["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
            except OSError:
                res["thp"] = None
            for kind in ("numpy", "thp", "hostmalloc"):
                bufs = {}
                for name, arr in (("msgs", msgs4), ("off", off4), ("sz", sz4), ("sigs", sigs4), ("pubs", pubs4),
                                  ("out", out4)):
                    bufs[name] = tile.host_array(arr.shape, arr.dtype, kind)
                    bufs[name][...] = arr
                reg = tile.HostRegistration(*[b for b in bufs.values()]) if kind != "hostmalloc" else None
                if reg:
                    reg.__enter__()
                pool = tile.Pool([0], 131072, 4, tile.max_span(off4, sz4, 131072))
                pool.run(bufs["msgs"], bufs["off"], bufs["sz"], bufs["sigs"], bufs["pubs"], bufs["out"])
                t = time.perf_counter()
                for _ in range(3):
                    _, _, st = pool.run(bufs["msgs"], bufs["off"], bufs["sz"], bufs["sigs"], bufs["pubs"], bufs["out"])
                dt = time.perf_counter() - t
                pool.close()
                if reg:
                    reg.__exit__(None, None, None)
                r = {"memory": kind, "stream": k * n, "verifies_per_s": 3 * k * n / dt,
                     "h2d_GBps": 3 * st["h2d_bytes"] / dt / 1e9, "direct": st["direct_batches"],
                     "ok": bool(np.array_equal(bufs["out"], np.tile(expect, k)))}
                res["runs"].append(r)
                print(json.dumps(r), flush=True)
                del bufs
    if args.bench_leg:
        # bench.py's own host-fed leg in this process (A/B against the runs above)
        import bench
        for rep in range(args.bench_leg):
            hf = bench.host_fed(wl, 0, eng.info(), 1, 3, 131072, 4, 4)
            r = {"bench_leg": rep, "verifies_per_s": hf["value"], "runs": hf["stream_run_seconds"]}
            res["runs"].append(r)
            print(json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    wl.free()
    eng.close()


if __name__ == "__main__":
    main()
