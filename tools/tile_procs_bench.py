#!/usr/bin/env python3
"""Verify tiles as separate processes on one GPU (run on the box), the way
fdctl runs them: each of K processes owns one verify tile (ring, tcache,
pipe with its own streams and hardware queues), signs its own single-signer
transactions, waits at a barrier, then runs them through the tile unpaced
(fd_ed25519_hip_latency_run).  Reports the aggregate transactions/s over the
union of the runs proper (each tile's setup excluded; common_s is how long
all K ran at once).  The parent never touches the GPU: children are
started with the spawn method.

    python tools/tile_procs_bench.py --procs 1,2,4,6,8 --batch 4096 --txns 400000
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(rank, args, barrier, q):
    sys.path.insert(0, REPO)
    import numpy as np
    from firedancer_amd import ed25519, tile, workload
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    pay, _ = workload.txn_payloads(eng, args.txns, 1000 + rank, msg_sz=200)
    eng.close()
    tile.latency_run(pay[:20000], 0.0, slot_cnt=args.slots, batch_sigs=args.batch)   # warm-up
    barrier.wait()
    t0 = time.time()
    lat, v, res = tile.latency_run(pay, 0.0, slot_cnt=args.slots, batch_sigs=args.batch, ring_depth=1 << 14,
                                   gpu_parse=args.gpu_parse)
    t1 = time.time()
    # the run proper (the tile's own clock, after its pipe and ring are set
    # up): it ended at t1 and lasted txns / achieved rate
    run0 = t1 - len(pay) / res["achieved_txn_per_s"]
    q.put({"rank": rank, "t0": run0, "t1": t1, "setup_s": run0 - t0, "txns": len(pay),
           "txn_per_s": res["achieved_txn_per_s"],
           "p99_ms": float(np.percentile(lat * 1e3, 99)), "all_success": bool((v == 0).all())})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,2,4,6,8")
    ap.add_argument("--txns", type=int, default=2000000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--gpu-parse", action="store_true")
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    for k in [int(x) for x in args.procs.split(",")]:
        barrier, q = ctx.Barrier(k), ctx.Queue()
        ps = [ctx.Process(target=child, args=(r, args, barrier, q)) for r in range(k)]
        for p in ps:
            p.start()
        rs = [q.get(timeout=600) for _ in range(k)]
        for p in ps:
            p.join(timeout=60)
        if any(p.exitcode != 0 for p in ps):
            print(json.dumps({"procs": k, "error": [p.exitcode for p in ps]}), flush=True)
            return 1
        window = max(r["t1"] for r in rs) - min(r["t0"] for r in rs)
        common = min(r["t1"] for r in rs) - max(r["t0"] for r in rs)
        total = sum(r["txns"] for r in rs)
        print(json.dumps({"procs": k, "batch_sigs": args.batch, "slots": args.slots,
                          "parse": "gpu" if args.gpu_parse else "host",
                          "txn_per_s": total / window, "window_s": window,
                          "common_s": common, "per_proc_txn_per_s": [round(r["txn_per_s"]) for r in rs],
                          "setup_s_max": max(r["setup_s"] for r in rs),
                          "p99_ms_max": max(r["p99_ms"] for r in rs),
                          "all_success": all(r["all_success"] for r in rs)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
