#!/usr/bin/env python3
"""Verify-tile layer throughput / latency sweep on one GPU (run on the box):
GPU-signed single-signer transactions through the tango-style ring and the
batched tile core (fd_ed25519_hip_latency_run), unpaced, for several batch
sizes and slot counts.  Prints one JSON object.

    python tools/tile_bench.py [--txns 400000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=400000)
    ap.add_argument("--batches", default="256,4096,16384,65536")
    ap.add_argument("--slots", default="3")
    ap.add_argument("--modes", default="host,gpu", help="parse on the host, the GPU, or both")
    ap.add_argument("--tiles", default="1", help="verify tiles (threads) on the GPU, comma list")
    args = ap.parse_args()
    from firedancer_amd import ed25519, tile, workload
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    t = time.perf_counter()
    pay, size = workload.txn_payloads(eng, args.txns, 99, msg_sz=200)
    gen_s = time.perf_counter() - t
    eng.close()
    # host-side parse cost alone (what the tile does per frag before staging)
    t = time.perf_counter()
    ok = sum(tile.txn_parse(bytes(pay[i])) is not None for i in range(2000))
    parse_us_py = (time.perf_counter() - t) / 2000 * 1e6
    out = {"txns": args.txns, "payload_bytes": size, "gen_seconds": gen_s, "parse_ok": ok,
           "python_parse_call_us": parse_us_py, "runs": []}
    tile.latency_run(pay[:20000], 0.0, slot_cnt=2, batch_sigs=4096)   # warm-up: code objects, pinned pools
    for mode in args.modes.split(","):
     for tiles in [int(x) for x in args.tiles.split(",")]:
      for slots in [int(s) for s in args.slots.split(",")]:
        for b in [int(x) for x in args.batches.split(",")]:
            lat, v, res = tile.latency_run(pay, 0.0, slot_cnt=slots, batch_sigs=b, ring_depth=1 << 14,
                                           gpu_parse=(mode == "gpu"), tiles=tiles)
            ms = lat * 1e3
            out["runs"].append({"parse": mode, "tiles": tiles, "batch_sigs": b, "slots": slots,
                                "txn_per_s": res["achieved_txn_per_s"],
                                "p50_ms": float(np.percentile(ms, 50)), "p99_ms": float(np.percentile(ms, 99)),
                                "batches": res["batches"], "overruns": res["ring_overruns"],
                                "all_success": bool((v == 0).all())})
            print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
