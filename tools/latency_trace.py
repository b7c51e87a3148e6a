#!/usr/bin/env python3
"""C5 latency mode at one offered load, for a kernel / copy trace: run it
under rocprofv3 --kernel-trace --memory-copy-trace and read the timeline
of each batch with tools/latency_timeline.py.

    python tools/latency_trace.py [--txns 20000] [--rate 1000000] [--slots 4] [--batch 256]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import ed25519, tile, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=20000)
    ap.add_argument("--rate", type=float, default=1.0e6)
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--gpu-parse", action="store_true")
    args = ap.parse_args()
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    pay, _ = workload.txn_payloads(eng, args.txns, 4242, msg_sz=200)
    eng.close()
    tile.latency_run(pay[:2000], 0.0, slot_cnt=args.slots, batch_sigs=args.batch)   # warm
    lat, v, res = tile.latency_run(pay, args.rate, slot_cnt=args.slots, batch_sigs=args.batch,
                                   gpu_parse=args.gpu_parse)
    ms = lat * 1e3
    print(json.dumps({"offered": args.rate, "achieved": res["achieved_txn_per_s"], "batches": res["batches"],
                      "p50_ms": float(np.percentile(ms, 50)), "p99_ms": float(np.percentile(ms, 99)),
                      "ok": bool((v == 0).all())}), flush=True)


if __name__ == "__main__":
    main()
