#!/usr/bin/env python3
"""Where the deployed multi-tile rate is capped: the
fdctl-topology harness (oracle/_ref/mux/mux_harness, the reference's
fd_mux_tile over one shared quic -> verify link) with no verify work:

  publish_only      the producer (the quic tile's side) alone, no reader:
                    its own publish rate (memcpy + fd_mcache_publish);
  filter_all K      K reference fd_mux_tile loops reading the shared link,
                    each filtering every frag in before_frag (fd_mux.c:387):
                    the run loop's per-frag cost and the credit coupling of
                    K reliable readers, with nothing behind them.

Unpaced, --txns 200-byte payloads (the C5 size), every thread on a physical
core of its own on the GPU's node (as bench.py's deployed leg), 3 runs each;
one JSON line per configuration.  Run on the box:

    python tools/mux_cap_probe.py [--txns 2000000] [--tiles 1,2,4,8]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=2000000)
    ap.add_argument("--tiles", default="1,2,4,8")
    ap.add_argument("--runs", type=int, default=3)
    args = ap.parse_args()
    from firedancer_amd import tile
    mux = os.path.join(REPO, "oracle", "_ref", "mux", "mux_harness")
    try:
        from firedancer_amd import ed25519
        eng = ed25519.Engine(0, max_chunk=4096)
        cores = tile.physical_cores(tile.device_cpus(eng.info()))
        eng.close()
    except Exception:   # no GPU: any physical cores
        cores = tile.physical_cores(os.sched_getaffinity(0))
    d = tempfile.mkdtemp(prefix="muxcap")
    path = os.path.join(d, "pay.bin")
    pay = np.zeros((args.txns, 200), np.uint8)
    pay[:, 0] = 1
    tile.write_payload_file(path, pay)
    configs = [("publish_only", 0)] + [("filter_all", int(k)) for k in args.tiles.split(",")]
    try:
        for kind, k in configs:
            need = 2 + k
            cpus = ",".join(map(str, cores[:need])) if len(cores) >= need else None
            rates, spins = [], []
            for r in range(args.runs):
                cmd = [mux, kind, path, os.path.join(d, "out.bin"), "--app", f"mc{os.getpid() % 10000}{r}",
                       "--depth", "16384", "--log-path", ""]
                if k:
                    cmd += ["--tiles", str(k)]
                if cpus:
                    cmd += ["--cpus", cpus]
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
                if p.returncode != 0:
                    raise SystemExit(f"{kind} {k}: rc {p.returncode} {p.stderr[-400:]}")
                res = json.loads(p.stdout.strip().splitlines()[-1])
                rates.append(res["txn_per_s"])
                spins.append(res["producer_credit_spins"])
            print(json.dumps({"kind": kind, "tiles": k, "txns": args.txns, "msg_sz": 200,
                              "txn_per_s_runs": [round(x) for x in rates], "txn_per_s_median": float(np.median(rates)),
                              "producer_credit_spins_runs": spins,
                              "cpus": cpus or "unpinned (not enough physical cores)"}), flush=True)
    finally:
        for f in os.listdir(d):
            os.unlink(os.path.join(d, f))
        os.rmdir(d)


if __name__ == "__main__":
    main()
