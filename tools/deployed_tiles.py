#!/usr/bin/env python3
"""K verify tiles on the deployed path, one GPU (run on the box): one
fd_verify_hip_service --tiles K, and K copies of the reference's tile
runtime (oracle/_ref/mux/mux_harness verify_hip, each its own process: a
producer, the sandboxed tile under fd_mux_tile, a dedup-side consumer), tile
k taking the frags with seq % K == k of the same quic stream, as the
reference's verify tiles share the quic link (fd_verify.c:36-47).  Unpaced;
the aggregate is the frags all tiles verified over the slowest tile's time.

Each harness runs 3 spinning threads and the service one per tile, so K
tiles take 4K cores: on a 16-core lease, K <= 4 says something about the
path, larger K about the lease.

    python tools/deployed_tiles.py [--tiles 1,2,4] [--txns 400000] [--batch 4096] [--slots 3] [--mode host-parse]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
import uuid

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="1,2,4")
    ap.add_argument("--txns", type=int, default=400000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--mode", choices=["zero-copy", "host-parse", "gpu-parse"], default="host-parse")
    ap.add_argument("--pin", action="store_true", help="everything on the GPU's NUMA-node CPUs")
    args = ap.parse_args()
    from firedancer_amd import ed25519, tile, workload
    mux = os.path.join(REPO, "oracle", "_ref", "mux", "mux_harness")
    svc_bin = os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service")
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    pay, _ = workload.txn_payloads(eng, args.txns, 8087, msg_sz=200)
    node = sorted(tile.device_cpus(eng.info())) if args.pin else []
    eng.close()

    def pin():
        if node:
            os.sched_setaffinity(0, node)
    tmp = tempfile.mkdtemp(prefix="dtiles")
    path = os.path.join(tmp, "pay.bin")
    tile.write_payload_file(path, pay)
    mode = {"zero-copy": ["--zero-copy"], "gpu-parse": ["--gpu-parse"], "host-parse": []}[args.mode]
    try:
        for k in [int(x) for x in args.tiles.split(",")]:
            for r in range(args.runs):
                app = uuid.uuid4().hex[:10]
                svc = subprocess.Popen([svc_bin, "--prefix", f"/fd_vhip_{app}_", "--tiles", str(k), "--batch",
                                        str(args.batch), "--slots", str(args.slots), *mode],
                                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, preexec_fn=pin)
                hs = []
                try:
                    line = svc.stdout.readline()
                    if not line.startswith("ready"):
                        raise SystemExit(f"service did not start: {line!r} {svc.stderr.read()[-500:]}")
                    t0 = time.perf_counter()
                    hs = [subprocess.Popen([mux, "verify_hip", path, os.path.join(tmp, f"out{i}.bin"), "--app", app,
                                            "--rr-cnt", str(k), "--rr-idx", str(i), "--depth", "16384",
                                            "--timeout", "100", "--log-path", ""],
                                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, preexec_fn=pin)
                          for i in range(k)]
                    outs = [h.communicate(timeout=150) for h in hs]
                    wall = time.perf_counter() - t0
                    for h, (o, e) in zip(hs, outs):
                        if h.returncode != 0:
                            raise SystemExit(f"harness rc {h.returncode}: {e[-500:]}")
                    if svc.wait(timeout=60) != 0:
                        raise SystemExit(f"service rc {svc.returncode}: {svc.stderr.read()[-500:]}")
                finally:
                    for h in hs:
                        if h.poll() is None:
                            h.kill()
                    if svc.poll() is None:
                        svc.kill()
                res = [json.loads(o.strip().splitlines()[-1]) for o, _ in outs]
                verified = sum(x["published"] for x in res)
                slowest = max(x["seconds"] for x in res)
                print(json.dumps({"tiles": k, "run": r, "mode": args.mode, "batch": args.batch, "slots": args.slots,
                                  "pinned": bool(node), "txns": args.txns, "verified": verified,
                                  "all_verified": verified == args.txns,
                                  "txn_per_s": verified / slowest,
                                  "per_tile_txn_per_s": [round(x["published"] / x["seconds"]) for x in res],
                                  "wall_s_incl_start": round(wall, 3)}), flush=True)
    finally:
        for f in os.listdir(tmp):
            os.unlink(os.path.join(tmp, f))
        os.rmdir(tmp)


if __name__ == "__main__":
    main()
