#!/usr/bin/env python3
"""Where the deployed path's latency tail sits (run on the box): the verify
tile under the reference's fd_mux_tile (oracle/_ref/mux/mux_harness) with
the GPU service behind it, as bench.py's latency_mode_deployed leg runs it,
at one offered rate, a few runs.  For every run: p50 / p99 / max and where
in the stream (frag index, in tenths of the run) the frags slower than
--slow-ms lie, and the run's latencies saved to gpurun_out/ for a closer
look.

    python tools/deployed_probe.py [--mode zero-copy|host-parse] [--rate 700000] [--runs 3] [--txns 300000]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import uuid

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["zero-copy", "host-parse", "gpu-parse"], default="zero-copy")
    ap.add_argument("--rate", type=float, default=700000.0)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--txns", type=int, default=300000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--slow-ms", type=float, default=5.0)
    ap.add_argument("--hw-queues", type=int, default=0, help="GPU_MAX_HW_QUEUES for the service (0: HIP's default)")
    ap.add_argument("--pin", action="store_true", help="service and harness on the GPU's NUMA-node CPUs (as bench.py)")
    ap.add_argument("--service", default=os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service"),
                    help="service binary (an A/B build's; its stderr profile lines are printed)")
    args = ap.parse_args()
    from firedancer_amd import ed25519, tile, workload
    mux = os.path.join(REPO, "oracle", "_ref", "mux", "mux_harness")
    svc_bin = args.service
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    pay, _ = workload.txn_payloads(eng, args.txns, 4711, msg_sz=200)
    node = sorted(tile.device_cpus(eng.info())) if args.pin else []
    eng.close()

    def pin():
        if node:
            os.sched_setaffinity(0, node)
    tmp = tempfile.mkdtemp(prefix="dprobe")
    path = os.path.join(tmp, "pay.bin")
    tile.write_payload_file(path, pay)
    mode = {"zero-copy": ["--zero-copy"], "gpu-parse": ["--gpu-parse"], "host-parse": []}[args.mode]
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    env = dict(os.environ)
    if args.hw_queues:
        env["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    for r in range(args.runs):
        app = uuid.uuid4().hex[:10]
        svc = subprocess.Popen([svc_bin, "--prefix", f"/fd_vhip_{app}_", "--tiles", "1", "--batch", str(args.batch),
                                "--slots", str(args.slots), *mode], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               text=True, preexec_fn=pin, env=env)
        line = svc.stdout.readline()
        if not line.startswith("ready"):
            raise SystemExit(f"service did not start: {line!r} {svc.stderr.read()[-500:]}")
        lat_path = os.path.join(tmp, "lat.bin")
        try:
            p = subprocess.run([mux, "verify_hip", path, os.path.join(tmp, "out.bin"), "--app", app, "--depth", "16384",
                                "--rate", str(args.rate), "--timeout", "100", "--log-path", "", "--lat-out", lat_path],
                               capture_output=True, text=True, timeout=150, preexec_fn=pin)
            if p.returncode != 0:
                raise SystemExit(f"harness rc {p.returncode}: {p.stderr[-500:]}")
            svc.wait(timeout=60)
            for ln in svc.stderr.read().splitlines():
                if "profile" in ln:
                    print(ln, flush=True)
        finally:
            if svc.poll() is None:
                svc.kill()
        res = json.loads(p.stdout.strip().splitlines()[-1])
        ms = np.fromfile(lat_path, np.uint32).astype(np.float64) * 1e-6
        slow = np.nonzero(ms > args.slow_ms)[0]
        tenths = np.bincount((slow * 10) // max(len(ms), 1), minlength=10).tolist() if slow.size else [0] * 10
        np.save(os.path.join(REPO, "gpurun_out", f"dprobe_{args.mode}_{r}.npy"), ms.astype(np.float32))
        print(json.dumps({"mode": args.mode, "batch": args.batch, "slots": args.slots, "hw_queues": args.hw_queues, "pinned": bool(node), "run": r, "rate": args.rate, "achieved": res["txn_per_s"],
                          "producer_credit_spins": res.get("producer_credit_spins"),
                          "consumer_idle_spins": res.get("consumer_idle_spins"),
                          "p50_ms": float(np.percentile(ms, 50)), "p99_ms": float(np.percentile(ms, 99)),
                          "max_ms": float(ms.max()), "slow_frags": int(slow.size),
                          "slow_first_last": [int(slow[0]), int(slow[-1])] if slow.size else None,
                          "slow_by_tenth_of_run": tenths}), flush=True)
    for f in os.listdir(tmp):
        os.unlink(os.path.join(tmp, f))
    os.rmdir(tmp)


if __name__ == "__main__":
    main()
