#!/usr/bin/env python3
"""The deployed path's ceiling without a GPU: the verify tile
(integration/fd_verify_hip.c) under the reference's fd_mux_tile
(oracle/_ref/mux/mux_harness) with the CPU stand-in service in parse-only
mode (oracle/_ref/mux/ref_vservice --parse-only: the reference's
fd_txn_parse and trailer, no signature check, every frag SUCCESS) behind
the same shared-memory links.  Unpaced, so the rate is what the producer ->
tile -> links -> stand-in -> tile -> consumer chain carries when verification
costs nothing: the bound the GPU service's deployed peak can approach.
Test infrastructure (the stand-in and the harness are oracle/ builds).

    python tools/chain_ceiling.py [--txns 400000] [--runs 3] [--cpus 0-7]
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


def payloads(n, msg_sz=200, seed=5):
    """n single-signer legacy transactions of workload.txn_payloads' shape,
    random signature and keys (parse-only: nothing is verified)"""
    from firedancer_amd import workload
    head = bytes([1, 0, 1]) + workload._cu16(3)
    fixed = len(head) + 32 * 3 + 32 + 1 + 1 + 1 + 2
    data_len = msg_sz - fixed - len(workload._cu16(max(msg_sz - fixed - 1, 0)))
    tail = bytes([1, 2, 2, 0, 1]) + workload._cu16(data_len)
    m_len = len(head) + 32 * 3 + 32 + len(tail) + data_len
    rng = np.random.default_rng(seed)
    pay = rng.integers(0, 256, (n, 1 + 64 + m_len), dtype=np.uint8)
    pay[:, 0] = 1
    p = 65
    pay[:, p:p + len(head)] = np.frombuffer(head, np.uint8)
    p += len(head) + 32 * 3 + 32
    pay[:, p:p + len(tail)] = np.frombuffer(tail, np.uint8)
    return pay


def parse_cpus(s):
    out = []
    for part in s.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=400000)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--cpus", default="", help="pin the stand-in and the harness to these CPUs")
    args = ap.parse_args()
    from firedancer_amd import tile
    mux = os.path.join(REPO, "oracle", "_ref", "mux")
    cpus = parse_cpus(args.cpus) if args.cpus else []

    def pin():
        if cpus:
            os.sched_setaffinity(0, cpus)
    tmp = tempfile.mkdtemp(prefix="chain")
    path = os.path.join(tmp, "pay.bin")
    tile.write_payload_file(path, payloads(args.txns))
    try:
        for r in range(args.runs):
            app = uuid.uuid4().hex[:10]
            svc = subprocess.Popen([os.path.join(mux, "ref_vservice"), "--prefix", f"/fd_vhip_{app}_", "--tiles", "1",
                                    "--parse-only", "--log-path", ""], stdout=subprocess.PIPE,
                                   stderr=subprocess.PIPE, text=True, preexec_fn=pin)
            try:
                line = svc.stdout.readline()
                if not line.startswith("ready"):
                    raise SystemExit(f"stand-in did not start: {line!r}")
                p = subprocess.run([os.path.join(mux, "mux_harness"), "verify_hip", path, os.path.join(tmp, "out.bin"),
                                    "--app", app, "--depth", "16384", "--timeout", "100", "--log-path", ""],
                                   capture_output=True, text=True, timeout=150, preexec_fn=pin)
                if p.returncode != 0:
                    raise SystemExit(f"harness rc {p.returncode}: {p.stderr[-500:]}")
                svc.wait(timeout=60)
            finally:
                if svc.poll() is None:
                    svc.kill()
            res = json.loads(p.stdout.strip().splitlines()[-1])
            print(json.dumps({"run": r, "txns": args.txns, "txn_per_s": res["txn_per_s"],
                              "published": res["published"], "cpus": args.cpus or "unpinned",
                              "producer_credit_spins": res.get("producer_credit_spins"),
                              "consumer_idle_spins": res.get("consumer_idle_spins")}), flush=True)
    finally:
        for f in os.listdir(tmp):
            os.unlink(os.path.join(tmp, f))
        os.rmdir(tmp)


if __name__ == "__main__":
    main()
