#!/usr/bin/env python3
"""K verify tiles on the deployed path in fdctl's topology, one GPU (run on
the box).  One harness process (oracle/_ref/mux/mux_harness --tiles K, the
reference's tile runtime compiled from its sources) holds the topology
fdctl builds: ONE quic -> verify link published by one producer thread (the
quic tile), K sandboxed verify tiles under fd_mux_tile that all read it and
keep seq % K == their kind id (src/app/fdctl/run/tiles/fd_verify.c:36-47,
verify_tile_count, src/app/fdctl/config/default.toml:535), K verify -> dedup
links read by one consumer thread (the dedup tile).  Behind the tiles one
fd_verify_hip_service --tiles K, its link pairs served by ceil(K / L)
threads (--links-per-thread L).  Every thread is pinned to its own physical
core of the GPU's NUMA node, and L is the smallest that keeps all spinning
threads -- K + 2 in the harness, ceil(K / L) in the service -- within the
lease's cores (16 on the box).  Unpaced: the rate is every verified frag
over the harness's stream time.  Beside it, the reference's own
fd_tile_verify (CPU verify) in the same topology with the same K.

    python tools/deployed_tiles.py [--tiles 1,2,4,8] [--txns 600000] [--batch 4096] [--slots 3] [--runs 2]
"""
import argparse
import json
import math
import os
import subprocess
import sys
import tempfile
import uuid

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def physical_cores(cpus):
    """one logical CPU per physical core, in the order given"""
    seen, out = set(), []
    for c in cpus:
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            out.append(c)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="1,2,4,8")
    ap.add_argument("--txns", type=int, default=600000)
    ap.add_argument("--ref-txns", type=int, default=120000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--cores", type=int, default=0, help="spinning-thread budget (default: the lease's CPU share)")
    ap.add_argument("--mode", choices=["zero-copy", "host-parse", "gpu-parse"], default="host-parse")
    args = ap.parse_args()
    from firedancer_amd import ed25519, tile, workload
    mux = os.path.join(REPO, "oracle", "_ref", "mux", "mux_harness")
    svc_bin = os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service")
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    pay, _ = workload.txn_payloads(eng, args.txns, 8087, msg_sz=200)
    node = physical_cores(sorted(tile.device_cpus(eng.info())))
    eng.close()
    cores = args.cores or workload.host_cores()[0]
    tmp = tempfile.mkdtemp(prefix="dtiles")
    path, path_ref = os.path.join(tmp, "pay.bin"), os.path.join(tmp, "pay_ref.bin")
    tile.write_payload_file(path, pay)
    tile.write_payload_file(path_ref, pay[:args.ref_txns])
    mode = {"zero-copy": ["--zero-copy"], "gpu-parse": ["--gpu-parse"], "host-parse": []}[args.mode]

    def cpu_list(cs):
        return ",".join(str(c) for c in cs)
    try:
        for k in [int(x) for x in args.tiles.split(",")]:
            per = 1
            while k + 2 + math.ceil(k / per) > cores and per < k:
                per += 1
            svc_threads = math.ceil(k / per)
            need = k + 2 + svc_threads
            if len(node) < need:
                raise SystemExit(f"{k} tiles need {need} physical cores, the GPU's node has {len(node)}")
            svc_cpus, h_cpus = node[:svc_threads], node[svc_threads:need]
            for r in range(args.runs):
                app = uuid.uuid4().hex[:10]
                svc = subprocess.Popen([svc_bin, "--prefix", f"/fd_vhip_{app}_", "--tiles", str(k), "--batch",
                                        str(args.batch), "--slots", str(args.slots), "--links-per-thread", str(per),
                                        "--cpus", cpu_list(svc_cpus), *mode],
                                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                h = None
                try:
                    line = svc.stdout.readline()
                    if not line.startswith("ready"):
                        raise SystemExit(f"service did not start: {line!r} {svc.stderr.read()[-500:]}")
                    h = subprocess.run([mux, "verify_hip", path, os.path.join(tmp, "out.bin"), "--app", app,
                                        "--tiles", str(k), "--depth", "16384", "--timeout", "100", "--log-path", "",
                                        "--cpus", cpu_list(h_cpus)], capture_output=True, text=True, timeout=150)
                    if h.returncode != 0:
                        raise SystemExit(f"harness rc {h.returncode}: {h.stderr[-500:]}")
                    if svc.wait(timeout=60) != 0:
                        raise SystemExit(f"service rc {svc.returncode}: {svc.stderr.read()[-500:]}")
                finally:
                    if svc.poll() is None:
                        svc.kill()
                res = json.loads(h.stdout.strip().splitlines()[-1])
                ref = subprocess.run([mux, "verify", path_ref, os.path.join(tmp, "out_ref.bin"), "--tiles", str(k),
                                      "--depth", "16384", "--timeout", "100", "--log-path", "", "--cpus",
                                      cpu_list(h_cpus)], capture_output=True, text=True, timeout=150)
                rres = json.loads(ref.stdout.strip().splitlines()[-1]) if ref.returncode == 0 else {"error": ref.stderr[-300:]}
                print(json.dumps({
                    "tiles": k, "run": r, "mode": args.mode, "batch": args.batch, "slots": args.slots,
                    "txns": args.txns, "verified": res["published"], "all_frags_consumed": res["frags"] == args.txns,
                    "txn_per_s": res["txn_per_s"], "seconds": res["seconds"],
                    "threads": {"harness": res["threads"], "service": svc_threads, "links_per_thread": per,
                                "total": res["threads"] + svc_threads, "core_budget": cores},
                    "producer_credit_spins": res["producer_credit_spins"],
                    "consumer_idle_spins": res["consumer_idle_spins"],
                    "reference_tiles_txn_per_s": rres.get("txn_per_s"), "reference_txns": args.ref_txns,
                    "topology": "one quic->verify link, K tiles seq % K, K verify->dedup links, one consumer"}),
                    flush=True)
    finally:
        for f in os.listdir(tmp):
            os.unlink(os.path.join(tmp, f))
        os.rmdir(tmp)


if __name__ == "__main__":
    main()
