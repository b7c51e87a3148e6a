#!/usr/bin/env python3
"""Verify tiles as sandboxed processes behind one GPU service process (the
deployment shape of integration/fd_verify_hip.c; run on the box).

For each K: one fd_verify_hip_service for K tiles, and K tile-side
processes (firedancer_amd/_lib/fd_shlink_producer: maps its two links,
enters seccomp strict mode, streams its transactions and takes the
verdict frags back, as the tile's during_frag / after_credit do).  Every
tile streams its own GPU-signed single-signer transactions; the service's
per-tile stream time runs from its first frag to the end of the stream, and
the aggregate is all tiles' transactions over the longest stream time (the
producers start together).  Verdicts are checked (all SUCCESS).

    python tools/service_bench.py [--tiles 1,2,4,6] [--txns 1000000] [--batch 4096] [--gpu-parse | --zero-copy]
                                  [--links-per-thread L]
"""
import argparse
import json
import multiprocessing as mp
import os
import subprocess
import sys
import tempfile
import time
import uuid

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVICE = os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service")
PRODUCER = os.path.join(REPO, "firedancer_amd", "_lib", "fd_shlink_producer")


def gen(paths, txns, q):
    """payload files, one per tile, signed on the GPU (in a child process,
    so the parent never holds the GPU while the service runs)"""
    sys.path.insert(0, REPO)
    from firedancer_amd import ed25519, tile, workload
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    q.put(sorted(tile.device_cpus(eng.info())))
    for k, path in enumerate(paths):
        pay, _ = workload.txn_payloads(eng, txns, 7000 + k, msg_sz=200)
        tile.write_payload_file(path, pay)
    eng.close()
    q.put(True)


def physical_cores(cpus):
    """one logical CPU per physical core among cpus (the lowest SMT
    sibling), in order"""
    out, seen = [], set()
    for c in sorted(cpus):
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
    ap.add_argument("--tiles", default="1,2,4,6")
    ap.add_argument("--txns", type=int, default=1000000, help="transactions per tile")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--gpu-parse", action="store_true")
    ap.add_argument("--zero-copy", action="store_true", help="the service DMAs payloads from the txn links in place")
    ap.add_argument("--links-per-thread", type=int, default=1, help="tiles one service thread serves")
    ap.add_argument("--hw-queues", type=int, default=16, help="GPU_MAX_HW_QUEUES of the service process")
    ap.add_argument("--service", default=SERVICE, help="service binary (an A/B build's)")
    ap.add_argument("--producer", default=PRODUCER, help="tile-side binary (the same A/B build's: the frag protocol)")
    ap.add_argument("--producer-profile", action="store_true",
                    help="the tile side's cycles per txn (fd_shlink_producer --profile: runs unsandboxed)")
    ap.add_argument("--pin", choices=["none", "node", "cores"], default="node",
                    help="node: the service and the tile processes on the CPUs of the GPU's NUMA node (default); "
                         "cores: each tile process and each service link thread on a physical core of its own "
                         "there, as fdctl pins tiles; none: wherever the OS puts them")
    args = ap.parse_args()
    ks = [int(x) for x in args.tiles.split(",")]
    tmp = tempfile.mkdtemp(prefix="svcb")
    paths = [os.path.join(tmp, f"p{k}.bin") for k in range(max(ks))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=gen, args=(paths, args.txns, q))
    p.start()

    def take():
        """the generator's next message; fails at once if it died"""
        import queue
        for _ in range(600):
            try:
                return q.get(timeout=1)
            except queue.Empty:
                if not p.is_alive():
                    raise SystemExit(f"payload generator exited with {p.exitcode}")
        raise SystemExit("payload generator: no answer in 600 s")
    node_cpus = take()
    take()
    p.join(timeout=60)
    pin = None
    if args.pin in ("node", "cores") and node_cpus:
        def pin():
            os.sched_setaffinity(0, node_cpus)
    cores = physical_cores(node_cpus) if args.pin == "cores" else []
    out = []
    for k in ks:
        app = uuid.uuid4().hex[:10]
        prefix = f"/fd_vhip_{app}_"
        env = dict(os.environ, GPU_MAX_HW_QUEUES=str(args.hw_queues))
        svc_cpus = ["--cpus", ",".join(str(c) for c in cores[k:2 * k])] if len(cores) >= 2 * k else []
        svc = subprocess.Popen([args.service, "--prefix", prefix, "--tiles", str(k), "--batch", str(args.batch), *svc_cpus,
                                "--slots", str(args.slots), *(["--gpu-parse"] if args.gpu_parse else []),
                                *(["--zero-copy"] if args.zero_copy else []),
                                *(["--links-per-thread", str(args.links_per_thread)] if args.links_per_thread != 1 else [])],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, preexec_fn=pin)
        line = svc.stdout.readline()
        if not line.startswith("ready"):
            raise SystemExit(f"service did not start: {line!r} {svc.stderr.read()[-2000:]}")
        t0 = time.time()
        def pin_core(c):
            return lambda: os.sched_setaffinity(0, {c})
        prods = [subprocess.Popen([args.producer, f"{prefix}{i}_txn", f"{prefix}{i}_vd", paths[i],
                                   *(["--profile"] if args.producer_profile else [])],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                  preexec_fn=pin_core(cores[i]) if len(cores) >= 2 * k else pin) for i in range(k)]
        ok = True
        for pr in prods:
            so, se = pr.communicate(timeout=300)
            ok &= pr.returncode == 0 and len(so) >= args.txns and so[:args.txns].count(0) == args.txns
            for ln in se.decode(errors="replace").splitlines():
                if "profile" in ln:
                    print(ln, file=sys.stderr)
        wall = time.time() - t0
        so, se = svc.communicate(timeout=120)
        res = json.loads(so.strip().splitlines()[-1])
        for ln in se.splitlines():
            if "profile" in ln:
                print(ln, file=sys.stderr)
        secs = []
        for ln in se.splitlines():   # "fd_verify_hip_service: tile k: N txns in B batches, S s, D device bytes"
            if ": tile " in ln and " txns in " in ln:
                secs.append(float(ln.split(" batches, ")[1].split(" s,")[0]))
        agg = sum(res["txns"]) / max(secs) if secs else None
        out.append({"tiles": k, "txns_per_tile": args.txns, "txn_per_s": agg, "per_tile_txn_per_s":
                    [args.txns / s for s in secs], "wall_s_incl_producer_start": wall, "service_rc": svc.returncode,
                    "verdicts_all_success": ok, "shared_device_bytes": res["shared_device_bytes"],
                    "tile_device_bytes": res["tile_device_bytes"]})
        print(json.dumps(out[-1]), flush=True)
        for kind in ("txn", "vd"):
            for i in range(k):
                try:
                    os.unlink(f"/dev/shm{prefix}{i}_{kind}")
                except OSError:
                    pass
    for path in paths:
        os.unlink(path)
    print(json.dumps({"service_bench": out, "batch": args.batch, "slots": args.slots, "gpu_parse": args.gpu_parse, "zero_copy": args.zero_copy,
                      "links_per_thread": args.links_per_thread,
                      "hw_queues": args.hw_queues, "pin": args.pin, "cores_used": 2 * max(ks) if args.pin == "cores" else None, "node_cpus": len(node_cpus)}))


if __name__ == "__main__":
    main()
