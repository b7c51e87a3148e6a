#!/usr/bin/env python3
"""Benchmark: ed25519 batch verification on MI355X.

A step is one verification pass (hash, decode, dsm kernels) over this rank's
batch of BASELINE.json's C2 workload -- 1,048,576 signatures, messages of
64-1232 B, 2% invalid -- resident in HBM (generated on the device by the
library's own batch signer, firedancer_amd/workload.py).  With N GPUs each
rank verifies its own shard (different signatures, no collective: weak
scaling); value = signatures verified by all ranks / max-over-ranks time.

Printed on rank 0 as one JSON line, with:
  roofline      INT32 VALU roofline of the dominant kernel (dsm), from the
                SURVEY.md §8(d) frozen per-verify op count and the kernel's
                mean duration measured with HIP events on its stream
  cpu_baseline  the reference's own fd_ed25519_verify (compiled from its
                sources into oracle/_ref) on this host's cores, over a bounded
                sample of the same workload (rank 0, N=1 only)

    python bench.py [--gpus N] [--steps K] [--warmup W]

With --gpus N > 1 and no launcher environment (WORLD_SIZE unset), bench.py
starts its N ranks itself, as child processes created before anything
touches a GPU (rank r on device r, gloo for the barrier and the
max-over-ranks); under torchrun it uses the launcher's ranks.  Every rank
must hold a distinct device (checked by PCI address) unless
--allow-shared-device is given (a one-GPU rehearsal).

No rank can hang the others: the gloo group has a 120 s timeout, every
rank's setup (device check, engine, workload) runs under a guard and all
ranks agree on its outcome in one collective before anything else, so a
failure on any rank makes every rank exit non-zero right away; when
bench.py started the ranks itself, it ends the others once one has failed.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "ed25519 verifies/sec at 1/8 GPUs; % INT32 VALU roofline; p99 batch latency"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


GLOO_TIMEOUT_S = float(os.environ.get("FD_BENCH_GLOO_TIMEOUT_S", "120"))
RANK_GRACE_S = 30.0


def spawn_ranks(gpus):
    """--gpus N without a launcher: N child processes of this script, rank r
    on device r, started before this process touches any GPU; returns the
    exit code (the worst rank's).  Once a rank has failed, the others get
    RANK_GRACE_S to finish (they normally fail the same agreement at once)
    and are then ended, so a dead rank never keeps the job waiting."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    failed_at = None
    while any(p.poll() is None for p in procs):
        if failed_at is None and any(p.poll() not in (None, 0) for p in procs):
            failed_at = time.time()
        if failed_at is not None and time.time() - failed_at > RANK_GRACE_S:
            for p in procs:
                if p.poll() is None:
                    log(f"[launcher] ending rank pid {p.pid}: another rank failed {RANK_GRACE_S:.0f} s ago")
                    p.kill()
        time.sleep(0.2)
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return (bad[0] if bad[0] > 0 else 2) if bad else 0


def dist_setup(gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        log(f"[rank {rank}] --gpus {gpus} but the launcher started {world} ranks")
        sys.exit(2)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo reports its connections on stdout: keep stdout for the one
        # JSON line (fd 1 points at stderr while the group forms)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        from datetime import timedelta
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=GLOO_TIMEOUT_S))
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return rank, local, world


def all_gather(obj, world):
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def allreduce_max(x, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(x, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_has(flag):
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    return flag in line.split()
    except OSError:
        pass
    return False


def cpu_baseline(wl, gpu_codes, sample, reps, workload_name="C2"):
    """Reference CPU verify (oracle/_ref) on `sample` signatures of the workload,
    one pthread per core of this process's share.  Also checks the reference's
    verdicts against the GPU's on the sample."""
    from firedancer_amd import workload
    ref_dir = os.path.join(REPO, "oracle", "_ref")
    flavour = "avx512" if cpu_has("avx512ifma") and cpu_has("avx512vbmi") else "portable"
    path = os.path.join(ref_dir, f"libfdref_{flavour}.so")
    kind = "reference"
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.fdref_verify_many.restype = ctypes.c_long
    lib.fdref_verify_many.argtypes = [ctypes.c_ulong] + [ctypes.c_void_p] * 6 + [ctypes.c_int, ctypes.c_ulong]
    n = min(sample, wl.n)
    sizes = wl.sizes[:n].astype(np.uint64)
    off = np.zeros(n, np.uint64)
    np.cumsum(sizes[:-1], out=off[1:])
    nbytes = int(sizes.sum())
    msgs = wl.msgs.download(np.uint8, max(nbytes, 1))
    sigs = wl.sigs.download(np.uint8, 64 * n)
    pubs = wl.pubs.download(np.uint8, 32 * n)
    sz = wl.sizes[:n].astype(np.uint32)
    out = np.zeros(n, np.int8)
    threads, cores_src = workload.host_cores()
    ns = lib.fdref_verify_many(n, msgs.ctypes.data, off.ctypes.data, sz.ctypes.data, sigs.ctypes.data,
                               pubs.ctypes.data, out.ctypes.data, threads, reps)
    if ns <= 0:
        return None
    rate = n * reps / (ns * 1e-9)
    box = workload.box_cores()
    proj = rate / threads * box["physical_cores"] if box["physical_cores"] else None
    return {"value": rate, "unit": "verifies/s", "cores": threads, "kind": kind,
            "box": box,
            "box_projection": {"verifies_per_s": proj, "basis": "per_core x box physical_cores",
                               "note": "a projection, not a measurement: this lease may use `cores` of the box; "
                                       "linear per physical core, SMT siblings not counted"},
            "sample": f"first {n} signatures of the {workload_name} workload x {reps} passes, fd_ed25519_verify of the "
                      f"reference's {flavour} backend (compiled from its sources), {threads} pthreads",
            "cores_source": cores_src,
            "scope": "the host cores this process may use (cores_source), measured on rank 0 in the same run "
                     "after the GPU steps",
            "seconds": ns * 1e-9, "per_core": rate / threads,
            "verdicts_equal_gpu": bool(np.array_equal(out, gpu_codes[:n]))}


def config_c1(eng, args, inflight):
    """C1 (BASELINE.json configs[0]): 16,384 single-signer ~200-byte
    signatures, all valid -- the reference's own CPU case.  The reference's
    fd_ed25519_verify on this host's cores (20 passes) next to this engine
    on one GPU (20 launches of the 16K batch, device-resident)."""
    from firedancer_amd import ed25519
    wl = ed25519.DeviceWorkload(eng, 16384, 200, 200, 0, seed=args.seed + 1)
    for _ in range(3):
        wl.verify()
    eng.sync()
    t = time.perf_counter()
    for _ in range(20):
        wl.verify()
    eng.sync()
    gpu_s = time.perf_counter() - t
    out = wl.out.download(np.int8, wl.n)
    # the same batch with `inflight` launches in flight on one-stream engines
    engs = [ed25519.Engine(device=eng.info()["device"], max_chunk=wl.n, half=args.half, one_stream=True)
            for _ in range(max(inflight, 1))]
    eouts = [e.alloc(wl.n) for e in engs]

    def run_k(k):
        e, o = engs[k % len(engs)], eouts[k % len(engs)]
        e.verify_dev(wl.n, wl.msgs.ptr, wl.off.ptr, wl.sz.ptr, wl.sigs.ptr, wl.pubs.ptr, o.ptr, e.stream)
    for k in range(len(engs)):
        run_k(k)
    for e in engs:
        e.sync()
    t = time.perf_counter()
    for k in range(80):
        run_k(k)
    for e in engs:
        e.sync()
    gpu_p = time.perf_counter() - t
    ok_p = all(bool((o.download(np.int8, wl.n) == 0).all()) for o in eouts)
    for o in eouts:
        o.free()
    for e in engs:
        e.close()
    cpu = cpu_baseline(wl, out, wl.n, 20, workload_name="C1")
    wl.free()
    return {"signatures": 16384, "msg_sz": 200, "gpu_verifies_per_s": 20 * 16384 / gpu_s,
            "gpu_ms_per_batch": gpu_s * 1e3 / 20, "all_valid": bool((out == 0).all()),
            "pipelined": {"batches_in_flight": len(engs), "gpu_verifies_per_s": 80 * 16384 / gpu_p,
                          "all_valid": ok_p},
            "cpu_reference": cpu}


def config_c3(eng, args, inflight):
    """C3 (BASELINE.json configs[2]): multi-signer transactions with
    fd_ed25519_verify_batch_single_msg's semantics -- 1..12 signatures
    (uniform) over one shared 200-byte message each, all valid -- as a
    device-resident batch of 65,536 transactions: the per-signature verify,
    then the per-transaction combine (fd_ed25519_hip_txn_combine_dev).
    Parity of this path is in tests/test_gpu_c3.py."""
    rng = np.random.default_rng(args.seed + 3)
    ntxn, msz = 65536, 200
    cnt = rng.integers(1, 13, ntxn).astype(np.uint32)
    first = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint32)
    nsig = int(cnt.sum())
    off = np.repeat(np.arange(ntxn, dtype=np.uint64) * msz, cnt)
    sz = np.full(nsig, msz, np.uint32)
    bufs = [eng.alloc(ntxn * msz + 16), eng.alloc(8 * nsig).upload(off), eng.alloc(4 * nsig).upload(sz),
            eng.alloc(64 * nsig), eng.alloc(32 * nsig), eng.alloc(nsig), eng.alloc(4 * ntxn).upload(first),
            eng.alloc(4 * ntxn).upload(cnt), eng.alloc(ntxn)]
    msgs, d_off, d_sz, sigs, pubs, out, d_first, d_cnt, tout = bufs
    eng.gen_dev(nsig, args.seed + 3, 0, msgs.ptr, ntxn * msz, d_off.ptr, d_sz.ptr, sigs.ptr, pubs.ptr)

    def run():
        eng.verify_dev(nsig, msgs.ptr, d_off.ptr, d_sz.ptr, sigs.ptr, pubs.ptr, out.ptr)
        eng.txn_combine_dev(ntxn, out.ptr, d_first.ptr, d_cnt.ptr, tout.ptr)
    for _ in range(2):
        run()
    eng.sync()
    t = time.perf_counter()
    for _ in range(10):
        run()
    eng.sync()
    dt = time.perf_counter() - t
    codes = tout.download(np.int8, ntxn)
    # the same batches with `inflight` of them in flight on one-stream
    # engines (as the C2 steps and the pool's slots run): a batch's phases
    # fill the previous batch's dsm tail
    from firedancer_amd import ed25519
    engs = [ed25519.Engine(device=eng.info()["device"], max_chunk=nsig, half=args.half, one_stream=True)
            for _ in range(max(inflight, 1))]
    eouts = [(e.alloc(nsig), e.alloc(ntxn)) for e in engs]

    def run_k(k):
        e, (o, to) = engs[k % len(engs)], eouts[k % len(engs)]
        e.verify_dev(nsig, msgs.ptr, d_off.ptr, d_sz.ptr, sigs.ptr, pubs.ptr, o.ptr, e.stream)
        e.txn_combine_dev(ntxn, o.ptr, d_first.ptr, d_cnt.ptr, to.ptr, e.stream)
    for k in range(len(engs)):
        run_k(k)
    for e in engs:
        e.sync()
    t = time.perf_counter()
    for k in range(20):
        run_k(k)
    for e in engs:
        e.sync()
    dtp = time.perf_counter() - t
    ok_p = all(bool((to.download(np.int8, ntxn) == 0).all()) for _, to in eouts)
    for o, to in eouts:
        o.free()
        to.free()
    for e in engs:
        e.close()
    for b in bufs:
        b.free()
    return {"txns": ntxn, "signatures": nsig, "sigs_per_txn": "1..12 uniform, one shared 200-byte message",
            "gpu_txn_per_s": 10 * ntxn / dt, "gpu_verifies_per_s": 10 * nsig / dt,
            "gpu_ms_per_batch": dt * 1e3 / 10, "all_success": bool((codes == 0).all()),
            "pipelined": {"batches_in_flight": len(engs), "gpu_txn_per_s": 20 * ntxn / dtp,
                          "gpu_verifies_per_s": 20 * nsig / dtp, "all_success": ok_p}}


SUSTAINED_PEAK = ("the highest paced rate at which one run keeps achieved/offered >= 0.99, bisected (5 runs) between "
                  "0.5x and 1x the median of 3 unpaced runs")


def sustained_rate(run_at, unpaced, steps=5, lo_frac=0.5, keep=0.99):
    """C5's peak: the highest offered rate at which one
    paced run keeps achieved / offered >= keep, found by bisection between
    lo_frac x and 1 x the unpaced median (an unpaced run overshoots what
    the paced path sustains, so 95% of it was not a load the path held).
    run_at(rate) -> achieved txn/s.  -> (rate, [[offered, achieved/offered]...])"""
    lo, hi, trail = lo_frac * unpaced, unpaced, []
    for _ in range(steps):
        mid = 0.5 * (lo + hi)
        a = run_at(mid)
        trail.append([round(mid, 1), round(a / mid, 4)])
        if a / mid >= keep:
            lo = mid
        else:
            hi = mid
    return lo, trail


class keep_off:
    """For the with-block, every thread of this process (and the children
    started with `child_mask`) off the physical cores the latency legs'
    spinning threads are pinned to, SMT siblings included: the Python main
    thread and the HIP runtime's helper threads float over the node
    otherwise, and one of them woken on a spinning thread's CPU takes a
    scheduler slice from it (a pause of milliseconds), or on its sibling
    halves its speed for a while (the path delivering at half the offered
    rate for ~10 ms: tools/episode_shape.py, profiles/r6_c5_episodes.txt).
    Restored afterwards; a no-op with --no-isolate-cores or when the node
    has no CPU to spare."""

    def __init__(self, spin, node, enabled):
        from firedancer_amd import tile
        busy = set().union(*(tile.core_siblings(c) for c in spin)) if spin else set()
        others = sorted(set(node) - busy) if spin else []
        self.mask = others if enabled and others else None
        self.saved = {}

    def child_mask(self, node):
        return self.mask or node

    def __enter__(self):
        if self.mask:
            for t in os.listdir("/proc/self/task"):
                try:
                    self.saved[int(t)] = os.sched_getaffinity(int(t))
                    os.sched_setaffinity(int(t), self.mask)
                except OSError:   # a thread that ended meanwhile
                    pass
        return self

    def __exit__(self, *exc):
        for t, m in self.saved.items():
            try:
                os.sched_setaffinity(t, m)
            except OSError:
                pass
        return False


def latency_mode(eng, args, device):
    """C5: the verify tile's latency mode.  Signed single-signer Solana
    transactions (~200-byte messages, GPU-signed) are published into a
    tango-style mcache/dcache ring by a producer thread at a fixed offered
    load; the verify-tile core (fd_ed25519_hip_vtile: parse, dedup,
    batch_single_msg verify) pulls them and submits batches of up to
    `batch` signatures (sooner when the ring is drained and a slot is free).
    Latency = due publish time -> verdict on the host.  Peak = the highest
    paced rate one run sustains (sustained_rate); then 50/80/95% of it."""
    from firedancer_amd import tile, workload
    n = args.latency_txns
    pay, _ = workload.txn_payloads(eng, n, args.seed + 77, msg_sz=200)
    ok = True
    # the producer and the tile each on a physical core of its own on the
    # GPU's node, as fdctl pins tiles: floating, the two threads can share a
    # core (SMT siblings, or other work), and the tile's per-frag rate then
    # varied run to run by 1.6x (profiles/r6_c5_stage_trace.txt)
    cores = tile.physical_cores(tile.device_cpus(eng.info()))
    if args.pin_threads and len(cores) >= 2:
        tile.latency_set_cpus(cores[0], cores[1])

    def run_at(rate):
        nonlocal ok
        lat, v, res = tile.latency_run(pay, rate, device=device, slot_cnt=args.latency_slots,
                                       batch_sigs=args.latency_batch, ring_depth=4096)
        ok &= bool((v == 0).all())
        return res["achieved_txn_per_s"]

    spin = cores[:2] if args.pin_threads and len(cores) >= 2 else None
    if args.pipe_split_waves:
        tile.pipe_set_split_waves(args.pipe_split_waves)
    try:
        with keep_off(spin, tile.device_cpus(eng.info()), args.isolate_cores):
            return latency_mode_loads(args, run_at, pay, n, device, lambda: ok, spin)
    finally:
        tile.latency_set_cpus(-1, -1)


def latency_mode_loads(args, run_at, pay, n, device, verdicts_ok, cpus):
    from firedancer_amd import tile
    unpaced = [run_at(0.0) for _ in range(3)]
    peak, trail = sustained_rate(run_at, float(np.median(unpaced)))
    out = {"batch_sigs": args.latency_batch, "slots_in_flight": args.latency_slots,
           "threads": (f"producer on CPU {cpus[0]}, tile on CPU {cpus[1]} (physical cores of the GPU's node)"
                       if cpus else "unpinned"),
           "other_threads": ("kept off those cores and their SMT siblings" if cpus and args.isolate_cores
                             else "anywhere on the node"),
           "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES") or 4), "txns_per_run": n,
           "msg_sz": 200, "peak_txn_per_s": peak, "peak": SUSTAINED_PEAK, "peak_search": trail,
           "unpaced_median_txn_per_s": float(np.median(unpaced)), "unpaced_runs_txn_per_s": unpaced,
           "ring": "tango-style mcache/dcache, depth 4096", "verdicts_ok": verdicts_ok(), "loads": []}
    # each load five times; p50 / p99 / max are over every transaction of
    # the five runs pooled (a run is ~0.05-0.1 s, so one host hiccup of a
    # few milliseconds is its whole p99: pooling keeps such events in the
    # tail instead of choosing a run after the fact), each run's own p99
    # beside them
    for frac in (0.5, 0.8, 0.95):
        runs, pooled = [], []
        for _ in range(5):
            lat, v, res = tile.latency_run(pay, frac * peak, device=device, slot_cnt=args.latency_slots,
                                           batch_sigs=args.latency_batch, ring_depth=4096)
            ms = lat * 1e3
            pooled.append(ms)
            runs.append({"offered_txn_per_s": res["offered_txn_per_s"], "achieved_txn_per_s": res["achieved_txn_per_s"],
                         "p99_ms": float(np.percentile(ms, 99)), "batches": res["batches"],
                         "ratio": res["achieved_txn_per_s"] / res["offered_txn_per_s"],
                         "ring_overruns": res["ring_overruns"]})
            out["verdicts_ok"] &= bool((v == 0).all())
        ms = np.concatenate(pooled)
        offered = float(np.mean([r["offered_txn_per_s"] for r in runs]))
        achieved = float(np.mean([r["achieved_txn_per_s"] for r in runs]))
        out["loads"].append({"offered_frac_of_peak": frac, "offered_txn_per_s": offered, "achieved_txn_per_s": achieved,
                             "achieved_over_offered": achieved / offered,
                             "p50_ms": float(np.percentile(ms, 50)), "p99_ms": float(np.percentile(ms, 99)),
                             "max_ms": float(ms.max()), "samples": int(ms.size), "percentiles": "pooled over 5 runs",
                             "p99_ms_runs": [r["p99_ms"] for r in runs],
                             "achieved_over_offered_runs": [round(r["ratio"], 4) for r in runs],
                             "batches": sum(r["batches"] for r in runs),
                             "ring_overruns": sum(r["ring_overruns"] for r in runs)})
    return out


def latency_deployed(eng, args):
    """C5 on the deployed path: the sandboxed verify
    tile (integration/fd_verify_hip.c) under the reference's own tile
    runtime -- fd_mux_tile, its mcache / dcache links and seccomp filter,
    compiled from the reference's sources as the harness
    oracle/_ref/mux/mux_harness -- with the product's GPU service process
    (fd_verify_hip_service, 256-signature batches, --deployed-slots of them
    in flight, each on its own hardware queue) behind its shared-memory
    links.  A producer publishes GPU-signed single-signer transactions into
    the quic -> verify link at a fixed offered load, each frag's tsorig its
    due time; the dedup side takes (now - tsorig) for every verified frag
    the tile publishes (src/disco/mux/fd_mux.c:548-559,
    src/app/fdctl/run/tiles/fd_verify.c:152-153).  Peak = the highest paced
    rate one run sustains (sustained_rate); then 50 / 80 / 95% of it, five runs each, percentiles over all
    five runs' frags pooled.  Beside it, the reference's own fd_tile_verify
    (CPU verify, one tile) in the same harness at 50 / 80 / 95% of its own
    peak: the CPU baseline of this leg.  The headline value is untouched:
    this leg measures the host runtime the verification plugs into."""
    import subprocess
    import tempfile
    import uuid
    from firedancer_amd import tile, workload
    mux = os.path.join(REPO, "oracle", "_ref", "mux", "mux_harness")
    svc_bin = os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service")
    if not (os.path.exists(mux) and os.path.exists(svc_bin)):
        return {"error": "oracle/_ref/mux or the service binary not built"}
    n, n_ref = args.deployed_txns, args.deployed_ref_txns
    pay, _ = workload.txn_payloads(eng, n, args.seed + 91, msg_sz=200)
    tmp = tempfile.mkdtemp(prefix="c5dep")
    path, path_ref = os.path.join(tmp, "pay.bin"), os.path.join(tmp, "pay_ref.bin")
    tile.write_payload_file(path, pay)
    tile.write_payload_file(path_ref, pay[:n_ref])
    svc_mode = ["--zero-copy"] if args.deployed_mode == "zero-copy" else (
        ["--gpu-parse"] if args.deployed_mode == "gpu-parse" else [])
    # the service and the tile's harness on the CPUs of the GPU's NUMA node,
    # as fdctl pins its tiles (tools/service_bench.py does the same)
    node = sorted(tile.device_cpus(eng.info()))
    # and each spinning thread on a physical core of its own (the harness's
    # producer, consumer and tile; the service's link thread), as fdctl pins
    # one tile per core
    cores = tile.physical_cores(node)
    per_thread = args.pin_threads and len(cores) >= 4
    # a hardware queue per slot: with two per slot (16), every batch of the
    # service's took ~0.8 ms at p99 even at the reference tile's loads
    # (profiles/r6_c5_launch_bump.txt)
    svc_queues = max(4, args.deployed_slots)
    harness_cpus = ["--cpus", ",".join(map(str, cores[:3]))] if per_thread else []
    service_cpus = ["--cpus", str(cores[3])] if per_thread else []

    iso = keep_off(cores[:4] if per_thread else None, node, args.isolate_cores)

    def pin():
        if node:
            os.sched_setaffinity(0, iso.child_mask(node))

    def delivered(r):
        """a run's achieved rate: its frags over the span from its start to
        the last verified frag delivered (the harness's own `txn_per_s`
        also counts the quiescence check after it, up to a housekeeping
        interval of each tile)"""
        return r.get("txn_per_s_delivered", r["txn_per_s"])

    def run(kind, rate, pay_path=None):
        """one harness run -> (its JSON line, latencies in ms)"""
        app = uuid.uuid4().hex[:10]
        svc = None
        if kind == "verify_hip":
            svc = subprocess.Popen([svc_bin, "--prefix", f"/fd_vhip_{app}_", "--tiles", "1", "--batch",
                                    str(args.latency_batch), "--slots", str(args.deployed_slots),
                                    "--hw-queues", str(svc_queues), *svc_mode, *service_cpus,
                                    *(["--split-waves", str(args.pipe_split_waves)] if args.pipe_split_waves else [])],
                                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, preexec_fn=pin)
            line = svc.stdout.readline()
            if not line.startswith("ready"):
                raise RuntimeError(f"service did not start: {line!r} {svc.stderr.read()[-500:]}")
        lat_path = os.path.join(tmp, f"lat_{app}.bin")
        try:
            pay_path = pay_path or (path if kind == "verify_hip" else path_ref)
            p = subprocess.run([mux, kind, pay_path, os.path.join(tmp, "out.bin"),
                                "--app", app, "--depth", "16384", "--rate", str(rate), "--timeout", "100",
                                "--log-path", "", "--lat-out", lat_path, *harness_cpus], capture_output=True, text=True,
                               timeout=150,
                               preexec_fn=pin)
            if p.returncode != 0:
                raise RuntimeError(f"harness {kind} rc {p.returncode}: {p.stderr[-500:]}")
            if svc is not None and svc.wait(timeout=60) != 0:
                raise RuntimeError(f"service rc {svc.returncode}: {svc.stderr.read()[-500:]}")
        finally:
            if svc is not None and svc.poll() is None:
                svc.kill()
            for f in os.listdir("/dev/shm"):
                if f.startswith(f"fd_vhip_{app}_"):
                    try:
                        os.unlink(os.path.join("/dev/shm", f))
                    except OSError:
                        pass
        res = json.loads(p.stdout.strip().splitlines()[-1])
        lat = np.fromfile(lat_path, np.uint32).astype(np.float64) * 1e-6
        os.unlink(lat_path)
        keep = os.environ.get("FD_BENCH_LAT_DIR")   # tail analysis (tools/episode_shape.py): every run's samples
        if keep:
            os.makedirs(keep, exist_ok=True)
            np.save(os.path.join(keep, f"{kind}_{int(rate)}_{app}.npy"), lat.astype(np.float32))
        return res, lat

    def sweep(kind, runs, txns):
        # the peak: the highest paced rate one run sustains (as latency_mode)
        published = []

        def run_at(rate):
            r = run(kind, rate)[0]
            published.append(r["published"] == txns)
            return delivered(r)

        unpaced = [run_at(0) for _ in range(3)]
        peak, trail = sustained_rate(run_at, float(np.median(unpaced)))
        out = {"peak_txn_per_s": peak, "peak": SUSTAINED_PEAK, "peak_search": trail,
               "unpaced_median_txn_per_s": float(np.median(unpaced)), "unpaced_runs_txn_per_s": unpaced,
               "txns_per_run": txns, "loads": [], "published_all": all(published)}
        for frac in (0.5, 0.8, 0.95):
            pooled, per_run = [], []
            for _ in range(runs):
                res, lat = run(kind, frac * peak)
                pooled.append(lat)
                per_run.append(res)
                out["published_all"] &= res["published"] == txns
            ms = np.concatenate(pooled)
            achieved = float(np.mean([delivered(r) for r in per_run]))
            out["loads"].append({"offered_frac_of_peak": frac, "offered_txn_per_s": frac * peak,
                                 "achieved_txn_per_s": achieved, "achieved_over_offered": achieved / (frac * peak),
                                 "p50_ms": float(np.percentile(ms, 50)), "p99_ms": float(np.percentile(ms, 99)),
                                 "max_ms": float(ms.max()), "samples": int(ms.size),
                                 "percentiles": f"pooled over {runs} runs",
                                 "p99_ms_runs": [r["lat_p99_us"] * 1e-3 for r in per_run],
                                 "achieved_over_offered_runs": [round(delivered(r) / (frac * peak), 4)
                                                                for r in per_run]})
        return out
    def at_rates(rates, runs):
        """the GPU tile at absolute offered loads (the reference tile's own
        rates and multiples of its peak): pooled p50 / p99 / max per rate.
        A run lasts about a second at the reference's rates (its 40K-txn
        file), 0.5 s at ten times its peak (the 300K file)."""
        out, rp = [], ref["peak_txn_per_s"]
        for label, rate in rates:
            f = path_ref if rate <= rp else path   # the reference tile's own transactions at its rates
            txns = n_ref if f == path_ref else n
            pooled, per_run = [], []
            for _ in range(runs):
                res, lat = run("verify_hip", rate, f)
                pooled.append(lat)
                per_run.append(res)
            ms = np.concatenate(pooled)
            out.append({"load": label, "offered_txn_per_s": rate, "txns_per_run": txns,
                        "achieved_txn_per_s": float(np.mean([delivered(r) for r in per_run])),
                        "published_all": all(r["published"] == txns for r in per_run),
                        "p50_ms": float(np.percentile(ms, 50)), "p99_ms": float(np.percentile(ms, 99)),
                        "max_ms": float(ms.max()), "samples": int(ms.size), "percentiles": f"pooled over {runs} runs"})
        return out
    try:
        with iso:
            hip = sweep("verify_hip", 5, n)
            ref = sweep("verify", 2, n_ref)
            rp = ref["peak_txn_per_s"]
            matched = at_rates([(f"{f:g} x reference tile peak", f * rp) for f in (0.5, 0.8, 0.95, 10.0, 100.0)],
                               args.deployed_matched_runs) if args.deployed_matched_runs > 0 else None
    finally:
        for f in os.listdir(tmp):
            os.unlink(os.path.join(tmp, f))
        os.rmdir(tmp)
    hip.update({"batch_sigs": args.latency_batch, "slots_in_flight": args.deployed_slots,
                "hw_queues": svc_queues,
                "cpus": f"{len(node)} CPUs of the GPU's NUMA node (service and harness pinned)" if node else "unpinned",
                "threads": (f"harness producer / consumer / tile on CPUs {cores[:3]}, service link thread on CPU "
                            f"{cores[3]} (physical cores)" if per_thread else "not pinned per thread"),
                "other_threads": "kept off those cores and their SMT siblings" if iso.mask else "anywhere on the node",
                "service_mode": args.deployed_mode, "msg_sz": 200,
                "path": "producer -> quic_verify mcache/dcache (reference tango) -> fd_tile_verify_hip under the "
                        "reference's fd_mux_tile, its seccomp filter installed -> shlink -> fd_verify_hip_service "
                        "(GPU) -> shlink -> after_credit publish -> verify_dedup mcache -> consumer",
                "latency": "due time (tsorig) -> verified frag received on the out link",
                "runtime": "the tile runtime (fd_mux, tango, metrics) is the reference's, compiled from its sources "
                           "as the harness oracle/_ref/mux/mux_harness; verification runs in the product's service"})
    hip["cpu_baseline_reference_tile"] = dict(ref, tile="the reference's fd_tile_verify (fd_verify.c, CPU verify, "
                                                        "AVX-512 build) in the same harness, one tile")
    if matched is not None:
        # the two tiles at the same absolute offered load: the reference
        # tile's 50 / 80 / 95% (its loads above), then 10x and 100x its peak
        # (100x is above the GPU tile's own peak when that is below ~5.8M:
        # then it measures the backlog of an overloaded tile)
        ref_at = {l["offered_frac_of_peak"]: l for l in ref["loads"]}
        for m in matched:
            f = m["offered_txn_per_s"] / rp
            r = ref_at.get(round(f, 2))
            m["reference_tile"] = ({"p50_ms": r["p50_ms"], "p99_ms": r["p99_ms"], "max_ms": r["max_ms"]} if r
                                   else "above the reference tile's peak: it cannot carry this load")
            m["above_gpu_tile_peak"] = m["offered_txn_per_s"] > hip["peak_txn_per_s"]
        hip["loads_at_reference_rates"] = matched
    return hip


def host_fed(wl, device, info, world, reps, batch, slots, copies):
    """The host-fed path: the C2 signatures from host memory (page-locked,
    as a deployment registers its dcache once) through the pool's feeder
    thread (fd_ed25519_hip_pool_run, one thread on the GPU's NUMA node):
    per batch, H2D of the messages' byte range and of msg_off / msg_sz /
    sigs / pubs, verify, D2H of the codes into the caller's array, `slots`
    batches in flight.  Measured as a continuous stream -- the 1M set
    `copies` times back to back, so the pipeline fills and drains once --
    and as single 1M passes.  Reported beside the device-resident value
    (never as it), with the PCIe bound it is up against: the H2D rate of a
    plain pinned copy over the bytes a signature moves."""
    from firedancer_amd import tile
    import contextlib
    n = wl.n
    mb = wl.msg_bytes
    # Every rank reaches every collective below whatever happens to its own
    # leg (a rank that raised before a barrier would hang the others): each
    # stage runs under a guard and the ranks agree on the outcome first.
    err = [None]

    def guarded(fn):
        if err[0] is None:
            try:
                return fn()
            except Exception as ex:  # reported below, on every rank
                err[0] = ex
        return None

    def agree(what):
        if allreduce_sum(0 if err[0] is None else 1, world) != 0:
            raise RuntimeError(f"host-fed leg failed on a rank ({what}): {err[0]!r}")

    near = tile.NearDevice(info)
    res = {}
    with contextlib.ExitStack() as stack:
        def prepare():
            msgs1 = wl.msgs.download(np.uint8, mb)
            off1 = wl.off.download(np.uint64, n)
            sigs1 = wl.sigs.download(np.uint8, 64 * n)
            pubs1 = wl.pubs.download(np.uint8, 32 * n)
            res["expect1"] = wl.expect.download(np.int8, n)
            # the stream's host buffers are first touched on the GPU's NUMA node
            with near:
                res["msgs"] = np.concatenate([msgs1] * copies + [np.zeros(16, np.uint8)])
                res["off"] = np.concatenate([off1 + np.uint64(c * mb) for c in range(copies)])
                res["sz"] = np.tile(wl.sizes.astype(np.uint32), copies)
                res["sigs"], res["pubs"] = np.tile(sigs1, copies), np.tile(pubs1, copies)
                res["out"] = np.ones(copies * n, np.int8)
            pool = tile.Pool([device], batch, slots, tile.max_span(res["off"], res["sz"], batch))
            stack.callback(pool.close)
            res["pool"] = pool
            t = time.perf_counter()
            stack.enter_context(tile.HostRegistration(res["msgs"], res["off"], res["sz"], res["sigs"], res["pubs"],
                                                      res["out"]))
            res["reg_s"] = time.perf_counter() - t
            # warm-up: a whole stream (clocks, DMA engines, page tables)
            pool.run(res["msgs"], res["off"], res["sz"], res["sigs"], res["pubs"], res["out"])

        guarded(prepare)
        agree("setup")
        barrier(world)
        t0 = time.perf_counter()

        def stream():
            runs, st = [], None
            for _ in range(reps):
                _, sec, st = res["pool"].run(res["msgs"], res["off"], res["sz"], res["sigs"], res["pubs"], res["out"])
                runs.append(sec)
            res["runs"], res["st"] = runs, st
        guarded(stream)
        dt = time.perf_counter() - t0
        barrier(world)
        agree("stream")
        ok = bool(np.array_equal(res["out"], np.tile(res["expect1"], copies)))

        def single():
            t1 = time.perf_counter()
            for _ in range(reps):
                res["pool"].run(res["msgs"][:mb + 16], res["off"][:n], res["sz"][:n], res["sigs"][:64 * n],
                                res["pubs"][:32 * n], res["out"][:n])
            res["dt1"] = time.perf_counter() - t1
        guarded(single)
    agree("single pass")
    st, runs, dt1, reg_s = res["st"], res["runs"], res["dt1"], res["reg_s"]
    dt_max = allreduce_max(dt, world)
    ok_all = allreduce_sum(0 if ok else 1, world) == 0
    h2d = tile.h2d_gbps(device, 256 << 20, 8)
    bytes_per_sig = st["h2d_bytes"] / (copies * n)
    bound = h2d * 1e9 / bytes_per_sig if h2d > 0 else None
    rate = world * copies * n * reps / dt_max
    return {"value": rate, "unit": "verifies/s", "per_gpu": rate / world, "n_gpus": world,
            "stream": f"the {n}-signature C2 set {copies} times back to back ({copies * n} signatures) x {reps}",
            "single_pass_verifies_per_s_per_gpu": n * reps / dt1,
            "stream_run_seconds": runs,
            "batch_sigs": batch, "slots_in_flight": slots,
            "h2d_bytes_per_signature": bytes_per_sig, "achieved_h2d_GBps_per_gpu": rate / world * bytes_per_sig / 1e9,
            "pinned_copy_h2d_GBps": h2d, "pcie_bound_verifies_per_s_per_gpu": bound,
            "frac_of_pcie_bound": (rate / world / bound) if bound else None,
            "direct_batches": st["direct_batches"], "staged_batches": st["staged_batches"],
            "register_seconds": reg_s, "verdicts_match_labels": ok_all,
            "host_buffers_numa_cpus": f"{len(near.cpus)} CPUs of the GPU's NUMA node" if near.cpus else "unknown",
            "path": "host SoA (page-locked) -> per-batch H2D (messages as one DMA of their span) -> verify -> "
                    "D2H codes; fd_ed25519_hip_pool_run, one feeder thread pinned to the GPU's NUMA node"}


# the verdict-stream SHA-256 of the whole 64M C4 stream (seed 0xC4C4, 1M-signature
# generation chunks), every code of which the reference's AVX-512 fd_ed25519_verify
# checked in rounds 1-3 (profiles/r3_parity_stream_64M.json)
C4_STREAM_DIGEST = "11b24458a5f5f3f3b9da0dd24ef066725e4fd8930c0ff61570c5f21348417503"
C4_STREAM_SEED = 0xC4C4
C4_CHUNK = 1 << 20


def host_stream(n, sizes, window, chunk, fill, pool_run, world, alloc=np.zeros, register=None):
    """Streams this rank's shard of n signatures from host memory through
    its GPU's feeder, `window` signatures at a time, so the host holds one
    window whatever n is (C4: 64M signatures are ~48 GB of messages).

      fill(i0, m, msgs, sigs, pubs) writes shard signatures [i0, i0+m) into
        the window views given (messages back to back, sizes[i0:i0+m]) and
        returns their expected codes (int8[m]); called per `chunk`
      pool_run(msgs, off, sz, sigs, pubs, out) verifies one window from the
        host arrays (codes into out) and returns its seconds

    Every window starts on all ranks together (a barrier) and its time is
    the max over ranks, so the sum over windows is the time in which all the
    GPUs streamed the whole job; refilling a window (here from the GPU's own
    generator, in deployment the NIC and the quic tiles) is outside it.
    Each stage runs under a guard and the ranks agree on its outcome before
    the next collective, so a failure on one rank fails every rank and none
    is left in a barrier.  Returns the rank's codes too (for the stream
    digest)."""
    import hashlib
    err = [None]

    def guarded(fn):
        if err[0] is None:
            try:
                return fn()
            except Exception as ex:  # agreed on below, on every rank
                err[0] = ex
        return None

    def agree(what):
        if allreduce_sum(0 if err[0] is None else 1, world) != 0:
            raise RuntimeError(f"host stream failed on a rank ({what}): {err[0]!r}")

    W = max(1, min(window, n))
    nwin = -(-n // W)
    cs = np.zeros(n + 1, np.uint64)
    np.cumsum(sizes, dtype=np.uint64, out=cs[1:])
    cap = max(int(cs[min(n, (w + 1) * W)] - cs[w * W]) for w in range(nwin))
    arr = {}

    def setup():
        arr["msgs"] = alloc(cap + 16, np.uint8)
        arr["off"], arr["sz"] = alloc(W, np.uint64), alloc(W, np.uint32)
        arr["sigs"], arr["pubs"], arr["out"] = alloc(64 * W, np.uint8), alloc(32 * W, np.uint8), alloc(W, np.int8)
    guarded(setup)
    agree("window allocation")
    host_bytes = sum(a.nbytes for a in arr.values())
    codes = np.zeros(n, np.int8)
    dig = hashlib.sha256()
    win_s, mism = [], 0
    import contextlib
    t_wall = time.perf_counter()
    with contextlib.ExitStack() as stack:
        if register is not None:
            guarded(lambda: stack.enter_context(register(*arr.values())))
            agree("window registration")
        for w in range(nwin):
            i0, i1 = w * W, min(n, (w + 1) * W)
            m, base = i1 - i0, int(cs[i0])
            expect = np.zeros(m, np.int8)

            def refill():
                arr["off"][:m] = cs[i0:i1] - np.uint64(base)
                arr["sz"][:m] = sizes[i0:i1]
                for c0 in range(i0, i1, chunk):
                    c1 = min(i1, c0 + chunk)
                    b0, b1 = int(cs[c0]) - base, int(cs[c1]) - base
                    expect[c0 - i0:c1 - i0] = fill(c0, c1 - c0, arr["msgs"][b0:b1], arr["sigs"][64 * (c0 - i0):64 * (c1 - i0)],
                                                   arr["pubs"][32 * (c0 - i0):32 * (c1 - i0)])
            guarded(refill)
            agree(f"window {w} refill")
            if w == 0:   # warm-up pass over the first window, untimed: clocks, DMA engines, IOMMU mappings
                guarded(lambda: pool_run(arr["msgs"][:int(cs[i1]) - base + 16], arr["off"][:m], arr["sz"][:m],
                                         arr["sigs"][:64 * m], arr["pubs"][:32 * m], arr["out"][:m]))
                agree("warm-up")
            barrier(world)
            sec = guarded(lambda: pool_run(arr["msgs"][:int(cs[i1]) - base + 16], arr["off"][:m], arr["sz"][:m],
                                           arr["sigs"][:64 * m], arr["pubs"][:32 * m], arr["out"][:m]))
            agree(f"window {w} stream")
            win_s.append(allreduce_max(sec, world))
            out = arr["out"][:m]
            codes[i0:i1] = out
            dig.update(out.tobytes())
            mism += int((out != expect).sum())
    wall = time.perf_counter() - t_wall
    return {"windows": nwin, "window_signatures": W, "window_seconds_max_over_ranks": win_s,
            "stream_seconds": float(sum(win_s)), "wall_seconds_with_refill": wall,
            "host_window_bytes": int(host_bytes), "label_mismatches": mism,
            "rank_digest": dig.hexdigest()}, codes


def _mem_available():
    """MemAvailable of this node in bytes (/proc/meminfo), or None"""
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return None


def _memlock_limit():
    """RLIMIT_MEMLOCK's soft limit in bytes, or None when unlimited"""
    import resource
    soft, _ = resource.getrlimit(resource.RLIMIT_MEMLOCK)
    return None if soft == resource.RLIM_INFINITY else int(soft)


def c4_window_preflight(window, sizes, world, chunk, local_world=None):
    """Before any rank pins its C4 window: the windows of
    all the node's ranks must fit in half of its MemAvailable, and each in
    RLIMIT_MEMLOCK when that is finite.  A window that does not fit shrinks
    (to a multiple of `chunk` when at least one chunk fits): the stream is
    counter-based per signature, so the verdicts and the digest do not
    depend on the window.  Every rank takes the smallest rank's window, so
    all run the same number of windows (their barriers pair up), and all
    fail together, before pinning anything, when not one signature fits.
    -> (window, record)"""
    n = len(sizes)
    W = max(1, min(window, n))
    bps = (float(np.mean(sizes)) if n else 0.0) + 8 + 4 + 64 + 32 + 1   # message, off, sz, sig, pub, code
    avail, memlock = _mem_available(), _memlock_limit()
    local = int(local_world or os.environ.get("LOCAL_WORLD_SIZE") or world)
    budget = None if avail is None else 0.5 * avail / max(local, 1)
    if memlock is not None:
        budget = memlock if budget is None else min(budget, memlock)
    fit = W if budget is None else int(budget // bps)
    W2 = W if fit >= W else ((fit // chunk) * chunk if fit >= chunk else fit)
    W2 = int(-allreduce_max(-float(W2), world))
    rec = {"requested_window": int(window), "window": W2, "bytes_per_signature_est": round(bps, 1),
           "ranks_on_node": local, "mem_available_bytes": avail, "memlock_limit_bytes": memlock,
           "budget_bytes_per_rank": budget, "shrunk": W2 < W}
    if W2 < 1:
        raise RuntimeError(f"C4 pre-flight: no window fits ({rec})")
    return W2, rec


def c4_host_fed(eng, device, info, rank, world, n, index_base, cfg, seed, window, batch, slots):
    """C4 as north_star defines it: the 64M-signature stream sharded over
    the GPUs with per-GPU host feeders (src/app/fdctl/run/tiles/
    fd_verify.c:46's seq % verify_tile_count).  Each rank streams its
    contiguous shard [index_base, index_base + n) from page-locked host
    windows through a one-device pool (fd_ed25519_hip_pool_run, one feeder
    thread on the GPU's NUMA node).  The windows are filled 1M signatures at
    a time from the device generator with the stream's seed and 1M chunk
    boundaries -- byte for byte the stream whose every code the reference
    checked (tools/parity_stream.py) -- so the concatenated verdict digest
    must equal C4_STREAM_DIGEST."""
    from firedancer_amd import ed25519, tile, workload
    import hashlib
    import resource
    sizes = workload.msg_sizes(seed, index_base, n, cfg["lo"], cfg["hi"])
    near = tile.NearDevice(info)

    def alloc(count, dtype):
        with near:   # first touch on the GPU's NUMA node
            return np.zeros(count, dtype)

    def fill(i0, m, msgs, sigs, pubs):
        wl = ed25519.DeviceWorkload(eng, m, cfg["lo"], cfg["hi"], cfg["ppm"], seed=seed, index_base=index_base + i0)
        try:
            if wl.msg_bytes != msgs.nbytes:
                raise RuntimeError(f"chunk at {index_base + i0}: {wl.msg_bytes} message bytes, window has {msgs.nbytes}")
            wl.msgs.download_into(msgs)
            wl.sigs.download_into(sigs)
            wl.pubs.download_into(pubs)
            return wl.expect.download(np.int8, m)
        finally:
            wl.free()
    pool = []   # made by the first (warm-up) call, under host_stream's guard: a rank whose pool fails is agreed on
    st = {}
    calls = [0]

    def run(msgs, off, sz, sigs, pubs, out):
        if not pool:
            pool.append(tile.Pool([device], batch, slots))
        _, sec, s = pool[0].run(msgs, off, sz, sigs, pubs, out)
        calls[0] += 1
        if calls[0] > 1:   # host_stream's first call is its untimed warm-up pass: not in the byte count
            for k, v in s.items():
                st[k] = st.get(k, 0) + v
        return sec
    window, preflight = c4_window_preflight(window, sizes, world, C4_CHUNK)
    try:
        res, codes = host_stream(n, sizes, window, C4_CHUNK, fill, run, world, alloc=alloc,
                                 register=tile.HostRegistration)
    finally:
        for p in pool:
            p.close()
    digests = all_gather(res["rank_digest"], world)
    if world > 1:
        everything = all_gather(codes.tobytes(), world)
        stream_digest = hashlib.sha256(b"".join(everything)).hexdigest()
    else:
        stream_digest = res["rank_digest"]
    mism_all = int(allreduce_sum(res["label_mismatches"], world))
    total = world * n
    rate = total / res["stream_seconds"]
    h2d = tile.h2d_gbps(device, 256 << 20, 8)
    bps = st.get("h2d_bytes", 0) / max(n, 1)
    bound = h2d * 1e9 / bps if h2d > 0 and bps > 0 else None
    whole = total == cfg["n"] and seed == C4_STREAM_SEED and (cfg["lo"], cfg["hi"], cfg["ppm"]) == (64, 1232, 20000)
    rss = allreduce_max(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024.0, world)
    return {"value": rate, "unit": "verifies/s", "per_gpu": rate / world, "n_gpus": world,
            "stream": f"{total} signatures (seed {seed:#x}), {n} per rank from host memory in "
                      f"{res['windows']} window(s) of {res['window_signatures']}",
            "stream_seconds": res["stream_seconds"], "window_seconds_max_over_ranks": res["window_seconds_max_over_ranks"],
            "wall_seconds_with_refill": res["wall_seconds_with_refill"],
            "host_window_bytes_per_rank": res["host_window_bytes"], "peak_rss_bytes_max_over_ranks": rss,
            "window_preflight": preflight,
            "batch_sigs": batch, "slots_in_flight": slots,
            "h2d_bytes_per_signature": bps, "achieved_h2d_GBps_per_gpu": rate / world * bps / 1e9,
            "pinned_copy_h2d_GBps": h2d, "pcie_bound_verifies_per_s_per_gpu": bound,
            "frac_of_pcie_bound": (rate / world / bound) if bound else None,
            "direct_batches": st.get("direct_batches"), "staged_batches": st.get("staged_batches"),
            "verdicts_match_labels": mism_all == 0, "label_mismatches": mism_all,
            "rank_digests": digests, "stream_digest": stream_digest,
            "reference_checked_digest": C4_STREAM_DIGEST if whole else None,
            "digest_equal": (stream_digest == C4_STREAM_DIGEST) if whole else None,
            "path": "page-locked host window -> per-batch H2D (messages as one DMA of their span) -> verify -> D2H "
                    "codes; fd_ed25519_hip_pool_run, one feeder thread on the GPU's NUMA node, per rank"}


def config_c4(eng, device, info, rank, world, args):
    """C4 in the default run (BASELINE.json configs[3]): the 64M-signature
    stream (seed 0xC4C4) sharded over the N ranks of this job, rank r its
    contiguous 64M/N, each streamed from bounded page-locked host windows
    through its own GPU's feeder (c4_host_fed), so that every `bench.py
    --gpus N` line -- the driver's SCALE runs included -- carries north
    star's C4 curve point beside the C2 headline (strong scaling: the
    stream's size is fixed, its time is the max over ranks per window).
    The concatenated verdict digest is compared with the one whose every
    code the reference's AVX-512 verify checked (C4_STREAM_DIGEST)."""
    from firedancer_amd import workload
    cfg = dict(workload.CONFIGS["C4"])
    total = args.c4_signatures
    if total % world:
        raise ValueError(f"--c4-signatures {total} does not split over {world} ranks")
    cfg["n"] = total
    n = total // world
    res = c4_host_fed(eng, device, info, rank, world, n, rank * n, cfg, C4_STREAM_SEED, args.host_window,
                      args.host_batch, args.host_slots)
    res.update({"scaling": "strong", "signatures_total": total, "signatures_per_rank": n,
                "shard": "rank r streams signatures [r*n, (r+1)*n) of the stream (fd_verify.c:46's seq % "
                         "verify_tile_count, as contiguous shards so each rank's host window is one range)",
                "rss_note": "peak RSS of the whole bench process (the C2 host-fed leg's 4 x 1M set included)"})
    return res


def pmc_traffic(n):
    """HBM bytes per dsm launch from the committed PMC summary (rocprofv3
    FETCH_SIZE + WRITE_SIZE passes, tools/pmc_summary.py), scaled to n.
    The dsm kernel's loads are 16 B per lane (global_load_dwordx4), for
    which gfx950's FETCH_SIZE reports half the bytes
    (MI355X_MICROARCH.md, HBM): reads are doubled; WRITE_SIZE is exact for
    16-B stores."""
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(path))["fd_ed25519_dsm_kernel"]
        per_sig = 2.0 * d["hbm_read_bytes_per_signature"] + d["hbm_write_bytes_per_signature"]
        return per_sig * n, os.path.relpath(path, REPO)
    except (OSError, KeyError, ValueError):
        return None, None


def pmc_issue_rate(cu_cnt):
    """The dsm kernel's VALU issue rate from the committed PMC summary:
    wave-instructions (SQ_INSTS_VALU) per SIMD over the kernel's active
    cycles (GRBM_GUI_ACTIVE, summed over the 8 XCDs), i.e. cycles per
    VALU wave-instruction per SIMD (the measured issue
    costs are 2.5 for 32-bit VOP2 ops, 4.2-4.4 for VOP3, 5.2 for the
    32x32->64 multiply-add)."""
    try:
        d = json.load(open(os.path.join(REPO, "profiles", "pmc_latest.json")))["fd_ed25519_dsm_kernel"]["per_dispatch"]
        return d["GRBM_GUI_ACTIVE"] / 8.0 / (d["SQ_INSTS_VALU"] / (cu_cnt * 4))
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None


def pmc_valu_per_sig():
    """Executed INT32+INT64 VALU instructions per signature (= per lane:
    one signature per lane) of the dsm kernel (rocprofv3
    SQ_INSTS_VALU_INT32/INT64 x 64 / signatures, committed summary)."""
    try:
        d = json.load(open(os.path.join(REPO, "profiles", "pmc_latest.json")))["fd_ed25519_dsm_kernel"]
        return d["SQ_INSTS_VALU_INT32_per_signature"] + d["SQ_INSTS_VALU_INT64_per_signature"]
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n", type=int, default=0, help="signatures per GPU (default: the config's)")
    ap.add_argument("--seed", type=int, default=None,
                    help="workload seed (default 0x5EED; C4: 0xC4C4, the stream the reference checked)")
    ap.add_argument("--cpu-sample", type=int, default=1048576)
    ap.add_argument("--cpu-reps", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--half", default="extended", choices=["extended", "strict"],
                    help="half-size scalar bound (A/B only; same verdicts)")
    ap.add_argument("--latency-batch", type=int, default=256)
    ap.add_argument("--latency-slots", type=int, default=8,
                    help="latency-mode batches in flight, one hardware queue each (see --hw-queues): 8 peak at "
                         "4.4M txn/s with the 4-slot p99, 4 at 3.3M")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES of this process (HIP's default is 4), set before its first HIP call "
                         "unless the environment names more; 0 leaves it.  8, a queue per latency slot: 16 here "
                         "beside the deployed leg's service (8) put every deployed batch at ~0.7 ms p99 "
                         "(profiles/r6_c5_launch_bump.txt)")
    ap.add_argument("--dev-kernargs", action="store_true",
                    help="leave HIP's kernel arguments in device memory (its default on this GPU; A/B)")
    ap.add_argument("--latency-txns", type=int, default=400000, help="0 disables the latency mode")
    ap.add_argument("--pipe-split-waves", type=int, default=0,
                    help="latency legs: small batches' group equation over 2, 4 or 8 waves "
                         "(fd_ed25519_hip_pipe_set_split_waves, the service's --split-waves; 0: the library's)")
    ap.add_argument("--no-isolate-cores", dest="isolate_cores", action="store_false",
                    help="latency legs: leave this process's other threads and the children's unpinned ones free "
                         "to run on the spinning threads' cores (A/B)")
    ap.add_argument("--no-pin-threads", dest="pin_threads", action="store_false",
                    help="C5 legs: leave the producer / tile / service threads unpinned (A/B)")
    ap.add_argument("--deployed-txns", type=int, default=300000,
                    help="C5 on the deployed path (the tile under fd_mux_tile + the GPU service): txns per run, "
                         "0 disables")
    ap.add_argument("--deployed-ref-txns", type=int, default=40000,
                    help="the reference tile's runs in the same harness (its CPU baseline)")
    ap.add_argument("--deployed-slots", type=int, default=8,
                    help="batches in flight in the deployed C5 leg's service (one hardware queue each): 8 carries "
                         "4.5M txn/s at the 4-slot p50, 4 saturate at 2.7M (profiles/r4_deployed_batch_slots_curve.txt)")
    ap.add_argument("--deployed-matched-runs", type=int, default=3,
                    help="runs per load of the deployed GPU tile at the reference tile's own absolute rates "
                         "(loads_at_reference_rates); 0 disables")
    ap.add_argument("--deployed-mode", default="host-parse", choices=["zero-copy", "gpu-parse", "host-parse"],
                    help="the GPU service's mode for the deployed C5 leg")
    ap.add_argument("--host-reps", type=int, default=3, help="host-fed stream passes (0 disables)")
    ap.add_argument("--host-copies", type=int, default=4, help="host-fed stream: the set this many times")
    ap.add_argument("--host-batch", type=int, default=131072)
    ap.add_argument("--host-slots", type=int, default=3,
                    help="batches in flight per GPU in the pool (70.1-70.5M/s at 3, 66-71M/s at 2 or 4: "
                         "profiles/r3_pool_h2d_serialize_ab.txt)")
    ap.add_argument("--host-first", action="store_true", help="run the host-fed leg first (A/B)")
    ap.add_argument("--host-window", type=int, default=8 << 20,
                    help="C4 host-fed stream: signatures per page-locked host window (the host holds one)")
    ap.add_argument("--c4-signatures", type=int, default=64 << 20,
                    help="the C4 stream leg of a C2 run (config_c4): signatures in the whole stream, split over the "
                         "ranks; 0 disables")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight on the GPU (steps alternate between this many engines); "
                         "0: 4 for C2-like configs, 2 for a strong-scaling stream (one call of many chunks, "
                         "pipelined inside the engine)")
    ap.add_argument("--one-stream", default="auto", choices=["auto", "0", "1"],
                    help="engines of the timed steps keep to one stream (no decode side stream); "
                         "auto: when 3 or more batches are in flight")
    ap.add_argument("--allow-shared-device", action="store_true",
                    help="let ranks share a GPU (one-GPU rehearsal of --gpus N; n_gpus then counts devices)")
    args = ap.parse_args()
    # read by the HIP runtime when it starts (the first HIP call, below):
    # the latency-mode slots each get a hardware queue instead of pairing up
    # on HIP's default 4 (a batch on a shared queue waits for the one ahead)
    if args.hw_queues and int(os.environ.get("GPU_MAX_HW_QUEUES") or 0) < args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))
    # kernel arguments in host memory, as the verify service runs (unless
    # the environment says otherwise): the in-process tile's five launches
    # per batch take ~7 us instead of ~15 us; C2's few launches per 1M
    # signatures do not notice (profiles/r6_c5_launch_bump.txt)
    if not args.dev_kernargs:
        os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "0")

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)
    rank, local, world = dist_setup(args.gpus)
    from firedancer_amd import ed25519, workload

    cfg = dict(workload.CONFIGS[args.config])
    n = args.n or cfg["n"]
    strong = bool(cfg.get("total"))
    if args.seed is None:
        args.seed = C4_STREAM_SEED if strong else 0x5EED
    if strong:  # cfg n is the whole stream: this rank verifies its contiguous share
        n = (n + world - 1) // world
    # setup under a guard on every rank, then one agreement (an all-gather
    # of each rank's outcome and device) before anything else: a rank that
    # fails here never leaves the others waiting in a later collective
    st = {}

    def setup():
        ndev = int(os.environ.get("FD_BENCH_FAKE_DEVICE_COUNT", ed25519.device_count()))   # test hook (CPU tests)
        if local >= ndev and not args.allow_shared_device:
            raise RuntimeError(f"local rank {local} but only {ndev} visible GPU(s)")
        st["device"] = local % max(ndev, 1)
        st["eng"] = ed25519.Engine(device=st["device"], max_chunk=min(n, 1 << 20), half=args.half)
        st["info"] = st["eng"].info()
        log(f"[rank {rank}] engine {st['info']}")
        t = time.perf_counter()
        st["wl"] = ed25519.DeviceWorkload(st["eng"], n, cfg["lo"], cfg["hi"], cfg["ppm"], seed=args.seed,
                                          index_base=rank * n)
        st["gen_s"] = time.perf_counter() - t
        log(f"[rank {rank}] generated {n} signatures ({st['wl'].msg_bytes / 1e6:.1f} MB of messages) "
            f"in {st['gen_s']:.2f} s")
        i = st["info"]
        return f"{i['pci_domain']:04x}:{i['pci_bus']:02x}:{i['pci_device']:02x}"
    try:
        mine = ("ok", setup())
    except Exception as ex:   # agreed on below, by every rank
        mine = ("failed", f"{ex}")
        log(f"[rank {rank}] {ex}")
    if os.environ.get("FD_BENCH_DIE_RANK") == str(rank):   # test hook: a rank lost before the agreement
        os._exit(3)
    outcome = all_gather(mine, world)
    bad = [(r, m) for r, (k, m) in enumerate(outcome) if k != "ok"]
    if bad:
        if rank == 0 or mine[0] != "ok":
            log(f"[rank {rank}] setup failed on rank(s) {[r for r, _ in bad]}: {bad}")
        return 2
    devices = [m for _, m in outcome]
    n_dev = len(set(devices))
    if n_dev != world and not args.allow_shared_device:
        log(f"[rank {rank}] ranks share devices: {devices}")
        return 2
    device, eng, info, wl, gen_s = st["device"], st["eng"], st["info"], st["wl"], st["gen_s"]

    inflight = args.inflight or (2 if strong else 4)
    one_stream = inflight >= 3 if args.one_stream == "auto" else args.one_stream == "1"
    hf_first = None
    # (round 2 ran the host-fed leg first: its rate depended on where the
    # pool's slot streams landed on the hardware queues.  The cause was two
    # batches crossing PCIe at once, which moves fewer bytes than one; the
    # pool now lets one batch's H2D run at a time (its kernels overlap the
    # next copy), at the same rate wherever the streams land, so the leg runs
    # last again; --host-first remains for the A/B)
    if args.host_first and args.host_reps > 0:   # the host-fed leg before the engine's timed passes
        try:
            hf_first = host_fed(wl, device, info, world, args.host_reps, args.host_batch, args.host_slots,
                                args.host_copies)
        except Exception as ex:  # the same on every rank (host_fed agrees first); never fatal
            log(f"[rank {rank}] host-fed leg failed: {ex!r}")
    # batches in flight: consecutive steps alternate between `inflight`
    # engines (each its own streams, work arrays and lane tables; the base
    # tables are shared), so a step's hash/scalar/decode run beside the
    # previous step's dsm and fill its tail -- the last waves of a
    # persistent kernel whose items last ~1 ms -- as the pool's and the
    # verify tile's slots do.  Every step still verifies all n signatures.
    # With 3+ in flight the batches overlap one another enough that each
    # engine keeps to one stream (FD_ED25519_HIP_FLAG_ONE_STREAM, as the
    # pool's slots do): 4 one-stream engines measured 107.7-108.7M/s against
    # 104.9-105.5M/s for 2 engines with the decode side stream
    # (profiles/r2_inflight_streams_ab.txt; extra streams share the process's
    # 4 hardware queues).  With 8 queues (--hw-queues), 4 / 6 / 8 one-stream
    # engines measured 100.4 / 98.0 / 100.6M/s on one box: 4 stays
    # (profiles/r4h_inflight_ab_hwq8.jsonl).
    if one_stream:
        engines = [ed25519.Engine(device=device, max_chunk=min(n, 1 << 20), half=args.half, one_stream=True)
                   for _ in range(inflight)]
        outs = [e.alloc(n) for e in engines]
    else:
        engines = [eng] + [ed25519.Engine(device=device, max_chunk=min(n, 1 << 20), half=args.half)
                           for _ in range(inflight - 1)]
        outs = [wl.out] + [e.alloc(n) for e in engines[1:]]

    def step(s):
        e, o = engines[s % len(engines)], outs[s % len(engines)]
        e.verify_dev(n, wl.msgs.ptr, wl.off.ptr, wl.sz.ptr, wl.sigs.ptr, wl.pubs.ptr, o.ptr, e.stream)

    def sync_all():
        for e in engines:
            e.sync()
    for s in range(args.warmup):
        step(s)
    sync_all()

    barrier(world)
    sync_all()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(s)
    sync_all()
    t1 = time.perf_counter()
    barrier(world)
    elapsed = allreduce_max(t1 - t0, world)
    mism_inflight = 0
    used = {s % len(engines) for s in range(max(args.warmup, args.steps))}   # K or W below the depth: some idle
    for i, o in enumerate(outs):
        if o is wl.out:
            continue
        if i in used:
            mism_inflight += int((o.download(np.int8, n) != wl.expect.download(np.int8, n)).sum())
        o.free()
    for e in engines:
        if e is not eng:
            e.close()
    # per-kernel durations: a separate pass of the same steps with HIP events
    # around each phase on the engine stream (the phases then run in sequence;
    # in the timed region above a chunk's decode overlaps its hash + scalar,
    # dsm runs alone either way)
    eng.timing(True)
    for _ in range(args.steps):
        wl.verify()
    eng.sync()
    phase_ms, launches = eng.timing_read()
    eng.timing(False)

    # full-size verdict check: every code equals the class label's reference code
    out = wl.out.download(np.int8, n)
    expect = wl.expect.download(np.int8, n)
    mism = int((out != expect).sum()) + mism_inflight
    mism_all = int(allreduce_sum(mism, world))
    if mism:
        log(f"[rank {rank}] VERDICT MISMATCH on {mism} of {n} signatures")

    total = world * n * args.steps
    value = total / elapsed
    ms_step = elapsed * 1e3 / args.steps

    # roofline (dsm = dominant kernel)
    ops = workload.ops_per_verify(wl.sizes)
    clock = eng.clock_mhz() * 1e6
    peak = clock * info["cu_cnt"] * 64 * 2 / 1e12
    per_launch = {k: v / max(launches, 1) for k, v in phase_ms.items()}
    # a launch is one chunk of at most max_chunk signatures: ops per launch
    # are the step's ops over its chunk count
    chunks = -(-n // info["max_chunk"])
    dsm_ops = float(ops["dsm"].sum()) / chunks
    achieved = dsm_ops / (per_launch["dsm"] * 1e-3) / 1e12 if per_launch["dsm"] > 0 else None
    path_ms = sum(per_launch.values())
    path_ops = float(ops["total"].sum()) / chunks
    path_achieved = path_ops / (path_ms * 1e-3) / 1e12 if path_ms > 0 else None

    cpu = c1 = c3 = None
    if rank == 0 and not args.no_cpu_baseline:
        # the reference CPU path on the host's cores in the same run, N=1 and
        # N>1 alike (the other ranks wait at the barrier below)
        try:
            cpu = cpu_baseline(wl, out, args.cpu_sample, args.cpu_reps)
        except Exception as ex:  # reported, never fatal for the GPU number
            log(f"cpu baseline failed: {ex!r}")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not strong:
        try:
            c1 = config_c1(eng, args, inflight)
        except Exception as ex:  # reported, never fatal for the GPU number
            log(f"C1 leg failed: {ex!r}")
        try:
            c3 = config_c3(eng, args, inflight)
        except Exception as ex:  # reported, never fatal for the GPU number
            log(f"C3 leg failed: {ex!r}")
            c3 = {"error": repr(ex)}
    barrier(world)
    hf = hf_first
    if args.host_reps > 0 and hf is None:
        try:
            if strong:   # C4: the rank's shard streamed from bounded host windows
                hf = c4_host_fed(eng, device, info, rank, world, n, rank * n, cfg, args.seed, args.host_window,
                                 args.host_batch, args.host_slots)
            else:
                hf = host_fed(wl, device, info, world, args.host_reps, args.host_batch, args.host_slots,
                              args.host_copies)
        except Exception as ex:  # reported, never fatal for the device-resident number
            log(f"[rank {rank}] host-fed leg failed: {ex!r}")
    c4 = None
    if not strong and args.c4_signatures > 0:
        try:
            c4 = config_c4(eng, device, info, rank, world, args)
        except Exception as ex:  # the same on every rank (the stream agrees on every stage); never fatal
            log(f"[rank {rank}] C4 stream leg failed: {ex!r}")
            c4 = {"error": repr(ex)}
    lat = None
    if rank == 0 and world == 1 and args.latency_txns > 0 and not strong:
        try:
            lat = latency_mode(eng, args, device)
        except Exception as ex:  # reported, never fatal for the device-resident number
            log(f"latency mode failed: {ex!r}")
            lat = {"error": repr(ex)}
    lat_dep = None
    if rank == 0 and world == 1 and args.deployed_txns > 0 and not strong:
        try:
            lat_dep = latency_deployed(eng, args)
        except Exception as ex:  # reported, never fatal for the device-resident number
            log(f"deployed latency leg failed: {ex!r}")
            lat_dep = {"error": repr(ex)}
    traffic, traffic_src = pmc_traffic(min(n, info["max_chunk"]))
    # executed (not algorithmic) instruction rate of the dsm kernel: the
    # half-size formulation executes fewer operations than the reference's
    # algorithm counted above, so both are reported
    valu = pmc_valu_per_sig()
    sig_launch = min(n, info["max_chunk"])
    executed = (valu * sig_launch / (per_launch["dsm"] * 1e-3) / 1e12) if valu and per_launch["dsm"] > 0 else None

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "verifies/s",
            "n_gpus": n_dev,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: seeded keys/messages generated and signed on the GPU (fd_ed25519_hip_gen_dev), "
                    "2% corrupted by class (fd_ed25519_hip_corrupt_dev)",
            "config": {"workload": f"{args.config}: {n} signatures per GPU"
                                   + (f" ({world * n} in the stream)" if strong else "")
                                   + f", message size uniform [{cfg['lo']},{cfg['hi']}] B, {cfg['ppm'] / 1e4:.1f}% invalid",
                       "signatures_per_gpu": n, "parallelism": f"shard x{world} (independent batches, no collective)",
                       "devices": devices,
                       "batches_in_flight": inflight,
                       "engine_streams": "one per engine" if one_stream else "two per engine (decode side stream)",
                       "codes": "reference AVX-512 backend"},
            "roofline": {"bound": "valu-int32", "kernel": "fd_ed25519_dsm_kernel",
                         "achieved": achieved, "peak": peak, "unit": "TOPS",
                         "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                         "traffic_unit": "bytes per launch (HBM read+write: rocprofv3 2 x FETCH_SIZE (gfx950 16-B/lane "
                                         "correction) + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "ops_per_launch": dsm_ops, "launch_ms": per_launch["dsm"],
                         "executed": {"achieved": executed, "frac": (executed / peak) if executed else None,
                                      "unit": "TOPS (INT32+INT64 VALU lane-instructions / s)",
                                      "valu_per_signature": valu, "source": traffic_src,
                                      "cycles_per_valu_instruction_per_simd": pmc_issue_rate(info["cu_cnt"]),
                                      "issue_note": "the peak assumes a wave64 instruction every 2 cycles per SIMD; "
                                                    "measured issue costs are 2.5 (VOP2), 4.2-4.4 (VOP3), 5.2 "
                                                    "(32x32->64 mad, 68% of dsm's instructions): DESIGN.md 2.4"},
                         "path": {"achieved": path_achieved, "frac": (path_achieved / peak) if path_achieved else None,
                                  "ops_per_verify_mean": path_ops * chunks / n, "ms_per_launch": path_ms},
                         "signatures_per_launch": min(n, info["max_chunk"])},
            "kernel_ms_per_launch": per_launch,
            "kernel_timing": "HIP events around each phase on the engine stream, in a separate pass of the same "
                             "steps on one engine (phases in sequence); in the timed region consecutive steps "
                             "alternate between config.batches_in_flight engines (config.engine_streams), so "
                             "a step's phases run beside the other steps' dsm",
            "cpu_baseline": cpu,
            "gpu_over_cpu": (value / cpu["value"]) if cpu else None,
            "gpu_over_cpu_scope": "per lease: these GPUs against the host cores this job may use (cpu_baseline.cores)",
            "gpu_over_box_cpu": (value / cpu["box_projection"]["verifies_per_s"])
            if cpu and cpu["box_projection"]["verifies_per_s"] else None,
            "gpu_over_box_cpu_scope": "these GPUs against cpu_baseline.box_projection (every physical core of the "
                                      "machine, projected from the measured per-core rate)",
            "host_fed": hf,
            "config_c4": c4,
            "latency_mode": lat,
            "latency_mode_deployed": lat_dep,
            "config_c1": c1,
            "config_c3": c3,
            "verdicts_match_reference_labels": mism_all == 0,
            "verdict_mismatches": mism_all,
            "invalid_fraction": float((expect != 0).mean()),
            "gen_seconds": gen_s,
        }
        print(json.dumps(line), flush=True)
    wl.free()
    eng.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if mism_all == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
