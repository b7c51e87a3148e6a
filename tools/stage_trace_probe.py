#!/usr/bin/env python3
"""Where C5's slow frags spend their time: the in-process
latency mode (tango-style ring -> verify tile -> pipe slots) at one offered
load, with the stage-trace build of the library
(tools/build_variant.sh stagetrace "" -DFD_ED25519_HIP_AB_STAGE_TRACE=1),
which stamps every frag (due, published, pulled, its batch) and every batch
(submit entered, last launch enqueued, seen done, resolved, slots in flight
when it went out).  A frag's latency splits into

    producer   published - due          (the producer thread late)
    ring       pulled - published       (the tile not pulling)
    batching   batch submit - pulled    (waiting for its batch to go out)
    launch     enqueued - submit        (host time in the launches)
    gpu        done seen - enqueued     (GPU round trip + poll delay)
    resolve    resolved - done seen
    deliver    verdict - resolved

and the tool prints, for the frags above --slow-ms and for the rest, the
mean of each part, the slow clusters (runs of consecutive slow frags) with
the stage that grew, and the batches around each cluster.

    python tools/stage_trace_probe.py [--rate 4e6 | --frac 0.95] [--runs 5] [--txns 300000] [--out gpurun_out/stage]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

PARTS = ("producer", "ring", "batching", "launch", "gpu", "resolve", "deliver")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=0.0, help="offered txn/s (0: --frac of the unpaced median)")
    ap.add_argument("--frac", type=float, default=0.95)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--txns", type=int, default=300000)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--slow-ms", type=float, default=0.45)
    ap.add_argument("--pin", action="store_true", help="producer and tile on two physical cores of the GPU's node")
    ap.add_argument("--lib", default=os.path.join(REPO, "build", "variants", "stagetrace", "libfd_ed25519_hip.so"))
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "stage"))
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(args.slots))
    os.environ["FD_ED25519_HIP_LIB"] = args.lib
    from firedancer_amd import ed25519, tile, workload
    lib = ed25519.library()
    lib.fd_ed25519_hip_stage_trace_frags.argtypes = [ctypes.c_void_p] * 4
    lib.fd_ed25519_hip_stage_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int]
    lib.fd_ed25519_hip_stage_trace_read.restype = ctypes.c_ulong
    os.makedirs(args.out, exist_ok=True)
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    if args.pin:
        cores = tile.physical_cores(tile.device_cpus(eng.info()))
        tile.latency_set_cpus(cores[0], cores[1])
        print("pinned producer / tile to CPUs", cores[:2], flush=True)
    n = args.txns
    pay, _ = workload.txn_payloads(eng, n, 4242, msg_sz=200)
    eng.close()

    def run(rate, keep=True):
        # np.full, not np.zeros: zeros come from untouched pages, and the
        # first touch inside the run (a huge page zeroed) stalled the thread
        # that stamps them
        due, pub, pull = (np.full(n, -1.0) for _ in range(3))
        bat = np.full(n, 0, np.uint64)
        lib.fd_ed25519_hip_stage_trace_frags(due.ctypes.data, pub.ctypes.data, pull.ctypes.data, bat.ctypes.data)
        buf = np.zeros((1 << 18, 8))
        lib.fd_ed25519_hip_stage_trace_read(buf.ctypes.data, 0, 1)   # reset
        lat, v, res = tile.latency_run(pay, rate, slot_cnt=args.slots, batch_sigs=args.batch, ring_depth=4096)
        nb = lib.fd_ed25519_hip_stage_trace_read(buf.ctypes.data, 1 << 18, 1)
        lib.fd_ed25519_hip_stage_trace_frags(None, None, None, None)
        assert (v == 0).all()
        return dict(lat=lat, due=due, pub=pub, pull=pull, bat=bat, batches=buf[:nb].copy(), res=res)

    for _ in range(2):
        run(0.0)   # warm-up
    rate = args.rate
    if rate <= 0:
        peaks = [run(0.0)["res"]["achieved_txn_per_s"] for _ in range(3)]
        rate = args.frac * float(np.median(peaks))
        print(f"unpaced peaks {[round(p / 1e6, 3) for p in peaks]} M -> offered {rate / 1e6:.3f} M", flush=True)
    summary = {"offered_txn_per_s": rate, "pinned": args.pin, "runs": []}
    for k in range(args.runs):
        r = run(rate)
        b = r["batches"]   # t_submit, t_enq, t_done, t_resolved, seq, sig_cnt, txn_cnt, in_flight
        seq = b[:, 4].astype(np.int64)
        by_seq = np.full(int(seq.max()) + 1, -1, np.int64)
        by_seq[seq] = np.arange(len(b))
        idx = by_seq[r["bat"].astype(np.int64)]
        ok = idx >= 0
        bb = b[idx]
        t_verdict = r["due"] + r["lat"]
        parts = np.stack([r["pub"] - r["due"], r["pull"] - r["pub"], bb[:, 0] - r["pull"], bb[:, 1] - bb[:, 0],
                          bb[:, 2] - bb[:, 1], bb[:, 3] - bb[:, 2], t_verdict - bb[:, 3]], 1) * 1e3
        ms = r["lat"] * 1e3
        slow = (ms > args.slow_ms) & ok
        rec = {"achieved_txn_per_s": r["res"]["achieved_txn_per_s"], "p50_ms": float(np.percentile(ms, 50)),
               "p99_ms": float(np.percentile(ms, 99)), "max_ms": float(ms.max()), "slow_frags": int(slow.sum()),
               "batches": int(len(b)), "mean_batch_txns": float(b[:, 6].mean()),
               "in_flight_at_submit_hist": np.bincount(b[:, 7].astype(int), minlength=9).tolist(),
               "tile_ns_per_frag_p50": float(np.median(np.diff(r["pull"])) * 1e9),
               "parts_ms_typical": dict(zip(PARTS, np.round(parts[~slow & ok].mean(0), 4).tolist())),
               "parts_ms_slow": dict(zip(PARTS, np.round(parts[slow].mean(0), 4).tolist())) if slow.any() else None,
               "gpu_ms_batches_p50_p99_max": np.round(np.percentile((b[:, 2] - b[:, 1]) * 1e3, [50, 99, 100]), 4).tolist(),
               "launch_ms_batches_p50_p99_max": np.round(np.percentile((b[:, 1] - b[:, 0]) * 1e3, [50, 99, 100]),
                                                         4).tolist(),
               "clusters": []}
        # clusters: runs of slow frags (gaps of < 50 frags merge)
        si = np.nonzero(slow)[0]
        if len(si):
            cuts = np.nonzero(np.diff(si) > 50)[0]
            starts, ends = np.r_[si[0], si[cuts + 1]], np.r_[si[cuts], si[-1]]
            t0 = r["due"][0]
            for a, e in zip(starts, ends):
                sel = np.arange(a, e + 1)
                sel = sel[slow[sel]]
                pm = parts[sel].mean(0)
                # the batches of this cluster: their GPU and launch times, in-flight counts
                bs = np.unique(r["bat"][sel].astype(np.int64))
                bi = by_seq[bs]
                bi = bi[bi >= 0]
                rec["clusters"].append({
                    "frags": [int(a), int(e)], "t_ms": round(float((r["due"][a] - t0) * 1e3), 3),
                    "max_ms": round(float(ms[a:e + 1].max()), 3), "parts_ms": dict(zip(PARTS, np.round(pm, 4).tolist())),
                    "grew": PARTS[int(np.argmax(pm - parts[~slow & ok].mean(0)))],
                    "batch_gpu_ms_max": round(float(((b[bi, 2] - b[bi, 1]) * 1e3).max()), 4) if len(bi) else None,
                    "batch_launch_ms_max": round(float(((b[bi, 1] - b[bi, 0]) * 1e3).max()), 4) if len(bi) else None,
                    "in_flight_max": int(b[bi, 7].max()) if len(bi) else None})
        summary["runs"].append(rec)
        np.savez_compressed(os.path.join(args.out, f"run{k}.npz"), lat=r["lat"], due=r["due"], pub=r["pub"],
                            pull=r["pull"], bat=r["bat"], batches=b)
        print(json.dumps(rec), flush=True)
    json.dump(summary, open(os.path.join(args.out, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
