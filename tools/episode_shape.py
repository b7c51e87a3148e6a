#!/usr/bin/env python3
"""Shape of the deployed leg's latency episodes: reads the per-frag
latencies bench.py keeps with FD_BENCH_LAT_DIR=DIR (one .npy per harness
run, samples in the order the consumer received the frags, named
KIND_RATE_APP.npy) and, for every run whose max exceeds --slow-ms, prints
where the episode starts (frag index and its due time, index / rate), how
many frags it covers, its peak, and the rise / fall rates: a pause of the
path shows as latency rising by 1 / rate per frag (frags keep arriving,
none is served) up to the pause's length, then falling at the path's
surplus rate while the backlog drains.

    python tools/episode_shape.py DIR [--slow-ms 1.0] [--windows OUT.npz] [--delete]

--windows keeps each slow run's samples around its episode (the box's
gpurun_out/ is copied back only under 64 MiB); --delete removes DIR's
files afterwards.
"""
import argparse
import glob
import json
import os

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--slow-ms", type=float, default=1.0)
    ap.add_argument("--windows", default=None)
    ap.add_argument("--delete", action="store_true")
    args = ap.parse_args()
    windows = {}
    files = sorted(glob.glob(os.path.join(args.dir, "*.npy")))
    n_slow = 0
    for f in files:
        kind, rate, _ = os.path.basename(f)[:-4].rsplit("_", 2)
        rate = float(rate)
        ms = np.load(f).astype(np.float64)
        if not ms.size or ms.max() <= args.slow_ms:
            continue
        n_slow += 1
        slow = np.nonzero(ms > args.slow_ms)[0]
        a, b = int(slow[0]), int(slow[-1])
        pk = int(np.argmax(ms))
        base = float(np.median(ms))
        lo, hi = max(0, a - 2000), min(ms.size, b + 2000)
        windows[os.path.basename(f)[:-4]] = np.stack([np.arange(lo, hi, dtype=np.float64), ms[lo:hi]]).astype(np.float32)
        rise = (ms[pk] - ms[a]) / max(pk - a, 1)   # ms per frag
        fall = (ms[pk] - ms[b]) / max(b - pk, 1)
        print(json.dumps({
            "run": os.path.basename(f), "kind": kind, "rate": rate, "frags": int(ms.size),
            "p50_ms": round(base, 4), "max_ms": round(float(ms.max()), 3),
            "episode_first_last": [a, b], "episode_frags": b - a + 1,
            "episode_start_s": round(a / rate, 4) if rate > 0 else None,
            "peak_at": pk, "rise_ms_per_frag": rise, "rise_if_paused_ms_per_frag": (1e3 / rate) if rate > 0 else None,
            "fall_ms_per_frag": fall,
            "pause_estimate_ms": round(float(ms[pk] - base), 3),
            "slow_runs_of_separate_episodes": int(np.sum(np.diff(slow) > 1000) + 1)}))
    print(json.dumps({"runs": len(files), "runs_with_episode": n_slow, "slow_ms": args.slow_ms}))
    if args.windows and windows:
        np.savez_compressed(args.windows, **windows)
    if args.delete:
        for f in files:
            os.unlink(f)


if __name__ == "__main__":
    main()
