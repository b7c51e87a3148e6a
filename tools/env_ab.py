#!/usr/bin/env python3
"""A/B of engine launch options read from the environment at engine creation,
on the C2 workload: for each spec (comma-separated VAR=VAL, "-" for the
defaults) a fresh engine verifies the same signatures; whole-step wall time
over K steps (no per-phase events), verdicts checked; specs interleaved.

    python tools/env_ab.py N STEPS REPS SPEC...
    e.g. python tools/env_ab.py 1048576 20 3 - FD_ED25519_HIP_OVERLAP=0
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, workload  # noqa: E402

VARS = ("FD_ED25519_HIP_OVERLAP", "FD_ED25519_HIP_QUAD_MAX", "FD_ED25519_HIP_OCT_MAX")


def run(spec, n, steps, cfg):
    for v in VARS:
        os.environ.pop(v, None)
    if spec != "-":
        for kv in spec.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    eng = ed25519.Engine(device=0, max_chunk=min(n, 1 << 20))
    wl = ed25519.DeviceWorkload(eng, n, cfg["lo"], cfg["hi"], cfg["ppm"], seed=0x5EED, index_base=0)
    for _ in range(2):
        wl.verify()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        wl.verify()
    eng.sync()
    dt = time.perf_counter() - t0
    ok = bool((wl.out.download(np.int8, n) == wl.expect.download(np.int8, n)).all())
    wl.free()
    eng.close()
    return n * steps / dt, ok


if __name__ == "__main__":
    n, steps, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    cfg = dict(workload.CONFIGS["C2"])
    for rep in range(reps):
        for spec in sys.argv[4:]:
            v, ok = run(spec, n, steps, cfg)
            print(f"{spec:60s} rep={rep}: {v / 1e6:.2f}M verifies/s verdicts_ok={ok}", flush=True)
