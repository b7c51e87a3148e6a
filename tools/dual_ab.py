#!/usr/bin/env python3
"""A/B of an engine launch option read from the environment at engine
creation (default FD_ED25519_HIP_DUAL: dual-stream chunking; also
FD_ED25519_HIP_OVERLAP: decode beside hash + scalar) on the C2 workload:
alternating engines with the option off / on, same signatures, whole-step
wall time over K steps (no per-phase events), verdicts checked.

    python tools/dual_ab.py [N] [STEPS] [ENVVAR]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, workload  # noqa: E402


def run(dual, n, steps, cfg, var):
    os.environ[var] = "1" if dual else "0"
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    var = sys.argv[3] if len(sys.argv) > 3 else "FD_ED25519_HIP_DUAL"
    cfg = dict(workload.CONFIGS["C2"])
    for rep in range(3):
        for dual in (0, 1):
            v, ok = run(dual, n, steps, cfg, var)
            print(f"n={n} {var}={dual} rep={rep}: {v / 1e6:.2f}M verifies/s verdicts_ok={ok}", flush=True)
