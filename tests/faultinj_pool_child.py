"""Child process of tests/test_gpu_pool_fault.py: runs with
FD_ED25519_HIP_LIB pointing at the fault-injection build
(libfd_ed25519_hip_faultinj.so, -DFD_ED25519_HIP_HOST_FAULT=1), whose pool
fails the second batch's launch after that batch's copies from the
caller's arrays are on the stream.  For registered (direct DMA) and
unregistered (staged) inputs: the run must report the injected error, the
first batch's verdicts must have landed, the pool must run a one-batch job
afterwards, and unregistering the arrays then deleting the pool must not
hang.  Prints one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from firedancer_amd import ed25519, tile
    assert os.path.basename(ed25519.LIB_PATH) == "libfd_ed25519_hip_faultinj.so", ed25519.LIB_PATH
    batch, nb, m = 1024, 5, 120
    n = batch * nb
    eng = ed25519.Engine(0, max_chunk=n)
    wl = ed25519.DeviceWorkload(eng, n, m, m, 0, seed=91)
    msgs = wl.msgs.download(np.uint8, wl.msg_bytes)
    off = wl.off.download(np.uint64, n)
    sz = np.full(n, m, np.uint32)
    sigs = wl.sigs.download(np.uint8, 64 * n)
    pubs = wl.pubs.download(np.uint8, 32 * n)
    wl.free()
    eng.close()
    res = {}
    for mode in ("direct", "staged"):
        pool = tile.Pool([0], batch, 3, msg_cap=batch * m + 64)
        out = np.full(n, 77, np.int8)
        reg = tile.HostRegistration(msgs, off, sz, sigs, pubs, out) if mode == "direct" else None
        if reg:
            reg.__enter__()
        err = None
        st = {}
        try:
            _, _, st = pool.run(msgs, off, sz, sigs, pubs, out)
        except ed25519.HipError as e:
            err = str(e)
        first_ok = bool((out[:batch] == 0).all())
        again = np.full(batch, 77, np.int8)
        codes, _, _ = pool.run(msgs, off[:batch], sz[:batch], sigs[:64 * batch], pubs[:32 * batch], again)
        if reg:
            reg.__exit__(None, None, None)
        pool.close()
        res[mode] = {"error": err, "first_batch_ok": first_ok, "rerun_ok": bool((codes == 0).all()),
                     "stats": {k: int(v) for k, v in st.items()}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
