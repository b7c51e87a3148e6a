#!/usr/bin/env python3
"""GPU round trip of one pipe batch (fd_ed25519_hip_pipe_submit -> poll),
from the slot's own t_submit / t_done: one batch in flight at a time, then
slot_cnt in flight back to back -- what a verify tile's (or the GPU
service's) batches of --batch single-signer signatures see.

    python tools/pipe_latency_probe.py [--batch 4096] [--slots 3] [--reps 50] [--split 2|4|8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, tile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--msg-sz", type=int, default=200)
    ap.add_argument("--split", type=int, default=None, help="fd_ed25519_hip_pipe_set_split_waves (A/B: 2, 4, 8)")
    args = ap.parse_args()
    if args.split is not None:
        tile.pipe_set_split_waves(args.split)
    n, m = args.batch, args.msg_sz
    eng = ed25519.Engine(0, max_chunk=max(n, 4096))
    wl = ed25519.DeviceWorkload(eng, n, m, m, 0, seed=77)
    msgs = wl.msgs.download(np.uint8, wl.msg_bytes)
    off = wl.off.download(np.uint64, n)
    sigs = wl.sigs.download(np.uint8, 64 * n)
    pubs = wl.pubs.download(np.uint8, 32 * n)
    wl.free()
    eng.close()
    pipe = tile.Pipe(0, args.slots, sig_cap=n, msg_cap=n * m + 64, txn_cap=n)

    def stage(s):
        a = tile.Pipe.arrays(s)
        a["msgs"][:len(msgs)] = msgs
        a["msg_off"][:n] = off
        a["msg_sz"][:n] = m
        a["sigs"][:64 * n] = sigs
        a["pubs"][:32 * n] = pubs
        return s

    res = {}
    for depth in (1, args.slots):
        rt, t0 = [], time.perf_counter()
        done = 0
        inflight = 0
        while done < args.reps:
            while inflight < depth:
                s = pipe.acquire()
                if s is None:
                    break
                stage(s)
                assert pipe.submit(s, n, len(msgs), 0) == 0
                inflight += 1
            s = pipe.poll(True)
            c = s.contents
            rt.append((c.t_done - c.t_submit) * 1e3)
            assert (np.ctypeslib.as_array(c.sig_out, (n,)) == 0).all()
            pipe.release(s)
            inflight -= 1
            done += 1
        while inflight:
            pipe.release(pipe.poll(True))
            inflight -= 1
        dt = time.perf_counter() - t0
        res[f"in_flight_{depth}"] = {"round_trip_ms_p50": float(np.percentile(rt, 50)),
                                     "round_trip_ms_p90": float(np.percentile(rt, 90)),
                                     "verifies_per_s": args.reps * n / dt}
    pipe.close()
    print(json.dumps({"batch": n, "slots": args.slots, "msg_sz": m, "split_waves": args.split, **res}))


if __name__ == "__main__":
    main()
