"""C4's host-fed leg on CPU (bench.host_stream with the generator and the
pool replaced by fakes): each rank streams its shard from bounded host
windows, the verdicts and the concatenated stream digest do not depend on
the window size or on how the stream is split over ranks, and a failure
on one rank at any stage fails every rank without leaving one in a
collective (gloo, world size 2 at 127.0.0.1)."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, REPO)

TOTAL = 6000
SEED = 0xC4C4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _code(g):
    return np.where(g % 7 == 3, -1, np.where(g % 11 == 5, -3, 0)).astype(np.int8)


def _fakes(index_base, fail=None):
    """fill: signature g's first 8 bytes hold g, byte 8 its code, its
    message is `size` bytes of (7g + 1) mod 256.  pool_run: recomputes each
    code from the window exactly as laid out (a message read at the wrong
    offset or size gives 99)."""
    from firedancer_amd import workload
    calls = {"fill": 0, "run": 0}

    def fill(i0, m, msgs, sigs, pubs):
        calls["fill"] += 1
        if fail == ("fill", calls["fill"]):
            raise OSError("generator failed (injected)")
        g = np.arange(index_base + i0, index_base + i0 + m, dtype=np.uint64)
        sz = workload.msg_sizes(SEED, index_base + i0, m, 1, 40)
        assert msgs.nbytes == int(sz.sum())
        msgs[:] = np.repeat(((g * np.uint64(7) + np.uint64(1)) % np.uint64(256)).astype(np.uint8), sz)
        s = sigs.reshape(m, 64)
        s[:, :8] = g.view(np.uint8).reshape(m, 8)
        s[:, 8] = _code(g).view(np.uint8)
        pubs[:] = 0
        return _code(g)

    def pool_run(msgs, off, sz, sigs, pubs, out):
        calls["run"] += 1
        if fail == ("run", calls["run"]):
            raise OSError("pool failed (injected)")
        s = sigs.reshape(-1, 64)
        for i in range(len(out)):
            g = int(s[i, :8].view(np.uint64)[0])
            want_sz = int(workload.msg_sizes(SEED, g, 1, 1, 40)[0])
            m = msgs[int(off[i]):int(off[i]) + int(sz[i])]
            ok = int(sz[i]) == want_sz and bool((m == (7 * g + 1) % 256).all())
            out[i] = s[i, 8].view(np.int8) if ok else 99
        return 0.001 * len(out) / 1000.0
    return fill, pool_run, calls


def _run(rank, world, window, fail=None):
    import bench
    from firedancer_amd import workload
    n = TOTAL // world
    base = rank * n
    sizes = workload.msg_sizes(SEED, base, n, 1, 40)
    fill, pool_run, calls = _fakes(base, fail)
    res, codes = bench.host_stream(n, sizes, window, 500, fill, pool_run, world)
    return res, codes, calls


def test_single_rank_windows_bound_host_memory_and_keep_the_stream():
    """One rank, windows of 700 / 2000 / the whole shard: the same codes and
    digest every time, every code equal to its label, and the host holds one
    window (its bytes grow with the window, not with the stream)."""
    seen = {}
    for window in (700, 2000, TOTAL):
        res, codes, calls = _run(0, 1, window)
        assert res["label_mismatches"] == 0
        assert np.array_equal(codes, _code(np.arange(TOTAL, dtype=np.uint64)))
        assert res["windows"] == -(-TOTAL // window) == calls["run"] - 1   # + the warm-up pass
        assert len(res["window_seconds_max_over_ranks"]) == res["windows"]
        seen[window] = res
    assert len({r["rank_digest"] for r in seen.values()}) == 1
    assert seen[700]["rank_digest"] == hashlib.sha256(_code(np.arange(TOTAL, dtype=np.uint64)).tobytes()).hexdigest()
    # a window of 700 signatures of <= 40-byte messages: about 700 x (40 + 109) bytes, far below the stream's
    assert seen[700]["host_window_bytes"] < 700 * (40 + 64 + 32 + 8 + 4 + 1) + 64
    assert seen[700]["host_window_bytes"] * 5 < seen[TOTAL]["host_window_bytes"]


def _worker(rank, world, port, q, window, fail_rank, fail):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    r, _, w = bench.dist_setup(world)
    try:
        res, codes, _ = _run(r, w, window, fail if r == fail_rank else None)
        everything = bench.all_gather(codes.tobytes(), w)
        outcome = ("ok", res["windows"], res["label_mismatches"], hashlib.sha256(b"".join(everything)).hexdigest(),
                   res["host_window_bytes"])
    except RuntimeError as ex:
        outcome = ("raised", str(ex)[:50])
    bench.barrier(w)   # both ranks reach this: none was left in a collective
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put((r, outcome))


def _world2(window, fail_rank=-1, fail=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, window, fail_rank, fail)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [o for _, o in res]


def test_two_ranks_stream_their_shards_and_agree():
    """World 2: each rank streams its contiguous half in windows of 800;
    both see every code equal to its label and the concatenated digest
    equals the one-rank stream's."""
    whole = hashlib.sha256(_code(np.arange(TOTAL, dtype=np.uint64)).tobytes()).hexdigest()
    out = _world2(800)
    assert [o[0] for o in out] == ["ok", "ok"], out
    assert all(o[1] == -(-(TOTAL // 2) // 800) and o[2] == 0 for o in out)
    assert out[0][3] == out[1][3] == whole
    assert all(o[4] < 800 * (40 + 64 + 32 + 8 + 4 + 1) + 64 for o in out)   # one window each


@pytest.mark.parametrize("fail_rank,fail", [(1, ("fill", 3)), (0, ("run", 2)), (1, ("run", 1))],
                         ids=["rank1-refill", "rank0-stream", "rank1-first-window"])
def test_a_failure_on_one_rank_fails_both(fail_rank, fail):
    out = _world2(800, fail_rank, fail)
    assert all(o[0] == "raised" and o[1].startswith("host stream failed on a rank") for o in out), out
