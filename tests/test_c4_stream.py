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


# ---- config_c4: the C4 stream leg of every default (C2) bench line --------

C4_TOTAL = 4000


def _c4_fakes(setattr_=setattr):
    """bench.config_c4 with the GPU replaced: a DeviceWorkload fake that
    writes C4's layout (the stream's own message sizes, seed 0xC4C4) and a
    pool fake that recomputes each code from the window as laid out."""
    import contextlib
    from firedancer_amd import ed25519, tile, workload

    class Buf:
        def __init__(self, a):
            self.a = a

        def download_into(self, dst):
            dst[:] = self.a

        def download(self, dtype, n):
            return self.a[:n].astype(dtype)

    class DeviceWorkload:
        def __init__(self, eng, m, lo, hi, ppm, seed, index_base):
            g = np.arange(index_base, index_base + m, dtype=np.uint64)
            sz = workload.msg_sizes(seed, index_base, m, lo, hi)
            self.msg_bytes = int(sz.sum())
            self.msgs = Buf(np.repeat(((g * np.uint64(7) + np.uint64(1)) % np.uint64(256)).astype(np.uint8), sz))
            s = np.zeros((m, 64), np.uint8)
            s[:, :8] = g.view(np.uint8).reshape(m, 8)
            s[:, 8] = _code(g).view(np.uint8)
            self.sigs, self.pubs = Buf(s.reshape(-1)), Buf(np.zeros(32 * m, np.uint8))
            self.expect = Buf(_code(g))

        def free(self):
            pass

    class Pool:
        def __init__(self, *a):
            pass

        def run(self, msgs, off, sz, sigs, pubs, out):
            s = sigs.reshape(-1, 64)
            for i in range(len(out)):
                g = int(s[i, :8].view(np.uint64)[0])
                ok = int(sz[i]) == int(workload.msg_sizes(SEED, g, 1, 64, 1232)[0]) and \
                    bool((msgs[int(off[i]):int(off[i]) + int(sz[i])] == (7 * g + 1) % 256).all())
                out[i] = s[i, 8].view(np.int8) if ok else 99
            return out, 0.001, {"h2d_bytes": 760 * len(out), "direct_batches": 1, "staged_batches": 0}

        def close(self):
            pass

    class Near:
        cpus = [0]

        def __init__(self, info):
            pass

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False
    setattr_(ed25519, "DeviceWorkload", DeviceWorkload)
    setattr_(tile, "Pool", Pool)
    setattr_(tile, "NearDevice", Near)
    setattr_(tile, "HostRegistration", lambda *a: contextlib.nullcontext())
    setattr_(tile, "h2d_gbps", lambda *a: 57.0)


class _Args:
    c4_signatures = C4_TOTAL
    host_window = 900
    host_batch = 256
    host_slots = 2


def _c4_whole_digest():
    return hashlib.sha256(_code(np.arange(C4_TOTAL, dtype=np.uint64)).tobytes()).hexdigest()


def _c4_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    from firedancer_amd import workload
    _c4_fakes()
    workload.CONFIGS["C4"] = dict(workload.CONFIGS["C4"])
    bench.C4_STREAM_DIGEST = _c4_whole_digest()   # the fake stream's own whole-stream digest
    r, _, w = bench.dist_setup(world)
    res = bench.config_c4(None, 0, {}, r, w, _Args())
    bench.barrier(w)
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put((r, res))


def test_config_c4_one_rank_carries_the_whole_stream_digest(monkeypatch):
    import bench
    _c4_fakes(monkeypatch.setattr)
    monkeypatch.setattr(bench, "C4_STREAM_DIGEST", _c4_whole_digest())
    res = bench.config_c4(None, 0, {}, 0, 1, _Args())
    assert res["digest_equal"] is True and res["stream_digest"] == _c4_whole_digest()
    assert res["scaling"] == "strong" and res["signatures_per_rank"] == C4_TOTAL
    assert res["label_mismatches"] == 0 and res["rank_digests"] == [res["stream_digest"]]
    assert res["frac_of_pcie_bound"] is not None and res["peak_rss_bytes_max_over_ranks"] > 0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config_c4_ranks_agree_on_the_concatenated_digest(world):
    """World 2 / 4 / 8 (gloo, the driver's scaling runs): the config_c4 key
    is present on every rank, each streamed its own contiguous shard, and
    all report the same concatenated digest, equal to the one-rank
    stream's (digest_equal true)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [o for _, o in sorted(q.get(timeout=240) for _ in procs)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r["digest_equal"] is True for r in res), res
    assert all(r["stream_digest"] == _c4_whole_digest() for r in res)
    assert all(r["rank_digests"] == res[0]["rank_digests"] for r in res) and len(res[0]["rank_digests"]) == world
    assert all(r["signatures_per_rank"] == C4_TOTAL // world and r["n_gpus"] == world for r in res)


# ---- config_c4's window pre-flight -------------------------

def _preflight_worker(rank, world, port, q, avail):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import bench
    from firedancer_amd import workload
    _c4_fakes()
    workload.CONFIGS["C4"] = dict(workload.CONFIGS["C4"])
    bench.C4_STREAM_DIGEST = _c4_whole_digest()
    # the node's free memory as the pre-flight sees it: rank 3's is smaller
    bench._mem_available = lambda: avail * (0.5 if rank == 3 else 1.0)
    bench._memlock_limit = lambda: None
    r, _, w = bench.dist_setup(world)
    try:
        res = bench.config_c4(None, 0, {}, r, w, _Args())
        out = ("ok", res["window_preflight"], res["stream_digest"], res["digest_equal"], res["host_window_bytes_per_rank"])
    except RuntimeError as ex:
        out = ("raised", str(ex)[:40])
    bench.barrier(w)
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put((r, out))


def _world8_preflight(avail):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_preflight_worker, args=(r, 8, port, q, avail)) for r in range(8)]
    for p in procs:
        p.start()
    res = [o for _, o in sorted(q.get(timeout=240) for _ in procs)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_preflight_shrinks_every_ranks_window_alike_and_keeps_the_digest():
    """World 8, 500 signatures per rank, --host-window 900: a node whose
    free memory holds (for 8 ranks, half of it) about 240 signatures per
    rank -- and rank 3 sees half that -- makes every rank stream in the
    smallest rank's window (the barriers pair up), before anything is
    pinned; the digest is the whole stream's."""
    bps = 648 + 109                            # C4's mean message (64..1232 B) + the rest of a signature
    res = _world8_preflight(avail=2 * 8 * 240 * bps)
    assert all(o[0] == "ok" for o in res), res
    pf = [o[1] for o in res]
    assert all(p["shrunk"] and p["requested_window"] == 900 for p in pf)
    assert len({p["window"] for p in pf}) == 1 and 90 <= pf[0]["window"] <= 130   # rank 3's ~120
    assert all(o[2] == _c4_whole_digest() and o[3] is True for o in res)
    assert all(o[4] < 140 * (1232 + 109) for o in res)   # one shrunk window of host memory each


def test_preflight_fails_every_rank_before_pinning_when_nothing_fits():
    res = _world8_preflight(avail=1000)
    assert all(o[0] == "raised" and o[1].startswith("C4 pre-flight: no window fits") for o in res), res


def test_preflight_keeps_a_window_that_fits(monkeypatch):
    import bench
    monkeypatch.setattr(bench, "_mem_available", lambda: 1 << 40)
    monkeypatch.setattr(bench, "_memlock_limit", lambda: None)
    from firedancer_amd import workload
    sizes = workload.msg_sizes(SEED, 0, 5000, 64, 1232)
    w, rec = bench.c4_window_preflight(2000, sizes, 1, 1 << 20)
    assert w == 2000 and not rec["shrunk"]
    monkeypatch.setattr(bench, "_memlock_limit", lambda: 300 * 760)   # a finite RLIMIT_MEMLOCK binds
    w, rec = bench.c4_window_preflight(2000, sizes, 1, 1 << 20)
    assert rec["shrunk"] and 250 <= w <= 300
