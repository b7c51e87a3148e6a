"""N>1 path on CPU: shard plan, counter-based workload shards, and the
bench's gloo coordination (barrier, max-over-ranks time, summed verdict
mismatches) with world_size 2 at 127.0.0.1."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shards_are_disjoint_and_cover_the_stream():
    n = 1000
    for world in (1, 2, 4, 8):
        seen = np.zeros(world * n, dtype=np.int32)
        for rank in range(world):
            base = rank * n  # bench.py: index_base = rank * n
            seen[base:base + n] += 1
        assert (seen == 1).all()


def test_workload_is_counter_based_across_shards():
    """Any rank can produce its shard alone: shard r of the stream equals the
    matching slice of the whole stream (sizes, keys, corruption draws)."""
    from firedancer_amd import workload
    seed, n, world = 77, 512, 4
    full_sz = workload.msg_sizes(seed, 0, n * world, 64, 1232)
    full_keys = workload.private_keys(seed, 0, n * world)
    full_cls, _ = workload.corruption(seed, 0, n * world, 20000)
    for r in range(world):
        assert np.array_equal(workload.msg_sizes(seed, r * n, n, 64, 1232), full_sz[r * n:(r + 1) * n])
        assert np.array_equal(workload.private_keys(seed, r * n, n), full_keys[r * n:(r + 1) * n])
        cls, _ = workload.corruption(seed, r * n, n, 20000)
        assert np.array_equal(cls, full_cls[r * n:(r + 1) * n])
    assert len(np.unique(full_keys, axis=0)) == n * world


def test_corruption_rate_and_classes():
    from firedancer_amd import workload
    cls, _ = workload.corruption(5, 0, 1 << 20, 20000)
    frac = (cls != 0).mean()
    assert 0.018 < frac < 0.022
    assert set(np.unique(cls).tolist()) == set(range(8))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    r, local, w = bench.dist_setup(world)
    bench.barrier(w)
    tmax = bench.allreduce_max(1.0 + r, w)
    msum = bench.allreduce_sum(3 * r, w)
    bench.barrier(w)
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put((r, local, w, tmax, msum))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_coordination(world):
    """bench.py's rank setup, barrier and max / sum over ranks at the
    driver's scaling worlds (gloo on the CPU)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [x[0] for x in res] == list(range(world))
    assert all(x[2] == world for x in res)
    assert all(x[3] == float(world) for x in res)                        # max over ranks of (1 + rank)
    assert all(x[4] == 3.0 * world * (world - 1) / 2 for x in res)      # sum over ranks of 3 * rank


def test_bench_spawns_its_ranks_without_a_launcher():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts two ranks itself
    (child processes, rank r on device r) which rendezvous over gloo and
    then refuse to run here: there is no GPU, so local rank 0 already has
    no device of its own -- the check that keeps two ranks from silently
    sharing one device (--gpus N was ignored)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "[rank 0] local rank 0 but only 0 visible GPU(s)" in r.stderr
    assert "[rank 1] local rank 1 but only 0 visible GPU(s)" in r.stderr
    assert r.stdout == ""


def _bench_ranks(extra_env, timeout=300):
    import subprocess
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=timeout, env=env)
    return r, time.time() - t0


def test_bench_one_rank_without_device_one_engine_failing():
    """Rank 1 has no device of its own while rank 0 has one (a test hook
    pretends one GPU is visible) and rank 0's engine then fails (there is no
    GPU here): both ranks reach the setup agreement, both exit non-zero
    promptly, none is left waiting in a collective."""
    r, dt = _bench_ranks({"FD_BENCH_FAKE_DEVICE_COUNT": "1"})
    assert r.returncode == 2, r.stderr[-3000:]
    assert "[rank 1] local rank 1 but only 1 visible GPU(s)" in r.stderr
    assert "[rank 0] engine_new failed" in r.stderr
    assert "setup failed on rank(s) [0, 1]" in r.stderr
    assert r.stdout == ""
    assert dt < 90, dt


def test_bench_rank_lost_before_the_agreement():
    """A rank that dies before the first collective (test hook: rank 1 exits
    at once): rank 0 leaves its collective on the gloo timeout (10 s here,
    120 s by default) or is ended by the launcher's grace period; the job
    exits non-zero within about that bound instead of the default 30
    minutes."""
    r, dt = _bench_ranks({"FD_BENCH_FAKE_DEVICE_COUNT": "2", "FD_BENCH_DIE_RANK": "1",
                          "FD_BENCH_GLOO_TIMEOUT_S": "10"})
    assert r.returncode != 0, r.stderr[-3000:]
    assert r.stdout == ""
    assert dt < 90, dt


def test_bench_rejects_a_launcher_world_that_differs_from_gpus():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 2 and "--gpus 2 but the launcher started 1 ranks" in r.stderr


class _Buf:
    def __init__(self, a):
        self.a = a

    def download(self, dtype, n):
        return self.a[:n].astype(dtype)


class _Workload:
    def __init__(self, n=64):
        self.n, self.msg_bytes = n, 16 * n
        self.msgs = _Buf(np.zeros(16 * n, np.uint8))
        self.off = _Buf(np.arange(n, dtype=np.uint64) * 16)
        self.sigs, self.pubs = _Buf(np.zeros(64 * n, np.uint8)), _Buf(np.zeros(32 * n, np.uint8))
        self.expect = _Buf(np.zeros(n, np.int8))
        self.sizes = np.full(n, 16, np.uint32)


def _host_fed_worker(rank, world, port, q, fail_rank):
    """bench.host_fed with the tile layer replaced by fakes: one rank's
    setup raises, the other's succeeds"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import contextlib
    import bench
    from firedancer_amd import tile

    class Pool:
        def __init__(self, *a):
            if rank == fail_rank:
                raise OSError("pinned allocation failed (injected)")

        def run(self, msgs, off, sz, sigs, pubs, out):
            out[:] = 0
            return out, 0.01, {"h2d_bytes": 100 * len(out), "direct_batches": 1, "staged_batches": 0}

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

    tile.Pool, tile.NearDevice = Pool, Near
    tile.HostRegistration = lambda *a: contextlib.nullcontext()
    tile.max_span = lambda *a: 1 << 20
    tile.h2d_gbps = lambda *a: 50.0
    r, _, w = bench.dist_setup(world)
    try:
        bench.host_fed(_Workload(), 0, {}, w, 2, 32, 2, 2)
        outcome = "ok"
    except RuntimeError as ex:
        outcome = "raised: " + str(ex)[:60]
    bench.barrier(w)   # both ranks got here: nobody was left waiting in a collective
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put((r, outcome))


@pytest.mark.parametrize("fail_rank", [0, 1, -1])
def test_host_fed_failure_is_agreed_by_every_rank(fail_rank):
    """A host-fed leg that fails on one rank fails on every rank, with no
    rank left blocked in a barrier (the leg's collectives are reached by all
    ranks whatever happens to their own setup); with no failure both
    succeed."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_fed_worker, args=(r, 2, port, q, fail_rank)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if fail_rank < 0:
        assert [o for _, o in res] == ["ok", "ok"]
    else:
        assert all(o.startswith("raised: host-fed leg failed on a rank (setup)") for _, o in res), res
