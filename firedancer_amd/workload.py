"""Synthetic workloads of SURVEY.md §8(d), shared by bench.py and the tests.

Every byte is a pure function of (seed, global signature index), computed by
a counter-based mixer (the splitmix64 finalizer), so a shard of a stream can
be produced on any GPU (fd_ed25519_hip_gen_dev / _corrupt_dev) and the same
bytes recomputed here on the host.  Definitions must match
firedancer_amd/csrc/fd_ed25519_gen.hip.

  C2  1,048,576 signatures, message size uniform in [64, 1232] B, 2% invalid
      (S+L, small-order A/R, undecodable A/R, non-canonical A, message bit
      flip), messages packed back to back at arbitrary byte offsets.
  C4  the C2 distribution as a 64M-signature stream, sharded over ranks.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
MSG_SALT = np.uint64(0xA0761D6478BD642F)
BAD_SALT = np.uint64(0xE7037ED1A0B428DB)
SIZE_SALT = np.uint64(0xD1B54A32D192ED03)

CONFIGS = {
    "C1": dict(n=16384, lo=200, hi=200, ppm=0),
    "C2": dict(n=1 << 20, lo=64, hi=1232, ppm=20000),
    # the C2 distribution as one 64M stream split over the ranks (strong scaling)
    "C4": dict(n=64 << 20, lo=64, hi=1232, ppm=20000, total=True),
}

# invalid classes of fd_ed25519_corrupt_kernel -> reference AVX-512 code
CLASS_NAMES = ["valid", "S_plus_L", "A_small_order", "R_small_order", "A_undecodable", "R_undecodable",
               "A_noncanonical_y", "msg_bitflip"]


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _ctr(salted_seed, idx):
    with np.errstate(over="ignore"):
        return np.uint64(salted_seed) + GOLDEN * (np.asarray(idx, dtype=np.uint64) + np.uint64(1))


def msg_sizes(seed, index_base, n, lo, hi):
    g = np.arange(index_base, index_base + n, dtype=np.uint64)
    x = mix64(_ctr(np.uint64(seed) ^ SIZE_SALT, g))
    return (np.uint64(lo) + x % np.uint64(hi - lo + 1)).astype(np.uint32)


def msg_offsets(sizes):
    off = np.zeros(len(sizes), dtype=np.uint64)
    if len(sizes) > 1:
        np.cumsum(sizes[:-1], dtype=np.uint64, out=off[1:])
    return off


def msg_buffer(seed, nbytes):
    """Host recomputation of the message buffer fd_ed25519_fill_random_kernel writes."""
    words = (nbytes + 7) // 8
    x = mix64(_ctr(np.uint64(seed) ^ MSG_SALT, np.arange(words, dtype=np.uint64)))
    return x.astype("<u8").view(np.uint8)[:nbytes].copy()


def private_keys(seed, index_base, n):
    """Host recomputation of the derived private keys ([n][32] bytes)."""
    g = np.arange(index_base, index_base + n, dtype=np.uint64)
    ctr = (g[:, None] * np.uint64(4) + np.arange(4, dtype=np.uint64)[None, :])
    x = mix64(_ctr(np.uint64(seed), ctr))
    return x.astype("<u8").view(np.uint8).reshape(n, 32)


def corruption(seed, index_base, n, ppm):
    """(class[n], selector[n]) as fd_ed25519_corrupt_kernel draws them."""
    g = np.arange(index_base, index_base + n, dtype=np.uint64)
    x = mix64(_ctr(np.uint64(seed) ^ BAD_SALT, g))
    bad = (x % np.uint64(1000000)) < np.uint64(ppm)
    cls = np.where(bad, 1 + ((x >> np.uint64(32)) % np.uint64(7)), 0).astype(np.uint8)
    return cls, (x >> np.uint64(40)).astype(np.uint64)


def _cu16(v):
    out = bytearray()
    while True:
        b, v = v & 0x7F, v >> 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def txn_payloads(engine, n, seed, msg_sz=200, index_base=0, signers=1):
    """n legacy Solana transactions (the verify tile's input format,
    src/ballet/txn/fd_txn.h) with `signers` signatures over a msg_sz-byte
    message each, keys derived from (seed, index), signed on the GPU
    (fd_ed25519_hip_sign_dev).  Message: header (signers, 0, 1), signers+2
    accounts (the signers' keys first), blockhash, one instruction with
    padding data.  Returns (payloads uint8 [n][size], size)."""
    k = signers
    head = bytes([k, 0, 1]) + _cu16(k + 2)
    fixed = len(head) + 32 * (k + 2) + 32 + 1 + 1 + 1 + 2
    data_len = msg_sz - fixed - len(_cu16(max(msg_sz - fixed - 1, 0)))
    assert data_len >= 0, "message too short"
    tail_hdr = bytes([1, k + 1, 2, 0, 1]) + _cu16(data_len)
    m_len = len(head) + 32 * (k + 2) + 32 + len(tail_hdr) + data_len
    rng = np.random.default_rng(seed)
    privs = private_keys(seed, index_base, n * k).reshape(n, k, 32)
    # public keys first (signing an empty message yields them)
    d_priv = engine.alloc(32 * n * k).upload(privs.reshape(-1))
    d_off = engine.alloc(8 * n * k).upload(np.zeros(n * k, np.uint64))
    d_sz = engine.alloc(4 * n * k).upload(np.zeros(n * k, np.uint32))
    d_msg = engine.alloc(16)
    d_sig, d_pub = engine.alloc(64 * n * k), engine.alloc(32 * n * k)
    engine.sign_dev(n * k, d_msg.ptr, d_off.ptr, d_sz.ptr, d_priv.ptr, d_sig.ptr, d_pub.ptr)
    engine.sync()
    pubs = d_pub.download(np.uint8, 32 * n * k).reshape(n, k, 32)
    msgs = np.zeros((n, m_len), np.uint8)
    p = 0
    msgs[:, p:p + len(head)] = np.frombuffer(head, np.uint8); p += len(head)
    msgs[:, p:p + 32 * k] = pubs.reshape(n, 32 * k); p += 32 * k
    msgs[:, p:p + 64] = rng.integers(0, 256, (n, 64), dtype=np.uint8); p += 64    # 2 more accounts
    msgs[:, p:p + 32] = rng.integers(0, 256, (n, 32), dtype=np.uint8); p += 32    # blockhash
    msgs[:, p:p + len(tail_hdr)] = np.frombuffer(tail_hdr, np.uint8); p += len(tail_hdr)
    msgs[:, p:] = rng.integers(0, 256, (n, m_len - p), dtype=np.uint8)
    # every signer signs its transaction's message
    d_m = engine.alloc(n * m_len).upload(msgs.reshape(-1))
    off = np.repeat(np.arange(n, dtype=np.uint64) * np.uint64(m_len), k)
    d_off2 = engine.alloc(8 * n * k).upload(off)
    d_sz2 = engine.alloc(4 * n * k).upload(np.full(n * k, m_len, np.uint32))
    engine.sign_dev(n * k, d_m.ptr, d_off2.ptr, d_sz2.ptr, d_priv.ptr, d_sig.ptr, d_pub.ptr)
    engine.sync()
    sigs = d_sig.download(np.uint8, 64 * n * k).reshape(n, 64 * k)
    for b in (d_priv, d_off, d_sz, d_msg, d_sig, d_pub, d_m, d_off2, d_sz2):
        b.free()
    size = 1 + 64 * k + m_len
    pay = np.empty((n, size), np.uint8)
    pay[:, 0] = k
    pay[:, 1:1 + 64 * k] = sigs
    pay[:, 1 + 64 * k:] = msgs
    return pay, size


def ops_per_verify(msg_sz):
    """SURVEY.md §8(d) frozen algorithmic INT32 op count per verify, split by
    phase kernel.  Unit costs (radix 2^25.5): mul 130, sqr 85, carried
    add/sub 30, uncarried add/sub 10, SHA-512 block 5400, misc 2000.
    Totals: 1381 mul + 1520 sqr + 806.5 add/sub + 1265.8 add_nr + SHA + misc.
    The reference's work is attributed to the kernel that stands in for it:
      hash   = SHA-512 blocks of R||A||M + mod-L reduction (1000)
      decode = the square roots of A and R (pow22523 = 251 sqr + 11 mul, + 10
               mul, 2 sqr each)
      scalar = nothing of the reference's: the half-size scalars are this
               engine's own preparation
      dsm    = the rest (double-scalar multiplication, table).
    The count is the reference algorithm's (frozen): the half-size
    formulation executes fewer operations for the same verdict, so the
    executed-instruction rate is reported separately from rocprof counters."""
    msg_sz = np.asarray(msg_sz, dtype=np.float64)
    blocks = np.ceil((81.0 + msg_sz) / 128.0)
    total = 1381 * 130 + 1520 * 85 + 806.5 * 30 + 1265.8 * 10 + 5400 * blocks + 2000
    hash_ = 5400 * blocks + 1000
    sqrt_ = 253 * 85 + 21 * 130
    dsm = total - hash_ - 2 * sqrt_
    return dict(total=total, hash=hash_, scalar=np.zeros_like(total), decode=np.full_like(total, 2 * sqrt_), dsm=dsm)


def box_cores(sysfs="/sys/devices/system/cpu"):
    """The whole machine's CPUs from its topology in sysfs, not from this
    process's cgroup or affinity: logical CPUs online, physical cores
    (distinct package/core pairs) and sockets.  None where unreadable."""
    import glob
    import os
    pairs, pkgs, logical = set(), set(), 0
    for d in glob.glob(os.path.join(sysfs, "cpu[0-9]*")):
        try:
            if open(os.path.join(d, "online")).read().strip() == "0":
                continue
        except OSError:
            pass   # cpu0 often has no "online" file: it is online
        try:
            pkg = int(open(os.path.join(d, "topology", "physical_package_id")).read())
            core = int(open(os.path.join(d, "topology", "core_id")).read())
        except (OSError, ValueError):
            continue
        logical += 1
        pairs.add((pkg, core))
        pkgs.add(pkg)
    if not logical:
        return {"logical_cpus": None, "physical_cores": None, "sockets": None, "source": sysfs}
    return {"logical_cpus": logical, "physical_cores": len(pairs), "sockets": len(pkgs),
            "source": f"{sysfs}/cpu*/topology (the machine, not the lease)"}


def host_cores():
    """CPU cores this process may use: the cgroup CPU quota (cpu.max, v2; or
    cpu.cfs_quota_us / cfs_period_us, v1) when one is set, else the
    scheduler's share the environment states ($OMP_NUM_THREADS, which the
    GPU box sets to the lease's CPU share), within the affinity mask.  On
    the GPU box the affinity shows the whole machine (256 CPUs)."""
    try:
        n_aff = len(__import__("os").sched_getaffinity(0))
    except (AttributeError, OSError):
        n_aff = __import__("os").cpu_count() or 1
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    env = __import__("os").environ.get("OMP_NUM_THREADS", "")
    share = int(env) if env.isdigit() and int(env) > 0 else None
    if quota is not None:
        n, src = min(n_aff, max(1, int(quota))), "cgroup cpu quota"
    elif share is not None:
        n, src = min(n_aff, share), "OMP_NUM_THREADS (lease share)"
    else:
        n, src = n_aff, "affinity mask"
    return max(1, n), {"affinity": n_aff, "cgroup_quota": quota, "omp_num_threads": share, "source": src}
