"""Test helper: Solana transaction payloads (legacy and v0), signed with the
oracle, in the wire format fd_txn_parse reads (src/ballet/txn/fd_txn.h,
https://docs.solana.com/developing/programming-model/transactions).  Also
the reference harness (oracle/_ref) entry points for the tile layer."""
import ctypes
import os
import random

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cu16(v):
    """compact-u16, minimal encoding."""
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def message(sig_cnt, accts, ro_signed=0, ro_unsigned=0, instrs=(), version=None, luts=(), blockhash=b"\x07" * 32):
    """Serialize a message. instrs: [(program_id, acct_idx_list, data)];
    luts (v0 only): [(addr32, writable_idx_list, readonly_idx_list)]."""
    m = bytearray()
    if version is not None:
        m.append(0x80 | version)
    m += bytes([sig_cnt, ro_signed, ro_unsigned])
    m += cu16(len(accts))
    for a in accts:
        m += a
    m += blockhash
    m += cu16(len(instrs))
    for prog, idx, data in instrs:
        m.append(prog)
        m += cu16(len(idx)) + bytes(idx)
        m += cu16(len(data)) + bytes(data)
    if version is not None:
        m += cu16(len(luts))
        for addr, w, r in luts:
            m += addr + cu16(len(w)) + bytes(w) + cu16(len(r)) + bytes(r)
    return bytes(m)


def txn(sigs, msg):
    return cu16(len(sigs)) + b"".join(sigs) + msg


class Signer:
    def __init__(self, oracle, seed):
        self.oracle = oracle
        self.rng = random.Random(seed)
        self.keys = []

    def key(self):
        priv = bytes(self.rng.getrandbits(8) for _ in range(32))
        pub = ctypes.create_string_buffer(32)
        self.oracle.oracle_ed25519_public_from_private(pub, priv)
        self.keys.append((priv, pub.raw))
        return priv, pub.raw

    def sign(self, msg, priv, pub):
        s = ctypes.create_string_buffer(64)
        self.oracle.oracle_ed25519_sign(s, msg, len(msg), pub, priv)
        return s.raw


def random_txn(signer, rng, nsig, v0=False, bad_sig=False, msg_pad=0, instr_n=1, lut_n=1):
    """A parseable transaction with nsig signers (pubkeys = first nsig
    account addresses), instr_n instructions (and, v0, lut_n address table
    lookups); bad_sig flips a bit of a random signature after signing."""
    keys = [signer.key() for _ in range(nsig)] if nsig <= 16 else [signer.key() for _ in range(2)] * ((nsig + 1) // 2)
    keys = keys[:nsig]
    extra = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(1 + rng.randrange(3))]
    accts = [k[1] for k in keys] + extra
    prog = len(accts) - 1
    data = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 40) + msg_pad))
    instrs = [(prog, [0, min(1, len(accts) - 1)], data)]
    for _ in range(instr_n - 1):
        instrs.append((prog, [rng.randrange(len(accts)) for _ in range(rng.randrange(4))],
                       bytes(rng.getrandbits(8) for _ in range(rng.randrange(12)))))
    luts = [(bytes(rng.getrandbits(8) for _ in range(32)), [0] * (1 + rng.randrange(2)), [1] * rng.randrange(3))
            for _ in range(lut_n)] if v0 else ()
    m = message(nsig, accts, ro_signed=0, ro_unsigned=1, instrs=instrs, version=0 if v0 else None, luts=luts)
    sigs = [signer.sign(m, priv, pub) for priv, pub in keys]
    if bad_sig:
        j = rng.randrange(nsig)
        s = bytearray(sigs[j])
        s[rng.randrange(64)] ^= 1 << rng.randrange(8)
        sigs[j] = bytes(s)
    return txn(sigs, m)


def mutate(rng, p):
    """A random structural mutation of a payload (bit flip, byte set,
    truncation, extension, insertion or deletion)."""
    p = bytearray(p)
    k = rng.randrange(6)
    if k == 0 and p:
        i = rng.randrange(len(p))
        p[i] ^= 1 << rng.randrange(8)
    elif k == 1 and p:
        p[rng.randrange(len(p))] = rng.choice([0, 1, 0x7F, 0x80, 0xFF, rng.randrange(256)])
    elif k == 2 and p:
        del p[rng.randrange(len(p)):]
    elif k == 3:
        p += bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 8)))
    elif k == 4:
        i = rng.randrange(len(p) + 1)
        p[i:i] = bytes([rng.randrange(256)])
    elif p:
        del p[rng.randrange(len(p))]
    return bytes(p)


def cpu_has_avx512ifma():
    try:
        flags = next(l for l in open("/proc/cpuinfo") if l.startswith("flags")).split()
        return "avx512ifma" in flags and "avx512vbmi" in flags
    except (OSError, StopIteration):
        return False


def ref_lib(flavour="portable"):
    """The reference compiled from its sources (oracle/_ref), or None.
    flavour: "portable" (fiat backend) or "avx512" (the production r43x6
    backend; None if this CPU lacks AVX-512 IFMA)."""
    if flavour == "avx512" and not cpu_has_avx512ifma():
        return None
    path = os.path.join(REPO, "oracle", "_ref", f"libfdref_{flavour}.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.fdref_txn_parse.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_void_p]
    lib.fdref_txn_parse.restype = ctypes.c_ulong
    lib.fdref_vtile_seq.argtypes = [ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong,
                                    ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
    lib.fdref_txn_parse_raw.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_void_p]
    lib.fdref_txn_parse_raw.restype = ctypes.c_ulong
    lib.fdref_after_frag.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_void_p]
    lib.fdref_after_frag.restype = ctypes.c_ulong
    lib.fdref_vtile_seq_frags.argtypes = [ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_ulong, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]
    return lib


TXN_MAX_SZ = 852                      # FD_TXN_MAX_SZ
TPU_DCACHE_MTU = 1232 + TXN_MAX_SZ + 2  # FD_TPU_DCACHE_MTU


def ref_parse_raw(lib, payload):
    """fd_txn_parse's fd_txn_t bytes (footprint long), or None."""
    buf = ctypes.create_string_buffer(TXN_MAX_SZ)
    r = lib.fdref_txn_parse_raw(payload, len(payload), buf)
    return buf.raw[:r] if r else None


def ref_after_frag(lib, payload):
    """The frag the reference verify tile's after_frag publishes, or None."""
    buf = ctypes.create_string_buffer(TPU_DCACHE_MTU)
    r = lib.fdref_after_frag(payload, len(payload), buf)
    return buf.raw[:r] if r else None


def ref_vtile_frags(lib, payloads, depth=16, map_cnt=64):
    """The sequential reference tile: verdicts, tags, and the published
    frag of every SUCCESS transaction (None otherwise)."""
    from firedancer_amd.tile import pack_payloads
    buf, off, sz = pack_payloads(payloads)
    n = len(payloads)
    v = np.zeros(n, np.int8)
    tags = np.zeros(n, np.uint64)
    fr = np.zeros((n, TPU_DCACHE_MTU), np.uint8)
    fsz = np.zeros(n, np.uint64)
    lib.fdref_vtile_seq_frags(n, buf.ctypes.data, off.ctypes.data, sz.ctypes.data, depth, map_cnt, v.ctypes.data,
                              tags.ctypes.data, fr.ctypes.data, fsz.ctypes.data)
    return v, tags, [fr[i, :int(fsz[i])].tobytes() if fsz[i] else None for i in range(n)]


def ref_parse(lib, payload):
    f = np.zeros(13, np.uint64)
    r = lib.fdref_txn_parse(payload, len(payload), f.ctypes.data)
    return (tuple(int(x) for x in f) if r else None), r


def ref_vtile(lib, payloads, depth=16, map_cnt=64):
    from firedancer_amd.tile import pack_payloads
    buf, off, sz = pack_payloads(payloads)
    n = len(payloads)
    v = np.zeros(n, np.int8)
    tags = np.zeros(n, np.uint64)
    lib.fdref_vtile_seq(n, buf.ctypes.data, off.ctypes.data, sz.ctypes.data, depth, map_cnt, v.ctypes.data,
                        tags.ctypes.data)
    return v, tags


def tile_workload(oracle, seed, n, p_bad=0.1, p_dup=0.1, p_junk=0.05, p_many=0.01):
    """n frags: valid txns of 1-12 signers, some with a bad signature, some
    duplicates of an earlier frag (near and far: across tcache evictions),
    some unparseable, some with 17+ signatures (ERR_SIG)."""
    rng = random.Random(seed)
    signer = Signer(oracle, seed)
    out = []
    for i in range(n):
        r = rng.random()
        if out and r < p_dup:
            back = rng.choice([1, 2, 5, 15, 16, 17, 40])
            out.append(out[max(0, len(out) - back)])
        elif r < p_dup + p_junk:
            base = out[-1] if out else random_txn(signer, rng, 1)
            out.append(mutate(rng, base))
        elif r < p_dup + p_junk + p_many:
            out.append(random_txn(signer, rng, 17 + rng.randrange(3)))
        else:
            nsig = rng.choice([1, 1, 1, 2, 2, 3, 4, 8, 12])
            # some with fd_txn_t trailers longer than the device's 64-byte slot
            many = rng.random() < 0.1
            out.append(random_txn(signer, rng, nsig, v0=rng.random() < 0.3, bad_sig=rng.random() < p_bad,
                                  msg_pad=rng.randrange(0, 600), instr_n=rng.randrange(5, 9) if many else 1,
                                  lut_n=rng.randrange(2, 5) if many else 1))
    return out
