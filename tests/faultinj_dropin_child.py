"""Child process of tests/test_gpu_dropin_fault.py: runs with
FD_ED25519_HIP_LIB pointing at the fault-injection build
(libfd_ed25519_hip_faultinj.so) and $FD_ED25519_HIP_FAULT_DROPIN naming the
drop-in launches that fail.  argv[1]: the policy ("abort" | "reject"),
argv[2]: calls before a reset (then as many after it, "reset" mode only
when argv[3] == "reset").  Signs one valid and one tampered signature with
the oracle (the checker) and prints one JSON line per drop-in call: its
code, the code the oracle gives, the drop-ins' status and launch count."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from firedancer_amd import ed25519
    assert os.path.basename(ed25519.LIB_PATH) == "libfd_ed25519_hip_faultinj.so", ed25519.LIB_PATH
    oracle = ctypes.CDLL(os.path.join(os.path.dirname(ed25519.LIB_PATH), "..", "..", "oracle", "liboracle_ed25519.so"))
    oracle.oracle_ed25519_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                           ctypes.c_char_p]
    oracle.oracle_ed25519_public_from_private.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    oracle.oracle_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_char_p,
                                             ctypes.c_int]
    priv, msg = bytes(range(1, 33)), b"drop-in failure policy" * 9
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_public_from_private(pub, priv)
    oracle.oracle_ed25519_sign(sig, msg, len(msg), pub.raw, priv)
    bad = bytearray(sig.raw)
    bad[40] ^= 4
    cases = [bytes(sig.raw), bytes(bad)]
    policy = {"abort": ed25519.DROPIN_ON_LOST_ABORT, "reject": ed25519.DROPIN_ON_LOST_REJECT}[sys.argv[1]]
    assert ed25519.dropin_set_on_lost(policy) == ed25519.DROPIN_ON_LOST_ABORT
    calls = int(sys.argv[2])

    def call(i):
        s = cases[i % 2]
        got = ed25519.verify(msg, s, pub.raw)
        want = oracle.oracle_ed25519_verify(msg, len(msg), s, pub.raw, 0)
        lost, rec = ed25519.dropin_status()
        print(json.dumps({"i": i, "got": got, "want": want, "lost": lost, "recoveries": rec,
                          "launches": ed25519.dropin_stats()[0]}), flush=True)
    for i in range(calls):
        call(i)
    if len(sys.argv) > 3 and sys.argv[3] == "reset":
        print(json.dumps({"reset": ed25519.dropin_reset()}), flush=True)
        for i in range(calls, 2 * calls):
            call(i)


if __name__ == "__main__":
    main()
