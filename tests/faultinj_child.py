"""Child process of tests/test_gpu_halfcheck.py: runs with
FD_ED25519_HIP_LIB pointing at the fault-injection build of the library
(libfd_ed25519_hip_faultinj.so) and verifies the sets in argv[1] (an .npz
of named signature sets) with every dsm form, plus the device's half-size
diagnostic on the k values given; writes the codes to argv[2]."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from firedancer_amd import ed25519
    assert os.path.basename(ed25519.LIB_PATH) == "libfd_ed25519_hip_faultinj.so", ed25519.LIB_PATH
    src = dict(np.load(sys.argv[1], allow_pickle=False))
    res = {}
    names = sorted({k.split("/")[0] for k in src if "/" in k})
    for dsm in ("oct", "quad", "wide"):
        for codes in ("avx512", "portable"):
            e = ed25519.Engine(0, max_chunk=1 << 14, dsm=dsm, codes=codes)
            for nm in names:
                d = {f: src[f"{nm}/{f}"] for f in ("msgs", "msg_off", "msg_sz", "sigs", "pubs")}
                res[f"{nm}/{dsm}/{codes}"] = e.verify_host(d["msgs"], d["msg_off"], d["msg_sz"], d["sigs"], d["pubs"])
            if dsm == "wide" and codes == "avx512":
                res["diag"] = e.diag_half_scalars(src["k_words"])
            e.close()
    np.savez(sys.argv[2], **res)


if __name__ == "__main__":
    main()
