"""fd_ed25519_hip_frag_assemble (include/fd_ed25519_hip_tile.h), the
verdict-frag protocol's tile side: payload | pad | trailer, the trailer
being the bytes after the payload and its 2-byte alignment pad in the frag
the reference's after_frag publishes (src/app/fdctl/run/tiles/
fd_verify.c:102-133: fd_txn_t, then the u16 payload_sz).  A tiny C driver,
built with gcc against the header alone, runs the helper on cases from
this file; the expected frags are built here independently.  CPU only."""
import os
import random
import struct
import subprocess

import pytest

from conftest import REPO

TXN_MTU, TXN_MAX_SZ = 1232, 852

DRIVER = r"""
#include <stdio.h>
#include <stdlib.h>
#include "fd_ed25519_hip_tile.h"
/* stdin: records of (u32 payload_sz, u32 trailer_sz, payload, trailer);
   stdout: per record u32 frag size, then the frag's bytes */
int main( void ) {
  static unsigned char pay[ 4096 ], tr[ 4096 ], dst[ FD_ED25519_HIP_TPU_DCACHE_MTU + 64 ];
  unsigned int h[ 2 ];
  while( fread( h, 4, 2, stdin )==2 ) {
    if( h[0]>sizeof(pay) || h[1]>sizeof(tr) ) return 2;
    if( fread( pay, 1, h[0], stdin )!=h[0] || fread( tr, 1, h[1], stdin )!=h[1] ) return 2;
    for( unsigned i=0; i<sizeof(dst); i++ ) dst[ i ] = 0xa5;
    unsigned int n = (unsigned int)fd_ed25519_hip_frag_assemble( dst, pay, h[0], tr, h[1] );
    fwrite( &n, 4, 1, stdout );
    fwrite( dst, 1, n, stdout );
  }
  return 0;
}
"""


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("fa")
    src, exe = d / "fa.c", d / "fa"
    src.write_text(DRIVER)
    san = ([f"-fsanitize={os.environ['FD_TEST_SANITIZE']}", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
           if os.environ.get("FD_TEST_SANITIZE") else [])   # tests/test_sanitizers.py
    r = subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-Werror", *san, "-I", os.path.join(REPO, "include"),
                        str(src), "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return str(exe)


def expected(payload, trailer):
    psz = len(payload)
    if psz > TXN_MTU or len(trailer) < 2 or len(trailer) > TXN_MAX_SZ + 2:
        return b""
    if struct.unpack_from("<H", trailer, len(trailer) - 2)[0] != psz:
        return b""
    return payload + b"\0" * (psz % 2) + trailer


def test_frag_assemble_cases(driver):
    rng = random.Random(7)
    cases = []
    for psz in (0, 1, 2, 63, 64, 65, 199, 200, 1231, 1232):
        body = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 40, 63, 851, 852])))
        good = body + struct.pack("<H", psz)
        payload = bytes(rng.getrandbits(8) for _ in range(psz))
        cases.append((payload, good))                                            # accepted
        cases.append((payload, body + struct.pack("<H", (psz + 1) & 0xffff)))    # another payload's trailer
        cases.append((payload, good[-1:]))                                       # too short
    cases.append((bytes(1233), bytes(10) + struct.pack("<H", 1233)))              # payload above the MTU
    cases.append((bytes(100), bytes(853) + struct.pack("<H", 100)))               # trailer above fd_txn_t's max
    cases.append((bytes(100), b""))                                               # no trailer
    blob = b"".join(struct.pack("<II", len(p), len(t)) + p + t for p, t in cases)
    r = subprocess.run([driver], input=blob, capture_output=True)
    assert r.returncode == 0
    out, i = [], 0
    while i < len(r.stdout):
        n = struct.unpack_from("<I", r.stdout, i)[0]
        out.append(r.stdout[i + 4:i + 4 + n])
        i += 4 + n
    assert len(out) == len(cases)
    for k, ((p, t), got) in enumerate(zip(cases, out)):
        assert got == expected(p, t), (k, len(p), len(t))
    assert sum(1 for g in out if g) == 10   # exactly the well-formed ones
