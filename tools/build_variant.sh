#!/bin/bash
# Build an experimental variant of libfd_ed25519_hip into build/variants/<name>/
# usage: tools/build_variant.sh NAME "EXTRA_HIPFLAGS" ["EXTRA_CFLAGS"]
set -e
NAME=$1; FLAGS=$2; CFL=$3
R=$(cd $(dirname $0)/.. && pwd)
OUT=$R/build/variants/$NAME
mkdir -p $OUT
make -s -C $R/firedancer_amd/csrc -j8 OBJ=$OUT/obj LIBDIR=$OUT LIB=$OUT/libfd_ed25519_hip.so EXTRA_HIPFLAGS="$FLAGS" EXTRA_CFLAGS="$CFL" >/dev/null
echo $OUT/libfd_ed25519_hip.so
