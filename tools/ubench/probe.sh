#!/bin/bash
# Environment probe for the GPU box: CPU features, core share, GPU clocks.
mkdir -p gpurun_out
{
  echo "== lscpu"; lscpu | head -30
  echo "== flags"; grep -m1 -o -w -E 'avx512ifma|avx512vbmi|avx512f|avx2|sha_ni' /proc/cpuinfo | sort -u | tr '\n' ' '; echo
  echo "== nproc $(nproc)  affinity $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"
  echo "== mem"; free -g | head -2
  echo "== rocminfo"; rocminfo | grep -E 'Marketing|Max Clock|Compute Unit|gfx950' | head -12
  echo "== rocm-smi"; rocm-smi --showclocks 2>/dev/null | head -20
} > gpurun_out/probe.txt 2>&1
