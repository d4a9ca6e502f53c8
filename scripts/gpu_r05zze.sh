#!/bin/bash
# C1 latency variants: -Os (code size of the single-wave kernels), the
# deflate parse's candidate tests per iteration (1 / 0 extra), interleaved
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05zze_lat.log
: > $O
for r in 1 2; do
  for v in "" os dual1 dual0; do
    lib=beast_amd/libbeast_pmd${v:+_$v}.so
    echo "== round $r variant ${v:-base}" >> $O
    BPMD_LIB=$lib timeout -k 10 120 python scripts/facade_latency.py 256 >> $O 2>&1 || { echo "lat $v failed"; tail $O; exit 1; }
  done
done
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 120 python scripts/diag_zstream.py 32 1024 > gpurun_out/r05zze_diag_zstream.log 2>&1 || { echo diag failed; tail gpurun_out/r05zze_diag_zstream.log; exit 2; }
grep -v amdgpu.ids $O
