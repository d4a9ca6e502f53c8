#!/bin/bash
# deflate phases after the multi-candidate parse (prof build)
set -o pipefail
mkdir -p gpurun_out
export BPMD_LIB=beast_amd/libbeast_pmd_prof.so
( DIAG_MSGS=65536 DIAG_SIZE=4096 DIAG_KIND=json timeout -k 10 200 python -u scripts/diag_deflate.py &&
  DIAG_MSGS=4096 DIAG_SIZE=65536 DIAG_KIND=json timeout -k 10 200 python -u scripts/diag_deflate.py &&
  DIAG_MSGS=4096 DIAG_SIZE=65536 DIAG_KIND=binary DIAG_LEVEL=1 timeout -k 10 200 python -u scripts/diag_deflate.py ) > gpurun_out/r05zd_diag_deflate_phases.log 2>&1 || { tail -20 gpurun_out/r05zd_diag_deflate_phases.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zd_diag_deflate_phases.log
