#!/bin/bash
# per-stream facade: per-phase cycles of the inflate and deflate kernels (prof build)
set -o pipefail
mkdir -p gpurun_out
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 300 python -u scripts/diag_zstream.py 72 > gpurun_out/r05o_diag_zstream.log 2>&1 || { tail -20 gpurun_out/r05o_diag_zstream.log; exit 1; }
cat gpurun_out/r05o_diag_zstream.log
