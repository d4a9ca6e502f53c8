#!/bin/bash
# per-stream inflater: where a fast-loop token's cycles go (laps build)
set -o pipefail
mkdir -p gpurun_out
BPMD_LIB=beast_amd/libbeast_pmd_laps.so timeout -k 10 300 python -u scripts/diag_zstream.py 40 4096 > gpurun_out/r05r_diag_zstream_laps.log 2>&1 || { tail -20 gpurun_out/r05r_diag_zstream_laps.log; exit 2; }
head -20 gpurun_out/r05r_diag_zstream_laps.log | grep -v amdgpu.ids
