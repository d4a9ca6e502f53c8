#!/bin/bash
# per-stream inflater: cycles per token against message size (prof build)
set -o pipefail
mkdir -p gpurun_out
for sz in 1024 4096 16384; do
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 300 python -u scripts/diag_zstream.py 40 $sz > gpurun_out/r05q_diag_zstream_$sz.log 2>&1 || { tail -20 gpurun_out/r05q_diag_zstream_$sz.log; exit 2; }
head -12 gpurun_out/r05q_diag_zstream_$sz.log | grep -v amdgpu.ids
done
