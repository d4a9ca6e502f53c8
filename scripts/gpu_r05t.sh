#!/bin/bash
# per-stream inflater: pfast phases (prof build)
set -o pipefail
TAG=${TAG:-r05t}
mkdir -p gpurun_out
for sz in 1024 16384; do
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 300 python -u scripts/diag_zstream.py 40 $sz > gpurun_out/${TAG}_diag_zstream_$sz.log 2>&1 || { tail -20 gpurun_out/${TAG}_diag_zstream_$sz.log; exit 2; }
head -14 gpurun_out/${TAG}_diag_zstream_$sz.log | grep -v amdgpu.ids
done
