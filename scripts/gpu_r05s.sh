#!/bin/bash
# per-stream inflater: wave-parallel inflate_fast -- parity, then where the time goes
set -o pipefail
TAG=${TAG:-r05s}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_stream.py tests/test_facade.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_zstream.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_zstream.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_zstream.log
for sz in 1024 16384; do
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 300 python -u scripts/diag_zstream.py 40 $sz > gpurun_out/${TAG}_diag_zstream_$sz.log 2>&1 || { tail -20 gpurun_out/${TAG}_diag_zstream_$sz.log; exit 2; }
head -12 gpurun_out/${TAG}_diag_zstream_$sz.log | grep -v amdgpu.ids
done
timeout -k 10 300 python -u scripts/facade_latency.py > gpurun_out/${TAG}_facade_latency.log 2>&1 || { tail -20 gpurun_out/${TAG}_facade_latency.log; exit 3; }
grep facade gpurun_out/${TAG}_facade_latency.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_c1_echo.log 2>&1 || { echo "c1 failed"; tail -20 gpurun_out/${TAG}_c1_echo.log; exit 4; }
grep "C1 echo" gpurun_out/${TAG}_c1_echo.log
