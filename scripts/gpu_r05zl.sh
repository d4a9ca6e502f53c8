#!/bin/bash
# per-stream inflater: pfast with the parallel replay -- parity, phases, latency, C1 (A/B vs the scalar replay)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zk}
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_zstream.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_zstream.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_zstream.log
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 300 python -u scripts/diag_zstream.py 40 1024 > gpurun_out/${TAG}_diag_zstream_1024.log 2>&1 || { tail -20 gpurun_out/${TAG}_diag_zstream_1024.log; exit 2; }
grep -E "whole call|pfast|outside|header" gpurun_out/${TAG}_diag_zstream_1024.log
for v in default; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L timeout -k 10 300 python -u scripts/facade_latency.py > gpurun_out/${TAG}_${v}_lat.log 2>&1 || { tail -5 gpurun_out/${TAG}_${v}_lat.log; exit 3; }
  echo "$v $(grep facade gpurun_out/${TAG}_${v}_lat.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_c1_echo.log 2>&1 || { tail -5 gpurun_out/${TAG}_c1_echo.log; exit 4; }
grep 'C1 echo' gpurun_out/${TAG}_c1_echo.log
