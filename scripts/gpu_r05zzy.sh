#!/bin/bash
# zstream: the dynamic header's code lengths wave-parallel (hdr_par + lenlens_par) -- parity, latency A/B, C1, phases
set -o pipefail
mkdir -p gpurun_out
T=r05zzy
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_stream.py tests/test_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
O=gpurun_out/${T}_lat.log
: > $O
for r in 1 2; do
  for hp in 1 0; do
    echo "== round $r hpar $hp" >> $O
    BPMD_ZSTREAM_HPAR=$hp timeout -k 10 120 python scripts/facade_latency.py 256 >> $O 2>&1 || { echo "lat failed"; tail $O; exit 2; }
  done
done
grep -E "==|facade per" $O
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${T}_c1_echo.log 2>&1 || { echo "c1 failed"; exit 3; }
grep "C1 echo" gpurun_out/${T}_c1_echo.log
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 120 python scripts/diag_zstream.py 32 1024 > gpurun_out/${T}_diag_zstream.log 2>&1 || { echo diag failed; exit 4; }
sed -n 3,6p gpurun_out/${T}_diag_zstream.log
