#!/bin/bash
# zstream header: register-resident code-length table -- parity, latency, C1, phases
set -o pipefail
mkdir -p gpurun_out
T=r05zzp
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_stream.py tests/test_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 120 python scripts/facade_latency.py 256 > gpurun_out/${T}_lat.log 2>&1 || { echo lat failed; exit 2; }
grep facade gpurun_out/${T}_lat.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${T}_c1_echo.log 2>&1 || { echo "c1 failed"; exit 3; }
grep "C1 echo" gpurun_out/${T}_c1_echo.log
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 120 python scripts/diag_zstream.py 32 1024 > gpurun_out/${T}_diag_zstream.log 2>&1 || { echo diag failed; exit 4; }
sed -n 3,16p gpurun_out/${T}_diag_zstream.log
