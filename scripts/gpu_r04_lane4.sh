#!/bin/bash
# lane4 bring-up: inflate parity in every kernel mode, then the C2 bench line.
set -o pipefail
TAG=${TAG:-r04b}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_inflate.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG}_inflate.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_inflate.log | head -30; exit 1; }
C2="--no-cpu-baseline --no-mixed --no-deflate --no-frame --no-exact"
timeout -k 10 200 python -u bench.py $C2 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err; rc=$?
echo "bench rc=$rc" >> gpurun_out/${TAG}_c2.err
[ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_c2.err; exit 2; }
tail -c 700 gpurun_out/${TAG}_c2.json
BPMD_INFLATE=lane3 timeout -k 10 200 python -u bench.py $C2 > gpurun_out/${TAG}_c2_lane3.json 2> gpurun_out/${TAG}_c2_lane3.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/${TAG}_c2_lane3.json'));print('lane3', d['value'], d['parity_ok'])"
