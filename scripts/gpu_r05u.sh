#!/bin/bash
# facade latency: idle GPU vs a spin kernel running on a side stream
set -o pipefail
TAG=${TAG:-r05u}
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/facade_latency.py > gpurun_out/${TAG}_facade_latency.log 2>&1 || { tail -20 gpurun_out/${TAG}_facade_latency.log; exit 3; }
BPMD_LAT_BUSY=8 timeout -k 10 300 python -u scripts/facade_latency.py >> gpurun_out/${TAG}_facade_latency.log 2>&1 || { tail -20 gpurun_out/${TAG}_facade_latency.log; exit 3; }
grep facade gpurun_out/${TAG}_facade_latency.log
