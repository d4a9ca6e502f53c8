#!/bin/bash
# product-build kernel durations of the facade's per-message calls (C1 shape)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05zzh_prof -o lat -- python scripts/facade_latency.py 256 > gpurun_out/r05zzh_lat.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r05zzh_lat.log; exit 1; }
find gpurun_out/r05zzh_prof -name "*kernel_stats.csv" | head -3
