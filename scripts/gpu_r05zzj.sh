#!/bin/bash
# which HIP calls the e2e pipeline's per-chunk batch calls make (32 chunks)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d gpurun_out/r05zzj_prof -o e2e -- python scripts/e2e.py --chunks 32 --depth 4 --reps 2 > gpurun_out/r05zzj_e2e.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r05zzj_e2e.log; exit 1; }
find gpurun_out/r05zzj_prof -name "*stats.csv"
