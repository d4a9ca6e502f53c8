#!/bin/bash
# C2 rocprof evidence + the default bench line (CPU baselines, C3, full C4/C5)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r02} bash scripts/profile.sh || { echo "profile failed rc=$?"; tail -20 gpurun_out/prof_${TAG:-r02}/err.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; tail -c 4000 gpurun_out/bench_full.json; tail -5 gpurun_out/bench_full.err; exit $rc
