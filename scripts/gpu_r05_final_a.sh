#!/bin/bash
# round-5 final evidence, part A: the whole GPU suite, the C1 echo, and every
# bench leg's kernel trace + PMC passes (scripts/profile_legs.sh), on one build
set -o pipefail
TAG=${TAG:-r05zz}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_c1_echo.log 2>&1 || { echo "c1 failed"; tail -20 gpurun_out/${TAG}_c1_echo.log; exit 2; }
grep "C1 echo" gpurun_out/${TAG}_c1_echo.log
TAG=$TAG bash scripts/profile_legs.sh || { echo "profile_legs failed"; tail -20 gpurun_out/prof_$TAG/err.log; exit 3; }
ls gpurun_out/prof_$TAG/*_pmc.csv
