#!/bin/bash
# level-dependent chunk history: parity, C4-shaped rate and size per level
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zi}
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_stream.py tests/test_gpu_reference_pins.py tests/test_facade.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_deflate.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_deflate.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_deflate.log
timeout -k 10 600 python -u scripts/deflate_levels.py 1 6 7 8 9 > gpurun_out/${TAG}_deflate_levels.log 2>&1 || { tail -10 gpurun_out/${TAG}_deflate_levels.log; exit 2; }
grep level gpurun_out/${TAG}_deflate_levels.log
