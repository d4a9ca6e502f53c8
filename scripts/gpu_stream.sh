#!/bin/bash
# per-stream inflater + facade / C1 echo tests on the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream_resume.py tests/test_gpu_stream.py tests/test_facade.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_stream.log 2>&1
rc=$?; tail -40 gpurun_out/pytest_stream.log; exit $rc
