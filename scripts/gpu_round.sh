#!/bin/bash
# One GPU call = a list of steps, each under its own time limit; the first
# failing step ends the call (no retries).  Replaces the per-experiment
# gpu_r0*.sh scripts of rounds 1-5.
#
# Usage: TAG=r06a bash scripts/gpu_round.sh STEP [STEP ...]
#   suite        the whole GPU test suite            -> gpurun_out/<TAG>_pytest_gpu.log
#   tests:<k>    GPU tests whose node id matches <k>  -> gpurun_out/<TAG>_pytest_<k>.log
#   c1           the C1 loopback echo                -> gpurun_out/<TAG>_c1_echo.log
#   bench        the default bench line              -> gpurun_out/<TAG>_bench.json
#   c2           C2 inflate only, 10 steps           -> gpurun_out/<TAG>_c2.json
#   ab           interleaved A/B of library variants on C2: VARIANTS="a b" ROUNDS=3
#                (a variant v is beast_amd/libbeast_pmd_<v>.so; "default" is the product)
#   prof         C2 rocprofv3 kernel trace + FETCH/WRITE + calibration (scripts/profile.sh)
#   legs         every other leg's kernel trace + PMC (scripts/profile_legs.sh)
#   sq           C2 SQ counters (scripts/pmc_sq.sh)  -> gpurun_out/<TAG>_c2_sq.txt
#   tcc          C2 and C4 L2 hit/miss + request counters -> gpurun_out/tcc_<TAG>/
#   diag         lane-kernel loop counters (prof build) -> gpurun_out/<TAG>_diag_lane3.txt
#   e2e          PCIe-inclusive rates                -> gpurun_out/<TAG>_e2e.json
#   shards       one 8-way shard's kernels per leg   -> gpurun_out/<TAG>_shards.log
#   bshard       one 8-way shard of C5 Beast payloads, L1 and L6, kernel trace -> gpurun_out/prof_bshard_<TAG>/
#   n2           the N2 harness at 64 threads, 1 and 16 KiB, GPU and CPU codec -> gpurun_out/<TAG>_n2_sweep.log
#   py:<script>  python scripts/<script> (args in PY_ARGS) -> gpurun_out/<TAG>_<script>.log
# Companions run on their own: scripts/ab_legs.sh (A/B of library variants on the
# C4 / C5 legs), scripts/ktrace.sh (C2-only kernel trace), scripts/prof_n2.sh (N2
# harness under rocprofv3 with the HIP API trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06}
mkdir -p gpurun_out
step() { echo "== $TAG $1 ($(date +%T))"; }
for s in "$@"; do
  case $s in
    suite)
      step suite
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 11; }
      tail -2 gpurun_out/${TAG}_pytest_gpu.log ;;
    tests:*)
      k=${s#tests:}; step "tests $k"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "$k" --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_pytest_${k//[^A-Za-z0-9_]/_}.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_${k//[^A-Za-z0-9_]/_}.log; exit 12; }
      tail -3 gpurun_out/${TAG}_pytest_${k//[^A-Za-z0-9_]/_}.log ;;
    c1)
      step c1
      timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread \
        > gpurun_out/${TAG}_c1_echo.log 2>&1 || { tail -20 gpurun_out/${TAG}_c1_echo.log; exit 13; }
      grep "C1 echo" gpurun_out/${TAG}_c1_echo.log ;;
    bench)
      step bench
      bash scripts/run_bench.sh ${TAG}_bench 900 "d['value'], d['parity_ok']" || exit 14
      wc -c gpurun_out/${TAG}_bench.json ;;
    c2)
      step c2
      bash scripts/run_bench.sh ${TAG}_c2 300 "d['value'], d['roofline']['kernel_ms'], d['parity_ok']" \
        --steps 10 --warmup 2 --no-cpu-baseline --no-mixed --no-deflate --no-frame --no-exact || exit 15 ;;
    ab)
      step "ab ${VARIANTS}"
      for r in $(seq ${ROUNDS:-3}); do
        for v in ${VARIANTS:-default}; do
          if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
          BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_ab_${v}_$r 300 \
            "'$v', d['value'], d['roofline']['kernel_ms'], d['parity_ok'], d.get('north_star',{}).get('c3',{}).get('deflate')" \
            --steps 10 --warmup 2 --no-cpu-baseline --no-mixed --no-frame --no-exact ${AB_ARGS} || exit 16
        done
      done ;;
    prof)
      step prof
      TAG=$TAG bash scripts/profile.sh || { tail -20 gpurun_out/prof_$TAG/err.log; exit 17; } ;;
    legs)
      step legs
      TAG=$TAG bash scripts/profile_legs.sh ${LEGS} || { tail -20 gpurun_out/prof_$TAG/err.log; exit 18; } ;;
    sq)
      step sq
      TAG=$TAG BENCH_ARGS="--no-mixed --no-deflate --no-frame --no-exact" bash scripts/pmc_sq.sh || exit 19
      python scripts/sq_summary.py gpurun_out/sq_$TAG > gpurun_out/${TAG}_c2_sq.txt && cat gpurun_out/${TAG}_c2_sq.txt ;;
    tcc)
      step tcc
      TAG=$TAG bash scripts/pmc_tcc.sh || exit 20 ;;
    diag)
      step diag
      python beast_amd/build.py prof > /dev/null || exit 21
      timeout -k 10 300 python -u scripts/diag_lane3.py > gpurun_out/${TAG}_diag_lane3.txt 2>&1 || { tail -20 gpurun_out/${TAG}_diag_lane3.txt; exit 21; }
      cat gpurun_out/${TAG}_diag_lane3.txt ;;
    e2e)
      step e2e
      timeout -k 10 300 python -u scripts/e2e.py > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 22; }
      cat gpurun_out/${TAG}_e2e.json ;;
    shards)
      step shards
      TAG=$TAG bash scripts/prof_shards.sh > gpurun_out/${TAG}_shards.log 2>&1 || { tail -10 gpurun_out/${TAG}_shards.log; exit 23; } ;;
    bshard)
      step bshard
      for L in 1 6; do TAG=$TAG LEVEL=$L bash scripts/prof_beast_shard.sh > gpurun_out/${TAG}_bshard_l$L.log 2>&1 || { tail -10 gpurun_out/${TAG}_bshard_l$L.log; exit 25; }; head -6 gpurun_out/${TAG}_bshard_l$L.log | cut -c1-160; done ;;
    n2)
      step n2
      TAG=$TAG THREADS="${THREADS:-64}" bash scripts/n2_sweep.sh || exit 26 ;;
    py:*)
      sc=${s#py:}; step "py $sc"
      timeout -k 10 ${PY_TIMEOUT:-300} python -u scripts/$sc $PY_ARGS > gpurun_out/${TAG}_${sc%.py}.log 2>&1 || { tail -30 gpurun_out/${TAG}_${sc%.py}.log; exit 24; }
      tail -${PY_TAIL:-30} gpurun_out/${TAG}_${sc%.py}.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== $TAG done ($(date +%T))"
