# round-6 check: bp tests, then the C5 Beast shards (default and the pass-2-off variant)
TAG=r06r bash scripts/gpu_round.sh "tests:test_gpu_inflate_bp" || exit 1
for L in 1 6; do echo "== default L$L"; timeout -k 10 300 python -u scripts/diag_beast_shard.py c5 $L 8 3 2>&1 | grep -v amdgpu.ids | cut -c1-200 || exit 5; done
TAG=r06r bash scripts/prof_beast_shard.sh | grep -v rocprim | head -12
