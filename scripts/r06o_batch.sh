TAG=r06o bash scripts/gpu_round.sh "tests:test_gpu_inflate_bp or test_gpu_configs or 64_threads or test_gpu_stream or test_gpu_zstream" || exit 1
for v in nofx default fx3; do for L in 1 6; do if [ $v = default ]; then LB=$GRAFT_REPO_ROOT/beast_amd/libbeast_pmd.so; else LB=$GRAFT_REPO_ROOT/beast_amd/libbeast_pmd_$v.so; fi; echo "== $v L$L"; BPMD_LIB=$LB timeout -k 10 300 python -u scripts/diag_beast_shard.py c5 $L 8 3 2>&1 | grep -v amdgpu.ids | cut -c1-200 || exit 5; done; done
TAG=r06o THREADS="64" bash scripts/n2_sweep.sh || exit 6
TAG=r06o VARIANTS="default" LEGS=c5_l1,c5_l6,c4_l6 bash scripts/ab_legs.sh || exit 7
