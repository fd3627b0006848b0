# density path: staged chunk rows for the index-order fp64 chains, candidate (-DLIDAR_SEQ_ROWS=2048, then 3072) against
# the product build (1024, then 2048), same box: the Tier R GPU tests on the candidate, then the bench's density leg alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abs; mkdir -p $O
CAND=$GRAFT_REPO_ROOT/tools/ablib/liblidar_cand.so
LIDAR_AMD_LIB=$CAND timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_r.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 11
for rep in 1 2; do
  for arm in cand prod; do
    if [ $arm = cand ]; then L=$CAND; else L=; fi
    LIDAR_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-extras --no-cpu-baseline --no-fp32-mfma-leg --no-standalone > $O/$arm$rep.json 2> $O/$arm$rep.err || exit 12
  done
done
