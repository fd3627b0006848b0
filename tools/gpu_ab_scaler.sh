# density path A/B, product vs tools/ablib/liblidar_cand.so (used for: the StandardScaler second pass split; the emulated
# chains' scan without scratch arrays or per-row branches), same box:
# the Tier R GPU tests on the product, then the bench's density leg alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/absc; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/tools/ablib/liblidar_cand.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_r.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 11
for rep in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then L=$BASE; else L=; fi
    LIDAR_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-extras --no-cpu-baseline --no-fp32-mfma-leg --no-standalone > $O/$arm$rep.json 2> $O/$arm$rep.err || exit 12
  done
done
LIDAR_AMD_LIB=$GRAFT_REPO_ROOT/lidar_ai_recommendation_software_amd/liblidar_amd_diag.so timeout -k 10 120 python tools/micro/pre_phases.py > $O/phases.log 2>&1 || exit 13
