# round 4: bench A/B of library builds at the driver's settings, arms alternating within each rep:
#   bash tools/gpu/r04_ab.sh OUT REPS "name=LIB [bench args]" ...   (LIB "-": the in-tree library)
# optional: TESTS=1 runs the Tier N GPU tests on the in-tree library first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; REPS=$2; shift 2; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread > $O/tests_new.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
A="--no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --steps 20 --warmup 5"
for rep in $(seq 1 $REPS); do
  for arm in "$@"; do
    name=${arm%%=*}; rest=${arm#*=}; lib=${rest%% *}; extra=""; [ "$lib" != "$rest" ] && extra=${rest#* }
    if [ "$lib" = "-" ]; then unset LIDAR_AMD_LIB; else export LIDAR_AMD_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python bench.py $A $extra --detail $O/${name}_$rep.json > $O/${name}_$rep.log 2>&1 || exit 21
  done
done
