# round 4: (1) the Tier N GPU tests on the current library, (2) bench A/B of the round-start library
# (tools/ablib/liblidar_head.so) against the current one, (3) the main-chain skip probes on the
# round-start library, (4) its evidence run (tests, bench, rocprof, PMC: tools/profile_round.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04a}; mkdir -p $O
HEAD_LIB=$GRAFT_REPO_ROOT/tools/ablib/liblidar_head.so
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }  # test failures go on; faults / timeouts stop
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread > $O/tests_new.log 2>&1; ok $?
A="--no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone --steps 20 --warmup 5"
for rep in 1 2; do
  LIDAR_AMD_LIB=$HEAD_LIB timeout -k 10 300 python bench.py $A --detail $O/ab_head_$rep.json > $O/ab_head_$rep.log 2>&1 || exit 21
  timeout -k 10 300 python bench.py $A --detail $O/ab_new_$rep.json > $O/ab_new_$rep.log 2>&1 || exit 22
done
P="--no-verify $A"
for arm in none l1 dense1 l1+dense1; do
  LIDAR_AMD_LIB=$HEAD_LIB timeout -k 10 300 python tools/skip_probe.py $arm $P --detail $O/skip_$arm.json > $O/skip_$arm.log 2>&1 || exit 31
done
export LIDAR_AMD_LIB=$HEAD_LIB
bash tools/profile_round.sh ${1:-r04a} tests || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 30
