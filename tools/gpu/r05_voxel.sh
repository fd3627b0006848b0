# round 5: the two-level voxel sort — its GPU tests, then rocprof kernel stats of the batched call for the
# round-start library and the new one, then FETCH/WRITE PMC passes of the new one
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_vox}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier_r.py -x -q --timeout 120 --timeout-method thread -k "voxel" \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 11; }
tail -2 $O/tests.log
R=$GRAFT_REPO_ROOT
for lib in tools/ablib/liblidar_eager.so lidar_ai_recommendation_software_amd/liblidar_amd.so; do
  t=$(basename $lib .so)
  (cd /tmp && export TMPDIR=/tmp && LIDAR_AMD_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$t -o p \
      -- python3 $R/tools/voxel_micro.py 32 0.05 > $R/$O/prof_$t.log 2>&1) || exit 12
done
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv \
     -d $R/$O/pmc_$c -o p -- python3 $R/tools/voxel_micro.py 32 0.05 > $R/$O/pmc_$c.log 2>&1) || exit 13
done
