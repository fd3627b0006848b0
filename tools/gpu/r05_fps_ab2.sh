# round 5: lazy FPS with LDS bucket records — tests, FPS alone (eager vs lazy), PMC traffic of one
# 128-frame FPS launch per library, then the SSG line A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_fps2}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread \
    -k "fps or nested or streaming or bench_shape" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
for lib in tools/ablib/liblidar_eager.so lidar_ai_recommendation_software_amd/liblidar_amd.so tools/ablib/liblidar_lazyk1.so; do
  echo "== $lib alone"
  LIDAR_AMD_LIB=$lib timeout -k 10 120 python tools/fps_scale.py 512 128,384 || exit 12
done
R=$GRAFT_REPO_ROOT
for lib in tools/ablib/liblidar_eager.so lidar_ai_recommendation_software_amd/liblidar_amd.so; do
  t=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && LIDAR_AMD_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv \
       -d $R/$O/pmc_${t}_$c -o p -- python3 $R/tools/fps_pmc.py 128 512 > $R/$O/pmc_${t}_$c.log 2>&1) || exit 13
  done
done
bash tools/ab.sh $O 2 "LIDAR_AMD_LIB=tools/ablib/liblidar_eager.so" "" "LIDAR_AMD_LIB=tools/ablib/liblidar_lazyk1.so"
