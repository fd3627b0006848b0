# same-box A/B of the round-3 FPS / chain changes against the round-start library
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab2; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/tools/ablib/liblidar_base.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier_r.py -x -q --timeout 120 --timeout-method thread > $O/tests_r.log 2>&1 || exit 11
for lib in base new; do
  if [ $lib = base ]; then export LIDAR_AMD_LIB=$BASE; else unset LIDAR_AMD_LIB; fi
  echo "== $lib" >> $O/fps.log
  timeout -k 10 200 python tools/fps_scale.py 1024,512 128 >> $O/fps.log 2>&1 || exit 12
  timeout -k 10 200 python tools/tier_r_leg.py >> $O/tier_r.log 2>&1 || exit 14
done
unset LIDAR_AMD_LIB
timeout -k 10 120 python tools/micro/fps_phases.py 128 > $O/phases.log 2>&1 || exit 13
timeout -k 10 120 python tools/micro/fps_phases.py 16 >> $O/phases.log 2>&1 || exit 13
bash tools/ab_args.sh $O 2 "LIDAR_AMD_LIB=$BASE --steps 20 --warmup 5" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 15
