# voxel A/B over libraries: kernel stats + FETCH_SIZE / WRITE_SIZE passes of tools/voxel_micro.py per library
# usage: bash tools/gpu/r05_vox_ab.sh TAG lib1.so [lib2.so ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
for lib in "$@"; do
  t=$(basename $lib .so); mkdir -p $O/$t
  (cd /tmp && export TMPDIR=/tmp && LIDAR_AMD_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/$O/$t/prof -o p -- python3 $R/tools/voxel_micro.py ${B:-32} ${VOXEL:-0.05} ${SCALE:-1} ${N:-65536} > $R/$O/$t/prof.log 2>&1) || exit 12
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && LIDAR_AMD_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv \
       -d $R/$O/$t/pmc_$c -o p -- python3 $R/tools/voxel_micro.py ${B:-32} ${VOXEL:-0.05} ${SCALE:-1} ${N:-65536} > $R/$O/$t/pmc_$c.log 2>&1) || exit 13
  done
done
