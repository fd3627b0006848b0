# voxel bucket kernel: rocprof kernel stats of diagnostic builds (wrong results by design)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_voxdiag}; shift
mkdir -p $O
R=$GRAFT_REPO_ROOT
for lib in "$@"; do
  t=$(basename $lib .so)
  (cd /tmp && export TMPDIR=/tmp && LIDAR_AMD_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/$O/prof_$t -o p -- python3 $R/tools/voxel_micro.py 32 0.05 > $R/$O/prof_$t.log 2>&1) || exit 12
  python3 - $R/$O/prof_$t $t <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'vx_' in r['Name']:
        print(sys.argv[2], r['Name'][:40], 'avg %.1f us' % (float(r['AverageNs']) / 1e3))
PY
done
