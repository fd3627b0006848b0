# SA2 grouped MLP alone on the product library and on the LIDAR_SA_ABL diagnostic builds (tools/micro/sa2_ablate.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abl; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python tools/micro/sa2_ablate.py >> $O/abl.log 2>> $O/err.log || exit 11
  for a in 1 2 4 3 7; do
    ABL=$a LIDAR_AMD_LIB=$GRAFT_REPO_ROOT/tools/ablib/liblidar_abl$a.so timeout -k 10 120 python tools/micro/sa2_ablate.py >> $O/abl.log 2>> $O/err.log || exit 12
  done
done
