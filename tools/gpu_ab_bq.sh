# SA1 ball queries answered inside the fused MLP kernel (bq bin, the default) vs a separate grid-query launch on
# the side stream (bq side, the MLP-only kernel on the main stream), on the double-buffered kernels, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abq; mkdir -p $O
bash tools/ab_args.sh $O 3 "--steps 20 --warmup 5 --bq side" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
