# CU-masked FPS side streams (main stream unrestricted) vs the default pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab3; mkdir -p $O
S="--steps 20 --warmup 5"
bash tools/ab_args.sh $O 2 "$S" "$S --fps-threads 1024 --side-cus 128" "$S --fps-threads 1024 --side-cus 96" \
  "$S --side-cus 128" "$S --fps-threads 1024 --side-cus 128 --side-layout stride" "$S --fps-threads 1024 --side-cus 160" > $O/ab.log 2>&1 || exit 15
