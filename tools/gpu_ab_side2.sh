set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abs2; mkdir -p $O
bash tools/ab_args.sh $O 1 "--steps 40 --warmup 5" "--steps 40 --warmup 5 --sa1-side 32" "--steps 20 --warmup 5 --sa1-side 32 --depth 4" "--steps 20 --warmup 5 --sa1-side 32 --slots 9" "--steps 20 --warmup 5 --sa1-side 64" > $O/ab.log 2>&1 || exit 12
