set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fw3; mkdir -p $O
bash tools/ab_args.sh $O 1 "--steps 20 --warmup 5 --fps-threads 0" "--steps 20 --warmup 5 --fps-threads 512" > $O/ab.log 2>&1 || exit 13
