# 1024-thread SA1 FPS workgroups in the pipeline (--fps-threads 1024) vs the default 512, on the round-3 kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abf; mkdir -p $O
bash tools/ab_args.sh $O 3 "--steps 20 --warmup 5 --fps-threads 1024" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
