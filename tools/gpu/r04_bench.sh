# bench line at the driver's settings (+ the rocprof kernel summary of the same command), precision probe
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04b}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.log 2> $O/bench.err || exit 13
timeout -k 10 300 python -u tools/precision_probe.py > $O/precision.log 2>&1 || exit 12
