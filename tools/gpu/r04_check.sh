# whole GPU suite, smoke, bench line at the driver's settings, precision probe
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04c}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA > $O/tests.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 14
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.log 2> $O/bench.err || exit 13
timeout -k 10 300 python -u tools/precision_probe.py > $O/precision.log 2>&1 || exit 12
