set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ff; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread -k "fps or streaming" > $O/tests.log 2>&1 || exit 11
bash tools/ab_args.sh $O 2 "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
