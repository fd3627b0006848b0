# the Tier N GPU tests, then an A/B of SA2's per-centre layer-1 term on the side streams (--q-side 1 / 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 11
bash tools/ab.sh -b "--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg --steps 20 --warmup 5" $O/ab 3 \
    "--q-side 1" "--q-side 0" > $O/ab.log 2>&1 || exit 15
