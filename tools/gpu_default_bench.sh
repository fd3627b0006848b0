# the bench with no flags (its defaults: 240 steps), as a driver run without arguments would see it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/def
timeout -k 10 900 python bench.py > gpurun_out/def/bench.json 2> gpurun_out/def/bench.err || exit 11
