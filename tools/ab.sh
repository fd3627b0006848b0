#!/bin/bash
# A/B of library builds and/or bench.py argument sets on the SSG line: every arm in one GPU call,
# arms alternating within each repetition (box-to-box spread is ~6 %, so only same-call arms compare).
#
#   bash tools/ab.sh [-t PYTEST_K] [-c CAND.so] [-b "BASE ARGS"] OUTDIR REPS "arm 1" "arm 2" ...
#
# An arm is bench.py arguments, optionally led by VAR=value tokens: "LIDAR_AMD_LIB=tools/ablib/x.so
# --fps-threads 1024".  -c CAND.so: a candidate library (built beforehand on the CPU, e.g.
# make -C lidar_ai_recommendation_software_amd/csrc OUT=$PWD/tools/ablib/x.so BUILD=build_x
# HIPFLAGS="... -DOPTION") on which tests/test_gpu_tier_n.py runs first (-t: its -k filter).
# Each arm's full record lands in OUTDIR/armI_REP.detail.json; a one-line summary is printed.
set -o pipefail
TESTK=""; CAND=""
BASE="--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg --no-standalone --steps 20 --warmup 5"
while getopts "t:c:b:" opt; do
  case $opt in
    t) TESTK=$OPTARG ;;
    c) CAND=$OPTARG ;;
    b) BASE=$OPTARG ;;
    *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
O=$1; REPS=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$O"
if [ -n "$CAND" ]; then
  LIDAR_AMD_LIB=$CAND timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 \
      --timeout-method thread ${TESTK:+-k "$TESTK"} > "$O/tests.log" 2>&1 || exit 11
fi
for rep in $(seq 1 "$REPS"); do
  i=0
  for arm in "$@"; do
    i=$((i + 1))
    envs=(); args=()
    for tok in $arm; do
      if [[ ${#args[@]} -eq 0 && $tok == *=* && $tok != -* ]]; then envs+=("$tok"); else args+=("$tok"); fi
    done
    D=$O/arm${i}_$rep.detail.json
    timeout -k 10 300 env "${envs[@]}" python bench.py $BASE "${args[@]}" --detail "$D" \
        > "$O/arm${i}_$rep.json" 2> "$O/arm${i}_$rep.err" || exit 12
    python - "$D" "$arm" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
p = d["pipeline"]
print("[%s]" % sys.argv[2], "value %.1f" % d["value"], "ms/step %.3f" % d["ms_per_step"],
      "frac %.3f" % d["roofline_grouped_mlp"]["frac"],
      "side %.2f main %.2f G=%d" % (p["side_ms_per_group"], p["main_ms_per_group"], p["batches_per_group"]),
      {k: round(v, 3) for k, v in d["kernel_ms_per_launch"].items()}, flush=True)
if d.get("roofline_standalone"):
    print("   standalone", {k: (round(v["avg_launch_ms"], 3), round(v["frac"], 3))
                           for k, v in d["roofline_standalone"].items()}, flush=True)
PY
  done
done
