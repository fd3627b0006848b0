#!/bin/bash
# A/B/... of bench.py argument sets on the SSG line, all arms in one GPU call, alternating:
#   bash tools/ab_args.sh OUTDIR REPS "arm1 args" "arm2 args" ...   (an arm may start with VAR=value)
set -o pipefail
O=$1; REPS=$2; shift 2
mkdir -p $O
BASE=${AB_BASE:-"--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg --no-standalone"}
for rep in $(seq 1 $REPS); do
  i=0
  for arm in "$@"; do
    i=$((i + 1))
    envs=(); args=()
    for tok in $arm; do
      if [[ ${#args[@]} -eq 0 && $tok == *=* && $tok != -* ]]; then envs+=("$tok"); else args+=("$tok"); fi
    done
    timeout -k 10 300 env "${envs[@]}" python bench.py $BASE "${args[@]}" > $O/arm${i}_$rep.json 2> $O/arm${i}_$rep.err || exit 1
    python - $O/arm${i}_$rep.json "$arm" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d["pipeline"]
print("[%s]" % sys.argv[2], "value %.1f" % d["value"], "ms/step %.3f" % d["ms_per_step"],
      "frac %.3f" % d["roofline_grouped_mlp"]["frac"],
      "side %.2f main %.2f G=%d" % (p["side_ms_per_group"], p["main_ms_per_group"], p["batches_per_group"]),
      {k: round(v, 3) for k, v in d["kernel_ms_per_launch"].items()}, flush=True)
if d.get("roofline_standalone"):
    print("   standalone", {k: (round(v["avg_launch_ms"], 3), round(v["frac"], 3)) for k, v in d["roofline_standalone"].items()},
          flush=True)
PY
  done
done
