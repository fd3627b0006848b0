set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06/host; mkdir -p $O; cd $R
for rep in 1 2; do
for t in 4 8 16; do
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-density --no-fp32-mfma-leg --no-standalone --no-cpu-baseline --no-extras --host-threads $t --detail $O/d_${t}_$rep.json > $O/b_${t}_$rep.json 2> $O/b_${t}_$rep.err || exit 12
python3 -c "
import json;d=json.load(open('$O/d_${t}_$rep.json'));print('threads $t rep $rep ssg', round(d['value'],1), 'host', round(d['ssg_host_feed']['value'],1))"
done
done
