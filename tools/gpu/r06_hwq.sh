set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06/hwq; mkdir -p $O; cd $R
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python -u tools/micro/queue_probe.py 12 > $O/probe8.log 2>&1 || exit 10
for rep in 1 2; do
for arm in "0 3" "8 3" "8 4" "8 5"; do
set -- $arm
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-density --no-fp32-mfma-leg --no-standalone --no-cpu-baseline --no-host-feed --hw-queues $1 --depth $2 --msg-depth $2 --detail $O/d_$1_$2_$rep.json > $O/b_$1_$2_$rep.json 2> $O/b_$1_$2_$rep.err || exit 11
python3 -c "
import json;d=json.load(open('$O/d_$1_$2_$rep.json'));m=d['other_configs']['configs[4]_msg_131k_bf16'];p=d['pipeline']
print('hwq $1 depth $2 rep $rep ssg', round(d['value'],1), 'frac', round(d['roofline_grouped_mlp']['frac'],3), 'main', round(p['main_ms_per_group'],2), 'side', round(p['side_ms_per_group'],2), 'fps', round(d['kernel_ms_per_launch']['sa1_fps'],2), '| msg', round(m['M_points_per_s'],1), {k:round(v,2) for k,v in m['chains_ms_per_group'].items()})"
done
done
