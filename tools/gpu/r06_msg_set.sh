set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06/msgset; mkdir -p $O; cd $R
for rep in 1 2; do
for st in "3 3 30" "2 3 30" "4 3 30" "3 2 30" "3 5 30" "2 2 30"; do
set -- $st
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-density --no-fp32-mfma-leg --no-standalone --no-cpu-baseline --no-host-feed --msg-depth $1 --msg-group $2 --msg-steps $3 --detail $O/d_$1_$2_$rep.json > $O/b_$1_$2_$rep.json 2> $O/b_$1_$2_$rep.err || exit 11
python3 -c "
import json,sys;d=json.load(open('$O/d_$1_$2_$rep.json'));m=d['other_configs']['configs[4]_msg_131k_bf16'];print('depth $1 G $2 rep $rep', round(m['M_points_per_s'],1), {k:round(v,2) for k,v in m['chains_ms_per_group'].items()}, 'sa1_fps', round(m['kernel_ms_per_launch']['sa1_fps'],2))"
done
done
