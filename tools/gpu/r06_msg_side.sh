set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06/msgside; mkdir -p $O; cd $R
for rep in 1 2; do
for ns in 0 128 32; do
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-density --no-fp32-mfma-leg --no-standalone --no-cpu-baseline --no-host-feed --msg-side-ns $ns --detail $O/d_${ns}_$rep.json > $O/b_${ns}_$rep.json 2> $O/b_${ns}_$rep.err || exit 11
python3 -c "
import json,sys;d=json.load(open('$O/d_${ns}_$rep.json'));m=d['other_configs']['configs[4]_msg_131k_bf16'];print('side_ns $ns rep $rep', round(m['M_points_per_s'],1), {k:round(v,2) for k,v in m['chains_ms_per_group'].items()}, {k:round(v,2) for k,v in m['kernel_ms_per_launch'].items()})"
done
done
