set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06/l1fuse; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -q --timeout 300 --timeout-method thread -k "fused_layer1 or msg or bf16" > $O/tests.log 2>&1 && timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -q --timeout 900 --timeout-method thread -k configs4 >> $O/tests.log 2>&1 || exit 11
for rep in 1 2; do
for arm in fuse nofuse; do
X=""; [ $arm = nofuse ] && X="--no-layer1-fuse"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-density --no-fp32-mfma-leg --no-standalone --no-cpu-baseline --no-host-feed $X --detail $O/d_${arm}_$rep.json > $O/b_${arm}_$rep.json 2> $O/b_${arm}_$rep.err || exit 12
python3 -c "
import json;d=json.load(open('$O/d_${arm}_$rep.json'));m=d['other_configs']['configs[4]_msg_131k_bf16'];k=m['kernel_ms_per_launch']
print('$arm rep $rep ssg', round(d['value'],1), '| msg', round(m['M_points_per_s'],1), {kk:round(v,2) for kk,v in m['chains_ms_per_group'].items()}, 'l1', round(k['sa2_layer1_points'],2), 'sa2', [round(k[x],2) for x in ('sa2_b0_group_mlp','sa2_b1_group_mlp','sa2_b2_group_mlp')])"
done
done
