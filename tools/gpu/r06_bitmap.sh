set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06/bitmap; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py tests/test_gpu_tier_r.py -q --timeout 300 --timeout-method thread -k "ball_query or bq or bench_shape or streaming or backbone or fused or radius" > $O/tests.log 2>&1 || exit 11
for rep in 1 2; do
for arm in base prod; do
if [ $arm = base ]; then L=$R/tools/ablib/base.so; else L=$R/lidar_ai_recommendation_software_amd/liblidar_amd.so; fi
LIDAR_AMD_LIB=$L timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-density --no-fp32-mfma-leg --no-standalone --no-cpu-baseline --no-host-feed --detail $O/d_${arm}_$rep.json > $O/b_${arm}_$rep.json 2> $O/b_${arm}_$rep.err || exit 12
python3 -c "
import json;d=json.load(open('$O/d_${arm}_$rep.json'));m=d['other_configs']['configs[4]_msg_131k_bf16'];c1=d['other_configs']['configs[1]_sa1_16k_f32']
print('$arm rep $rep ssg', round(d['value'],1), 'frac', round(d['roofline_grouped_mlp']['frac'],3), 'sa1', round(d['kernel_ms_per_launch']['sa1_group_mlp'],3), 'sa2q', round(d['kernel_ms_per_launch']['sa2_ball_query'],3), '| c1', round(c1['M_points_per_s'],1), '| msg', round(m['M_points_per_s'],1), {k:round(v,2) for k,v in m['chains_ms_per_group'].items()}, 'b2', round(m['kernel_ms_per_launch']['sa1_b2_group_mlp'],2), 'b1', round(m['kernel_ms_per_launch']['sa1_b1_group_mlp'],2), 'b0', round(m['kernel_ms_per_launch']['sa1_b0_group_mlp'],2))"
done
done
