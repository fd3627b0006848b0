#!/bin/bash
# Build an A/B variant of liblidar_amd.so with extra -D flags into ab/<name>/ (gitignored).
# usage: tools/ab_build.sh NAME "-DFLAG1 -DFLAG2"   then  LIDAR_AMD_LIB=ab/NAME/liblidar_amd.so python ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
D=$R/ab/$NAME; mkdir -p $D/build
C=$R/lidar_ai_recommendation_software_amd/csrc
objs=()
for f in $C/*.hip; do
  o=$D/build/$(basename ${f%.hip}).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-rdc -w $FLAGS -c $f -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/liblidar_amd.so "${objs[@]}"
echo "built $D/liblidar_amd.so"
