#!/bin/bash
# mkvar.sh <tag> <file.hip>... : lib_<tag> = current objects with the listed files from HEAD
set -e
cd "$(dirname "$0")/../event-camera-clustering-and-optical-flow-estimation_amd"
T=$1; shift
rm -rf build_exp/v_$T lib_$T; mkdir -p build_exp/v_$T/src lib_$T
cp build/*.o build_exp/v_$T/
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -DECC_CORNER_PROFILE=0 -DECC_TRACKER_PROFILE=0 -DECC_ARC_PROFILE=0 -DECC_DBSCAN_PROFILE=0 -DECC_KM_ACC_SUB=4 -fhip-fp32-correctly-rounded-divide-sqrt -fvisibility=hidden -Icsrc -I../include"
for f in "$@"; do
  git show HEAD:event-camera-clustering-and-optical-flow-estimation_amd/csrc/$f > build_exp/v_$T/src/$f
  /opt/rocm/bin/hipcc $FLAGS -c build_exp/v_$T/src/$f -o build_exp/v_$T/${f%.hip}.o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib_$T/libecc.so build_exp/v_$T/*.o -lpthread
echo built lib_$T
