#!/bin/bash
# mkflag.sh <tag> <file.hip> <-Dflags...> : lib_<tag> = current objects with <file.hip> (working tree)
# recompiled with the extra flags (A/B of build switches)
set -e
cd "$(dirname "$0")/../event-camera-clustering-and-optical-flow-estimation_amd"
T=$1; F=$2; shift 2
rm -rf build_exp/f_$T lib_$T; mkdir -p build_exp/f_$T lib_$T
cp build/*.o build_exp/f_$T/
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -DECC_CORNER_PROFILE=0 -DECC_TRACKER_PROFILE=0 -DECC_ARC_PROFILE=0 -DECC_DBSCAN_PROFILE=0 -DECC_KM_ACC_SUB=4 -fhip-fp32-correctly-rounded-divide-sqrt -fvisibility=hidden -Icsrc -I../include"
/opt/rocm/bin/hipcc $FLAGS "$@" -c csrc/$F -o build_exp/f_$T/${F%.hip}.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib_$T/libecc.so build_exp/f_$T/*.o -lpthread
echo built lib_$T
