#!/bin/bash
# A/B build: one source (SRC, default ba_chol_dag.hip) recompiled with extra -D switches, linked
# with the main build's other objects into tools/ubench/ab/liborbhip_<name>.so (probe it with
# ORBHIP_PROBE_LIB=... tools/probe_cholesky_dag.py, or load it as ORBHIP_LIB). Usage:
# [SRC=extract_kernels.hip] tools/build_ab.sh <name> -DX=0 ...
set -e
name=$1; shift
cd "$(dirname "$0")/../orb_slam3_ros2_amd/csrc"
out=../../tools/ubench/ab
mkdir -p $out/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math "$@" \
    -c ${SRC:-ba_chol_dag.hip} -o $out/$name/${SRC:-ba_chol_dag.hip}.o
objs=$(ls build/*.o | grep -v "build/${SRC:-ba_chol_dag.hip}" | grep -v "build/$(basename ${SRC:-ba_chol_dag.hip} .hip).o")
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o $out/liborbhip_$name.so $objs $out/$name/${SRC:-ba_chol_dag.hip}.o \
    -pthread -L/opt/rocm/lib -lrccl
echo built $out/liborbhip_$name.so
