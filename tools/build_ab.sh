#!/bin/bash
# Build A/B variants of libmpiv.so into build/ab_<name>.so (selected at run time with
# MPIV_LIB=...; tools/gpu_ab_lib.sh or tools/ab.py).  Usage: tools/build_ab.sh name "-DFOO=1 -DBAR=2" ...
set -eu
cd "$(dirname "$0")/../mpi_vision_amd/csrc"
mkdir -p ../../build
while [ $# -ge 2 ]; do
  n=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize -Wall \
      -DMPIV_SRC_HASH=\"ab_$n\" $flags -o ../../build/ab_$n.so abi.hip &
done
wait
ls -la ../../build/
