#!/bin/bash
# tools/ab.py "libs" (the bench legs' default routes) alternating two library builds: $1 and the in-tree one
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for pass in 0 1; do
  for so in "$1" mpi_vision_amd/libmpiv.so; do
    n=$(basename $so .so)_p$pass
    MPIV_LIB=$(pwd)/$so timeout -k 10 200 python -u tools/ab.py --only libs --iters ${ITERS:-20} > $OUT/libs_$n.jsonl 2> $OUT/libs_$n.err \
      || { echo "$n failed"; tail -3 $OUT/libs_$n.err; exit 1; }
  done
done
echo done
