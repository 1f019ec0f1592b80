#!/bin/bash
# Render-backward A/B across build/ab_*.so (tools/build_ab.sh) + SQ PMC passes of the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for so in $(ls build/ab_*.so 2>/dev/null); do
  n=$(basename $so .so)
  MPIV_LIB=$(pwd)/$so timeout -k 10 200 python -u tools/ab.py --only ${ONLY:-bwd} > $OUT/$n.jsonl 2> $OUT/$n.err \
    || { echo "$n failed"; tail -3 $OUT/$n.err; exit 1; }
  echo "== $n"; cat $OUT/$n.jsonl
done
[ "${PMC:-0}" = 1 ] || exit 0
ROOT=$(pwd); P=$ROOT/$OUT/pmcb; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$P/p$i" -o run \
    -- python3 -u "$ROOT/tools/pmc_bwd.py" > "$P/p$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$P/p$i.log"; exit 1; }
done
echo pmc done
