#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under its own limit) over any driver script:
#   tools/pmc_run.sh <out-name> <python script> [args...]   -> gpurun_out/<out-name>/p<k>/...
# then locally: python tools/pmc_table.py gpurun_out/<out-name> [kernel-substring]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); NAME=$1; shift; SCRIPT=$1; shift
OUT=$ROOT/gpurun_out/$NAME; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run \
    -- python3 -u "$ROOT/$SCRIPT" "$@" > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
done
echo "pmc passes done: $OUT"
