#!/bin/bash
# PMC passes (one counter group per run) for the plane-sweep kernel store modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcs; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for store in ${STORES:-lds tile}; do
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" \
              "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
              "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
              "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/s${store}_$i" -o run \
      -- python -u "$ROOT/tools/pmc_sweep.py" --store $store > "$OUT/s${store}_$i.log" 2>&1 \
      || { echo "pass $i store $store failed"; tail -3 "$OUT/s${store}_$i.log"; }
  done
done
echo done
