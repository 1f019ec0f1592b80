#!/bin/bash
# PMC passes (one counter group per run) for both render variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcr; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
V=${V:-8}
for variant in ${VARIANTS:-mv direct}; do
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
              "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
              "SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE" \
              "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
              "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/${variant}_$i" -o run \
      -- python -u "$ROOT/tools/pmc_render.py" --variant $variant --views $V > "$OUT/${variant}_$i.log" 2>&1 \
      || { echo "pass $i $variant failed"; tail -3 "$OUT/${variant}_$i.log"; }
  done
done
echo done
