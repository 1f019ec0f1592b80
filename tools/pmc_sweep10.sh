#!/bin/bash
# PMC passes (one counter group per run) of the plane sweep at few depths: the LDS-staged
# depth-per-lane kernel (direct=-1) and the pixel-per-lane one (direct=2), or ROUTES, D = ${D:-10}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc10; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for dr in ${ROUTES:--1 2}; do
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
              "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
              "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE" \
              "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/d${dr}_$i" -o run \
      -- python3 -u "$ROOT/tools/pmc_sweep10.py" --D ${D:-10} --direct $dr > "$OUT/d${dr}_$i.log" 2>&1 \
      || { echo "pass $i direct $dr failed"; tail -3 "$OUT/d${dr}_$i.log"; exit 1; }
  done
  (timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/d${dr}_stats" -o run \
      -- python3 -u "$ROOT/tools/pmc_sweep10.py" --D ${D:-10} --direct $dr --iters 20 > "$OUT/d${dr}_stats.log" 2>&1) \
    || { echo "stats direct $dr failed"; exit 1; }
done
echo done
