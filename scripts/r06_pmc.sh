#!/bin/bash
# Round 6: SQ PMC passes of one kernel (regex $KRE) of library $LIB on shape $SHAPE (M:N, K 4096),
# each counter set in its own rocprofv3 run over scripts/kernel_times.py, into gpurun_out/$RECORD/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${RECORD:-r06_pmc}"; mkdir -p "$OUT"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
         ${EXTRA:-}; do
  i=$((i+1)); rm -rf /tmp/pmc_$i
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d /tmp/pmc_$i -o pmc --output-format csv -- python3 scripts/kernel_times.py $LIB $SHAPE > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  mkdir -p "$OUT/p$i"; find /tmp/pmc_$i -name "*counter_collection.csv" -exec cp {} "$OUT/p$i/" \;
done
python3 scripts/pmc_to_json.py "$OUT" "$OUT/pmc.json" "$KRE" ${SHAPE%%:*} 4096 ${SHAPE##*:} 4 128 ${REV:-r06}
