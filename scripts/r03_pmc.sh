#!/bin/bash
# PMC passes on the bench GEMM (M = K = N = 4096, the default kernel: wq_horner16_kernel): the SQ
# wait/issue breakdown, instruction mix, clock, and HBM traffic (FETCH_SIZE doubled per the gfx950
# calibration + WRITE_SIZE), each counter set in its own rocprofv3 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/pmc"; mkdir -p "$OUT"
KRE=${KREGEX:-wq_horner16_kernel}
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d "$OUT/p$i" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-denoise --prewarm-ms 0 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_to_json.py "$OUT" "$OUT/pmc_gemm.json" "$KRE" 4096 4096 4096 4 128 "${GEMM_REV:-r04-horner16b}"
