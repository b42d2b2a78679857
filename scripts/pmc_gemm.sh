#!/bin/bash
# PMC passes (one counter set per pass) on the M=4096 ring GEMM: load-path diagnosis.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/pmcg"
mkdir -p "$OUT"
SETS=${PMC_SETS:-"TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum;TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum;TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum;TCC_HIT_sum TCC_MISS_sum;TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum;SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES;GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES;SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"}
IFS=';' read -ra SETARR <<< "$SETS"
for C in "${SETARR[@]}"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-wq_gemm8}" -d "$OUT/$tag" -o pmc --output-format csv -- python3 scripts/sweep.py ${SWEEP_M:-4096} > "$OUT/$tag.log" 2>&1
  rc=$?; echo "pmc $tag rc=$rc"
  case $rc in 0) ;; *) echo "stopping"; tail -5 "$OUT/$tag.log"; exit $rc;; esac
done
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.json"; cat "$OUT/summary.json"
