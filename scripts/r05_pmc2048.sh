#!/bin/bash
# Round 5: PMC passes on the C5 layer GEMM (M 2048 x K 4096 x N 4096: wq_gemm_exact_kernel, the
# staggered 128 x 256 tiles), each counter set in its own rocprofv3 run over scripts/kernel_times.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05_pmc2048"; mkdir -p "$OUT"
KRE=wq_gemm_exact_kernel
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1)); rm -rf /tmp/pmc2048_$i
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d /tmp/pmc2048_$i -o pmc --output-format csv -- python3 scripts/kernel_times.py diffusion-llm-rs_amd/lib/libdllm_hip.so 2048:4096 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  mkdir -p "$OUT/p$i"; find /tmp/pmc2048_$i -name "*counter_collection.csv" -exec cp {} "$OUT/p$i/" \;
done
python3 scripts/pmc_to_json.py "$OUT" "$OUT/pmc_gemm_2048.json" "$KRE" 2048 4096 4096 4 128 r05-exact-stag
