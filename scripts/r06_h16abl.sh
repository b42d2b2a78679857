#!/bin/bash
# Round 6: the headline kernel's ceiling by ablation -- lab build, M = K = N = 4096:
# -1 product, 340 no Horner rescale, 341 no rescale + A fragments built once (no loop VALU besides
# the MFMAs' B reads), 342 no DMA after the prologue, 343 MFMAs + LDS reads + barriers only.
# HIP-event A/B in one process, then one PMC pass (clock and MFMA busy per variant).  Timing only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_h16abl
mkdir -p $OUT
DLLM_LIB=lab timeout -k 10 300 python3 scripts/horner_ab.py -1 340 341 342 343 > $OUT/ab.json 2> $OUT/ab.err || { echo "ab failed"; tail -5 $OUT/ab.err; exit 1; }
cat $OUT/ab.json
DLLM_LIB=lab timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace \
  --kernel-include-regex wq_horner16 -d $OUT/pmc -o pmc --output-format csv -- python3 scripts/horner_ab.py -1 340 341 342 343 > $OUT/pmc.log 2>&1
echo "pmc rc=$?"
