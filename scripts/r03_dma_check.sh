#!/bin/bash
# Round-3 lab pass: Horner GEMM DMA-issue ablations (26 = no stores; 303 = + no X DMA; 304 = + no
# DMA at all) and the mid-M two-k-group tile A/B (300).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {   # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -${TAILN:-12} "gpurun_out/$name.log"
    return $rc
}
step dma_ab 300 python -u scripts/horner_ab.py -1 26 303 304 &&
step midkg2 200 python -u scripts/policy_ab.py 300 256 384
