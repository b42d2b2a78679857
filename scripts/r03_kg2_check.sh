#!/bin/bash
# Round-3 GPU pass for the KG2 Horner kernel (M = 2048 tiles), the attention priority A/B and the
# graph-captured 40-layer M-sweep: targeted parity tests (product build), lab A/Bs, the sweep.
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
step pt 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_diffusion.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread \
    -k "kv_attention or decode or linear_policy or first_call or horner or mid_m or exact_weights or full_size or diffusion or loop or c5" &&
step kg2_ab 300 python -u scripts/policy_ab.py 14 2048 1800 &&
step attn_ab 300 python -u scripts/attn_stag_ab.py &&
TAILN=40 step sweep 400 python -u bench.py --steps 10 --warmup 3 --sweep --no-cpu --no-denoise
