#!/bin/bash
# Round-3 GPU pass for the staggered attention schedule, the Horner-GEMM ablations and the
# 40-layer M-sweep: targeted parity tests (product build), then lab A/Bs, then the sweep.
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
step pt 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "kv_attention or decode or linear_policy or first_call" &&
step attn_ab 300 python -u scripts/attn_stag_ab.py &&
TAILN=40 step sweep 400 python -u bench.py --steps 10 --warmup 3 --sweep --no-cpu --no-denoise
