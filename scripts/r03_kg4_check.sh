#!/bin/bash
# Round-3 pass: mid-M k-group A/B (product = two k-groups; 300 one k-group, 301 / 302 four k-groups
# with a 2- / 3-stage ring) and the parity tests of the exact policy grid.
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
step pt 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "linear_policy or mid_m or split_k or int4_shapes or exact_weights or first_call" &&
step kg1 200 python -u scripts/policy_ab.py 300 256 320 384 448 &&
step kg4r2 200 python -u scripts/policy_ab.py 301 256 384 &&
step kg4r3 200 python -u scripts/policy_ab.py 302 256 384 &&
step dec16 300 python -u scripts/decode_ab.py 306 1 16 32
