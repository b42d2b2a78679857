#!/bin/bash
# Round-3 GPU pass: mid-M ring depth A/B (lab variants 300..302 = RING 3 / 4 / 8 against the
# product's 6), parity tests touching the changed policies, the attention priority check.
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
step pt 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "kv_attention or linear_policy or first_call or horner or mid_m or exact_weights or split_k or int4_shapes" &&
step ring3 200 python -u scripts/policy_ab.py 300 256 384 &&
step ring4 200 python -u scripts/policy_ab.py 301 256 384 &&
step ring8 200 python -u scripts/policy_ab.py 302 256 384 &&
step kg2 200 python -u scripts/policy_ab.py 14 1800 &&
step attn_ab 300 python -u scripts/attn_stag_ab.py 0 302
