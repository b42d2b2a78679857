#!/bin/bash
# decode lab + bench profile (kernel trace + PMC) in one GPU call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/decode_lab.py > gpurun_out/decode_lab.jsonl 2> gpurun_out/decode_lab.err
rc=$?; echo "decode_lab rc=$rc"; cat gpurun_out/decode_lab.jsonl; tail -5 gpurun_out/decode_lab.err
[ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh
