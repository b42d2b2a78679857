#!/bin/bash
# A/B of the fold-form exact kernel (128 x 256 tiles) against its Horner form (make variant VNAME=eh
# VFLAGS=-DDLLM_EXACT_HORNER=1): parity tests on the eh build, then scripts/gemm_ab.py on the C5 shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/eh; mkdir -p $OUT
EH=${EH:-diffusion-llm-rs_amd/lib/libdllm_hip_eh.so}
DLLM_LIB=$EH timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_diffusion.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "linear or psample or denoise" > $OUT/pt.log 2>&1
rc=$?; echo "pytest(eh) rc=$rc"; tail -3 $OUT/pt.log
[ $rc -ne 0 ] && exit $rc
LIBS=${LIBS:-diffusion-llm-rs_amd/lib/libdllm_hip.so,$EH} SHAPES=2048:4096,4096:2048,4096:4096 timeout -k 10 300 python scripts/gemm_ab.py > $OUT/ab.jsonl 2> $OUT/ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab.jsonl; exit $rc
