#!/bin/bash
# Horner-form exact GEMM check on one GPU box: the linear/p_sample parity tests on the product build,
# then a same-process A/B (lab build): 14 = fold-form exact policy, -1 = product (Horner where the
# 256 x 256 grid fills the chip), 4 = rounded-weight policy.  Output under gpurun_out/horner/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/horner; mkdir -p $OUT
hard() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_diffusion.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "${PT_K:-linear or psample or denoise}" > $OUT/pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pt.log | tail -15
if hard $rc || [ $rc -ne 0 ]; then exit $rc; fi
DLLM_LIB=lab VARS=${VARS:-14,-1,4} timeout -k 10 300 python scripts/exact_lab.py ${SHAPES:-4096:4096 8192:4096 4096:8192 4300:4096} \
  > $OUT/ab.jsonl 2> $OUT/ab.err
rc2=$?; echo "ab rc=$rc2"; cat $OUT/ab.jsonl; tail -3 $OUT/ab.err
[ $rc2 -ne 0 ] && exit $rc2
# (optional) builds of the same ABI: LIBS=a.so,b.so
if [ -n "${LIBS:-}" ]; then
  LIBS=$LIBS SHAPES=${AB_SHAPES:-4096:4096,8192:4096} timeout -k 10 300 python scripts/gemm_ab.py > $OUT/libs_ab.jsonl 2> $OUT/libs_ab.err
  rc3=$?; echo "libs ab rc=$rc3"; cat $OUT/libs_ab.jsonl; tail -3 $OUT/libs_ab.err
fi
