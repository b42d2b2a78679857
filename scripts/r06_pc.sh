#!/bin/bash
# Round 6: the producer/consumer Horner kernel (linear_pc.hip) -- parity tests on the 128 x 256 grids,
# then an interleaved A/B against the round-5 product (lib/libdllm_hip_base.so) on one box.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${RECORD:-r06_pc}; mkdir -p $OUT
hard() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_diffusion.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  -k "${TESTK:-policy_exact_integers or exact_weights_tight or horner_scale_spread or mid_m_paths or full_size_vs_torch or psample_fused or config5_per_step or overlap_bit_identical}" \
  > $OUT/pytest.txt 2>&1
r=$?; echo "pytest rc=$r"; tail -3 $OUT/pytest.txt
if hard $r; then exit $r; fi
LIBS=${LIBS:-diffusion-llm-rs_amd/lib/libdllm_hip_base.so,diffusion-llm-rs_amd/lib/libdllm_hip.so} \
SHAPES=${SHAPES:-2048:4096,4096:2048,3072:4096} ROUNDS=${ROUNDS:-3} \
  timeout -k 10 400 python scripts/gemm_ab.py > $OUT/ab.jsonl 2> $OUT/ab.err
r=$?; echo "ab rc=$r"; cat $OUT/ab.jsonl
exit $r
