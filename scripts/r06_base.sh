set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_base; mkdir -p $OUT
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench.jsonl 2> $OUT/bench.err || exit $?
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so SHAPES=4096:4096,2048:4096,4096:2048,4096:1024,4096:512 ROUNDS=2 \
  timeout -k 10 300 python scripts/gemm_ab.py > $OUT/shapes.jsonl 2> $OUT/shapes.err
