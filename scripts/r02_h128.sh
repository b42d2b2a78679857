set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/h128
DLLM_LIB=lab VARS=14,-1 timeout -k 10 200 python scripts/exact_lab.py 2048:4096 4096:2048 1024:8192 > gpurun_out/h128/base.jsonl 2> gpurun_out/h128/base.err || exit $?
DLLM_LAB_HORNER128=1 DLLM_LIB=lab VARS=14,-1 timeout -k 10 200 python scripts/exact_lab.py 2048:4096 4096:2048 1024:8192 > gpurun_out/h128/h128.jsonl 2> gpurun_out/h128/h128.err
rc=$?; cat gpurun_out/h128/*.jsonl; tail -3 gpurun_out/h128/h128.err; exit $rc
