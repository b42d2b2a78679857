#!/bin/bash
# Round-4 measurement batch (one gpurun call): each GPU step under its own timeout; a hard failure
# (abort, segfault, timeout) stops the batch.  Output under gpurun_out/r04_batch/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04_batch
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "step $name rc=$rc"; tail -c 400 $O/$name.out; echo
  case $rc in 124|134|137|139) echo "hard failure in $name; stopping"; exit $rc;; esac
  return 0
}
for s in ${STEPS:-tests chain quant horner shard}; do
  case $s in
    tests) step tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "${TESTK:-policy_exact or decode or psample or split_k or quantize_kv or resident}";;
    chain) step chain 200 python scripts/chain_ab.py
           DLLM_LIB=lab DLLM_DECODE_REDUCE_LAUNCH=1 step chain_launch 200 python scripts/chain_ab.py;;
    quant) step quant 150 python scripts/quant_kv_ab.py
           DLLM_LIB=lab DLLM_QUANT_RESIDENT=1 step quant_resident 150 python scripts/quant_kv_ab.py;;
    res) for m in 0 4 12; do
           DLLM_LIB=lab DLLM_QUANT_RESIDENT=1 DLLM_RES_LAB=$m step res_$m 150 python scripts/quant_kv_ab.py
         done;;
    ablate) step ablate 300 python scripts/horner_ab.py -1 316 26 305 318 317 314 315;;
    horner) step horner 200 python scripts/horner_ab.py -1 310 311 312
            for v in -1 310 311 312; do
              step pmc_fetch_$v 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex wq_horner -d $O/pmc_fetch_$v -o pmc --output-format csv -- python scripts/horner_ab.py $v
            done;;
    clock) for v in ${CLOCKV:--1 314 315 305 317}; do
             step clk_$v 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex wq_horner -d $O/clk_$v -o pmc --output-format csv -- python scripts/horner_ab.py $v
           done;;
    clkshard) i=0
           for C in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" "FETCH_SIZE" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
             i=$((i+1))
             LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so ROUNDS=1 SHAPES=${CSHAPES:-4096:1024,4096:512,4096:4096} step clkshard_$i 120 rocprofv3 --pmc $C --kernel-include-regex "wq_gemm_exact|wq_horner" -d $O/clkshard_$i -o pmc --output-format csv -- python scripts/gemm_ab.py
           done;;
    shape) step shape 200 python scripts/horner_ab.py -1 319 314 320;;
    h128) AB_M=2048 step h128 200 python scripts/horner_ab.py -1 323 -1 323
          AB_M=3000 step h128_3000 120 python scripts/horner_ab.py -1 323
          AB_M=4096 AB_N=2048 step h128_shard2 120 python scripts/horner_ab.py -1 323
;;
    h16) step h16 200 python scripts/horner_ab.py -1 328 -1 328 -1 328;;
    blas) step blas 120 python scripts/blas_shapes.py
          LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so ROUNDS=2 step shard_ab 200 python scripts/gemm_ab.py;;
    tp) DLLM_BENCH_BACKEND=gloo step tp_trace 400 rocprofv3 --kernel-trace -d $O/tp -o kt --output-format csv -- python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --tp-steps 4 --no-cpu;;
    tpstep) DLLM_BENCH_BACKEND=gloo step tp_step 300 rocprofv3 --kernel-trace -d $O/tpstep -o kt --output-format csv -- python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 scripts/tp_step_trace.py
            for f in $(ls $O/tpstep/*kernel_trace.csv 2>/dev/null); do python scripts/tp_step_trace.py --analyze $f > $O/tp_step_kernels.json; done;;
    pmcm) for m in 64 256; do
            k=$([ $m -le 64 ] && echo wq_decode || echo wq_gemm_exact)
            i=0
            for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
              i=$((i+1))
              MS=$m step pmc_m${m}_$i 120 rocprofv3 --pmc $C --kernel-include-regex $k -d $O/pmc_m${m}_$i -o pmc --output-format csv -- python scripts/pmc_chain.py
            done
          done;;
    shard) LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so ROUNDS=2 SHAPES=4096:4096,4096:2048,4096:1024,4096:512,2048:4096,2048:2048,2048:1024,2048:512 step shard_trace 300 rocprofv3 --kernel-trace --stats -d $O/shard -o kt --output-format csv -- python scripts/gemm_ab.py;;
  esac
done
echo batch done
