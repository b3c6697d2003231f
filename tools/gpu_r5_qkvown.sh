#!/bin/bash
# qkv forward on gemm4p under the auto policy vs on hipBLASLt: GEMM / GPT GPU tests, full step alternating
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_quant_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or mlp or linear or gpt or fallback or headline" > gpurun_out/r5_qkvown_tests.log 2>&1 || { tail -30 gpurun_out/r5_qkvown_tests.log; exit 1; }
tail -1 gpurun_out/r5_qkvown_tests.log
for i in 1 2 3; do
  for q in 1 0; do
    PHA_GEMM_AUTO_NT_OWN=$q timeout -k 10 400 python bench.py --no-resnet --steps 6 --warmup 3 > gpurun_out/r5_step_qkvown${q}_$i.log 2>&1 || { tail -20 gpurun_out/r5_step_qkvown${q}_$i.log; exit 1; }
    echo "qkv_own=$q run $i: $(tail -1 gpurun_out/r5_step_qkvown${q}_$i.log | cut -c150-230)"
  done
done
