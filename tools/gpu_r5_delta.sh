#!/bin/bash
# delta inside dQ: FA tests, FA roofline (backward), GPT bench A/B (PHA_FA_DELTA_PASS=1: separate pass)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/r5_delta_tests.log 2>&1 || { tail -30 gpurun_out/r5_delta_tests.log; exit 1; }
tail -2 gpurun_out/r5_delta_tests.log
for i in 1 2; do
  for d in inq pass; do
    if [ $d = pass ]; then export PHA_FA_DELTA_PASS=1; else unset PHA_FA_DELTA_PASS; fi
    timeout -k 10 400 python bench.py --no-resnet --steps 8 --warmup 3 > gpurun_out/r5_bench_delta_${d}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_delta_${d}_$i.log; exit 1; }
    echo "delta=$d run $i: $(tail -1 gpurun_out/r5_bench_delta_${d}_$i.log | cut -c150-200)"
  done
done
unset PHA_FA_DELTA_PASS
