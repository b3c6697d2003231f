#!/bin/bash
# cache-aware TN group_m + split rule: GEMM tests, then alternating GPT bench A/B (PHA_TN_GM=4 = old)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or tn or linear or bmm" > gpurun_out/r5_tngm_tests.log 2>&1 || { tail -30 gpurun_out/r5_tngm_tests.log; exit 1; }
tail -2 gpurun_out/r5_tngm_tests.log
for i in 1 2; do
  for g in model 4; do
    if [ $g = model ]; then unset PHA_TN_GM; else export PHA_TN_GM=$g; fi
    timeout -k 10 300 python bench.py --no-resnet --steps 10 --warmup 3 > gpurun_out/r5_bench_tngm_${g}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_tngm_${g}_$i.log; exit 1; }
    echo "gm=$g run $i: $(tail -1 gpurun_out/r5_bench_tngm_${g}_$i.log | cut -c150-200)"
  done
done
unset PHA_TN_GM
