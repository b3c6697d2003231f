#!/bin/bash
# GPT step with the in-tree TunableOp database (default) vs hipBLASLt heuristics only, alternating
mkdir -p gpurun_out
for i in 1 2; do
  for t in db off; do
    timeout -k 10 300 python bench.py --no-resnet --steps 10 --warmup 3 --gemm-tuning $t > gpurun_out/r5_bench_tuning_${t}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_tuning_${t}_$i.log; exit 1; }
    echo "tuning=$t run $i: $(tail -1 gpurun_out/r5_bench_tuning_${t}_$i.log | cut -c150-200)"
  done
done
