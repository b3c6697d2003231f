#!/bin/bash
# GPT-3 1.3B micro-batch 16 vs 32 per GPU (288 GB HBM: the larger batch fits), alternating
mkdir -p gpurun_out
for i in 1 2; do
  for mb in 16 32; do
    timeout -k 10 400 python bench.py --no-resnet --steps 8 --warmup 3 --micro-batch $mb > gpurun_out/r5_bench_mb${mb}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_mb${mb}_$i.log; exit 1; }
    echo "mb=$mb run $i: $(tail -1 gpurun_out/r5_bench_mb${mb}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("peak_mem_gb"))')"
  done
done
for i in 1; do
  for mb in 256 512; do
    timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --micro-batch $mb > gpurun_out/r5_bench_rn${mb}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_rn${mb}_$i.log; exit 1; }
    echo "resnet mb=$mb run $i: $(tail -1 gpurun_out/r5_bench_rn${mb}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("peak_mem_gb"))')"
  done
done
