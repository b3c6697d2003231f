#!/bin/bash
# GPT-3 1.3B micro-batch 32 / 48 / 64 alternating on one box (GPT only), with peak memory
mkdir -p gpurun_out
for i in 1 2; do
  for mb in 32 48 64; do
    timeout -k 10 400 python bench.py --no-resnet --micro-batch $mb --steps 8 --warmup 3 > gpurun_out/r5_mb${mb}_$i.log 2>&1 || { tail -20 gpurun_out/r5_mb${mb}_$i.log; exit 1; }
    echo "mb $mb run $i: $(tail -1 gpurun_out/r5_mb${mb}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k: v for k, v in d["config"].items() if "mem" in k.lower() or "peak" in k.lower()})')"
  done
done
