#!/bin/bash
# the driver's default bench invocation (no flags) on the current tree
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r5_bench_default_mb48.log 2>&1 || { tail -20 gpurun_out/r5_bench_default_mb48.log; exit 1; }
tail -1 gpurun_out/r5_bench_default_mb48.log | cut -c1-300
python -c "import json; d=json.loads(open('gpurun_out/r5_bench_default_mb48.log').read().strip().splitlines()[-1]); print({k: v for k, v in d['config'].items() if k in ('global_batch', 'peak_mem_gb', 'resnet50_samples_per_sec', 'resnet50_eager_samples_per_sec')})"
