#!/bin/bash
# the default GPT micro-batch picked from the free HBM on a real MI355X
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-resnet --steps 3 --warmup 2 > gpurun_out/r5_mbcheck.log 2>&1 || { tail -20 gpurun_out/r5_mbcheck.log; exit 1; }
grep "\[bench\]" gpurun_out/r5_mbcheck.log || true
python -c "import json; d=json.loads(open('gpurun_out/r5_mbcheck.log').read().strip().splitlines()[-1]); print(d['value'], d['config']['global_batch'], d['config'].get('peak_mem_gb'))"
