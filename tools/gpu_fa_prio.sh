#!/bin/bash
# FA wave-priority A/B, then the default bench twice with PHA_FA_PRIO=0 / 1.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python tools/fa_prio_ab.py > gpurun_out/fa_prio_ab.log 2>&1 || { tail -5 gpurun_out/fa_prio_ab.log; exit 1; }
cat gpurun_out/fa_prio_ab.log | grep rep
for p in 0 1 0 1; do
  PHA_FA_PRIO=$p timeout -k 10 300 python bench.py > gpurun_out/bench_prio$p.log 2>&1 || { tail -5 gpurun_out/bench_prio$p.log; exit 1; }
  echo "prio $p: $(grep -o '"value": [0-9.]*' gpurun_out/bench_prio$p.log | head -1) $(grep -o '"resnet50_samples_per_sec": [0-9.]*' gpurun_out/bench_prio$p.log)"
done
