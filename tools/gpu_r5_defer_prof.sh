#!/bin/bash
# kernel profiles of the GPT step with / without the deferred output-projection biases
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for d in 1 0; do
  PHA_GPT_DEFER_BIAS=$d timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_defer$d -o run -- python bench.py --steps 3 --warmup 2 --no-resnet > gpurun_out/prof_defer$d.log 2>&1 || { tail -5 gpurun_out/prof_defer$d.log; exit 1; }
  f=$(find /tmp/prof_defer$d -name "*results.db" | head -1)
  python tools/prof_db_summary.py "$f" 5 60 > gpurun_out/prof_defer${d}_summary.txt
done
