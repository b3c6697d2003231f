#!/bin/bash
# Alternating A/B of bench.py under two values of one environment variable; stops at the first
# failing run. usage: tools/ab_env.sh VAR "A B" REPS OUTFILE [extra bench args]
var=$1; vals=$2; reps=$3; out=$4; shift 4
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
: > gpurun_out/$out
for r in $(seq 1 $reps); do
  for v in $vals; do
    env $var=$v timeout -k 10 240 python bench.py --steps 10 --warmup 3 "$@" > gpurun_out/ab_tmp.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$var=$v rc=$rc" >> gpurun_out/$out; tail -20 gpurun_out/ab_tmp.log >> gpurun_out/$out; exit $rc; fi
    echo "$var=$v $(tail -1 gpurun_out/ab_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("resnet50_samples_per_sec"))')" >> gpurun_out/$out
  done
done
cat gpurun_out/$out
