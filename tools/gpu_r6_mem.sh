#!/bin/bash
# round 6: per-rank peak HBM of the BASELINE multi-GPU GPT layouts at two reduced depths, every
# rank of the job on this one card over gloo (tools/mem_rehearsal.py); fit + verdict by
# tools/mem_fit.py. One torchrun per (layout, depth), each under its own time limit.
mkdir -p gpurun_out
export PHA_DIST_BACKEND=gloo
out=gpurun_out/mem_r6_13b.jsonl
touch $out
port=29611
run() {  # nproc args...
  local n=$1; shift
  echo "[mem] n=$n $*"
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port tools/mem_rehearsal.py "$@" > gpurun_out/mem_run.log 2>&1
  local rc=$?
  port=$((port + 1))
  grep '^{"model"' gpurun_out/mem_run.log >> $out
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/mem_run.log; exit $rc; fi
  tail -1 $out
}
# BASELINE 2: GPT-3 1.3B fleet DP, the bench default micro-batch 48 per GPU (2 ranks shown)
# (DP2 mb48 and DP2 x TP4 measured in the first pass: gpurun_out/mem_r6.jsonl)
: &&
# BASELINE 4: GPT-3 1.3B DP2 x TP4, micro-batch 16 (bench default for non-DP layouts)
: &&
# BASELINE 5: GPT-3 13B sharding stage 3 + PP2 + recompute on 8 ranks, micro-batch 16
run 8 --model gpt3-13b --pp 2 --sharding-stage 3 --recompute --layers 4 --micro-batch 16 &&
run 8 --model gpt3-13b --pp 2 --sharding-stage 3 --recompute --layers 8 --micro-batch 16 &&
python tools/mem_fit.py $out > gpurun_out/mem_fit_r6.txt && cat gpurun_out/mem_fit_r6.txt
