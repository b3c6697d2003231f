#!/bin/bash
# Two ranks sharing the one GPU over gloo: the multi-rank DP path of bench.py (GPT + ResNet).
# (micro-batch 16: two ranks share the one card, and the default 48 needs 183 GB per rank)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
PHA_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --micro-batch 16 --steps 2 --warmup 2 > gpurun_out/rehearse2.log 2>&1
rc=$?
grep -E "metric|capture|Error|error" gpurun_out/rehearse2.log | cut -c1-400 | tail -6
exit $rc
