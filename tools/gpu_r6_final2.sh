#!/bin/bash
# round 6 session 3 end: smoke, the whole GPU suite, the default bench (GPT-3 1.3B + ResNet-50),
# BERT-base alternating PHA_WT_BATCH=1/0, then BERT and default-bench kernel profiles (stats only)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6g.log 2>&1 || { tail -5 gpurun_out/smoke_r6g.log; exit 1; }
tail -1 gpurun_out/smoke_r6g.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_gpu_r6g.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_r6g.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_r6g.log 2>&1 || { tail -5 gpurun_out/bench_r6g.log; exit 1; }
tail -1 gpurun_out/bench_r6g.log | cut -c1-400
for i in 1 2; do
  for c in 1 0; do
    PHA_WT_BATCH=$c timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_r6g_wt${c}_$i.log 2>&1 || { tail -5 gpurun_out/bench_bert_r6g_wt${c}_$i.log; exit 1; }
    echo "bert wtbatch=$c $i: $(tail -1 gpurun_out/bench_bert_r6g_wt${c}_$i.log | cut -c1-300)"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert_r6g -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert_r6g.log 2>&1 || { tail -5 gpurun_out/prof_bert_r6g.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6g -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof_r6g.log 2>&1 || { tail -5 gpurun_out/prof_r6g.log; exit 1; }
tail -1 gpurun_out/prof_r6g.log | cut -c1-200
