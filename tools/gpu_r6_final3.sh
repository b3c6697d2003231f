#!/bin/bash
# round 6 session 3 end: smoke, the whole GPU suite, the default bench (GPT-3 1.3B + ResNet-50),
# BERT-base x2 (no profiles: gpurun_out stays under 64 MiB)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6h.log 2>&1 || { tail -5 gpurun_out/smoke_r6h.log; exit 1; }
tail -1 gpurun_out/smoke_r6h.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_gpu_r6h.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_r6h.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_r6h.log 2>&1 || { tail -5 gpurun_out/bench_r6h.log; exit 1; }
tail -1 gpurun_out/bench_r6h.log | cut -c1-400
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_r6h_$i.log 2>&1 || { tail -5 gpurun_out/bench_bert_r6h_$i.log; exit 1; }
  echo "bert $i: $(tail -1 gpurun_out/bench_bert_r6h_$i.log | cut -c1-300)"
done
