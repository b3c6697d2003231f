#!/bin/bash
# round 6 (session 2): D=64 FA with pair-shared dropout hashes in dK/dV + the plain D=64 entry;
# tests, FA timing at the BERT shape, BERT-base rocprofv3 kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fa64b.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_fa64b.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/fa_bert_time.py > gpurun_out/fa_bert_time_fa64b.log 2>&1; grep -v amdgpu.ids gpurun_out/fa_bert_time_fa64b.log
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s14.log 2>&1
rc=$?; echo "bert: $(tail -1 gpurun_out/bench_bert_s14.log | cut -c1-330)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert2 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert2.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert2.log | cut -c1-200; exit $rc
