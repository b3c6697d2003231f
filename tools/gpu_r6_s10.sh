#!/bin/bash
# round 6 (session 2): SPREAD bitwise tests; own-policy GPT step with the shipped LV 8 vs SPREAD LV 40
# (alternating); BERT-base rocprofv3 kernel stats of the current tree
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_ring_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s10.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s10.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lv in 8 40; do
    PHA_GEMM_IMPL=own PHA_G4P_LV=$lv timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-resnet > gpurun_out/own_lv${lv}_$i.log 2>&1
    rc=$?; echo "own lv$lv $i: $(tail -1 gpurun_out/own_lv${lv}_$i.log | cut -c1-200)"; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert.log | cut -c1-300; exit $rc
