#!/bin/bash
# round 6: bias gradients from the TN weight-gradient GEMM (G4P_COLSUM) — tests, GEMM + linear
# tests, then the GPT step A/B (PHA_TN_COLSUM=0 / 1 alternating) and a rocprof of the default step
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tn_colsum_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tn_colsum_r6.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_tn_colsum_r6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_ring_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kern_r6s5.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_kern_r6s5.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 0 1; do
    PHA_TN_COLSUM=$v timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-resnet > gpurun_out/ab_colsum_${v}_$i.log 2>&1
    rc=$?; echo "colsum=$v run $i: $(tail -1 gpurun_out/ab_colsum_${v}_$i.log | cut -c1-160)"; [ $rc -ne 0 ] && exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/prof_cs -o run -- python bench.py --steps 3 --warmup 2 --no-resnet > gpurun_out/prof_colsum.log 2>&1 || { tail -5 gpurun_out/prof_colsum.log; exit 1; }
f=$(find /tmp/prof_cs -name "*results.db" | head -1)
timeout 200 python tools/prof_db_summary.py "$f" 5 45 > gpurun_out/gpt3_r6_colsum_kernels.txt
head -14 gpurun_out/gpt3_r6_colsum_kernels.txt
