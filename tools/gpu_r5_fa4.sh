#!/bin/bash
# FA forward v4: correctness, then forward timing v3 vs v4 at the GPT shape
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fwd_v2_v3 or fwd_v4" > gpurun_out/r5_fa4_tests.log 2>&1 || { tail -30 gpurun_out/r5_fa4_tests.log; exit 1; }
tail -2 gpurun_out/r5_fa4_tests.log
for m in v3 v4; do
  PHA_FA_FWD=$m timeout -k 10 200 python tools/fa_roofline.py > gpurun_out/r5_fa4_roof_$m.log 2>&1 || { tail -20 gpurun_out/r5_fa4_roof_$m.log; exit 1; }
  echo "== $m"; grep -i "fwd\|forward" gpurun_out/r5_fa4_roof_$m.log | head -6
done
