#!/bin/bash
# NT products own vs library at micro-batch 48, then full-step auto vs own alternating
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/nt_mb48_ab.py > gpurun_out/r5_nt_mb48.log 2>&1 || { tail -20 gpurun_out/r5_nt_mb48.log; exit 1; }
cat gpurun_out/r5_nt_mb48.log | grep -v amdgpu.ids
for i in 1 2; do
  for impl in auto own; do
    PHA_GEMM_IMPL=$impl timeout -k 10 400 python bench.py --no-resnet --steps 6 --warmup 3 > gpurun_out/r5_step_${impl}_$i.log 2>&1 || { tail -20 gpurun_out/r5_step_${impl}_$i.log; exit 1; }
    echo "$impl run $i: $(tail -1 gpurun_out/r5_step_${impl}_$i.log | cut -c150-260)"
  done
done
