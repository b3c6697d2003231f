#!/bin/bash
# HBM ceilings; library-free GEMM policy vs default at micro-batch 32
mkdir -p gpurun_out
timeout -k 10 120 python tools/bw_probe.py > gpurun_out/r5_bw_probe.log 2>&1 || { tail -20 gpurun_out/r5_bw_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_bw_probe.log
for m in auto own; do
  PHA_GEMM_IMPL=$m timeout -k 10 400 python bench.py --no-resnet --steps 8 --warmup 3 > gpurun_out/r5_bench_impl_$m.log 2>&1 || { tail -20 gpurun_out/r5_bench_impl_$m.log; exit 1; }
  echo "impl=$m: $(tail -1 gpurun_out/r5_bench_impl_$m.log | cut -c150-200)"
done
