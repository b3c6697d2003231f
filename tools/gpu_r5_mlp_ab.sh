#!/bin/bash
# MLP chain A/B in the GPT step: epi (default: gemm4p GELU epilogue fwd, library dX + HIP dGELU pass)
# vs force (gemm4w GELU fwd, gemm4w dGELU + bias-grad epilogue bwd)
mkdir -p gpurun_out
for i in 1 2; do
  for m in epi force; do
    PHA_FUSED_MLP=$m timeout -k 10 300 python bench.py --no-resnet --steps 10 --warmup 3 > gpurun_out/r5_bench_mlp_${m}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_mlp_${m}_$i.log; exit 1; }
    echo "mlp=$m run $i: $(tail -1 gpurun_out/r5_bench_mlp_${m}_$i.log | cut -c150-200)"
  done
done
