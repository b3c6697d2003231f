#!/bin/bash
# folded-bias add-LN tests, LN backward A/B, then an alternating GPT bench A/B (PHA_GPT_DEFER_BIAS 1 / 0)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layer_norm or deferred or mlp or bdrln or dropout_residual" > gpurun_out/r5_defer_tests.log 2>&1 || { tail -30 gpurun_out/r5_defer_tests.log; exit 1; }
tail -2 gpurun_out/r5_defer_tests.log
timeout -k 10 120 python tools/ln_xs_bench.py > gpurun_out/r5_ln_xs.log 2>&1 || { tail -20 gpurun_out/r5_ln_xs.log; exit 1; }
cat gpurun_out/r5_ln_xs.log
for i in 1 2; do
  for d in 1 0; do
    PHA_GPT_DEFER_BIAS=$d timeout -k 10 300 python bench.py --no-resnet --steps 10 --warmup 3 > gpurun_out/r5_bench_defer${d}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_defer${d}_$i.log; exit 1; }
    echo "defer=$d run $i: $(tail -1 gpurun_out/r5_bench_defer${d}_$i.log | cut -c150-200)"
  done
done
