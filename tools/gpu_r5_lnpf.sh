#!/bin/bash
# prefetching LN backward: tests, micro A/B, GPT bench A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "layer_norm or conv or route" > gpurun_out/r5_lnpf_tests.log 2>&1 || { tail -30 gpurun_out/r5_lnpf_tests.log; exit 1; }
tail -2 gpurun_out/r5_lnpf_tests.log
timeout -k 10 120 python tools/ln_bwd_ab.py > gpurun_out/r5_ln_bwd_ab.log 2>&1 || { tail -20 gpurun_out/r5_ln_bwd_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_ln_bwd_ab.log
for i in 1 2; do
  for pf in 1 0; do
    PHA_LN_BWD_PF=$pf timeout -k 10 300 python bench.py --no-resnet --steps 10 --warmup 3 > gpurun_out/r5_bench_lnpf${pf}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_lnpf${pf}_$i.log; exit 1; }
    echo "lnpf=$pf run $i: $(tail -1 gpurun_out/r5_bench_lnpf${pf}_$i.log | cut -c150-200)"
  done
done
