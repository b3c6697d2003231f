#!/bin/bash
# LN backward next-row prefetch: numerics tests, microbenchmark A/B, whole-step A/B.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q -k "layer_norm" --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_ln.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ln.log
if [ $rc -ne 0 ]; then exit $rc; fi
for pf in 1 0 1 0; do
  PHA_LN_BWD_PF=$pf timeout -k 10 120 python tools/bench_ln.py > gpurun_out/ln_pf$pf.log 2>&1 || { tail -3 gpurun_out/ln_pf$pf.log; exit 1; }
  echo "pf $pf: $(grep 32768 gpurun_out/ln_pf$pf.log)"
done
for pf in 1 0 1 0; do
  PHA_LN_BWD_PF=$pf timeout -k 10 300 python bench.py > gpurun_out/bench_lnpf$pf.log 2>&1 || { tail -5 gpurun_out/bench_lnpf$pf.log; exit 1; }
  echo "bench pf $pf: $(grep -o '"value": [0-9.]*' gpurun_out/bench_lnpf$pf.log | head -1)"
done
