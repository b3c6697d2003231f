#!/bin/bash
# fp32 path tests + fp32 ResNet timing (new fp32-output tiles), FA wave-priority A/B, then the
# default bench with PHA_FA_PRIO=0 / 1 alternated.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_fp32_paths_gpu.py -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_fp32.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fp32.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/bench_fp32.py resnet hip > gpurun_out/fp32_resnet_hip.log 2>&1 || { tail -5 gpurun_out/fp32_resnet_hip.log; exit 1; }
grep resnet gpurun_out/fp32_resnet_hip.log
timeout -k 10 300 python tools/gen_static_op_benchmark.py gpurun_out/static_op_benchmark_mi355x.json > gpurun_out/op_bench.log 2>&1 || { tail -5 gpurun_out/op_bench.log; exit 1; }
tail -3 gpurun_out/op_bench.log
timeout -k 10 300 python tools/fa_prio_ab.py > gpurun_out/fa_prio_ab.log 2>&1 || { tail -5 gpurun_out/fa_prio_ab.log; exit 1; }
grep rep gpurun_out/fa_prio_ab.log
for p in 0 1 0 1; do
  PHA_FA_PRIO=$p timeout -k 10 300 python bench.py > gpurun_out/bench_prio$p.log 2>&1 || { tail -5 gpurun_out/bench_prio$p.log; exit 1; }
  echo "prio $p: $(grep -o '"value": [0-9.]*' gpurun_out/bench_prio$p.log | head -1) $(grep -o '"resnet50_samples_per_sec": [0-9.]*' gpurun_out/bench_prio$p.log)"
done
