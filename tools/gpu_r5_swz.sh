#!/bin/bash
# conflict-free BK=32 LDS swizzle in gemm256: conv numerics, LDS counters, per-conv table, ResNet bench
mkdir -p gpurun_out/resnet_pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py tests/test_resnet_unit.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or bn or batch_norm or resnet or gemm256 or grouped or stem" > gpurun_out/r5_swz_tests.log 2>&1 || { tail -30 gpurun_out/r5_swz_tests.log; exit 1; }
tail -1 gpurun_out/r5_swz_tests.log
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d /tmp/pmc_swz -o run --output-format csv -- python3 bench.py --model resnet50 --steps 2 --warmup 1 --graph off > gpurun_out/resnet_pmc/swz.log 2>&1 || { tail -3 gpurun_out/resnet_pmc/swz.log; exit 1; }
d=$(dirname $(find /tmp/pmc_swz -name "*counter_collection.csv" | head -1))
timeout 120 python tools/pmc_summary.py gpurun_out/resnet_pmc/summary_swz.txt $d
python - gpurun_out/resnet_pmc/summary_swz.txt <<'PY'
import re, sys
t = open(sys.argv[1]).read().split('\n')
for i in range(len(t) - 1):
    if 'gemm256_kernel' in t[i]:
        print(t[i].strip()[:70], dict(re.findall(r'(dispatches|lds_conflict_rate)=(\S+)', t[i + 1])))
PY
timeout -k 10 400 python -u tools/resnet_conv_table.py 256 > gpurun_out/r5_conv_table_swz.log 2>&1 || { tail -20 gpurun_out/r5_conv_table_swz.log; exit 1; }
head -3 gpurun_out/r5_conv_table_swz.log | tail -2
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_swz_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_swz_$i.log; exit 1; }
  echo "run $i: $(tail -1 gpurun_out/r5_bench_swz_$i.log | cut -c100-200)"
done
