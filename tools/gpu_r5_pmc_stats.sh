#!/bin/bash
# LDS bank conflicts of the conv kernels with the BN-statistics epilogue on vs off
mkdir -p gpurun_out/resnet_pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=/tmp/resnet_pmc_s
for st in 1 0; do
  PHA_CONV_BN_STATS=$st timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/s$st -o run --output-format csv -- python3 bench.py --model resnet50 --steps 2 --warmup 1 --graph off > gpurun_out/resnet_pmc/stats$st.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/resnet_pmc/stats$st.log; exit $rc; }
  d=$(dirname $(find $O/s$st -name "*counter_collection.csv" | head -1))
  timeout 120 python tools/pmc_summary.py gpurun_out/resnet_pmc/summary_stats$st.txt $d
  echo "== stats $st"; python - gpurun_out/resnet_pmc/summary_stats$st.txt <<'PY'
import re, sys
t = open(sys.argv[1]).read().split('\n')
for i in range(len(t) - 1):
    if 'gemm256_kernel' in t[i]:
        m = dict(re.findall(r'(dispatches|lds_conflict_rate)=(\S+)', t[i + 1]))
        print(t[i].strip()[:70], m)
PY
done
