#!/bin/bash
# default bench (GPT-3 1.3B + ResNet-50): this tree vs the session-2 final library (libpha_kernels_r6f.so,
# commit 1ab4001) alternating on one box; the old library runs with the new Python paths off
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then
      PHA_KERNELS_LIB=libpha_kernels_r6f.so PHA_LN_DROP_FUSED=0 PHA_WT_BATCH=0 timeout -k 10 300 python bench.py > gpurun_out/bench_s31_${v}_$i.log 2>&1
    else
      timeout -k 10 300 python bench.py > gpurun_out/bench_s31_${v}_$i.log 2>&1
    fi
    rc=$?; echo "$v $i: $(tail -1 gpurun_out/bench_s31_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('resnet50', d.get('extra', '')))" 2>&1 | cut -c1-200)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
