#!/bin/bash
# round 6 (session 2): whole GPU suite on the current tree, then the GPT step with the TN SPREAD default
# vs the plain TN schedule (PHA_G4P_TN_LV=0), alternating
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_gpu_s17.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_s17.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  for lv in 40 0; do
    PHA_G4P_TN_LV=$lv timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-resnet > gpurun_out/tnlv_${lv}_$i.log 2>&1
    rc=$?; echo "tn lv$lv $i: $(tail -1 gpurun_out/tnlv_${lv}_$i.log | cut -c150-250)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
