#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/g4p_groupm_tn_sweep.py > gpurun_out/r5_groupm_tn.log 2>&1 || { tail -20 gpurun_out/r5_groupm_tn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_groupm_tn.log
