#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert3 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert3.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert3.log | cut -c1-200; exit $rc
