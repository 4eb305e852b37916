#!/bin/bash
# Round 3: the default bench line (as the driver runs it, with the CPU baseline).
set -u
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.e+]*\|"frac": [0-9.]*' gpurun_out/final/bench.log | tr '\n' ' ')"
exit $rc
