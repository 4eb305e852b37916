#!/bin/bash
# Round 3: extended-key parity (minus the windows), config 5 bench with the
# 2-quad XK loop, the GCP configs 1-2 line with its full CPU baseline, and an
# A/B of the base kernel's client-loop unroll (4 vs 2 quads).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_keys.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "eval_keys or sweep_keys or slice or errors" > gpurun_out/gpu_keys.log 2>&1
rc=$?; echo "pytest keys rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/gpu_keys.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload r128n6 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r128x.log 2>&1
rc=$?; echo "bench r128n6 (config 5) rc=$rc"; tail -1 gpurun_out/bench_r128x.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload gcp --steps 5 --warmup 2 > gpurun_out/bench_gcp.log 2>&1
rc=$?; echo "bench gcp rc=$rc"; tail -1 gpurun_out/bench_gcp.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
VARIANTS="default u2 default u2" STEPS=10 bash scripts/gpu_ab.sh
