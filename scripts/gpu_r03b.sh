#!/bin/bash
# Round 3, extended key set: its GPU parity tests, then the bench on
# config 4 (R=64 n=7) and config 5 as stated (R=128 n=6, extended keys).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_keys.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "eval_keys or sweep_keys or slice or errors" > gpurun_out/gpu_keys.log 2>&1
rc=$?; echo "pytest keys rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/gpu_keys.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r64.log 2>&1
rc=$?; echo "bench r64n7 rc=$rc"; tail -1 gpurun_out/bench_r64.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload r128n6 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r128x.log 2>&1
rc=$?; echo "bench r128n6 (config 5) rc=$rc"; tail -1 gpurun_out/bench_r128x.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload r128n6_base --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r128b.log 2>&1
rc=$?; echo "bench r128n6_base rc=$rc"; tail -1 gpurun_out/bench_r128b.log | cut -c1-400
exit $rc
