#!/bin/bash
# Round 3: S32/V32 kernels: GPU suite and benches (each checked against its
# oracle fixture), then the fixed per-launch cost experiment (gpu_r03q.sh).
set -u
mkdir -p gpurun_out/r
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r/gpu_tests.log | head; exit $rc; }
for wl in r64n7 r128n6_base r128n6; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/r/bench_$wl.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
bash scripts/gpu_r03q.sh
