#!/bin/bash
# Round 3: top-K seed pre-pass: GPU suite, benches, shard kernel times.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head; exit $rc; }
for wl in r64n7 r128n6_base r128n6; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/bench_$wl.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u scripts/shard_ablate.py 0 > gpurun_out/shard_seed.log 2>&1
rc=$?; echo "shards rc=$rc $(grep ablate gpurun_out/shard_seed.log)"
exit $rc
