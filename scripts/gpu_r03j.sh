#!/bin/bash
# Round 3: host-unranked chunk starts + ticket prefetch: GPU suite, bench,
# per-shard kernel times of an 8-way split (the N=8 step bound).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/bench.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/shard_balance.py --parts 8 > gpurun_out/shard8.log 2>&1
rc=$?; echo "shard rc=$rc"; grep -E "^(equal|cost)" gpurun_out/shard8.log
exit $rc
