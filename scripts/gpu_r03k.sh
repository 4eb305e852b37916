#!/bin/bash
# Round 3: kernel time vs chunks per wave, full sweep and an 8-way shard split.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cpw in 4 8 16 32; do
  BOTE_CHUNKS_PER_WAVE=$cpw timeout -k 10 300 python -u scripts/shard_balance.py --parts 8 --reps 2 > gpurun_out/shard8_$cpw.log 2>&1
  rc=$?; echo "cpw=$cpw shard rc=$rc $(grep -E '^cost' gpurun_out/shard8_$cpw.log)"; [ $rc -ne 0 ] && exit $rc
  BOTE_CHUNKS_PER_WAVE=$cpw timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$cpw.log 2>&1
  rc=$?; echo "cpw=$cpw full $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/bench_$cpw.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
