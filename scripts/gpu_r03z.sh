#!/bin/bash
# Round 3: A/B of the top-K seed's sample size (sample steps per wave 4, 8
# (default), 16): bench step time (checked against the fixture) and shards.
set -u
mkdir -p gpurun_out/z
export PYTHONUNBUFFERED=1
for lib in s16 main s4 s16 main s4; do
  P=fantoch_amd/lib/libbote_hip.so; [ $lib != main ] && P=fantoch_amd/lib_$lib/libbote_hip.so
  BOTE_LIB_PATH=$P timeout -k 10 300 python -u bench.py --workload r64n7 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/z/bench_$lib.log 2>&1
  rc=$?; echo "bench $lib rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/z/bench_$lib.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
  BOTE_LIB_PATH=$P timeout -k 10 300 python -u scripts/shard_ablate.py 0 > gpurun_out/z/shards_$lib.log 2>&1
  rc=$?; echo "shards $lib rc=$rc $(grep ablate gpurun_out/z/shards_$lib.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
