#!/bin/bash
# Round 3: cost of the block top-K (screen + merges) per shard size, from the
# ablation build (BOTE_ABLATE bit 4 = no top-K, 16 = no digest; results are
# wrong when set); then the seed kernel that skips the keys' common high
# bytes: GPU suite, R=64 bench, per-dispatch trace.
set -u
mkdir -p gpurun_out/v
export PYTHONUNBUFFERED=1
BOTE_LIB_PATH=fantoch_amd/lib_abl/libbote_hip.so timeout -k 10 300 python -u scripts/shard_ablate.py 0 4 16 > gpurun_out/v/ablate.log 2>&1
rc=$?; grep ablate gpurun_out/v/ablate.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/v/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/v/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --workload r64n7 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/v/bench_r64n7.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/v/bench_r64n7.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v/trace -o run -- python3 scripts/shard_ablate.py 0 > gpurun_out/v/trace.log 2>&1
rc=$?; echo "trace rc=$rc $(grep ablate gpurun_out/v/trace.log)"; [ $rc -ne 0 ] && exit $rc
# A/B: a sample of 8 steps per wave (lib_s8) against 1 (the default), same box
for lib in s8 main s8; do
  P=fantoch_amd/lib/libbote_hip.so; [ $lib = s8 ] && P=fantoch_amd/lib_s8/libbote_hip.so
  BOTE_LIB_PATH=$P timeout -k 10 300 python -u bench.py --workload r64n7 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/v/bench_$lib.log 2>&1
  rc=$?; echo "bench $lib rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/v/bench_$lib.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
  BOTE_LIB_PATH=$P timeout -k 10 300 python -u scripts/shard_ablate.py 0 > gpurun_out/v/shards_$lib.log 2>&1
  rc=$?; echo "shards $lib rc=$rc $(grep ablate gpurun_out/v/shards_$lib.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
