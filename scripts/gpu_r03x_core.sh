#!/bin/bash
# Round 3 (r03x): seed sample chunks of 8 consecutive steps: suite, benches, shards
# the per-step overhead cuts: GPU suite, three benches, per-dispatch trace of
# 1/1 .. 1/64 shards.
set -u
mkdir -p gpurun_out/x
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/x/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/x/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/x/gpu_tests.log | head; exit $rc; }
for wl in r64n7 r128n6_base r128n6; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/x/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/x/bench_$wl.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x/trace -o run -- python3 scripts/shard_ablate.py 0 > gpurun_out/x/trace.log 2>&1
rc=$?; echo "trace rc=$rc $(grep ablate gpurun_out/x/trace.log)"
exit $rc
