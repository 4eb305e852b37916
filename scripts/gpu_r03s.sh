#!/bin/bash
# Round 3: per-step overhead cuts (radix-select seed, 1024-thread merges,
# one-group samples): GPU suite, R=64 bench, per-dispatch trace of shards.
set -u
mkdir -p gpurun_out/s
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/s/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/s/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --workload r64n7 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/s/bench_r64n7.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/s/bench_r64n7.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s/trace -o run -- python3 scripts/shard_ablate.py 0 > gpurun_out/s/trace.log 2>&1
rc=$?; echo "trace rc=$rc $(grep ablate gpurun_out/s/trace.log)"
exit $rc
