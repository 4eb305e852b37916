#!/bin/bash
# Round 3 (re-entry): smoke, the whole GPU suite (incl. the extended key set),
# bench config 4 (R=64 n=7) and config 5 as stated (R=128 n=6, extended keys),
# the 10-key R=128 line, and a kernel trace of config 5.
set -u
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u __graft_entry__.py > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r64.log 2>&1
rc=$?; echo "bench r64n7 rc=$rc"; tail -1 gpurun_out/bench_r64.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload r128n6 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r128x.log 2>&1
rc=$?; echo "bench r128n6 (config 5) rc=$rc"; tail -1 gpurun_out/bench_r128x.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload r128n6_base --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r128b.log 2>&1
rc=$?; echo "bench r128n6_base rc=$rc"; tail -1 gpurun_out/bench_r128b.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r03d_x_trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload r128n6 > gpurun_out/prof/r03d_x_trace.log 2>&1
rc=$?; echo "trace rc=$rc"
exit $rc
