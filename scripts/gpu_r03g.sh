#!/bin/bash
# Round 3: pipelined bench steps + fix-up early exit: GPU suite, bench N=1,
# N=2 rehearsal (gloo, one GPU), and a kernel trace of the N=1 bench.
set -u
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-330; [ $rc -ne 0 ] && exit $rc
BOTE_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/rehearsal2.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; tail -1 gpurun_out/rehearsal2.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r03g_trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof/r03g_trace.log 2>&1
rc=$?; echo "trace rc=$rc"
exit $rc
