#!/bin/bash
# Round 3, first call: smoke, GPU suite, bench N=1, the N=2 rehearsal on one
# GPU (gloo), and the device-assert build against oracle fixtures.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u __graft_entry__.py > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "ratio|passed|failed|Error" gpurun_out/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
BOTE_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/rehearsal2.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; tail -1 gpurun_out/rehearsal2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/refuse2.log 2>&1
echo "refusal rc=$? (nonzero expected)"; tail -1 gpurun_out/refuse2.log
BOTE_LIB_PATH=fantoch_amd/lib_debug/libbote_hip.so timeout -k 10 300 python -u scripts/debug_check.py > gpurun_out/debug_check.log 2>&1
rc=$?; echo "debug rc=$rc"; tail -6 gpurun_out/debug_check.log
exit $rc
