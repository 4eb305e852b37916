#!/bin/bash
# Round evidence: smoke, full GPU suite, bench (with CPU baseline), rocprofv3 trace + PMC passes.
set -u
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
TAG=${TAG:-r01}
timeout -k 10 300 python -u __graft_entry__.py > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -1; [ $rc -ne 0 ] && exit $rc
TAG=$TAG bash scripts/gpu_profile.sh
