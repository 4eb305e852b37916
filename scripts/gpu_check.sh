#!/bin/bash
# One GPU session: smoke -> parity tests -> bench.  Stops at the first fault/timeout.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u __graft_entry__.py > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 400 --timeout-method thread ${PYTEST_K:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -3 gpurun_out/bench.log
exit $rc2
