#!/bin/bash
# One GPU call: the -m gpu suite (unless SKIP_TESTS=1), then an A/B bench of
# library variants (VARIANTS="default rx ...", see scripts/gpu_ab.sh).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
VARIANTS="${VARIANTS:-default}" bash scripts/gpu_ab.sh
