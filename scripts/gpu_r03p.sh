#!/bin/bash
# Round 3 evidence for the current kernels: smoke, GPU suite, then rocprofv3
# kernel trace + separate PMC passes for R=64 n=7 and both R=128 n=6 sweeps.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/smoke.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head; exit $rc; }
for wl in r64n7 r128n6_base r128n6; do
  TAG=r03p_$wl WL=$wl bash scripts/gpu_profile.sh
  rc=$?; echo "profile $wl rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
