#!/bin/bash
# Parity of the group kernel (forced on every n>=4 case) + default suites + A/B bench.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
BOTE_SWEEP_KERNEL=group timeout -k 10 300 $T tests/test_gpu_golden.py > gpurun_out/ab_golden_group.log 2>&1
rc=$?; echo "golden(group) rc=$rc"; tail -4 gpurun_out/ab_golden_group.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 $T tests/test_gpu_golden.py tests/test_gpu_parity.py > gpurun_out/ab_parity.log 2>&1
rc=$?; echo "parity(default) rc=$rc"; tail -4 gpurun_out/ab_parity.log; [ $rc -ne 0 ] && exit $rc
for K in group fast; do
  BOTE_SWEEP_KERNEL=$K timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_bench_$K.log 2>&1
  rc=$?; echo "bench $K rc=$rc"; grep -o '"value": [0-9.e+]*\|"kernel_ms_avg": [0-9.]*\|"kernel_path": "[a-z]*"\|"frac": [0-9.]*' gpurun_out/ab_bench_$K.log | tr '\n' ' '; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
