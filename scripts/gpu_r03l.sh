#!/bin/bash
# Round 3: wave_topk with lane-held candidates (readlane) vs the previous
# library: full sweep and 1/8, 1/64 shards (kernel ms), then the GPU suite.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in prev default; do
  if [ $v = default ]; then unset BOTE_LIB_PATH; else export BOTE_LIB_PATH=fantoch_amd/lib_$v/libbote_hip.so; fi
  timeout -k 10 300 python -u scripts/shard_ablate.py 0 > gpurun_out/topk_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(grep ablate gpurun_out/topk_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
unset BOTE_LIB_PATH
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/gpu_tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/bench.log | tr '\n' ' ')"
exit $rc
