#!/bin/bash
# A/B timing of library variants (scripts/build_variant.sh NAME FLAGS):
#   VARIANTS="default v1 v2" [WL=r64n7] [ABL="0 1 16"] bash scripts/gpu_ab.sh
# Each variant runs bench.py (no CPU baseline); the digest/valid must agree.
# With ABL set, scripts/ablate.py runs on fantoch_amd/lib_abl (built with
# -DBOTE_ABLATION) for those masks.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for V in ${VARIANTS:-default}; do
  if [ "$V" = default ]; then unset BOTE_LIB_PATH; else export BOTE_LIB_PATH=fantoch_amd/lib_$V/libbote_hip.so; fi
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --workload ${WL:-r64n7} > gpurun_out/ab_$V.log 2>&1
  rc=$?; echo "$V rc=$rc $(grep -o '"kernel_ms_avg": [0-9.]*\|"ms_per_step": [0-9.]*\|"valid": [0-9]*\|"digest": [0-9]*' gpurun_out/ab_$V.log | tr '\n' ' ')"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$V.log; exit $rc; }
done
unset BOTE_LIB_PATH
if [ -n "${ABL:-}" ]; then
  BOTE_LIB_PATH=fantoch_amd/lib_abl/libbote_hip.so timeout -k 10 300 python -u scripts/ablate.py $ABL > gpurun_out/ab_ablate.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_ablate.log; exit $rc
fi
exit 0
