#!/bin/bash
# Round 3 final evidence: gpu_r03t.sh (suite, benches, shard trace), smoke,
# the N=2 rehearsal, then rocprofv3 trace + PMC passes of the final kernels.
set -u
bash scripts/gpu_r03x_core.sh || exit $?
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/x/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/x/smoke.log)"; [ $rc -ne 0 ] && exit $rc
BOTE_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/x/rehearsal2.log 2>&1
rc=$?; echo "rehearsal2 rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"fixture": "[a-z ]*' gpurun_out/x/rehearsal2.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
for wl in r64n7; do
  TAG=r03x_$wl WL=$wl bash scripts/gpu_profile.sh
  rc=$?; echo "profile $wl rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
