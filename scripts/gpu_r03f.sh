#!/bin/bash
# Round 3: group geometry chosen by pick_group_geometry (no env) vs XK at 768.
set -u
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
run() {  # tag, env bd ("" = automatic), bench args
  BOTE_GROUP_BD=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $3 > gpurun_out/ab/$1_${2:-auto}.log 2>&1
  rc=$?; echo "$1 bd=${2:-auto} rc=$rc $(tail -1 gpurun_out/ab/$1_${2:-auto}.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["config"].get("block"), d["config"].get("grid"), d["config"].get("lds_bytes"), d.get("roofline",{}).get("kernel_ms_avg"))' 2>&1 | tail -1)"
  return $rc
}
run x 768 "--workload r128n6 --steps 3 --warmup 1" || exit 1
run x "" "--workload r128n6 --steps 3 --warmup 1" || exit 1
run b "" "--workload r128n6_base --steps 3 --warmup 1" || exit 1
run a "" "--steps 10 --warmup 2" || exit 1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests_auto.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/ab/tests_auto.log)"
exit $rc
