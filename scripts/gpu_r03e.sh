#!/bin/bash
# Round 3: group-kernel workgroup size A/B (BOTE_GROUP_BD env) on config 5
# (extended keys), the 10-key R=128 sweep and R=64 n=7, plus parity at 384/512.
set -u
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
run() {  # tag, env bd, bench args
  BOTE_GROUP_BD=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $3 > gpurun_out/ab/$1_$2.log 2>&1
  rc=$?; echo "$1 bd=$2 rc=$rc $(tail -1 gpurun_out/ab/$1_$2.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["config"].get("block"), d["config"].get("grid"), d["config"].get("lds_bytes"), d.get("roofline",{}).get("kernel_ms_avg"))' 2>&1 | tail -1)"
  return $rc
}
for bd in 256 384 512; do run x $bd "--workload r128n6 --steps 3 --warmup 1" || exit 1; done
for bd in 256 384 512 640 768; do run b $bd "--workload r128n6_base --steps 3 --warmup 1" || exit 1; done
for bd in 256 384 512; do run a $bd "--steps 10 --warmup 2" || exit 1; done
for bd in 384 512; do
  BOTE_GROUP_BD=$bd timeout -k 10 600 python -u -m pytest tests/test_gpu_keys.py tests/test_gpu_fixtures.py -m gpu -x -q --timeout 300 --timeout-method thread -k "windows or full_r64n7 or sweep_keys" > gpurun_out/ab/tests_$bd.log 2>&1
  rc=$?; echo "tests bd=$bd rc=$rc $(tail -1 gpurun_out/ab/tests_$bd.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
