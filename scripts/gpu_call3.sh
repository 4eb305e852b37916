set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="default w5 old" bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 python -u scripts/oracle_full_sweep.py --workload r64n7 --threads 16 --chunk 4194304 --partial --sweep-begin 209715200 --sweep-end 230686720 --state gpurun_out/box3_chunks.jsonl > gpurun_out/box3.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/oracle_full_sweep.py --workload r64n7 --threads 16 --chunk 4194304 --partial --sweep-begin 608174080 --state gpurun_out/box3_chunks.jsonl >> gpurun_out/box3.log 2>&1 || exit $?
tail -1 gpurun_out/box3.log
