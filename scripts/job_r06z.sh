# oracle_full_sweep.py chunks of a contiguous R=128 n=6 range on the box's CPUs
# (SWEEP_BEGIN: the first chunk; KEYS=1: the extended key set); state to gpurun_out/$TAG/
set -u
TAG=${TAG:-r06z}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1100 python -u scripts/oracle_full_sweep.py --workload r128n6 --threads 16 --chunk ${CHUNK:-4194304} --partial \
  --rank-begin ${RANK_BEGIN:-1700000000} --rank-end ${RANK_END:-2000000000} --sweep-begin ${SWEEP_BEGIN:-1700000000} \
  --time-limit ${SECONDS_LIMIT:-960} --keys ${KEYS:-0} --state $O/r128n6_chunks.jsonl > $O/oracle.log 2>&1
echo "rc=$? $(tail -1 $O/oracle.log)"
