set -u
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 1100 python -u scripts/oracle_full_sweep.py --workload r128n6 --threads 16 --chunk 4194304 --partial \
  --rank-begin 1700000000 --rank-end 2000000000 --sweep-begin 1700000000 --time-limit 960 \
  --state $O/r128n6_chunks.jsonl > $O/oracle.log 2>&1
echo "rc=$? $(tail -1 $O/oracle.log)"
