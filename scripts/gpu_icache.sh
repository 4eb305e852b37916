set -u
mkdir -p gpurun_out/ic
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/ic/avail.txt 2>&1
echo "list rc=$?"
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INSTS_[A-Z_]*" gpurun_out/ic/avail.txt | sort -u | tr '\n' ' '
echo
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_REQ --output-format csv -d gpurun_out/ic/p1 -o run -- $B > gpurun_out/ic/p1.log 2>&1
echo "pmc rc=$?"
