set -u
O=gpurun_out/r06r
mkdir -p $O
STEPS="shardsteps bench" TAG=r06r BWLS="gcp" BSTEPS=10 VARIANTS=default bash scripts/gpu_job.sh || exit 1
BOTE_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/rehearsal8.log 2>&1 || { echo "rehearsal rc=$?"; tail -5 $O/rehearsal8.log; exit 1; }
echo "rehearsal8: $(grep -o '"value": [0-9.e+]*\|"fixture": "[^"]*' $O/rehearsal8.log | tr '\n' ' ' | cut -c1-200)"
