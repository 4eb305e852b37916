set -u
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 300 python -u __graft_entry__.py > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2; do
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests_$i.log 2>&1 || { echo "tests $i rc=$?"; tail -8 $O/tests_$i.log; exit 1; }
  echo "tests $i: $(tail -1 $O/tests_$i.log)"
done
