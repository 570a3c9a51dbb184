set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6/g2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -25 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
export JSP_SERVICE_IDLE_MS=30 PHASE_OUT=$OUT
timeout -k 10 240 python -u tools/phase_probe.py > $OUT/phase_probe.txt 2>&1; rc=$?
cat $OUT/phase_probe.txt; exit $rc
