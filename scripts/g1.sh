set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6/g1; mkdir -p $OUT
export JSP_SERVICE_IDLE_MS=30
timeout -k 10 180 python -u tools/phase_probe.py > $OUT/phase_probe.txt 2>&1 || { echo PROBE_FAIL; tail -30 $OUT/phase_probe.txt; exit 1; }
cat $OUT/phase_probe.txt
unset JSP_SERVICE_IDLE_MS
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $OUT/bench_detail.json > $OUT/bench_driver.json 2> $OUT/bench_driver.err
rc=$?; tail -c 3000 $OUT/bench_driver.json; tail -5 $OUT/bench_driver.err; exit $rc
