set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6/${TAG:-g3}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 $OUT/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
SECONDS=0; timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $OUT/bench_detail.json > $OUT/bench_driver.json 2> $OUT/bench_driver.err
rc=$?; wc -c $OUT/bench_driver.json; echo "bench wall ${SECONDS}s"; tail -c 5000 $OUT/bench_driver.json; tail -3 $OUT/bench_driver.err; exit $rc
