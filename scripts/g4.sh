set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6/${TAG:-svc}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -30 $OUT/pytest.log; exit $rc; }
timeout -k 10 300 python -u tools/svc_probe.py 1000 2,3,5 > $OUT/svc_probe.txt 2>&1; rc=$?; cat $OUT/svc_probe.txt; exit $rc
