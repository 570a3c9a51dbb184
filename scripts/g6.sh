set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6/${TAG:-anctab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { tail -30 $OUT/pytest.log; exit $rc; }
timeout -k 10 300 python -u tools/devpath_loop.py 5,3 3 > $OUT/devpath.txt 2>&1; rc=$?; cat $OUT/devpath.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/svc_probe.py 1000 3,5 > $OUT/svc_probe.txt 2>&1; rc=$?; grep "timing=" $OUT/svc_probe.txt; exit $rc
