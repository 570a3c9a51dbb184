set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/grp_pytest.log 2>&1 || { tail -40 gpurun_out/grp_pytest.log; exit 1; }
tail -2 gpurun_out/grp_pytest.log
timeout -k 10 120 python tools/stamps_walk.py 5 1 20 > gpurun_out/walkstamps5g.log 2>&1 || exit $?
head -4 gpurun_out/walkstamps5g.log; grep -A3 "tally tiles" gpurun_out/walkstamps5g.log
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/grp_hostapi.txt 2>&1 || exit $?
cat gpurun_out/grp_hostapi.txt
