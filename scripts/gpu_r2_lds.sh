set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lds_pytest.log 2>&1 || { tail -30 gpurun_out/lds_pytest.log; exit 1; }
tail -2 gpurun_out/lds_pytest.log
timeout -k 10 120 python tools/stamps_walk.py 5 1 20 > gpurun_out/lds_st5.log 2>&1 || exit $?
grep "row 400" gpurun_out/lds_st5.log
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/lds_hostapi.txt 2>&1 || exit $?
grep "cfg" gpurun_out/lds_hostapi.txt
