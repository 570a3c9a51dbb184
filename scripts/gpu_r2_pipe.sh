set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_pytest.log 2>&1 || { tail -40 gpurun_out/pipe_pytest.log; exit 1; }
tail -2 gpurun_out/pipe_pytest.log
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/pipe_hostapi.txt 2>&1 || exit $?
cat gpurun_out/pipe_hostapi.txt
JSP_NO_PIPE=1 timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/nopipe_hostapi.txt 2>&1 || exit $?
cat gpurun_out/nopipe_hostapi.txt
