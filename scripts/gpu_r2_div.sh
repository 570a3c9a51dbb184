set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/div_pytest.log 2>&1 || { tail -40 gpurun_out/div_pytest.log; exit 1; }
tail -2 gpurun_out/div_pytest.log
timeout -k 10 200 python3 tools/tally_probe.py > gpurun_out/div_tally.txt 2>&1 || { cat gpurun_out/div_tally.txt; exit 1; }
cat gpurun_out/div_tally.txt
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/div_hostapi.txt 2>&1 || exit $?
cat gpurun_out/div_hostapi.txt
