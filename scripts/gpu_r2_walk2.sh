# walker change: engine parity suite, then cfg5/cfg3 host-API and kernel times
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/walk2_pytest.log 2>&1 || { tail -30 gpurun_out/walk2_pytest.log; exit 1; }
tail -2 gpurun_out/walk2_pytest.log
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/walk2_hostapi.txt 2>&1 || exit $?
cat gpurun_out/walk2_hostapi.txt
