# resident service: parity tests, then the host-API latency probe
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_service_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/svc_pytest.log 2>&1 || { tail -30 gpurun_out/svc_pytest.log; exit 1; }
tail -3 gpurun_out/svc_pytest.log
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/svc_hostapi.txt 2>&1 || exit $?
cat gpurun_out/svc_hostapi.txt
timeout -k 10 120 tools/diag/launch_probe2 > gpurun_out/floor_probe.txt 2>&1 || exit $?
echo done
