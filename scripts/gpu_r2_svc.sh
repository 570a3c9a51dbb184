# resident service: parity tests, the phase probe, the bench line
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_service_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/svc_pytest.log 2>&1 || { tail -30 gpurun_out/svc_pytest.log; exit 1; }
tail -3 gpurun_out/svc_pytest.log
timeout -k 10 200 python3 tools/svc_probe.py 2000 > gpurun_out/svc_probe.txt 2>&1 || { cat gpurun_out/svc_probe.txt; exit 1; }
cat gpurun_out/svc_probe.txt
timeout -k 10 400 python bench.py > gpurun_out/svc_bench.json 2> gpurun_out/svc_bench.err || { tail gpurun_out/svc_bench.err; exit 1; }
echo bench-ok
