# quick iteration: GPU tests, host-API probe, stamps of cfg2 from idle
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/it_hostapi.txt 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 2 60 1 > gpurun_out/it_stamps2_idle.log 2>&1 || exit $?
echo all-done
