set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/walk_hostapi.txt 2>&1 || exit $?
echo all-done
