# GPU parity tests + per-kernel breakdown (each step time-limited, stop on failure)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/breakdown.py > gpurun_out/breakdown.log 2>&1 || exit $?
cat gpurun_out/breakdown.log
