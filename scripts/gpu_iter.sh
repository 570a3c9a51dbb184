# Iteration: GPU parity tests, short bench, kernel trace, b2b stamps (diag build)
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --trials 300 --cpu-seconds 2 > gpurun_out/bench.log 2>&1 || exit $?
cat gpurun_out/bench.log | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_iter" -o run --output-format csv -- python3 "$R/bench.py" --trials 0 --cpu-seconds 0 > "$R/gpurun_out/prof_iter.log" 2>&1 || exit $?
cd "$R"
if [ -f tools/diag/libjsplace.so ]; then
timeout -k 10 120 python tools/stamps.py 2 40 20 > gpurun_out/stamps2_b2b.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 4 15 5 > gpurun_out/stamps4_b2b.log 2>&1 || exit $?
fi
echo iter-done
