set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --trials 300 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --trials 0 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1
echo "prof rc=$?"
