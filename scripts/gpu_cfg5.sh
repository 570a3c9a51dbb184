# GPU parity tests, then kernel traces of cfg5 in both shapes
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
echo pytest-ok
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/cfg5_f$f" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 5 --steps 20 --fused $f > "$R/gpurun_out/cfg5_f$f.log" 2>&1 || exit $?
done
echo done
