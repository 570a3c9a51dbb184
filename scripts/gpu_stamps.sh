# Diagnostic: per-workgroup stamp timelines (diag build) + dispatch probe
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/diag/dispatch_probe > gpurun_out/dispatch_probe.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 2 60 > gpurun_out/stamps2.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 1 60 > gpurun_out/stamps1.log 2>&1 || exit $?
echo stamps-done
