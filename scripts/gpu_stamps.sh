# Diagnostic: per-workgroup stamp timelines (diag build), idle-start and back-to-back
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py 2 60 1 > gpurun_out/stamps2_idle.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 2 60 20 > gpurun_out/stamps2_b2b.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 4 20 5 > gpurun_out/stamps4_b2b.log 2>&1 || exit $?
echo stamps-done
