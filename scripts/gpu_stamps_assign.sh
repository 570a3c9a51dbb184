cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps_assign.py 4 20 > gpurun_out/stamps_assign4.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps_assign.py 3 20 >> gpurun_out/stamps_assign4.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps_assign.py 5 20 >> gpurun_out/stamps_assign4.log 2>&1 || exit $?
