# launch + completion floor of the host path (tools/launch_probe2.hip) next to
# the library's host-API phases
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 tools/diag/launch_probe2 > gpurun_out/floor_probe.txt 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 tools/diag/launch_probe2 > gpurun_out/floor_probe_hostkernarg.txt 2>&1 || exit $?
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/floor_hostapi.txt 2>&1 || exit $?
echo done
