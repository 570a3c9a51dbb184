set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
nproc > gpurun_out/g1_cpu.txt; grep -m1 "model name" /proc/cpuinfo >> gpurun_out/g1_cpu.txt; grep -m1 flags /proc/cpuinfo | tr ' ' '\n' | grep -E "avx2|avx512f" | tr '\n' ' ' >> gpurun_out/g1_cpu.txt
python3 -c "import os;print('affinity',len(os.sched_getaffinity(0)), 'omp', os.environ.get('OMP_NUM_THREADS'))" >> gpurun_out/g1_cpu.txt
timeout -k 10 120 ./tools/diag/launch_probe > gpurun_out/g1_probe.txt 2>&1 || exit $?
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/g1_hostapi.txt 2>&1 || exit $?
echo done
