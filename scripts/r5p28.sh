#!/bin/bash
# call-entry prefetch: service GPU tests, then the cold-recovery A/B (warm=0 vs default)
out=gpurun_out/r5/${1:-p28}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -60 $out/pytest.log; exit 2; }
tail -2 $out/pytest.log
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
cpus=$(cat /sys/devices/system/node/node$node/cpulist)
timeout -k 10 400 taskset -c $cpus python tools/warm_ab.py 50 2 > $out/warm_ab.txt 2>&1 || { cat $out/warm_ab.txt; exit 3; }
grep -v amdgpu.ids $out/warm_ab.txt
