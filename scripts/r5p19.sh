#!/bin/bash
out=gpurun_out/r5/${1:-p19}
mkdir -p $out
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
timeout -k 10 300 taskset -c $(cat /sys/devices/system/node/node$node/cpulist) python tools/split_probe.py > $out/split_probe.txt 2>&1 || { cat $out/split_probe.txt; exit 3; }
grep -v amdgpu.ids $out/split_probe.txt
