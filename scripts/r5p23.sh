#!/bin/bash
out=gpurun_out/r5/${1:-p23}
mkdir -p $out
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
timeout -k 10 300 taskset -c $(cat /sys/devices/system/node/node$node/cpulist) python tools/stop_probe.py > $out/stop.txt 2>&1 || { cat $out/stop.txt; exit 3; }
timeout -k 10 300 taskset -c $(cat /sys/devices/system/node/node$node/cpulist) python tools/bracket_probe.py 40 >> $out/stop.txt 2>&1 || { cat $out/stop.txt; exit 3; }
grep -v amdgpu.ids $out/stop.txt
