#!/bin/bash
# the service stop's anatomy: a service-shaped persistent kernel stopped from the host, then the engine's own stop
out=gpurun_out/r5/${1:-p25}
mkdir -p $out
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
cpus=$(cat /sys/devices/system/node/node$node/cpulist)
timeout -k 10 120 taskset -c $cpus tools/bin/stop_anatomy > $out/anatomy.txt 2>&1 || { cat $out/anatomy.txt; exit 3; }
cat $out/anatomy.txt
timeout -k 10 300 taskset -c $cpus python tools/stop_probe.py > $out/stop.txt 2>&1 || { cat $out/stop.txt; exit 4; }
grep -v amdgpu.ids $out/stop.txt
