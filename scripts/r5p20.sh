#!/bin/bash
out=gpurun_out/r5/${1:-p20}
mkdir -p $out
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
for c in 3 5; do
timeout -k 10 300 taskset -c $(cat /sys/devices/system/node/node$node/cpulist) python tools/gap_probe.py "" $c >> $out/gap.txt 2>&1 || { cat $out/gap.txt; exit 3; }
done
grep -v amdgpu.ids $out/gap.txt
