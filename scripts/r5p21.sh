#!/bin/bash
out=gpurun_out/r5/${1:-p21}
mkdir -p $out
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
for h in "" wait_delay_ns=4000 wait_delay_ns=8000 wait_delay_ns=12000; do
echo "hooks: $h" >> $out/split.txt
timeout -k 10 300 taskset -c $(cat /sys/devices/system/node/node$node/cpulist) python tools/split_probe.py "$h" >> $out/split.txt 2>&1 || { cat $out/split.txt; exit 3; }
done
grep -v amdgpu.ids $out/split.txt
