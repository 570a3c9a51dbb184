#!/bin/bash
out=gpurun_out/r5/${1:-p22}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py tests/test_multi_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -60 $out/pytest.log; exit 2; }
tail -2 $out/pytest.log
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
for h in "" wait_delay_ns=12000; do
echo "hooks: $h" >> $out/split.txt
timeout -k 10 300 taskset -c $(cat /sys/devices/system/node/node$node/cpulist) python tools/split_probe.py "$h" >> $out/split.txt 2>&1 || { cat $out/split.txt; exit 3; }
done
grep -v amdgpu.ids $out/split.txt
