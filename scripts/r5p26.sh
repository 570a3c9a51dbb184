#!/bin/bash
# the stop waits on an event behind the service: service + engine GPU tests, the stop probe, the driver bench line
out=gpurun_out/r5/${1:-p26}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -60 $out/pytest.log; exit 2; }
tail -2 $out/pytest.log
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
cpus=$(cat /sys/devices/system/node/node$node/cpulist)
timeout -k 10 300 taskset -c $cpus python tools/stop_probe.py > $out/stop.txt 2>&1 || { cat $out/stop.txt; exit 3; }
grep -v amdgpu.ids $out/stop.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 4; }
python -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step']);print({k:v for k,v in d.items() if 'patch' in k or 'host_api' in k})"
