#!/bin/bash
# branch-free leaf sums in the resident evaluation: service + engine GPU tests, eval stamps, svc_probe, the driver bench line
out=gpurun_out/r5/${1:-p31}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -60 $out/pytest.log; exit 2; }
tail -2 $out/pytest.log
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
cpus=$(cat /sys/devices/system/node/node$node/cpulist)
timeout -k 10 200 taskset -c $cpus python tools/svc_probe.py 1000 2 > $out/svc_eval.txt 2>&1 || { cat $out/svc_eval.txt; exit 3; }
grep -v amdgpu $out/svc_eval.txt
timeout -k 10 200 taskset -c $cpus python tools/split_probe.py > $out/split.txt 2>&1 || { cat $out/split.txt; exit 5; }
grep -v amdgpu $out/split.txt
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 4; }
python -c "import json;d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_api_step_p50_us'],d['cpu_baseline']['gpu_over_best_cpu']);print(d['host_api_breakdown']);print(d['patched_step_us'])"
