#!/bin/bash
# split-service stamps (cfg3, cfg5) and the driver bench line with equal-sample cold legs
out=gpurun_out/r5/${1:-p27}
mkdir -p $out
node=$(cat /sys/bus/pci/devices/$(python -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print(b.value.decode().lower())")/numa_node)
cpus=$(cat /sys/devices/system/node/node$node/cpulist)
timeout -k 10 300 taskset -c $cpus python tools/svc_probe.py 500 3,5 > $out/svc_probe.txt 2>&1 || { cat $out/svc_probe.txt; exit 3; }
grep -v amdgpu.ids $out/svc_probe.txt
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 4; }
python - <<PY
import json
d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'])
print('cfg2', d['cold_recovery']['vs_cpu'])
print('cfg2 parked', d['cold_recovery_parked'].get('vs_cpu'))
for c in ('cfg3','cfg5'):
    print(c, d['configs'][c]['host_api_cold_recovery'].get('vs_cpu'))
PY
