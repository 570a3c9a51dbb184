#!/bin/bash
# the settle's reading of the tiles' lines, prefetched: service GPU tests, then the bench's cold legs
out=gpurun_out/r5/${1:-p32}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -60 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 4; }
python - <<PY
import json
d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['host_api_step_p50_us'], d['cpu_baseline']['gpu_over_best_cpu'])
for c in ('cfg3','cfg5'):
    hc=d['configs'][c]['host_api_cold_recovery']
    print(c, d['configs'][c]['host_api_resident'], {g: (hc[g]['p50_us'], hc[g]['p99_us'], hc[g]['patch_p50_us'], hc[g]['place_p50_us']) for g in ('gap_1ms','gap_10ms')})
    print('  cpu', {g: (v['best_cpu_p50_us'], v['best_cpu_p99_us']) for g, v in hc['vs_cpu'].items()})
for n in ('cold_recovery','cold_recovery_parked'):
    print(n, {g: (v['gpu_p50_us'], v['gpu_p99_us'], v['best_cpu_p50_us'], v['best_cpu_p99_us']) for g, v in d[n]['vs_cpu'].items()})
PY
