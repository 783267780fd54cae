#!/bin/bash
# Time the in-tree library and every variants/libgncde_*.so on one GPU box.
#   tools/bench_variants.sh            config 2 (bench.py)
#   tools/bench_variants.sh 3,5        configs 3 / 5 (tools/bench_configs.py)
export TMPDIR=/tmp
cfg=${1:-2}
out=gpurun_out/variants.log; : > $out
for lib in "" variants/libgncde_*.so; do
  name=${lib:-in-tree}
  if [ "$cfg" = "2" ]; then
    GNCDE_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/v.json 2>/dev/null || { echo "FAIL $name" >> $out; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/v.json').read().strip().split('\n')[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['kernel_ms'])" "$name" >> $out
  else
    GNCDE_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs $cfg > gpurun_out/v.json 2>/dev/null || { echo "FAIL $name" >> $out; exit 1; }
    python -c "
import json,sys
for l in open('gpurun_out/v.json'):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[1], d['config'], d['ms_per_solve'])" "$name" >> $out
  fi
done
cat $out
