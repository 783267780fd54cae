#!/bin/bash
# Time bench.py (config 2) on the in-tree library and on every variants/libgncde_*.so (GPU box).
export TMPDIR=/tmp
out=gpurun_out/variants.log; : > $out
for lib in "" variants/libgncde_*.so; do
  GNCDE_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/v.json 2>/dev/null || { echo "FAIL $lib" >> $out; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/v.json').read().strip().split('\n')[-1]); print(sys.argv[1] or 'in-tree', d['ms_per_step'], d['roofline']['kernel_ms'])" "$lib" >> $out
done
cat $out
