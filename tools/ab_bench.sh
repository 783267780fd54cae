#!/bin/bash
# A/B timing of two builds of libgncde_hip.so on one box (config-2 bench, alternating runs).
# Usage: tools/ab_bench.sh OLD_SO [ROUNDS]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
OLD=$1; R=${2:-3}
for r in $(seq 1 "$R"); do
  for v in old new; do
    if [ $v = old ]; then export GNCDE_LIB=$PWD/$OLD GNCDE_LIB_UNVERIFIED=1; else unset GNCDE_LIB; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --train-steps 0 > gpurun_out/ab_$v.log 2>&1 || exit $?
    echo "$v $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
  done
done
