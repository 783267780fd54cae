#!/bin/bash
# A/B of the persistent solve's hand-off variants on one box (GPU), alternating: the counter barriers (default),
# tagged granules (GNCDE_SOLVE_GRANULES=1) and granules polling one stale pair (+ GNCDE_GRAN_POLL1=1), over config 5's
# persistent solve at B = ${AB_B:-16 32} (tools/bench_configs.py).  AB_ROUNDS (default 3) alternations.
export TMPDIR=/tmp
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for v in counter gran poll1; do
    for B in ${AB_B:-16 32}; do
      unset GNCDE_SOLVE_GRANULES GNCDE_GRAN_POLL1
      if [ $v != counter ]; then export GNCDE_SOLVE_GRANULES=1; fi
      if [ $v = poll1 ]; then export GNCDE_GRAN_POLL1=1; fi
      timeout -k 10 200 python tools/bench_configs.py --configs 5 --quick --batch5 $B --reps 3 > gpurun_out/ab5_${v}_$B.log 2>&1 || exit $?
      echo "$v B=$B $(grep -o '"ms_per_solve": [0-9.]*' gpurun_out/ab5_${v}_$B.log | paste -sd' ' | cut -c1-300)"
    done
  done
done
