#!/bin/bash
# A/B of library builds / switches on one box (GPU): abtest/libgncde_old.so (GNCDE_LIB, provenance check waived),
# the in-tree build, and the in-tree build with GNCDE_GRAN_POLL1=1, alternating, over config 5's persistent solve at
# B = ${AB_B:-16 32} (tools/bench_configs.py).
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in old new poll1; do
    for B in ${AB_B:-16 32}; do
      unset GNCDE_LIB GNCDE_LIB_UNVERIFIED GNCDE_GRAN_POLL1
      if [ $v = old ]; then export GNCDE_LIB=$PWD/abtest/libgncde_old.so GNCDE_LIB_UNVERIFIED=1; fi
      if [ $v = poll1 ]; then export GNCDE_GRAN_POLL1=1; fi
      timeout -k 10 200 python tools/bench_configs.py --configs 5 --quick --batch5 $B --reps 3 > gpurun_out/ab5_${v}_$B.log 2>&1 || exit $?
      echo "$v B=$B $(grep -o '"ms_per_solve": [0-9.]*' gpurun_out/ab5_${v}_$B.log | paste -sd' ' | cut -c1-300)"
    done
  done
done
