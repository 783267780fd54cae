#!/bin/bash
# A/B of two library builds on one box (GPU): abtest/libgncde_old.so (GNCDE_LIB, provenance check waived) against
# the in-tree build, alternating, over config 5's persistent solve at B = ${AB_B:-16 32} (tools/bench_configs.py).
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in old new; do
    for B in ${AB_B:-16 32}; do
      if [ $v = old ]; then export GNCDE_LIB=$PWD/abtest/libgncde_old.so GNCDE_LIB_UNVERIFIED=1; else unset GNCDE_LIB GNCDE_LIB_UNVERIFIED; fi
      timeout -k 10 200 python tools/bench_configs.py --configs 5 --quick --batch5 $B --reps 3 > gpurun_out/ab5_${v}_$B.log 2>&1 || exit $?
      echo "$v B=$B $(grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*' gpurun_out/ab5_${v}_$B.log | paste -sd' ' | cut -c1-400)"
    done
  done
done
