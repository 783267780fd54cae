export TMPDIR=/tmp
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export GNCDE_LIB=$PWD/abtest/libgncde_old.so GNCDE_LIB_UNVERIFIED=1; else unset GNCDE_LIB; fi
    timeout -k 10 120 python tools/bench_configs.py --configs 5 --reps 5 > gpurun_out/ab5_$v.log 2>&1 || exit $?
    echo "$v $(grep -m1 tsit5pid\" gpurun_out/ab5_$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_solve"])')"
  done
done
