#!/bin/bash
# A/B of library builds on one box (GPU): AB_LIBS="base <dir>..." (base = the in-tree build), alternating twice,
# over tools/bench_configs.py --configs ${AB_CFGS:-3}.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
for round in 1 2; do
  for v in ${AB_LIBS:-base}; do
    if [ "$v" = base ]; then L=""; else L=$(pwd)/$v/libgncde_hip.so; fi
    echo "== $v"
    GNCDE_LIB=$L GNCDE_LIB_UNVERIFIED=1 timeout -k 10 200 python tools/bench_configs.py --configs ${AB_CFGS:-3} --reps 3 2>&1 | grep -v bf16 | grep '^{' | cut -c1-170 || exit $?
  done
done
