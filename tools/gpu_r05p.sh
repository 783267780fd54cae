#!/bin/bash
# Round 5 (GPU box): the persistent solve's sample queue (one launch past the resident groups): the GPU suite, then
# config 5 at B = 48 / 64 with the queue vs the chunked launches (GNCDE_SOLVE_CHUNKED=1), alternating.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/p_pytest_gpu.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 6 gpurun_out/p_pytest_gpu.log | cut -c1-250
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  for v in 0 1; do
    for B in 48 64; do
      GNCDE_SOLVE_CHUNKED=$v timeout -k 10 200 python tools/bench_configs.py --configs 5 --quick --batch5 $B --reps 3 > gpurun_out/p_cfg5_C${v}_B$B_$r.jsonl 2>&1 || exit $?
      echo "chunked=$v B=$B $(grep -o '"ms_per_solve": [0-9.]*' gpurun_out/p_cfg5_C${v}_B$B_$r.jsonl | paste -sd' ')"
    done
  done
done
echo r05p done
