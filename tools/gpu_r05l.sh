#!/bin/bash
# Round 5 (GPU box): the GPU suite after folding the stage combination into the forms launch, then config 3 timings.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/l_pytest_gpu.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 8 gpurun_out/l_pytest_gpu.log | cut -c1-250
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/l_cfg3_$r.jsonl 2>&1 || exit $?
  echo "$(grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*' gpurun_out/l_cfg3_$r.jsonl | paste -sd' ' | cut -c1-300)"
done
echo r05l done
