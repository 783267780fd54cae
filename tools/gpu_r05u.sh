#!/bin/bash
# Round 5 (GPU box): the bf16-storage solve's LDS coefficient cache: parity (cache vs reload, bf16 tests, config 5
# tests), then config 5 at B = 16 with and without the cache, alternating.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_configs.py::test_rows_solve_coef_cache_bitwise" tests/test_gpu_bf16.py \
  "tests/test_gpu_configs.py::test_rows_pid_batch_independent" "tests/test_gpu_configs.py::test_rows_solve_sample_queue_bitwise" \
  "tests/test_gpu_configs.py::test_config5_pid_record_backward_equals_replay" > gpurun_out/u_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 4 gpurun_out/u_tests.log | cut -c1-250
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2 3; do
  for v in 1 0; do
    GNCDE_SOLVE_COEF_CACHE=$v timeout -k 10 200 python tools/bench_configs.py --configs 5 --quick --batch5 16 --reps 3 > gpurun_out/u_cfg5_C${v}_$r.jsonl 2>&1 || exit $?
    echo "cache=$v $(grep -o '"ms_per_solve": [0-9.]*\|"steps_max_rel_diff_vs_fp32": [0-9.]*' gpurun_out/u_cfg5_C${v}_$r.jsonl | paste -sd' ')"
  done
done
echo r05u done
