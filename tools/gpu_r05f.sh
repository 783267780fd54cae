#!/bin/bash
# Round 5 (GPU box): tagged-granule hand-offs in the persistent solve — the persistent-path tests first (verbose,
# bounded), then config 5 at B = 16 / 32 / 64, then the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_gpu_configs.py::test_config5_exact_shape_pid_replay" \
  "tests/test_gpu_configs.py::test_rows_pid_against_host_paced" \
  "tests/test_gpu_configs.py::test_rows_pid_batch_independent" \
  "tests/test_gpu_configs.py::test_rows_grid_against_host_paced_and_oracle" \
  "tests/test_gpu_configs.py::test_config5_reference_tgb_grid_vs_oracle" \
  "tests/test_gpu_configs.py::test_config5_pid_record_backward_equals_replay" \
  "tests/test_gpu_parity.py" > gpurun_out/f_sel.log 2>&1; rc=$?; echo "sel-tests rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/f_sel.log | cut -c1-160 | tail -30
case $rc in 0) ;; *) exit $rc;; esac
for B in 16 32 64; do
  timeout -k 10 300 python tools/bench_configs.py --configs 5 --quick --batch5 $B --reps 3 > gpurun_out/f_cfg5_B${B}.jsonl 2>&1 || exit $?
  echo "B=$B"; grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*' gpurun_out/f_cfg5_B${B}.jsonl | paste -sd' '
done
timeout -k 10 300 python tools/bench_grad_configs.py --configs 5 > gpurun_out/f_grad5.jsonl 2>&1 || exit $?
cut -c1-200 gpurun_out/f_grad5.jsonl | grep '^{'
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/tall_f.log 2>&1; echo "tests rc=$?"
tail -n 8 gpurun_out/tall_f.log
echo r05f done
