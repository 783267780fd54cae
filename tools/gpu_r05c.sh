#!/bin/bash
# Round 5 (GPU box): the new / previously failing tests verbose; config 5 fp32 vs bf16-storage persistent solve at
# B = 16 / 32 / 64 with one and two workgroups per CU; config 5 gradient timings (record vs replay); the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_gpu_configs.py::test_rows_pid_against_host_paced" \
  "tests/test_gpu_configs.py::test_config5_pid_record_backward_equals_replay" \
  "tests/test_gpu_grad.py::test_stage_record_matches_recompute" \
  "tests/test_gpu_grad.py::test_pid_solve_gradient_matches_oracle" > gpurun_out/c_sel.log 2>&1; rc=$?; echo "sel-tests rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/c_sel.log | cut -c1-150
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/bench_grad_configs.py --configs 5 > gpurun_out/c_grad5.jsonl 2>&1 || exit $?
cut -c1-220 gpurun_out/c_grad5.jsonl | grep '^{'
for B in 16 32 64; do
  for W in 1 2; do
    GNCDE_SOLVE_WG_PER_CU=$W timeout -k 10 300 python tools/bench_configs.py --configs 5 --quick --batch5 $B --reps 2 \
      > gpurun_out/c_cfg5_B${B}_W${W}.jsonl 2>&1 || exit $?
    echo "B=$B W=$W"; grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*\|"steps_max_rel_diff_vs_fp32": [0-9.]*\|"rel_dev_vs_fp32": [0-9.e-]*' gpurun_out/c_cfg5_B${B}_W${W}.jsonl | paste -sd' '
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tall_c.log 2>&1; echo "tests rc=$?"
tail -n 12 gpurun_out/tall_c.log
echo r05c done
