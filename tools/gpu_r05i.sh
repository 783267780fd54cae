#!/bin/bash
# Round 5 (GPU box): the parity tests of the read-out tile variants and the solve's hand-off variants, the PID
# gradient test (diagnostics), config 3 with five- vs two-tile read-out workgroups, config 5 counters vs granules.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_gpu_configs.py::test_readout_tiles_bitwise" "tests/test_gpu_configs.py::test_rows_solve_granule_handoffs_bitwise" \
  "tests/test_gpu_configs.py::test_barrier_fault_is_reported" \
  "tests/test_gpu_grad.py::test_pid_solve_gradient_matches_oracle" > gpurun_out/i_tests.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "PASSED|FAILED|Error|worst|all:|l[0-9]\.param" gpurun_out/i_tests.log | cut -c1-220 | head -60
case $rc in 0|1) ;; *) exit $rc;; esac
for r in 1 2; do
  for v in 5 2; do
    GNCDE_READOUT_TILES=$v timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/i_cfg3_T${v}_$r.jsonl 2>&1 || exit $?
    echo "tiles=$v $(grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*' gpurun_out/i_cfg3_T${v}_$r.jsonl | paste -sd' ' | cut -c1-300)"
  done
done
AB_ROUNDS=1 bash tools/ab_config5.sh || exit $?
echo r05i done
