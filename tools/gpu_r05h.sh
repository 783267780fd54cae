#!/bin/bash
# Round 5 (GPU box): the five-tile CDE read-out (parity test, then config 3 A/B against GNCDE_READOUT_TILES=2), the
# granule hand-off A/B on config 5 (tools/ab_config5.sh), then the barrier fault test and the PID gradient test.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_gpu_configs.py::test_readout_tiles_bitwise" > gpurun_out/h_readout.log 2>&1; rc=$?; echo "readout-test rc=$rc"
grep -E "PASSED|FAILED|Error|error" gpurun_out/h_readout.log | cut -c1-200 | head -20
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  for v in 5 2; do
    GNCDE_READOUT_TILES=$v timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/h_cfg3_T${v}_$r.jsonl 2>&1 || exit $?
    echo "tiles=$v $(grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*' gpurun_out/h_cfg3_T${v}_$r.jsonl | paste -sd' ' | cut -c1-300)"
  done
done
bash tools/ab_config5.sh || exit $?
timeout -k 10 400 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_configs.py::test_barrier_fault_is_reported" \
  "tests/test_gpu_grad.py::test_pid_solve_gradient_matches_oracle" > gpurun_out/h_sel.log 2>&1; echo "sel rc=$?"
grep -E "PASSED|FAILED|ERROR|redrawn|worst" gpurun_out/h_sel.log | cut -c1-160
echo r05h done
