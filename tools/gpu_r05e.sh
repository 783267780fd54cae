#!/bin/bash
# Round 5 (GPU box): the re-screened PID gradient tests, the config-3 end-to-end gradient and the reference TGB grid
# tests verbose; the driver's bench command under rocprofv3 --kernel-trace --stats; the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 800 python -u -m pytest -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
  "tests/test_gpu_grad.py::test_pid_solve_gradient_matches_oracle" \
  "tests/test_gpu_configs.py::test_config3_exact_shape_trajectory_and_gradient" \
  "tests/test_gpu_configs.py::test_config5_reference_tgb_grid_vs_oracle" > gpurun_out/e_sel.log 2>&1; rc=$?; echo "sel-tests rc=$rc"
grep -E "PASSED|FAILED|ERROR|redrawn|moves|skipped|worst|window|record vs" gpurun_out/e_sel.log | cut -c1-200
case $rc in 124|134|137|139) exit $rc;; esac
(cd /tmp && rm -rf "$R/gpurun_out/prof_e" && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$R/gpurun_out/prof_e" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
   > "$R/gpurun_out/prof_e.log" 2>&1); rc=$?; echo "prof rc=$rc"; grep '^{' gpurun_out/prof_e.log | cut -c1-300
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/tall_e.log 2>&1; echo "tests rc=$?"
tail -n 8 gpurun_out/tall_e.log
echo r05e done
