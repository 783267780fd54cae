#!/bin/bash
# Round 5 (GPU box): A/B of the granule hand-offs (in-tree) against the counter hand-offs (abtest/libgncde_old.so,
# commit 072f6b5) on config 5, then the fault test and the rows PID gradient test.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_config5.sh || exit $?
timeout -k 10 400 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_configs.py::test_barrier_fault_is_reported" \
  "tests/test_gpu_grad.py::test_pid_solve_gradient_matches_oracle" > gpurun_out/g_sel.log 2>&1; echo "sel rc=$?"
grep -E "PASSED|FAILED|ERROR|redrawn|worst" gpurun_out/g_sel.log | cut -c1-160
echo r05g done
