#!/bin/bash
# Round 5 (GPU box): overlapped forms (side stream, one evaluation ahead): parity tests, then config 3 with and
# without (GNCDE_FORMS_OVERLAP=0), alternating, and its kernel statistics.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_configs.py::test_forms_overlap_bitwise" "tests/test_gpu_configs.py::test_config3_exact_shape_trajectory_and_gradient" \
  "tests/test_gpu_configs.py::test_activation_record_matches_recompute" "tests/test_gpu_configs.py::test_readout_tiles_bitwise" \
  "tests/test_gpu_parity.py" > gpurun_out/q_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 4 gpurun_out/q_tests.log | cut -c1-250
case $rc in 0|1) ;; *) exit $rc;; esac
for r in 1 2; do
  for v in 1 0; do
    GNCDE_FORMS_OVERLAP=$v timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/q_cfg3_O${v}_$r.jsonl 2>&1 || exit $?
    echo "overlap=$v $(grep -o '"ms_per_solve": [0-9.]*' gpurun_out/q_cfg3_O${v}_$r.jsonl | head -1)"
  done
done
echo r05q done
