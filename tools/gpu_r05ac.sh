#!/bin/bash
# Round 5 (GPU box): the stage combination folded into the read-out epilogue (GNCDE_COMBO_FOLD).  Parity (placements bitwise, config 3 exact shape,
# activation record, generic parity), then config 3 alternating: ride (default) vs GNCDE_FORMS_RIDE=0 vs the HEAD build.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_configs.py::test_forms_overlap_bitwise" "tests/test_gpu_configs.py::test_config3_exact_shape_trajectory_and_gradient" \
  "tests/test_gpu_configs.py::test_activation_record_matches_recompute" "tests/test_gpu_configs.py::test_readout_tiles_bitwise" \
  tests/test_gpu_parity.py > gpurun_out/ac_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 4 gpurun_out/ac_tests.log | cut -c1-250
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2 3; do
  for v in old nofold fold; do
    unset GNCDE_LIB GNCDE_LIB_UNVERIFIED GNCDE_COMBO_FOLD
    if [ $v = old ]; then export GNCDE_LIB=$PWD/abtest/libgncde_old.so GNCDE_LIB_UNVERIFIED=1; fi
    if [ $v = nofold ]; then export GNCDE_COMBO_FOLD=0; fi
    timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/ac_cfg3_${v}_$r.jsonl 2>&1 || exit $?
    echo "$v $(grep -o '"ms_per_solve": [0-9.]*' gpurun_out/ac_cfg3_${v}_$r.jsonl | head -1)"
  done
done
echo r05ac done
