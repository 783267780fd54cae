#!/bin/bash
# Round 5 (GPU box): the read-out K loop with A operands formed a step ahead: parity, phase stamps, config 3 timing.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_gpu_configs.py::test_readout_tiles_bitwise" "tests/test_gpu_configs.py::test_config3_exact_shape_trajectory_and_gradient" > gpurun_out/o_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 gpurun_out/o_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
GNCDE_LIB=$PWD/build_alt/libgncde_hip.so timeout -k 10 200 python tools/diag_layer_stamps.py > gpurun_out/o_stamps_T5.txt 2>&1 || exit $?
grep -v Warning gpurun_out/o_stamps_T5.txt | tail -9
for r in 1 2; do
  for v in 5 2; do
    GNCDE_READOUT_TILES=$v timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/o_cfg3_T${v}_$r.jsonl 2>&1 || exit $?
    echo "tiles=$v $(grep -o '"ms_per_solve": [0-9.]*' gpurun_out/o_cfg3_T${v}_$r.jsonl | head -1)"
  done
done
echo r05o done
