#!/bin/bash
# Round 5 (GPU box): k_fused with the form's sums taken from the operand-build reads: fused parity tests and smoke,
# then config 2 A/B against the previous build (abtest/libgncde_old.so), alternating.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_configs.py::test_fused_configs_exact_shape_vs_oracle tests/test_gpu_models.py tests/test_gpu_bf16.py \
  tests/test_gpu_grad.py -k "fused or stage or config" > gpurun_out/r_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 4 gpurun_out/r_tests.log | cut -c1-250
case $rc in 0|1|5) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -2
bash tools/ab_bench.sh abtest/libgncde_old.so 4 || exit $?
echo r05r done
