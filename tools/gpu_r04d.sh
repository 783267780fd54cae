#!/bin/bash
# Round-4 config-5 batch (GPU box): the persistent-solve tests, config 5 at B = 16 and 64, the solve's phase stamps.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1; echo "tests rc=$?"
timeout -k 10 200 python tools/bench_configs.py --configs 5 > gpurun_out/cfg5.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs 5 --batch5 64 > gpurun_out/cfg5_64.jsonl 2>&1 || exit $?
GNCDE_LIB=$R/build_alt/libgncde_hip.so DIAG_SOLVE=1 timeout -k 10 120 python tools/diag_rows_stamps.py > gpurun_out/stamps5.log 2>&1
GNCDE_LIB=$R/build_alt/libgncde_hip.so DIAG_SOLVE=1 DIAG_B=32 timeout -k 10 120 python tools/diag_rows_stamps.py > gpurun_out/stamps5_32.log 2>&1
echo done
