#!/bin/bash
# Round-4 check batch (GPU box): config tests and gradient tests, then config 3 / 5 forward and gradient timings.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_grad.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t4.log 2>&1; echo "tests rc=$?"
timeout -k 10 200 python tools/bench_configs.py --configs ${CFGS:-3} > gpurun_out/cfg3.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_grad_configs.py --configs ${GCFGS:-3,5} > gpurun_out/grad3.jsonl 2>&1 || exit $?
GNCDE_LIB=$(pwd)/build_alt/libgncde_hip.so timeout -k 10 200 python tools/diag_bwd_stamps.py > gpurun_out/bwd3.log 2>&1
GNCDE_LIB=$(pwd)/build_alt/libgncde_hip.so DIAG_CFG=5 timeout -k 10 200 python tools/diag_bwd_stamps.py > gpurun_out/bwd5.log 2>&1
echo done
