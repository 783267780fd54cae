#!/bin/bash
# Round-4 measurement batch on the GPU box: new config tests, config 3/5 timings, kernel stats of config 3's forward
# and backward, and the persistent solve's phase stamps (GNCDE_LIB = the -DGNCDE_ROWS_STAMPS build in build_alt/).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -v --timeout 280 --timeout-method thread > gpurun_out/t2.log 2>&1
echo "tests rc=$?"
timeout -k 10 200 python tools/bench_configs.py --configs 3,5 > gpurun_out/cfg2.jsonl 2>&1 || exit $?
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof3" -o run -- \
   python "$R/tools/bench_configs.py" --configs 3 --reps 2 > "$R/gpurun_out/prof3.log" 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof3g" -o run -- \
   python "$R/tools/bench_grad_configs.py" --configs 3 --reps 1 > "$R/gpurun_out/prof3g.log" 2>&1) || exit $?
GNCDE_LIB=$R/build_alt/libgncde_hip.so DIAG_SOLVE=1 timeout -k 10 120 python tools/diag_rows_stamps.py > gpurun_out/stamps5.log 2>&1
echo "stamps rc=$?"
