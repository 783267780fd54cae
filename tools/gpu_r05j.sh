#!/bin/bash
# Round 5 final evidence, part 1 (GPU box): the GPU suite, smoke, the driver's exact bench command under rocprofv3
# --kernel-trace --stats, the FETCH_SIZE / WRITE_SIZE passes and the SQ passes of config 2's k_fused.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/j_pytest_gpu.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 6 gpurun_out/j_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_session.sh smoke profdrv pmc pmcsq || exit $?
echo r05j done
