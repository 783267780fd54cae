#!/bin/bash
# Round 5 checkpoint (GPU box): the full GPU suite, smoke, and the default bench run (the driver's N = 1 command).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/w_pytest_gpu.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 4 gpurun_out/w_pytest_gpu.log | cut -c1-250
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_session.sh smoke bench || exit $?
echo r05w done
