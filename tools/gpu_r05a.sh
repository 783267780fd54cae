#!/bin/bash
# Round-5 baseline (GPU box): the driver's exact bench command under rocprofv3 --kernel-trace --stats (its line and
# kernel statistics from one run), the GPU suite at HEAD, and the config 3-5 timings.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
(cd /tmp && rm -rf "$R/gpurun_out/prof_driver" && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$R/gpurun_out/prof_driver" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
   > "$R/gpurun_out/prof_driver.log" 2>&1); rc=$?; echo "prof rc=$rc"; tail -n 3 gpurun_out/prof_driver.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/bench_configs.py --configs 3,5 > gpurun_out/configs_a.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs 5 --batch5 64 > gpurun_out/cfg5_64_a.jsonl 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tall_a.log 2>&1; echo "tests rc=$?"
tail -n 5 gpurun_out/tall_a.log
echo r05a done
