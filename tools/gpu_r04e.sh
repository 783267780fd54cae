#!/bin/bash
# Round-4 final evidence (GPU box): the full GPU suite, then bench.py, its rocprofv3 kernel stats and PMC passes
# (the same command), the config timings and the gradient timings.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tall.log 2>&1; echo "tests rc=$?"
bash tools/gpu_session.sh bench prof pmc pmcsq || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs 3,4,5 > gpurun_out/configs_final.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs 5 --batch5 64 > gpurun_out/cfg5_64.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_grad_configs.py --configs 3,5 > gpurun_out/grad_final.jsonl 2>&1 || exit $?
bash tools/gpu_session.sh profgrad || exit $?
echo r04e done
