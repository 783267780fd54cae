#!/bin/bash
# Round-4 closing evidence (GPU box), after the late forward / reverse changes: the full GPU suite, the config
# timings (configs 3-5, config 5 at B = 64), the gradient timings and the kernel statistics of both.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tall.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python tools/bench_configs.py --configs 3,4,5 > gpurun_out/configs_final.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs 5 --batch5 64 > gpurun_out/cfg5_64.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_grad_configs.py --configs 3,5 > gpurun_out/grad_final.jsonl 2>&1 || exit $?
CFGS=3,5 bash tools/gpu_session.sh profcfg profgrad || exit $?
echo r04f done
