#!/bin/bash
# Round 5 final evidence, part 2 (GPU box): SQ / TCC counter passes over configs 3 and 5 (tools/pmc_configs.sh), the
# kernel statistics of both, their timings (B = 16 and 64 for config 5), the training-step gradients, and the
# persistent solve's phase stamps at B = 16 and 32 (stamps build in build_alt/).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 16 32; do
  DIAG_SOLVE=1 DIAG_B=$B GNCDE_LIB=$PWD/build_alt/libgncde_hip.so timeout -k 10 200 python tools/diag_rows_stamps.py > gpurun_out/k_solve_stamps_b$B.txt 2>&1 || exit $?
  echo "== solve stamps B=$B"; grep -v Warning gpurun_out/k_solve_stamps_b$B.txt | tail -22
done
CFGS="3 5" bash tools/gpu_session.sh pmccfg || exit $?
CFGS=3,5 bash tools/gpu_session.sh profcfg || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs 3,5 > gpurun_out/k_configs.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs 5 --quick --batch5 64 > gpurun_out/k_cfg5_b64.jsonl 2>&1 || exit $?
timeout -k 10 400 python tools/bench_grad_configs.py > gpurun_out/k_grad_configs.jsonl 2>&1 || exit $?
grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*\|"B": [0-9]*' gpurun_out/k_configs.jsonl gpurun_out/k_cfg5_b64.jsonl | paste -sd' ' | cut -c1-900
tail -n 4 gpurun_out/k_grad_configs.jsonl | cut -c1-300
echo r05k done
