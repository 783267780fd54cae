#!/bin/bash
# Round 5 (GPU box): config 3 with the stage combination folded into the forms launch vs separate k_combo launches
# (GNCDE_COMBO_SEPARATE=1), alternating; then the kernel statistics of both.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
for r in 1 2 3; do
  for v in 0 1; do
    GNCDE_COMBO_SEPARATE=$v timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/m_cfg3_S${v}_$r.jsonl 2>&1 || exit $?
    echo "separate=$v $(grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*' gpurun_out/m_cfg3_S${v}_$r.jsonl | head -2 | paste -sd' ' | cut -c1-200)"
  done
done
for v in 0 1; do
  (cd /tmp && rm -rf "$R/gpurun_out/m_prof$v" && GNCDE_COMBO_SEPARATE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$R/gpurun_out/m_prof$v" -o run -- python3 "$R/tools/bench_configs.py" --configs 3 --reps 2 > "$R/gpurun_out/m_prof$v.log" 2>&1) || exit $?
  head -8 gpurun_out/m_prof$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
echo r05m done
