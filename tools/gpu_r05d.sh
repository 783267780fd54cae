#!/bin/bash
# Round 5 (GPU box): the kink-screened tests verbose, the TGB bf16-storage run, config 5 at B = 16 / 32 / 64 (two
# workgroups per CU by default), the driver's bench command under rocprofv3 --kernel-trace --stats, the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 700 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_grad.py::test_stage_record_matches_recompute" \
  "tests/test_gpu_grad.py::test_pid_solve_gradient_matches_oracle" \
  "tests/test_gpu_run.py" > gpurun_out/d_sel.log 2>&1; rc=$?; echo "sel-tests rc=$rc"
grep -E "PASSED|FAILED|ERROR|redrawn|moves" gpurun_out/d_sel.log | cut -c1-180
case $rc in 124|134|137|139) exit $rc;; esac
for B in 16 32 64; do
  timeout -k 10 300 python tools/bench_configs.py --configs 5 --quick --batch5 $B --reps 3 > gpurun_out/d_cfg5_B${B}.jsonl 2>&1 || exit $?
  echo "B=$B"; grep -o '"config": "[^"]*"\|"ms_per_solve": [0-9.]*' gpurun_out/d_cfg5_B${B}.jsonl | paste -sd' '
done
(cd /tmp && rm -rf "$R/gpurun_out/prof_d" && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$R/gpurun_out/prof_d" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
   > "$R/gpurun_out/prof_d.log" 2>&1); rc=$?; echo "prof rc=$rc"; grep '^{' gpurun_out/prof_d.log | cut -c1-300
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tall_d.log 2>&1; echo "tests rc=$?"
tail -n 8 gpurun_out/tall_d.log
echo r05d done
