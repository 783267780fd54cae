#!/bin/bash
# Round 5 (GPU box): where the riding forms go (GNCDE_FORMS_RIDE = 1 split, 2 first hidden launch, 3 last), config 3
# alternating, then a kernel trace of config 3 (default placement).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_gpu_configs.py::test_forms_overlap_bitwise" > gpurun_out/y_tests.log 2>&1 || { tail -5 gpurun_out/y_tests.log; exit 1; }
for r in 1 2 3; do
  for v in 1 2 3; do
    GNCDE_FORMS_RIDE=$v timeout -k 10 200 python tools/bench_configs.py --configs 3 --reps 3 > gpurun_out/y_cfg3_${v}_$r.jsonl 2>&1 || exit $?
    echo "$v $(grep -o '"ms_per_solve": [0-9.]*' gpurun_out/y_cfg3_${v}_$r.jsonl | head -1)"
  done
done
cd /tmp && run_dir="$ROOTDIR/gpurun_out/prof_y" && rm -rf "$run_dir" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$run_dir" -o run -- \
    python3 "$ROOTDIR/tools/bench_configs.py" --configs 3 --reps 2 > "$ROOTDIR/gpurun_out/prof_y.log" 2>&1
echo "prof rc=$?"
echo r05y done
