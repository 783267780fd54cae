#!/bin/bash
# Run GPU steps on the gpurun box; each step has its own time limit and the session stops at the first
# crash / abort / timeout (exit 124, 134, 137, 139).  Usage: tools/gpu_session.sh STEP...
#   tests  : pytest -m gpu
#   smoke  : __graft_entry__.smoke()
#   bench  : python bench.py (default args)
#   prof   : rocprofv3 --kernel-trace --stats on bench.py (summary into gpurun_out/prof)
#   pmc    : rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes (separate runs)
#   profdrv: rocprofv3 --kernel-trace --stats on the driver's exact bench command (--gpus 1 --steps 20 --warmup 5)
#   pmccfg : SQ / TCC counter passes over tools/bench_configs.py for each config in $CFGS (tools/pmc_configs.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
ROOTDIR=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "FATAL in $name: stopping"; exit $rc;; esac
  return 0
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -s -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sel) run pytest_sel 900 python -u -m pytest ${SEL:-tests/test_gpu_grad.py} -v -s -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    benchtrain) run bench_train 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    bench8) run bench_quick 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    prof) (cd /tmp && run_dir="$ROOTDIR/gpurun_out/prof" && rm -rf "$run_dir" && \
           timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$run_dir" -o run -- \
             python3 "$ROOTDIR/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --train-steps 0 > "$ROOTDIR/gpurun_out/prof.log" 2>&1; \
           rc=$?; echo "prof rc=$rc"; tail -n 5 "$ROOTDIR/gpurun_out/prof.log"; \
           case $rc in 124|134|137|139) exit $rc;; esac) || exit $? ;;
    profdrv) (cd /tmp && run_dir="$ROOTDIR/gpurun_out/prof_driver" && rm -rf "$run_dir" && \
           timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$run_dir" -o run -- \
             python3 "$ROOTDIR/bench.py" --gpus 1 --steps 20 --warmup 5 > "$ROOTDIR/gpurun_out/prof_driver.log" 2>&1; \
           rc=$?; echo "profdrv rc=$rc"; tail -n 3 "$ROOTDIR/gpurun_out/prof_driver.log"; \
           case $rc in 124|134|137|139) exit $rc;; esac) || exit $? ;;
    pmccfg) for c in ${CFGS:-3 5}; do CFGS=$c bash tools/pmc_configs.sh || exit $?; echo "pmccfg $c done"; done ;;
    pmc) for ctr in FETCH_SIZE WRITE_SIZE; do
           (cd /tmp && run_dir="$ROOTDIR/gpurun_out/pmc_$ctr" && rm -rf "$run_dir" && \
            timeout -k 10 900 rocprofv3 --pmc $ctr --output-format csv -d "$run_dir" -o run -- \
              python3 "$ROOTDIR/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --train-steps 0 > "$ROOTDIR/gpurun_out/pmc_$ctr.log" 2>&1; \
            rc=$?; echo "pmc $ctr rc=$rc"; tail -n 3 "$ROOTDIR/gpurun_out/pmc_$ctr.log"; \
            case $rc in 124|134|137|139) exit $rc;; esac) || exit $?
         done ;;
    listctr) run listctr 300 rocprofv3 -L ;;
    profcfg) (cd /tmp && run_dir="$ROOTDIR/gpurun_out/profcfg" && rm -rf "$run_dir" && \
           timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$run_dir" -o run -- \
             python3 "$ROOTDIR/tools/bench_configs.py" --configs "${CFGS:-3,5}" --reps 2 > "$ROOTDIR/gpurun_out/profcfg.log" 2>&1; \
           rc=$?; echo "profcfg rc=$rc"; tail -n 5 "$ROOTDIR/gpurun_out/profcfg.log"; \
           case $rc in 124|134|137|139) exit $rc;; esac) || exit $? ;;
    proftrain) (cd /tmp && run_dir="$ROOTDIR/gpurun_out/proftrain" && rm -rf "$run_dir" && \
           timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$run_dir" -o run -- \
             python3 "$ROOTDIR/tools/bench_train.py" --steps 2 --warmup 1 > "$ROOTDIR/gpurun_out/proftrain.log" 2>&1; \
           rc=$?; echo "proftrain rc=$rc"; tail -n 5 "$ROOTDIR/gpurun_out/proftrain.log"; \
           case $rc in 124|134|137|139) exit $rc;; esac) || exit $? ;;
    configs) run configs 900 python tools/bench_configs.py ;;
    gradcfg) run gradcfg 900 python tools/bench_grad_configs.py ;;
    profgrad) (cd /tmp && run_dir="$ROOTDIR/gpurun_out/profgrad" && rm -rf "$run_dir" && \
           timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$run_dir" -o run -- \
             python3 "$ROOTDIR/tools/bench_grad_configs.py" --configs "${CFGS:-5}" --reps 1 > "$ROOTDIR/gpurun_out/profgrad.log" 2>&1; \
           rc=$?; echo "profgrad rc=$rc"; tail -n 5 "$ROOTDIR/gpurun_out/profgrad.log"; \
           case $rc in 124|134|137|139) exit $rc;; esac) || exit $? ;;
    pmcsq) i=0; for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
                          "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
                          "TCC_HIT_sum TCC_MISS_sum"; do
           i=$((i+1))
           (cd /tmp && run_dir="$ROOTDIR/gpurun_out/pmcsq_$i" && rm -rf "$run_dir" && \
            timeout -k 10 900 rocprofv3 --pmc $ctrs --output-format csv -d "$run_dir" -o run -- \
              python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --train-steps 0 > "$ROOTDIR/gpurun_out/pmcsq_$i.log" 2>&1; \
            rc=$?; echo "pmcsq $i rc=$rc"; tail -n 3 "$ROOTDIR/gpurun_out/pmcsq_$i.log"; \
            case $rc in 124|134|137|139) exit $rc;; esac) || exit $?
         done ;;
    pmctrain) i=0; for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
                          "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
                          "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
           i=$((i+1))
           (cd /tmp && run_dir="$ROOTDIR/gpurun_out/pmctrain_$i" && rm -rf "$run_dir" && \
            timeout -k 10 900 rocprofv3 --pmc $ctrs --output-format csv -d "$run_dir" -o run -- \
              python3 "$ROOTDIR/tools/bench_train.py" --steps 1 --warmup 0 --rk4-steps 10 > "$ROOTDIR/gpurun_out/pmctrain_$i.log" 2>&1; \
            rc=$?; echo "pmctrain $i rc=$rc"; tail -n 2 "$ROOTDIR/gpurun_out/pmctrain_$i.log"; \
            case $rc in 124|134|137|139) exit $rc;; esac) || exit $?
         done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done"
