#!/bin/bash
# SQ / TCC counter passes (one rocprofv3 --pmc run each) over tools/bench_configs.py --configs ${CFGS:-3} (GPU box).
export TMPDIR=/tmp
ROOTDIR=$(pwd)
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
            "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  out="$ROOTDIR/gpurun_out/pmccfg${CFGS:-3}_$i"
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d "$out" -o run -- \
     python3 "$ROOTDIR/tools/bench_configs.py" --configs "${CFGS:-3}" --reps 1 > "$out.log" 2>&1) || exit $?
done
echo done
