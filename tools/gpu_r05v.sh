#!/bin/bash
# Round 5 (GPU box): persistent-solve phase stamps at B = 16, fp32 and bf16 coefficient storage (stamps build).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in bf16_storage fp32; do
  DIAG_SOLVE=1 DIAG_B=16 DIAG_COMPUTE=$c GNCDE_LIB=$PWD/build_alt/libgncde_hip.so timeout -k 10 200 python tools/diag_rows_stamps.py > gpurun_out/v_stamps_$c.txt 2>&1 || exit $?
  echo "== $c"; grep -v "Warning\|amdgpu.ids" gpurun_out/v_stamps_$c.txt | tail -21
done
echo r05v done
