#!/bin/bash
# Round 5 (GPU box): phase stamps of config 3's CDE read-out launch (stamps build), five- and two-tile workgroups.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 5 2; do
  GNCDE_READOUT_TILES=$v GNCDE_LIB=$PWD/build_alt/libgncde_hip.so timeout -k 10 200 python tools/diag_layer_stamps.py > gpurun_out/n_stamps_T$v.txt 2>&1 || exit $?
  echo "== tiles $v"; cat gpurun_out/n_stamps_T$v.txt | grep -v Warning | tail -12
done
echo r05n done
