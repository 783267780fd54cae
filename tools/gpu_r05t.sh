#!/bin/bash
# Round 5 (GPU box): phase stamps of config 3's eight-wave five-tile read-out (stamps build).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
GNCDE_LIB=$PWD/build_alt/libgncde_hip.so timeout -k 10 200 python tools/diag_layer_stamps.py > gpurun_out/t_stamps.txt 2>&1 || exit $?
grep -v Warning gpurun_out/t_stamps.txt | tail -10
echo r05t done
