#!/bin/bash
# rocprofv3 kernel stats of tools/bench_configs.py --configs ${CFGS:-3} for the in-tree library and every
# variants/libgncde_*.so (GPU box); summaries in gpurun_out/profvar_<name>/.
export TMPDIR=/tmp
ROOTDIR=$(pwd)
for lib in "" variants/libgncde_*.so; do
  name=$(basename "${lib:-intree}" .so)
  (cd /tmp && GNCDE_LIB=${lib:+$ROOTDIR/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$ROOTDIR/gpurun_out/profvar_$name" -o run -- python3 "$ROOTDIR/tools/bench_configs.py" --configs "${CFGS:-3}" \
     --reps 1 > "$ROOTDIR/gpurun_out/profvar_$name.log" 2>&1) || exit $?
done
echo done
