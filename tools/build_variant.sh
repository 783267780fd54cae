#!/bin/bash
# Build an experimental variant of libgncde_hip.so: gncde_fused.hip recompiled with extra -D flags, linked with the
# in-tree objects of everything else.  Usage: tools/build_variant.sh NAME -DFLAG=1 ...  -> variants/libgncde_NAME.so
# (run with GNCDE_LIB=variants/libgncde_NAME.so).  The in-tree library is untouched.
set -e
cd "$(dirname "$0")/../perm-equiv-graph-neural-cdes_amd"
make -s -j8
name=$1; shift
mkdir -p ../variants build/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-pass-failed "$@" \
  -c csrc/gncde_fused.hip -o build/variants/fused_$name.o
objs=$(ls build/*.o | grep -v gncde_fused.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../variants/libgncde_$name.so $objs build/variants/fused_$name.o
echo "variants/libgncde_$name.so"
