#!/bin/bash
# Build an experimental variant of libgncde_hip.so: one translation unit recompiled with extra -D flags, linked with
# the in-tree objects of everything else.
#   tools/build_variant.sh NAME SOURCE -DFLAG=1 ...   (SOURCE e.g. gncde_fused, gncde_layer)
#   -> variants/libgncde_NAME.so, run with GNCDE_LIB=variants/libgncde_NAME.so.  The in-tree library is untouched.
set -e
cd "$(dirname "$0")/../perm-equiv-graph-neural-cdes_amd"
make -s -j8
name=$1; src=$2; shift 2
mkdir -p ../variants build/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-pass-failed "$@" \
  -c csrc/$src.hip -o build/variants/${src}_$name.o
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../variants/libgncde_$name.so $objs build/variants/${src}_$name.o
echo "variants/libgncde_$name.so"
