#!/bin/bash
# Builds a kernel variant of the product library: tools/build_variant.sh NAME [hipcc -D flags...]
# -> bidirectional-path-tracing_amd/lib/libbdpt_amd_NAME.so (select with BDPT_AMD_LIB=...).
# Rebuilds the BDPT megakernel translation unit with the flags;
# every other object comes from the default build (run make first).
set -e
cd "$(dirname "$0")/../bidirectional-path-tracing_amd"
NAME=$1; shift
O=lib/obj_$NAME
mkdir -p $O
F="--offload-arch=gfx950 ${OPT:--O3} -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I../include -Icsrc"
/opt/rocm/bin/hipcc $F "$@" -x hip -c csrc/bdpt_kernels.hip -o $O/k.o
OTHERS=$(ls lib/obj/*.o | grep -v -e '/bdpt_kernels.o$' -e '/tinyrender_main.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/k.o $OTHERS -ldl -o lib/libbdpt_amd_$NAME.so
echo lib/libbdpt_amd_$NAME.so
