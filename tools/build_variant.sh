#!/bin/bash
# Builds a kernel variant of the product library: tools/build_variant.sh NAME [hipcc -D flags...]
# -> bidirectional-path-tracing_amd/lib/libbdpt_amd_NAME.so (select with BDPT_AMD_LIB=...).
# Rebuilds the BDPT megakernel translation units (the default and the short-subpath
# build) with the flags (ALL=1: every HIP
# translation unit, e.g. for traversal changes the per-function kernels must see);
# every other object comes from the default build (run make first).
# HOST=1 also rebuilds the C-ABI host units with the flags.
set -e
cd "$(dirname "$0")/../bidirectional-path-tracing_amd"
NAME=$1; shift
O=lib/obj_$NAME
mkdir -p $O
F="--offload-arch=gfx950 ${OPT:--O3} -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -I../include -Icsrc"
if [ "${ALL:-0}" = "1" ]; then TUS="bdpt_kernels bdpt_kernels_deep bdpt_kernels_hbm bdpt_kernels_rr bdpt_kernels_rrc bdpt_kernels_split pt_kernels sample_state kat_kernels"
else TUS="bdpt_kernels bdpt_kernels_split"; fi
# HOST=1: the C-ABI translation units too (layout switches the upload must follow)
if [ "${HOST:-0}" = "1" ]; then TUS="$TUS bdpt_capi bdpt_multi"; fi
EXCL=""
for t in $TUS; do
  SRC=csrc/$t.hip; [ -f $SRC ] || SRC=csrc/$t.cpp
  /opt/rocm/bin/hipcc $F "$@" -x hip -c $SRC -o $O/$t.o &
  EXCL="$EXCL -e /$t.o\$"
done
wait
OTHERS=$(ls lib/obj/*.o | grep -v $EXCL -e '/tinyrender_main.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/*.o $OTHERS -ldl -o lib/libbdpt_amd_$NAME.so
echo lib/libbdpt_amd_$NAME.so
