#!/bin/bash
# Compile-time resource report of the frame kernel<false,false>: VGPRs, scratch,
# occupancy and code size (lines of ISA), optional extra hipcc flags as $@.
PKG="$(cd "$(dirname "$0")/../bidirectional-path-tracing_amd" && pwd)"
T=$(mktemp -d)
cd $T
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -I$PKG/csrc -I$PKG/../include "$@" -x hip \
  -c $PKG/csrc/bdpt_kernels.hip -o $T/k.o --save-temps -Rpass-analysis=kernel-resource-usage 2> $T/rem.txt < /dev/null
S=$(ls $T/*gfx950.s 2>/dev/null) || { echo "compile failed"; grep error $T/rem.txt | head; rm -rf $T; exit 1; }
grep -A12 'Name: _ZN4bdpt3dev17bdpt_frame_kernelILb0ELb0ELb0EE' $T/rem.txt | grep -E 'VGPRs:|VGPRs Spill|SGPRs:|Scratch|Occupancy|LDS Size' | sed 's/.*remark: *//' | sed "s/ \[-Rpass.*//" | tr "\n" " "
awk '/^_ZN4bdpt3dev17bdpt_frame_kernelILb0ELb0ELb0EE.*:/{f=1} f{print} /s_endpgm/{if(f)exit}' $S > $T/k.s
echo "isa_lines=$(wc -l < $T/k.s) scratch_ops=$(grep -c scratch_ $T/k.s) lanespill=$(grep -c v_writelane $T/k.s)"
cd /; rm -rf $T
