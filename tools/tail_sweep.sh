#!/bin/bash
# tools/shard_tail.py for each variant library given ("default" = the product build).
# usage: tools/tail_sweep.sh OUT.txt NAME... [-- shard_tail args]
cd "$(dirname "$0")/.."
OUT=$1; shift
NAMES=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do NAMES+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out
: > $OUT
for n in "${NAMES[@]}"; do
  if [ "$n" == "default" ]; then LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd.so
  else LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd_$n.so; fi
  echo "== $n" >> $OUT
  BDPT_AMD_LIB=$LIB timeout -k 10 150 python3 tools/shard_tail.py "$@" >> $OUT 2>gpurun_out/tail_$n.err || { echo "$n FAILED" >> $OUT; exit 1; }
done
