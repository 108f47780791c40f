#!/bin/bash
# Times the bench workload with each variant library given (names under
# bidirectional-path-tracing_amd/lib/libbdpt_amd_NAME.so; "default" = the product build).
# usage: tools/sweep_libs.sh OUT.txt NAME... [-- bench args]
cd "$(dirname "$0")/.."
OUT=$1; shift
NAMES=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do NAMES+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out
: > $OUT
for n in "${NAMES[@]}"; do
  if [ "$n" == "default" ]; then LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd.so
  else LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd_$n.so; fi
  BDPT_AMD_LIB=$LIB timeout -k 10 150 python3 bench.py --no-cpu --no-parity --steps 3 --warmup 1 "$@" > gpurun_out/sweep_$n.json 2>gpurun_out/sweep_$n.err || { echo "$n FAILED" >> $OUT; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['roofline']['kernel_ms'])" >> $OUT
  cat $OUT | tail -1
done
