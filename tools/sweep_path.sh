#!/bin/bash
# Path-tracer bench (bench.py --integrator path) for each variant library given.
# usage: tools/sweep_path.sh OUT.txt NAME... [-- bench args]
cd "$(dirname "$0")/.."
OUT=$1; shift
NAMES=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do NAMES+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out
: > $OUT
for n in "${NAMES[@]}"; do
  if [ "$n" == "default" ]; then LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd.so
  else LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd_$n.so; fi
  BDPT_AMD_LIB=$LIB timeout -k 10 150 python3 bench.py --integrator path --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/psweep_$n.json 2>gpurun_out/psweep_$n.err || { echo "$n FAILED" >> $OUT; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/psweep_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['config']['kernel_ms'])" >> $OUT
done
