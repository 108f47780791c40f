#!/bin/bash
# Times the bench workload under environment settings: tools/sweep_env.sh OUT.txt "VAR=v ..." ... [-- bench args]
cd "$(dirname "$0")/.."
OUT=$1; shift
SETS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out
: > $OUT
i=0
for e in "${SETS[@]}"; do
  i=$((i + 1))
  env $e timeout -k 10 200 python3 bench.py --no-cpu --no-parity --steps 3 --warmup 1 "$@" > gpurun_out/sweepenv_$i.json 2>gpurun_out/sweepenv_$i.err || { echo "$e FAILED" >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sweepenv_$i.json').read().strip().splitlines()[-1]); print('$e', d['value'], d['roofline']['kernel_ms'])" >> $OUT
  tail -1 $OUT
done
