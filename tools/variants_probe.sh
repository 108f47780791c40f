#!/bin/bash
# Probes each built variant library (tools/build_variant.sh) on the GPU box.
cd "$(dirname "$0")/.."
for v in "$@"; do
  echo "== $v"
  BDPT_AMD_LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd_$v.so timeout -k 10 200 python tools/probe.py ${PROBE_ARGS:-caustic 512 512 16} || exit 1
done
