cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
# the drain phase of the 1/8 row shard and the full frame (tail probe variant); the tail knobs
# re-swept on this build (drain shade fraction 5/8, 7/8; finer claims from 2x / 8x the grid's lanes)
BDPT_AMD_LIB=$L/libbdpt_amd_tailprobe.so timeout -k 10 200 python3 tools/tail_probe.py caustic 512 512 256 1 8 > gpurun_out/r5v_tail_probe.log 2>&1 || exit 1
for n in default tf5 tf7 tc2 tc8; do
  X=$L/libbdpt_amd.so; [ "$n" != "default" ] && X=$L/libbdpt_amd_$n.so
  echo "== $n" >> gpurun_out/r5v_tail.log
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 tools/shard_tail.py caustic 512 512 256 1 8 >> gpurun_out/r5v_tail.log 2>&1 || exit 1
done
