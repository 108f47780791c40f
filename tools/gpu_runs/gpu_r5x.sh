cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
# the frame's last samples to fewer, fuller waves (verdict item 6): 1 wave in 4 (k4) or 2 (k2)
# keeps claiming once the claims come within 1/4, 1/2 or 1 x the grid's lanes of the end
: > gpurun_out/r5x_tail.log
for n in default k4r1 k4r2 k4r4 k2r2 default; do
  X=$L/libbdpt_amd.so; [ "$n" != "default" ] && X=$L/libbdpt_amd_$n.so
  echo "== $n" >> gpurun_out/r5x_tail.log
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 tools/shard_tail.py caustic 512 512 256 1 8 >> gpurun_out/r5x_tail.log 2>&1 || exit 1
done
