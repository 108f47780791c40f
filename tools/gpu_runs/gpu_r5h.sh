cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# synth1m: the traversal tree's node order in HBM (depth-first, breadth-first, 3-level treelets)
: > gpurun_out/r5h_order.txt
for m in dfs bfs treelet dfs bfs treelet; do
  BDPT_NODE_ORDER=$m timeout -k 10 200 python3 bench.py --no-cpu --no-parity --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 > gpurun_out/r5h_$m.json 2> gpurun_out/r5h_$m.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5h_$m.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['roofline']['kernel_ms'])" >> gpurun_out/r5h_order.txt
done
cat gpurun_out/r5h_order.txt
