cd $GRAFT_REPO_ROOT
bash tools/gpu_runs/gpu_r5q.sh && bash tools/gpu_runs/gpu_r5r.sh
