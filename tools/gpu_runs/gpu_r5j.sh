cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# branch-free stack pushes / LDS-only pops when the wave's stacks allow (BDPT_PUSH3, BDPT_POP_LDS)
tools/gpu_steps.sh \
 "100 r5j_kat.log -- python -u -m pytest tests/test_gpu_kat.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'golden or kat or adversarial or full_traversal'" \
 "300 r5j_sweep.log -- tools/sweep_libs.sh gpurun_out/r5j_sweep.txt default nopush3 push3only poponly default nopush3 push3only poponly" \
 "200 r5j_sweep_s.log -- tools/sweep_libs.sh gpurun_out/r5j_sweep_s.txt default nopush3 -- --scene synth1m --width 1024 --height 1024 --spp 64"
