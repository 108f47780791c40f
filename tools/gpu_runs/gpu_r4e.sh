cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "200 r4e_sweep.log -- tools/sweep_libs.sh gpurun_out/r4e_sweep.txt default r3 va vb vd tail1 tail2 default r3" \
 "150 r4e_tail_default.log -- python tools/shard_tail.py caustic 512 512 256 1 8" \
 "150 r4e_tail_t1.log -- BDPT_AMD_LIB=bidirectional-path-tracing_amd/lib/libbdpt_amd_tail1.so python tools/shard_tail.py caustic 512 512 256 1 8" \
 "150 r4e_tail_t2.log -- BDPT_AMD_LIB=bidirectional-path-tracing_amd/lib/libbdpt_amd_tail2.so python tools/shard_tail.py caustic 512 512 256 1 8" \
 "100 r4e_rr_small.log -- python tools/rr_probe.py caustic 512 512 1"
