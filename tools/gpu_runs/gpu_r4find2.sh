cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
O=gpurun_out/orc_shard.npy
tools/gpu_steps.sh \
 "400 find2_oracle.log -- python -u tools/rr_shard_check.py oracle $O" \
 "120 find2_default.log -- python -u tools/rr_shard_check.py gpu $O" \
 "120 find2_tc0.log -- env BDPT_AMD_LIB=$L/libbdpt_amd_tc0.so python -u tools/rr_shard_check.py gpu $O" \
 "120 find2_es0.log -- env BDPT_AMD_LIB=$L/libbdpt_amd_es0.so python -u tools/rr_shard_check.py gpu $O" \
 "120 find2_ra0.log -- env BDPT_AMD_LIB=$L/libbdpt_amd_ra0.so python -u tools/rr_shard_check.py gpu $O" \
 "120 find2_ca0.log -- env BDPT_AMD_LIB=$L/libbdpt_amd_ca0.so python -u tools/rr_shard_check.py gpu $O"
