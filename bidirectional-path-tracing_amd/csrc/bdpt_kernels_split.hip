// The short-subpath build of the BDPT megakernel (BDPT_SPLIT_CONTINUE 1, chosen
// per render for rrDepth <= kSplitMaxRrDepth, bdpt_capi.cpp): the light
// subpath's ContinuePathRandomWalk (bdpt.h:211-215) and its loop test (:188) run
// before the eye subpath's start in the action sweep, so a light walk that ends
// starts its eye walk (bdpt.h:47-65) in the same shading step instead of
// waiting one loop iteration in ST_DEFER; the eye subpath's continuation
// (bdpt.h:152) becomes a body of its own. Same arithmetic in the same order per
// sample; every host-visible symbol gets a _split name.
#define BDPT_SPLIT_CONTINUE 1
#define bdpt_frame_kernel bdpt_frame_kernel_split
#define bdpt_sample_kernel bdpt_sample_kernel_split
#define frame_params_bytes frame_params_bytes_split
#define launch_frame launch_frame_split
#define launch_sample launch_sample_split
#define frame_kernel_blocks_per_cu frame_kernel_blocks_per_cu_split
#define frame_kernel_lds_stack frame_kernel_lds_stack_split
#define frame_kernel_block frame_kernel_block_split
#define light_vertex_fields light_vertex_fields_split
#include "bdpt_kernels.hip"
