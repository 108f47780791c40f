// The Russian-roulette build of the BDPT megakernel: the reference's NO_RR = 0
// branch (src/integrators/bdpt.h:18, :68, :129-132, :188, :201-204), selected
// per render by bdpt_frame_params.russian_roulette. Subpaths run past rrDepth
// while sampler.next() < rrProbability, so a sample draws an unbounded number of
// random numbers (the deep build's MT19937 rings continue past draw 226) and
// stores up to DevFrame::depth_cap - 1 light vertices. Same source as
// bdpt_kernels.hip; every host-visible symbol gets an _rr name.
#define BDPT_DEEP_RNG 1
#define BDPT_RR 1
#define bdpt_frame_kernel bdpt_frame_kernel_rr
#define bdpt_sample_kernel bdpt_sample_kernel_rr
#define frame_params_bytes frame_params_bytes_rr
#define launch_frame launch_frame_rr
#define launch_chain launch_chain_rr
#define bdpt_chain_kernel bdpt_chain_kernel_rr
#define launch_sample launch_sample_rr
#define frame_kernel_blocks_per_cu frame_kernel_blocks_per_cu_rr
#define frame_kernel_lds_stack frame_kernel_lds_stack_rr
#define frame_kernel_block frame_kernel_block_rr
#define light_vertex_fields light_vertex_fields_rr
#include "bdpt_kernels.hip"
