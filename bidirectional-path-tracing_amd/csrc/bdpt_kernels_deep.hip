// The deep-path build of the BDPT megakernel: rrDepth 29..1024, whose samples
// can draw past the first 227 outputs of their std::mt19937 (the lazy window
// of the default build). Same source as bdpt_kernels.hip with draws n >= 227
// continued from a per-lane ring of untempered MT19937 outputs in HBM
// (mt_u32_long, bdpt_device.hpp); every host-visible symbol gets a _deep name.
#define BDPT_DEEP_RNG 1
#define bdpt_frame_kernel bdpt_frame_kernel_deep
#define bdpt_sample_kernel bdpt_sample_kernel_deep
#define frame_params_bytes frame_params_bytes_deep
#define launch_frame launch_frame_deep
#define launch_sample launch_sample_deep
#define frame_kernel_blocks_per_cu frame_kernel_blocks_per_cu_deep
#define frame_kernel_lds_stack frame_kernel_lds_stack_deep
#define frame_kernel_block frame_kernel_block_deep
#define light_vertex_fields light_vertex_fields_deep
#include "bdpt_kernels.hip"
