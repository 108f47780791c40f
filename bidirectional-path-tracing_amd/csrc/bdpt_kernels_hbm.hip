// The BDPT megakernel for scenes whose BSDF records do not fit the LDS table
// budget (more than ~300 materials): the same source as bdpt_kernels.hip with
// the records read from HBM (BDPT_BSDF_TABLE 1, bsdf_of in bdpt_device.hpp);
// every host-visible symbol gets an _hbm name. Selected by bdpt_ctx_create's
// table layout (DevScene::lds_bsdf_off == kNoLds).
#define BDPT_BSDF_TABLE 1
#define bdpt_frame_kernel bdpt_frame_kernel_hbm
#define bdpt_sample_kernel bdpt_sample_kernel_hbm
#define frame_params_bytes frame_params_bytes_hbm
#define launch_frame launch_frame_hbm
#define launch_sample launch_sample_hbm
#define frame_kernel_blocks_per_cu frame_kernel_blocks_per_cu_hbm
#define frame_kernel_lds_stack frame_kernel_lds_stack_hbm
#define frame_kernel_block frame_kernel_block_hbm
#define light_vertex_fields light_vertex_fields_hbm
#include "bdpt_kernels.hip"
