// The Russian-roulette build for scenes with a dielectric (GlassBSDF): the same
// megakernel as bdpt_kernels_rr.hip plus BDPT_EXPRESS_CHAIN — a lone long walk's
// delta bounces (a subpath trapped in glass by total internal reflection, DESIGN.md
// §8) run back to back inside the express block, each closest hit walked by the
// whole wave, instead of one bounce per pass through the loop top, the walk loop and
// the sweep (Caustic 512^2 x 256: frames 42-45 s -> 35.8-37.4 s). The inline chain
// costs the build's register allocation (92 VGPR spills vs 10), so scenes that
// cannot trap a subpath (no GlassBSDF) keep bdpt_kernels_rr.hip (HardLight RR
// 82.9 vs 78.9 Msamples/s). Chosen per render (bdpt_capi.cpp); every host-visible
// symbol gets an _rrc name.
#define BDPT_DEEP_RNG 1
#define BDPT_RR 1
#define BDPT_EXPRESS_CHAIN 1
#define bdpt_frame_kernel bdpt_frame_kernel_rrc
#define bdpt_sample_kernel bdpt_sample_kernel_rrc
#define frame_params_bytes frame_params_bytes_rrc
#define launch_frame launch_frame_rrc
#define launch_chain launch_chain_rrc
#define bdpt_chain_kernel bdpt_chain_kernel_rrc
#define launch_sample launch_sample_rrc
#define frame_kernel_blocks_per_cu frame_kernel_blocks_per_cu_rrc
#define frame_kernel_lds_stack frame_kernel_lds_stack_rrc
#define frame_kernel_block frame_kernel_block_rrc
#define light_vertex_fields light_vertex_fields_rrc
#include "bdpt_kernels.hip"
