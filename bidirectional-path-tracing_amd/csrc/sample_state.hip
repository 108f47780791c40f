// The single-sample build: Integrator::render(const Ray&, Sampler&) of the
// reference's BDPT (bdpt.h:219-241), path tracer (path.h:235-245) and direct
// integrator (direct.h:449-462), one camera sample on one lane. Same sources as
// the frame kernels, compiled with BDPT_SAMPLER_STATE: every draw advances the
// caller's whole std::mt19937 state (mt_state_u32, bdpt_device.hpp) and camera
// splats are returned as a list (splat_add, bdpt_path.hpp). Only the sample
// kernels and their launchers exist in this translation unit.
#define BDPT_SAMPLER_STATE 1
#define BDPT_RR 2  // NO_RR 1 or 0 per launch (DevFrame::rr_mode)
#include "bdpt_kernels.hip"
#include "pt_kernels.hip"
