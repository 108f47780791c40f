/* TEST INFRASTRUCTURE (oracle). CPU restatement of the libm single-precision
 * functions the reference BDPT path calls, so that the oracle does not depend on
 * which libm variant the host happens to select.
 *
 * Third-party dependency (absent from /root/reference): GNU libc 2.35
 * (Ubuntu 2.35-0ubuntu3.11), sysdeps/ieee754/flt-32/{s_sinf.c,s_cosf.c,
 * sincosf.h,e_powf.c,e_exp2f_data.c,e_powf_log2_data.c,s_sincosf_data.c}
 * (the ARM optimized-routines algorithms), in the x86_64 "fma" multiarch build
 * that glibc's ifunc resolver selects on FMA+AVX2 CPUs (the machine the goldens
 * were produced on). Every double expression of the form a*b+c that GCC
 * contracted in that build is written as an explicit fma() here.
 * Reference call sites: src/core/math.h:125,142,178,213-217,224;
 * src/bsdfs/mixture.h:70,310. */
#ifndef TR_MATHF_H
#define TR_MATHF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

float tr_sinf(float x);
float tr_cosf(float x);
float tr_powf(float x, float y);
/* glibc 2.35 x86_64 fmaxf/fminf (maxss/minss based): on ordered operands the
 * SECOND argument is returned on ties (so fmaxf(-0,+0) = +0, fmaxf(+0,-0) = -0);
 * a NaN operand yields the other operand. Used where the reference calls
 * std::fmax / glm::fmax / glm::fclamp on floats. */
float tr_fmaxf(float x, float y);
float tr_fminf(float x, float y);

#ifdef __cplusplus
}
#endif
#endif
