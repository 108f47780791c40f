// The reference (written against MSVC) calls std::sqrtf / std::tanf / std::cosf /
// std::sinf / std::powf (reference src/core/math.h:124-242, src/bsdfs/glass.h:81,
// src/bsdfs/mixture.h:70, src/integrators/bdpt.h:52,:322). Those C++17 <cmath>
// names are not declared by libstdc++ 11, so this force-included header maps them
// to the C library functions of the same name. Nothing is replaced or stubbed:
// the calls still land in this machine's glibc libm.
#include <cmath>
namespace std { using ::sqrtf; using ::tanf; using ::cosf; using ::sinf; using ::powf; }
