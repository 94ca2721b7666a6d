// placeholder — replaced by the LM/Schur implementation
#include "orbhip_ba.h"
namespace orbhip {
struct BaWorkspace { int dummy; };
BaWorkspace* ba_create() { return new BaWorkspace(); }
void ba_destroy(BaWorkspace* ws) { delete ws; }
int ba_solve(BaWorkspace*, const orbhip_ba_problem*, orbhip_ba_result*, const volatile int*, hipStream_t) {
    return ORBHIP_ERR_UNSUPPORTED;
}
}  // namespace orbhip
