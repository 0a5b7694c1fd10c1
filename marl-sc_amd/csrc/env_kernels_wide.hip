// env_kernels_wide.hip -- the env kernels for 9-12 SKUs: env_kernels.hip compiled again with
// MSC_EK_WIDE (its launchers' *_w1 entry points), a translation unit of its own so the parts of
// the instantiations build in parallel (13-16 SKUs: env_kernels_wide2.hip).
#define MSC_EK_WIDE 1
#include "env_kernels.hip"
