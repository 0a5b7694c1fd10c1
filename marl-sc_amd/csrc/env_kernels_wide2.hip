// env_kernels_wide2.hip -- the env kernels for 13-16 SKUs (env_kernels.hip, MSC_EK_WIDE 2: the
// launchers' *_w2 entry points).
#define MSC_EK_WIDE 2
#include "env_kernels.hip"
