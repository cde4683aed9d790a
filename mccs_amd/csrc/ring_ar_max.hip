// ring_ar_max.hip — AllReduce ring kernels, reduction op Max (ring_ar_tu.h).
#include "ring_ar_tu.h"

MCCS_AR_TU(Max, mccs::OpMax)
MCCS_RING_TU_ACCESSORS(ar_max)
