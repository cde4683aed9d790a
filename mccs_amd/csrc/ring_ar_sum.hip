// ring_ar_sum.hip — AllReduce ring kernels, reduction op Sum (ring_ar_tu.h).
#include "ring_ar_tu.h"

MCCS_AR_TU(Sum, mccs::OpSum)
MCCS_RING_TU_ACCESSORS(ar_sum)
