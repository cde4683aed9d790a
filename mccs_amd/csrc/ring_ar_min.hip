// ring_ar_min.hip — AllReduce ring kernels, reduction op Min (ring_ar_tu.h).
#include "ring_ar_tu.h"

MCCS_AR_TU(Min, mccs::OpMin)
MCCS_RING_TU_ACCESSORS(ar_min)
