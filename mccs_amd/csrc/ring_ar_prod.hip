// ring_ar_prod.hip — AllReduce ring kernels, reduction op Prod (ring_ar_tu.h).
#include "ring_ar_tu.h"

MCCS_AR_TU(Prod, mccs::OpProd)
MCCS_RING_TU_ACCESSORS(ar_prod)
