// TEST INFRASTRUCTURE (oracle).  Prints the layout of this repo's
// include/mccs_devcomm.h with the same dumper as ref_layout.cpp so the two can
// be diffed byte for byte.
#include <cstddef>
#include "mccs_devcomm.h"
#include "layout_dump.inc"
