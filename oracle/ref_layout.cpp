// TEST INFRASTRUCTURE (oracle).  Compiles the reference's own device-ABI
// header, /root/reference/src/collectives/include/devcomm.h (which host g++
// accepts because align.h:19-26 stubs __host__/__device__), and prints its
// layout.  Built by oracle/Makefile into oracle/_ref/ref_layout; never shipped.
#include <cstddef>
#include "devcomm.h"
#include "layout_dump.inc"
