// version.cpp — library identification string.
#include "mccs_hip.h"

extern "C" size_t mccsCommConfigSize(void) { return sizeof(mccsCommConfig); }

extern "C" const char* mccs_hip_version(void) { return "mccs_amd 0.3.0 gfx950"; }
