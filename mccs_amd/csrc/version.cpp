// version.cpp — library identification string.
#include "mccs_hip.h"

extern "C" const char* mccs_hip_version(void) { return "mccs_amd 0.1.0 gfx950"; }
