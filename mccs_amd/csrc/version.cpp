// version.cpp — library identification string.
#include "mccs_hip.h"

extern "C" size_t mccsCommConfigSize(void) { return sizeof(mccsCommConfig); }

extern "C" mccsResult_t mccsCommConfigDefaultSized(mccsCommConfig* cfg, size_t size) {
  if (!cfg || size != sizeof(mccsCommConfig)) return mccsInvalidArgument;
  mccsCommConfigDefault(cfg);
  return mccsSuccess;
}

extern "C" const char* mccs_hip_version(void) { return "mccs_amd 0.4.0 gfx950"; }
