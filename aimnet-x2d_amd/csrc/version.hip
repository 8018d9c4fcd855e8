// Library identity and load check.
#include "aimx_common.h"

extern "C" const char* aimx_version(void) { return "aimx/0.1.0/gfx950"; }
