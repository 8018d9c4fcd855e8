// Library identity and load check.
#include "aimx_common.h"

extern "C" const char* aimx_version(void) { return "aimx/0.1.0/gfx950"; }

extern "C" int aimx_events_create(int32_t n, void** events) {
  if (n < 0 || (n > 0 && !events)) return AIMX_EARG;
  for (int32_t i = 0; i < n; ++i) {
    hipEvent_t e;
    const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (r != hipSuccess) {
      for (int32_t j = 0; j < i; ++j) (void)hipEventDestroy((hipEvent_t)events[j]);
      return (int)r;
    }
    events[i] = (void*)e;
  }
  return AIMX_OK;
}

extern "C" int aimx_events_destroy(int32_t n, void** events) {
  if (n < 0 || (n > 0 && !events)) return AIMX_EARG;
  for (int32_t i = 0; i < n; ++i)
    if (events[i]) AIMX_CHECK_HIP(hipEventDestroy((hipEvent_t)events[i]));
  return AIMX_OK;
}
