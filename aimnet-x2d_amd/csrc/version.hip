// Library identity and load check; the test-hook option table.
#include <cstring>
#include <mutex>

#include "aimx_common.h"

namespace {
// Options set through aimx_set_option: a few names, looked up at launch planning (host side). The
// common case — nothing set — is one relaxed load.
constexpr int kMaxOpts = 16;
struct Opt {
  char name[48];
  int64_t value;
};
Opt g_opts[kMaxOpts];
int g_nopts = 0;
std::mutex g_opt_mu;
}  // namespace

namespace aimx {
int64_t opt_i64(const char* name, int64_t dflt) {
  if (__atomic_load_n(&g_nopts, __ATOMIC_ACQUIRE) > 0) {
    std::lock_guard<std::mutex> lk(g_opt_mu);
    for (int i = 0; i < g_nopts; ++i)
      if (std::strcmp(g_opts[i].name, name) == 0) return g_opts[i].value;
  }
#ifdef AIMX_TUNING
  if (const char* e = getenv(name)) return (int64_t)atoll(e);
#endif
  return dflt;
}
}  // namespace aimx

extern "C" int aimx_set_option(const char* name, int64_t value) {
  if (!name || std::strlen(name) >= sizeof(Opt::name)) return AIMX_EARG;
  std::lock_guard<std::mutex> lk(g_opt_mu);
  for (int i = 0; i < g_nopts; ++i)
    if (std::strcmp(g_opts[i].name, name) == 0) {
      g_opts[i].value = value;
      return AIMX_OK;
    }
  if (g_nopts == kMaxOpts) return AIMX_EARG;
  std::strcpy(g_opts[g_nopts].name, name);
  g_opts[g_nopts].value = value;
  __atomic_store_n(&g_nopts, g_nopts + 1, __ATOMIC_RELEASE);
  return AIMX_OK;
}

extern "C" int aimx_clear_options(void) {
  std::lock_guard<std::mutex> lk(g_opt_mu);
  __atomic_store_n(&g_nopts, 0, __ATOMIC_RELEASE);
  return AIMX_OK;
}

extern "C" const char* aimx_version(void) { return "aimx/0.1.0/gfx950"; }
