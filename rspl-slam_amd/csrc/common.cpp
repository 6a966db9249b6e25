#include "common.hpp"

#include <cstring>

namespace rspl {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int load_blob(const char* path, std::vector<Tensor>& out) {
  out.clear();
  if (!path) {
    set_error("weights path is NULL");
    return RSPL_E_WEIGHTS;
  }
  FILE* f = fopen(path, "rb");
  if (!f) {
    set_error("cannot open weights %s", path);
    return RSPL_E_WEIGHTS;
  }
  auto rd = [&](void* p, size_t n) { return fread(p, 1, n, f) == n; };
  char magic[8];
  uint32_t count = 0;
  if (!rd(magic, 8) || memcmp(magic, "RSPLWT01", 8) || !rd(&count, 4)) {
    fclose(f);
    set_error("%s: not an RSPLWT01 blob", path);
    return RSPL_E_WEIGHTS;
  }
  out.resize(count);
  for (uint32_t i = 0; i < count; i++) {
    uint32_t nl = 0, nd = 0;
    if (!rd(&nl, 4) || nl > 4096) goto bad;
    out[i].name.resize(nl);
    if (!rd(&out[i].name[0], nl) || !rd(&nd, 4) || nd > 8) goto bad;
    out[i].dims.resize(nd);
    int64_t n = 1;
    for (uint32_t d = 0; d < nd; d++) {
      if (!rd(&out[i].dims[d], 8)) goto bad;
      n *= out[i].dims[d];
    }
    out[i].data.resize(n);
    if (!rd(out[i].data.data(), sizeof(float) * n)) goto bad;
  }
  fclose(f);
  return RSPL_OK;
bad:
  fclose(f);
  set_error("%s: truncated / malformed blob", path);
  return RSPL_E_WEIGHTS;
}

const Tensor* find(const std::vector<Tensor>& ts, const std::string& name, int64_t numel) {
  for (auto& t : ts)
    if (t.name == name) {
      if (numel >= 0 && (int64_t)t.data.size() != numel) {
        set_error("weight %s has %zu values, expected %lld", name.c_str(), t.data.size(), (long long)numel);
        return nullptr;
      }
      return &t;
    }
  set_error("weight %s missing from blob", name.c_str());
  return nullptr;
}

}  // namespace rspl

extern "C" const char* rspl_last_error(void) { return rspl::g_err; }
extern "C" const char* rspl_version(void) { return "rspl-mi355x 0.2 (gfx950)"; }
extern "C" int rspl_abi_version(void) { return RSPL_ABI_VERSION; }
