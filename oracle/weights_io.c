/* ORACLE (test infrastructure only): RSPLWT01 weight-blob reader. */
#include "oracle_common.h"

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

int orc_load_weights(const char* path, orc_weights* w) {
  memset(w, 0, sizeof(*w));
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  char magic[8];
  uint32_t count = 0;
  if (rd(f, magic, 8) || memcmp(magic, "RSPLWT01", 8) || rd(f, &count, 4)) { fclose(f); return -2; }
  w->t = (orc_tensor*)calloc(count, sizeof(orc_tensor));
  w->count = (int)count;
  for (uint32_t i = 0; i < count; i++) {
    orc_tensor* t = &w->t[i];
    uint32_t nl = 0, nd = 0;
    if (rd(f, &nl, 4) || nl >= sizeof(t->name) || rd(f, t->name, nl) || rd(f, &nd, 4) || nd > 4) {
      fclose(f); return -3;
    }
    t->name[nl] = 0;
    t->ndim = (int)nd;
    t->numel = 1;
    for (uint32_t d = 0; d < nd; d++) {
      if (rd(f, &t->dims[d], 8)) { fclose(f); return -3; }
      t->numel *= t->dims[d];
    }
    t->data = (float*)malloc(sizeof(float) * (size_t)t->numel);
    if (rd(f, t->data, sizeof(float) * (size_t)t->numel)) { fclose(f); return -3; }
  }
  fclose(f);
  return 0;
}

void orc_free_weights(orc_weights* w) {
  for (int i = 0; i < w->count; i++) free(w->t[i].data);
  free(w->t);
  memset(w, 0, sizeof(*w));
}

const float* orc_get(const orc_weights* w, const char* name, int64_t expect_numel) {
  for (int i = 0; i < w->count; i++)
    if (!strcmp(w->t[i].name, name)) {
      if (expect_numel >= 0 && w->t[i].numel != expect_numel) {
        fprintf(stderr, "oracle: %s has %lld values, expected %lld\n", name, (long long)w->t[i].numel,
                (long long)expect_numel);
        return NULL;
      }
      return w->t[i].data;
    }
  fprintf(stderr, "oracle: tensor %s missing\n", name);
  return NULL;
}
