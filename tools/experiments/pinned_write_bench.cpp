// Host write speed into the BA's pinned staging memory (hipHostMalloc Mapped | Coherent) vs pageable
// memory: 7 interleaved sequential streams of 4-byte stores + one of 32-byte records per "edge", the
// shape of rspl_ba_local's staging gather.  Prints ns per edge for each.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double run(char* base, int n) {
  int* a[6];
  for (int k = 0; k < 6; k++) a[k] = reinterpret_cast<int*>(base + (size_t)k * 4 * n);
  double* o = reinterpret_cast<double*>(base + (size_t)24 * n);
  const auto t0 = std::chrono::steady_clock::now();
  for (int rep = 0; rep < 20; rep++)
    for (int i = 0; i < n; i++) {
      for (int k = 0; k < 6; k++) a[k][i] = i + k + rep;
      o[4 * i] = i;
      o[4 * i + 1] = i + 1;
      o[4 * i + 2] = i + 2;
    }
  return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / (20.0 * n);
}

int main() {
  const int n = 23290;
  const size_t bytes = (size_t)56 * n;
  char* pin = nullptr;
  if (hipHostMalloc((void**)&pin, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  char* pin_nc = nullptr;
  if (hipHostMalloc((void**)&pin_nc, bytes, hipHostMallocMapped | hipHostMallocNonCoherent) != hipSuccess) return 1;
  std::vector<char> pg(bytes);
  run(pin, n); run(pin_nc, n); run(pg.data(), n);
  printf("ns per edge: pinned coherent %.2f, pinned non-coherent %.2f, pageable %.2f\n", run(pin, n), run(pin_nc, n),
         run(pg.data(), n));
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < 20; r++) memcpy(pin, pg.data(), bytes);
  printf("memcpy pageable -> pinned coherent: %.1f GB/s\n",
         20.0 * bytes / std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count());
  return 0;
}
