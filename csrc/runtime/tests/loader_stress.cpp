// Host stress driver for token_loader.cpp, built under ThreadSanitizer /
// AddressSanitizer by tests/test_token_data.py::test_loader_under_sanitizers
// (race + memory-error detection for the native runtime; GPU sanitizers are
// not available on this pool).  Many worker threads, a tiny ring, and a
// destroy while workers are blocked on a full ring.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
void* rn_loader_create(const char**, int, int, int, int, uint64_t, int, int, int, int, int, uint64_t, char*, int);
uint64_t rn_loader_next(void*, int64_t*);
void rn_loader_destroy(void*);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* paths[] = {argv[1]};
  char err[256];
  for (int mode = 0; mode < 2; ++mode) {
    void* h = rn_loader_create(paths, 1, 2, 4, 32, 7, 0, 1, mode, 8, 3, 0, err, sizeof err);
    if (!h) {
      std::fprintf(stderr, "create failed: %s\n", err);
      return 1;
    }
    std::vector<int64_t> buf(4 * 33);
    for (uint64_t k = 0; k < 200; ++k) {
      if (rn_loader_next(h, buf.data()) != k) return 3;
      for (int64_t v : buf)
        if (v < 0 || v >= 65536) return 4;
    }
    rn_loader_destroy(h);  // workers are parked on the full ring here
  }
  std::puts("loader stress ok");
  return 0;
}
