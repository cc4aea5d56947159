// Native token-shard data loader (host C++, no GPU code): the IO half of the
// training runtime.  The reference has no data pipeline at all (SURVEY.md §2.1:
// modules only; §2.3 N22 asks for synthetic generators, which
// replicann_amd/utils/data.py provides); this is the real-data counterpart for
// the LM configs: flat binary token shards (uint16 or uint32 little-endian,
// the "tokens.bin" layout GPT-2 pre-tokenisers write) are memory-mapped and
// worker threads cut (B, T+1) int64 windows into a ring of prefetch slots
// while the GPU runs the previous step.
//
// Determinism: batch k's content is a pure function of (seed, rank, world, k),
// independent of thread count and timing, so a run resumed at batch k sees the
// same stream as an uninterrupted one.
//
//   mode 0 (train):  B windows at uniformly random offsets (counter-based
//                    splitmix64 per (seed, rank, k, j)); a window never crosses
//                    a shard boundary.
//   mode 1 (eval):   non-overlapping windows (stride T, T+1 tokens incl. the
//                    shifted target) dealt round-robin over ranks:
//                    window w = (k*world + rank)*B + j, modulo the window count.
//
// C ABI (ctypes; see replicann_amd/utils/token_data.py):
//   rn_loader_create / rn_loader_next / rn_loader_num_tokens /
//   rn_loader_num_windows / rn_loader_destroy

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

struct Shard {
  const uint8_t* base = nullptr;
  size_t bytes = 0;
  uint64_t ntok = 0;
};

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Loader {
  std::vector<Shard> shards;
  std::vector<uint64_t> tok_prefix;  // cumulative usable start positions per shard (mode 0)
  std::vector<uint64_t> win_prefix;  // cumulative window counts per shard (mode 1)
  int elem = 2;
  int B = 0, T = 0, rank = 0, world = 1, mode = 0;
  uint64_t seed = 0;

  int nslots = 0;
  std::vector<std::vector<int64_t>> slots;
  std::vector<uint8_t> full;       // slot holds batch `slot_batch[s]`
  std::vector<uint64_t> slot_batch;
  uint64_t next_produce = 0;       // next batch index a worker claims
  uint64_t next_consume = 0;       // next batch index rn_loader_next returns
  bool stop = false;
  std::mutex m;
  std::condition_variable cv_full, cv_free;
  std::vector<std::thread> workers;

  ~Loader() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv_free.notify_all();
    cv_full.notify_all();
    for (auto& t : workers) t.join();
    for (auto& s : shards)
      if (s.base) munmap(const_cast<uint8_t*>(s.base), s.bytes);
  }

  inline int64_t tok(const Shard& s, uint64_t i) const {
    if (elem == 2) {
      uint16_t v;
      std::memcpy(&v, s.base + i * 2, 2);
      return v;
    }
    uint32_t v;
    std::memcpy(&v, s.base + i * 4, 4);
    return v;
  }

  void copy_window(const Shard& s, uint64_t start, int64_t* dst) const {
    const uint64_t n = (uint64_t)T + 1;
    for (uint64_t i = 0; i < n; ++i) dst[i] = tok(s, start + i);
  }

  // Shard index holding global position p of a prefix table (upper_bound - 1).
  static size_t locate(const std::vector<uint64_t>& prefix, uint64_t p) {
    return size_t(std::upper_bound(prefix.begin(), prefix.end(), p) - prefix.begin()) - 1;
  }

  void fill(uint64_t k, int64_t* out) const {
    const uint64_t W = (uint64_t)T + 1;
    for (int j = 0; j < B; ++j) {
      int64_t* dst = out + (size_t)j * W;
      if (mode == 0) {
        uint64_t h = splitmix64(seed ^ splitmix64(((uint64_t)rank << 40) ^ (k * (uint64_t)B + (uint64_t)j)));
        uint64_t p = h % tok_prefix.back();
        size_t s = locate(tok_prefix, p);
        copy_window(shards[s], p - tok_prefix[s], dst);
      } else {
        uint64_t w = ((k * (uint64_t)world + (uint64_t)rank) * (uint64_t)B + (uint64_t)j) % win_prefix.back();
        size_t s = locate(win_prefix, w);
        copy_window(shards[s], (w - win_prefix[s]) * (uint64_t)T, dst);
      }
    }
  }

  void worker() {
    for (;;) {
      uint64_t k;
      int s;
      {
        std::unique_lock<std::mutex> g(m);
        cv_free.wait(g, [&] { return stop || next_produce < next_consume + (uint64_t)nslots; });
        if (stop) return;
        k = next_produce++;
        s = int(k % (uint64_t)nslots);
      }
      fill(k, slots[s].data());
      {
        std::lock_guard<std::mutex> g(m);
        full[s] = 1;
        slot_batch[s] = k;
      }
      cv_full.notify_all();
    }
  }
};

void set_err(char* err, int len, const std::string& msg) {
  if (err && len > 0) std::snprintf(err, (size_t)len, "%s", msg.c_str());
}

}  // namespace

extern "C" {

void* rn_loader_create(const char** paths, int npaths, int elem_bytes, int B, int T, uint64_t seed, int rank,
                       int world, int mode, int nthreads, int nslots, uint64_t start_batch, char* err, int errlen) {
  if (npaths <= 0 || B <= 0 || T <= 0 || (elem_bytes != 2 && elem_bytes != 4) || world <= 0 || rank < 0 ||
      rank >= world || (mode != 0 && mode != 1)) {
    set_err(err, errlen, "invalid loader arguments");
    return nullptr;
  }
  auto* L = new Loader();
  L->elem = elem_bytes;
  L->B = B;
  L->T = T;
  L->seed = seed;
  L->rank = rank;
  L->world = world;
  L->mode = mode;
  L->tok_prefix.push_back(0);
  L->win_prefix.push_back(0);
  for (int i = 0; i < npaths; ++i) {
    int fd = open(paths[i], O_RDONLY);
    if (fd < 0) {
      set_err(err, errlen, std::string("cannot open ") + paths[i]);
      delete L;
      return nullptr;
    }
    struct stat st;
    fstat(fd, &st);
    Shard sh;
    sh.bytes = (size_t)st.st_size;
    sh.ntok = sh.bytes / (size_t)elem_bytes;
    if (sh.ntok < (uint64_t)T + 1) {
      close(fd);
      set_err(err, errlen, std::string("shard shorter than seq_len+1 tokens: ") + paths[i]);
      delete L;
      return nullptr;
    }
    void* p = mmap(nullptr, sh.bytes, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      set_err(err, errlen, std::string("mmap failed: ") + paths[i]);
      delete L;
      return nullptr;
    }
    madvise(p, sh.bytes, mode == 0 ? MADV_RANDOM : MADV_SEQUENTIAL);
    sh.base = static_cast<const uint8_t*>(p);
    L->shards.push_back(sh);
    L->tok_prefix.push_back(L->tok_prefix.back() + (sh.ntok - (uint64_t)T));   // valid starts: [0, ntok-T-1]
    L->win_prefix.push_back(L->win_prefix.back() + (sh.ntok - 1) / (uint64_t)T);
  }
  L->nslots = std::max(2, nslots);
  L->slots.assign(L->nslots, std::vector<int64_t>((size_t)B * (size_t)(T + 1)));
  L->full.assign(L->nslots, 0);
  L->slot_batch.assign(L->nslots, 0);
  L->next_produce = L->next_consume = start_batch;
  nthreads = std::max(1, std::min(nthreads, L->nslots));
  for (int t = 0; t < nthreads; ++t) L->workers.emplace_back([L] { L->worker(); });
  return L;
}

// Blocks until the next batch is ready and copies it (B*(T+1) int64) to dst.
// Returns the batch index it delivered.
uint64_t rn_loader_next(void* h, int64_t* dst) {
  auto* L = static_cast<Loader*>(h);
  uint64_t k;
  int s;
  {
    std::unique_lock<std::mutex> g(L->m);
    k = L->next_consume;
    s = int(k % (uint64_t)L->nslots);
    L->cv_full.wait(g, [&] { return L->full[s] && L->slot_batch[s] == k; });
  }
  std::memcpy(dst, L->slots[s].data(), L->slots[s].size() * sizeof(int64_t));
  {
    std::lock_guard<std::mutex> g(L->m);
    L->full[s] = 0;
    L->next_consume = k + 1;
  }
  L->cv_free.notify_all();
  return k;
}

uint64_t rn_loader_num_tokens(void* h) {
  auto* L = static_cast<Loader*>(h);
  uint64_t n = 0;
  for (auto& s : L->shards) n += s.ntok;
  return n;
}

uint64_t rn_loader_num_windows(void* h) { return static_cast<Loader*>(h)->win_prefix.back(); }

void rn_loader_destroy(void* h) { delete static_cast<Loader*>(h); }

}  // extern "C"
