// host_copy_stress.cpp — CPU sanitizer driver for the native staging-copy pool (csrc/host_copy.cpp,
// include/adfl_host.h). Built WITHOUT the HIP code, with -fsanitize=address,undefined or -fsanitize=thread
// (tools/sanitize/run.sh). Several caller threads share the pool (the channel's concurrent-receive
// case, tests/test_hostcopy.py::test_concurrent_callers), with ragged piece lists, zero-length pieces,
// odd offsets and explicit thread counts; every byte is checked.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "adfl_host.h"

static int run_caller(int id, int iters) {
  std::mt19937_64 rng(1234 + id);
  int bad = 0;
  for (int it = 0; it < iters; ++it) {
    const int n = 1 + (int)(rng() % 40);
    std::vector<std::vector<uint8_t>> src(n), dst(n);
    std::vector<void*> d(n);
    std::vector<const void*> s(n);
    std::vector<int64_t> b(n);
    for (int k = 0; k < n; ++k) {
      const int64_t len = (rng() % 4 == 0) ? 0 : (int64_t)(rng() % (it % 3 == 0 ? (3 << 20) : 70000));
      src[k].resize((size_t)len + 1);
      dst[k].assign((size_t)len + 1, 0xEE);
      for (int64_t i = 0; i < len; ++i) src[k][(size_t)i] = (uint8_t)(i * 31 + k + id);
      s[k] = src[k].data();
      d[k] = dst[k].data();
      b[k] = len;
    }
    const int threads = (int)(rng() % 20) - 2;  // <= 0: the default
    const int flags = (int)(rng() % 2);  // plain memcpy or streaming stores (ADFL_HOST_COPY_STREAM)
    if (adfl_host_copy_ex(d.data(), s.data(), b.data(), n, threads, flags) != 0) ++bad;
    for (int k = 0; k < n; ++k) {
      if (b[k] && std::memcmp(dst[k].data(), src[k].data(), (size_t)b[k]) != 0) ++bad;
      if (dst[k][(size_t)b[k]] != 0xEE) ++bad;  // nothing written past the piece
    }
  }
  return bad;
}

int main() {
  if (adfl_host_copy(nullptr, nullptr, nullptr, 1, 0) != -1) return 2;
  if (adfl_host_copy(nullptr, nullptr, nullptr, 0, 0) != 0) return 2;
  if (adfl_host_copy_ex(nullptr, nullptr, nullptr, 0, 0, 4) != -1) return 2;  // unknown flag
  const int callers = 8, iters = 12;
  std::vector<int> bad(callers, 0);
  std::vector<std::thread> ts;
  for (int c = 0; c < callers; ++c) ts.emplace_back([&, c] { bad[c] = run_caller(c, iters); });
  for (auto& t : ts) t.join();
  int total = 0;
  for (int v : bad) total += v;
  std::printf("host_copy_stress: %d callers x %d calls on a %d-thread pool, %d mismatches\n", callers, iters,
              adfl_host_threads(), total);
  return total ? 1 : 0;
}
