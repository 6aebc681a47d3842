// host_copy_stress.cpp — CPU sanitizer driver for the native staging-copy pool (csrc/host_copy.cpp,
// include/adfl_host.h). Built WITHOUT the HIP code, with -fsanitize=address,undefined or -fsanitize=thread
// (tools/sanitize/run.sh). Several caller threads share the pool (the channel's concurrent-receive
// case, tests/test_hostcopy.py::test_concurrent_callers), with ragged piece lists, zero-length pieces,
// odd offsets and explicit thread counts; every byte is checked.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "adfl_host.h"

// the wait callback of asynchronous jobs: a flag the test sets after submitting (the "D2H has landed")
struct Gate {
  std::atomic<int> open{0};
};
static int gate_wait(void* arg) {
  auto* g = static_cast<Gate*>(arg);
  while (!g->open.load(std::memory_order_acquire)) std::this_thread::yield();
  return 0;
}
static int failing_wait(void*) { return 7; }

// asynchronous jobs: several queued at once, each behind a gate opened in reverse order; sources written
// BEFORE the gate opens (the D2H filling the staging range), then every byte checked after the waits
static int run_async(int id, int iters) {
  std::mt19937_64 rng(999 + id);
  int bad = 0;
  for (int it = 0; it < iters; ++it) {
    const int jobs = 1 + (int)(rng() % 6);
    std::vector<std::vector<uint8_t>> src(jobs), dst(jobs);
    std::vector<Gate> gates(jobs);
    std::vector<int64_t> tickets(jobs);
    for (int j = 0; j < jobs; ++j) {
      const int64_t len = (int64_t)(rng() % (2 << 20));
      src[j].assign((size_t)len + 1, 0);
      dst[j].assign((size_t)len + 1, 0xEE);
      void* d = dst[j].data();
      const void* sp = src[j].data();
      tickets[j] = adfl_host_copy_submit(&d, &sp, &len, 1, (int)(rng() % 5) - 1, (int)(rng() % 2), gate_wait,
                                         &gates[j]);
      if (tickets[j] <= 0) ++bad;
    }
    for (int j = jobs - 1; j >= 0; --j) {
      for (size_t i = 0; i + 1 < src[j].size(); ++i) src[j][i] = (uint8_t)(i * 7 + j + id);
      gates[j].open.store(1, std::memory_order_release);
    }
    for (int j = 0; j < jobs; ++j) {
      if (adfl_host_copy_wait(tickets[j]) != 0) ++bad;
      const size_t len = src[j].size() - 1;
      if (len && std::memcmp(dst[j].data(), src[j].data(), len) != 0) ++bad;
      if (dst[j][len] != 0xEE) ++bad;
    }
  }
  // a failing wait callback: the status comes back, nothing is copied
  uint8_t a[4096] = {1}, b[4096] = {0};
  void* d = b;
  const void* sp = a;
  const int64_t len = sizeof(a);
  const int64_t t = adfl_host_copy_submit(&d, &sp, &len, 1, 0, 0, failing_wait, nullptr);
  if (adfl_host_copy_wait(t) != 7 || b[0] != 0) ++bad;
  return bad;
}

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
  if (adfl_host_copy_submit(nullptr, nullptr, nullptr, 1, 0, 0, nullptr, nullptr) != -1) return 2;
  if (adfl_host_copy_wait(0) != -1) return 2;
  const int callers = 8, iters = 12;
  std::vector<int> bad(2 * callers, 0);
  std::vector<std::thread> ts;
  for (int c = 0; c < callers; ++c) ts.emplace_back([&, c] { bad[c] = run_caller(c, iters); });
  for (int c = 0; c < callers; ++c) ts.emplace_back([&, c] { bad[callers + c] = run_async(c, iters); });
  for (auto& t : ts) t.join();
  int total = 0;
  for (int v : bad) total += v;
  std::printf("host_copy_stress: %d sync + %d async callers x %d calls on a %d-thread pool, %d mismatches\n",
              callers, callers, iters,
              adfl_host_threads(), total);
  return total ? 1 : 0;
}
