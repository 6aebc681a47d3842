// host_copy.cpp — parallel host staging copies (include/adfl_host.h): a persistent pool of std::threads
// that splits a list of memcpys into equal byte ranges. Used by the host-resident channel path to gather a
// CPU state dict into the pinned bucket and to scatter payloads back into per-tensor storage.

#include <emmintrin.h>

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "adfl_host.h"
#include "adfl_slq.h"

namespace {

constexpr int kMaxThreads = 8;  // host channel A/B on the GPU box: 8 and 4 beat 16 (profiles/r04/host_channel)
constexpr int64_t kMinBytesPerThread = 256 << 10;  // below this, extra threads cost more than they copy

// One list of copies. Synchronous jobs (adfl_host_copy_ex) borrow the caller's arrays and the caller's
// thread takes part; asynchronous jobs (adfl_host_copy_submit) own copies of them and run on the workers
// only, after an optional wait callback (a HIP event's completion: the D2H that fills the source).
struct Job {
  bool stream;  // ADFL_HOST_COPY_STREAM
  void* const* dsts;
  const void* const* srcs;
  const int64_t* prefix;  // prefix[k] = bytes before piece k; prefix[n] = total
  int64_t n;
  int parts;
  int (*wait_fn)(void*) = nullptr;
  void* wait_arg = nullptr;
  uint32_t* const* absmax = nullptr;  // ADFL_HOST_COPY_ABSMAX: piece k's max |fp32 bits| max'ed into *absmax[k]
  int next = 0;               // next unclaimed part (under the pool mutex)
  std::atomic<int> done{0};   // finished parts (incremented under the pool mutex; a waiter may spin on it)
  int status = 0;
  // owned storage of an asynchronous job
  std::vector<uint32_t*> own_absmax;
  std::vector<void*> own_dsts;
  std::vector<const void*> own_srcs;
  std::vector<int64_t> own_prefix;
};

constexpr int64_t kStreamBytes = 64 << 10;  // pieces at least this long take the streaming copy

// memcpy with non-temporal 16-byte stores (SSE2, baseline x86-64), for ADFL_HOST_COPY_STREAM: fresh
// per-tensor outputs nothing reads soon; streaming stores skip the read-for-ownership of every destination
// line. Into the pinned bucket the plain memcpy measured faster (tools/hostcopy_ab.py), so the gather does
// not ask for it. Weakly ordered: every part ends with _mm_sfence() (run_part) before it reports done.
void stream_copy(char* d, const char* s, size_t n) {
  size_t head = (16 - ((uintptr_t)d & 15)) & 15;
  if (head > n) head = n;
  std::memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  const size_t m = n & ~(size_t)63;
  for (size_t i = 0; i < m; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 48), e);
  }
  std::memcpy(d + m, s + m, n - m);
}

// max of |x| as the fp32 bit pattern with the sign cleared: the float order on non-NaN values, and every NaN
// (> 0x7f800000) wins — torch.max(torch.abs(t)) (quant.py:100), as the device kernels reduce it. Cloned for
// AVX-512 / AVX2 with the loader's run-time dispatch: the default x86-64 target has no unsigned 32-bit max
// (SSE4.1), and the scalar loop reduced 15 GB/s from cache against 110 GB/s with AVX-512 (this container).
// (hipcc also parses this file in its gfx950 pass, which has no x86 clones: the attribute is host-pass only;
// a ThreadSanitizer build runs the ifunc resolver before its runtime is up and crashes, so it is left out.)
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__) && !defined(__SANITIZE_THREAD__)
#define ADFL_X86_CLONES __attribute__((target_clones("avx512f", "avx2", "default")))
#else
#define ADFL_X86_CLONES
#endif
ADFL_X86_CLONES uint32_t absmax_bits(const uint32_t* w, size_t n) {
  uint32_t m = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t v = w[i] & 0x7fffffffu;
    m = v > m ? v : m;
  }
  return m;
}

void atomic_max(uint32_t* p, uint32_t v) {
  uint32_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v > cur && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
}

constexpr size_t kMaxBlock = 32 << 10;  // absmax copies: the block is reduced, then copied from cache

// Copy byte range [lo, hi) of the concatenated piece list.
void copy_range(const Job& j, int64_t lo, int64_t hi) {
  int64_t k = std::upper_bound(j.prefix, j.prefix + j.n + 1, lo) - j.prefix - 1;
  while (lo < hi && k < j.n) {
    const int64_t piece_end = j.prefix[k + 1];
    const int64_t take = std::min(hi, piece_end) - lo;
    if (take > 0) {
      const int64_t off = lo - j.prefix[k];
      char* d = static_cast<char*>(j.dsts[k]) + off;
      const char* s = static_cast<const char*>(j.srcs[k]) + off;
      if (j.absmax && j.absmax[k]) {
        uint32_t m = 0;
        for (int64_t b = 0; b < take; b += (int64_t)kMaxBlock) {
          const size_t len = (size_t)std::min<int64_t>((int64_t)kMaxBlock, take - b);
          m = std::max(m, absmax_bits(reinterpret_cast<const uint32_t*>(s + b), len / 4));
          if (j.stream && take >= kStreamBytes)
            stream_copy(d + b, s + b, len);
          else
            std::memcpy(d + b, s + b, len);
        }
        atomic_max(j.absmax[k], m);
      } else if (j.stream && take >= kStreamBytes) {
        stream_copy(d, s, (size_t)take);
      } else {
        std::memcpy(d, s, (size_t)take);
      }
      lo += take;
    }
    ++k;
  }
}

// One part of a job; returns the wait callback's status (nonzero: nothing copied).
int run_part(const Job& j, int p) {
  if (j.wait_fn) {
    const int st = j.wait_fn(j.wait_arg);  // every part waits: a part never runs before its source is ready
    if (st != 0) return st;
  }
  const int64_t total = j.prefix[j.n];
  int64_t lo = total * p / j.parts, hi = total * (p + 1) / j.parts;
  if (j.absmax) {  // parts split at fp32 words: a part reduces whole elements
    lo &= ~(int64_t)3;
    hi = p + 1 == j.parts ? total : hi & ~(int64_t)3;
  }
  copy_range(j, lo, hi);
  _mm_sfence();  // the streaming stores are visible before this part counts as done
  return 0;
}

// Persistent workers over a FIFO of jobs: a worker claims the next unclaimed part of the oldest job that has
// one. A synchronous caller also works on its own job; an asynchronous job is left to the workers.
class Pool {
 public:
  static Pool& get() {
    static Pool* pool = new Pool();  // never destroyed: worker threads outlive static destruction order
    return *pool;
  }

  int size() const { return (int)workers_.size() + 1; }
  int workers() const { return (int)workers_.size(); }

  // pin every worker to `cpus` (the GPU's NUMA node: the staging copies then run next to the pinned buckets
  // and the GPU's PCIe root)
  int bind(const int32_t* cpus, int32_t n) {
#ifdef __linux__
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int32_t i = 0; i < n; ++i)
      if (cpus[i] >= 0 && cpus[i] < CPU_SETSIZE) CPU_SET(cpus[i], &set);
    if (CPU_COUNT(&set) == 0) return -1;
    for (auto& h : handles_)
      if (pthread_setaffinity_np(h, sizeof(set), &set) != 0) return -1;
    return 0;
#else
    (void)cpus;
    (void)n;
    return -1;
#endif
  }

  void run(Job& job) {
    push(&job);
    int p;
    while ((p = claim_own(&job)) >= 0) finish(&job, run_part(job, p));
    wait(&job);
  }

  void push(Job* job) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      queue_.push_back(job);
      queued_.fetch_add(1, std::memory_order_relaxed);
    }
    cv_.notify_all();
  }

  int wait(Job* job) {
    // spin first: a channel call's copies finish within microseconds of each other, and a thread woken from
    // a condition variable (and a deep C-state) costs tens of microseconds each time
    const auto t0 = std::chrono::steady_clock::now();
    while (job->done.load(std::memory_order_acquire) != job->parts) {
      if (std::chrono::steady_clock::now() - t0 > spin_) {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return job->done.load(std::memory_order_acquire) == job->parts; });
        break;
      }
      _mm_pause();
    }
    std::lock_guard<std::mutex> lk(mu_);  // the status, written before the last part counted
    return job->status;
  }

 private:
  // threads = the CPUs this process may run on (its affinity mask, not the machine's count: a container or a
  // job share may see fewer), at most kMaxThreads, or ADFL_HOST_THREADS when set (1 = the caller only)
  static int pool_threads() {
    int hw = (int)std::thread::hardware_concurrency();
#ifdef __linux__
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) hw = CPU_COUNT(&set);
#endif
    int n = std::min(hw > 0 ? hw : 4, kMaxThreads);
    if (const char* e = std::getenv("ADFL_HOST_THREADS")) {
      const int v = std::atoi(e);
      if (v >= 1) n = std::min(v, 64);
    }
    return n;
  }

  // ADFL_HOST_SPIN_US (default 200): how long an idle worker, or a waiting caller, spins before sleeping
  static std::chrono::microseconds spin_time() {
    long us = 200;
    if (const char* e = std::getenv("ADFL_HOST_SPIN_US")) us = std::max(0L, std::atol(e));
    return std::chrono::microseconds(us);
  }

  Pool() : spin_(spin_time()) {
    const int n = pool_threads() - 1;
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
    for (auto& t : workers_) {
      handles_.push_back(t.native_handle());
      t.detach();
    }
  }

  // the caller's claim on its own (synchronous) job
  int claim_own(Job* job) {
    std::lock_guard<std::mutex> lk(mu_);
    if (job->next >= job->parts) return -1;
    const int p = job->next++;
    if (job->next == job->parts) drop(job);
    return p;
  }

  void drop(Job* job) {  // a fully claimed job leaves the queue (under mu_)
    for (auto it = queue_.begin(); it != queue_.end(); ++it)
      if (*it == job) {
        queue_.erase(it);
        queued_.fetch_sub(1, std::memory_order_relaxed);
        return;
      }
  }

  void finish(Job* job, int status) {
    std::lock_guard<std::mutex> lk(mu_);
    if (status != 0 && job->status == 0) job->status = status;
    const int parts = job->parts;  // read before the count: a spinning waiter may free the job right after it
    if (job->done.fetch_add(1, std::memory_order_acq_rel) + 1 == parts) done_cv_.notify_all();
  }

  void loop() {
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      while (queued_.load(std::memory_order_relaxed) == 0 && std::chrono::steady_clock::now() - t0 < spin_)
        _mm_pause();
      Job* job;
      int p;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !queue_.empty(); });
        job = queue_.front();
        p = job->next++;
        if (job->next == job->parts) {
          queue_.pop_front();
          queued_.fetch_sub(1, std::memory_order_relaxed);
        }
      }
      finish(job, run_part(*job, p));
    }
  }

  std::vector<std::thread> workers_;
  std::vector<std::thread::native_handle_type> handles_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Job*> queue_;
  std::atomic<int> queued_{0};  // jobs in queue_ (idle workers spin on it before sleeping)
  const std::chrono::microseconds spin_;
};

int64_t build_prefix(const int64_t* nbytes, void* const* dsts, const void* const* srcs, int64_t n,
                     std::vector<int64_t>& prefix) {
  prefix.assign((size_t)n + 1, 0);
  for (int64_t k = 0; k < n; ++k) {
    if (nbytes[k] < 0 || (nbytes[k] > 0 && (!dsts[k] || !srcs[k]))) return -1;
    prefix[k + 1] = prefix[k] + nbytes[k];
  }
  return prefix[n];
}

int parts_for(int64_t total, int nthreads, int available) {
  int parts = nthreads > 0 ? std::min<int>(nthreads, available) : available;
  return (int)std::max<int64_t>(1, std::min<int64_t>(parts, total / kMinBytesPerThread));
}

}  // namespace

extern "C" {

int32_t adfl_host_threads(void) { return Pool::get().size(); }

int adfl_host_copy(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n, int32_t nthreads) {
  return adfl_host_copy_ex(dsts, srcs, nbytes, n, nthreads, 0);
}

int adfl_host_copy_ex(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n, int32_t nthreads,
                      int32_t flags) {
  if (n < 0 || (n > 0 && (!dsts || !srcs || !nbytes)) || (flags & ~ADFL_HOST_COPY_STREAM)) return ADFL_E_ARG;
  std::vector<int64_t> prefix;
  const int64_t total = build_prefix(nbytes, dsts, srcs, n, prefix);
  if (total < 0) return ADFL_E_ARG;
  if (total == 0) return ADFL_OK;
  Pool& pool = Pool::get();
  Job job;
  job.stream = (flags & ADFL_HOST_COPY_STREAM) != 0;
  job.dsts = dsts;
  job.srcs = srcs;
  job.prefix = prefix.data();
  job.n = n;
  job.parts = parts_for(total, nthreads, pool.size());
  if (job.parts == 1) {
    run_part(job, 0);
    return ADFL_OK;
  }
  pool.run(job);
  return ADFL_OK;
}

int64_t adfl_host_copy_submit(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n,
                              int32_t nthreads, int32_t flags, int (*wait_fn)(void*), void* wait_arg) {
  return adfl_host_copy_submit_absmax(dsts, srcs, nbytes, n, nthreads, flags, wait_fn, wait_arg, nullptr);
}

int64_t adfl_host_copy_submit_absmax(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n,
                                     int32_t nthreads, int32_t flags, int (*wait_fn)(void*), void* wait_arg,
                                     uint32_t* const* absmax_bits) {
  if (n < 0 || (n > 0 && (!dsts || !srcs || !nbytes)) || (flags & ~ADFL_HOST_COPY_STREAM)) return ADFL_E_ARG;
  Job* job = new Job();
  const int64_t total = build_prefix(nbytes, dsts, srcs, n, job->own_prefix);
  bool fp32_words = true;
  for (int64_t k = 0; absmax_bits && k < n; ++k)
    if ((nbytes[k] & 3) || ((uintptr_t)srcs[k] & 3)) fp32_words = false;
  if (total < 0 || !fp32_words) {
    delete job;
    return ADFL_E_ARG;
  }
  if (absmax_bits) {
    job->own_absmax.assign(absmax_bits, absmax_bits + n);
    job->absmax = job->own_absmax.data();
  }
  job->own_dsts.assign(dsts, dsts + n);
  job->own_srcs.assign(srcs, srcs + n);
  job->stream = (flags & ADFL_HOST_COPY_STREAM) != 0;
  job->dsts = job->own_dsts.data();
  job->srcs = job->own_srcs.data();
  job->prefix = job->own_prefix.data();
  job->n = n;
  job->wait_fn = wait_fn;
  job->wait_arg = wait_arg;
  Pool& pool = Pool::get();
  // the workers only (the caller returns at once); at least one part, so the wait callback always runs
  job->parts = pool.workers() > 0 ? parts_for(std::max<int64_t>(total, 1), nthreads, pool.workers()) : 1;
  if (pool.workers() == 0) {  // no worker threads on this host: run it here
    job->status = run_part(*job, 0);
    job->done.store(job->parts, std::memory_order_release);
  } else {
    pool.push(job);
  }
  return reinterpret_cast<int64_t>(job);
}

int adfl_host_bind(const int32_t* cpus, int32_t n) {
  if (!cpus || n < 1) return ADFL_E_ARG;
  return Pool::get().bind(cpus, n) == 0 ? ADFL_OK : ADFL_E_ARG;
}

int adfl_host_copy_done(int64_t ticket) {
  if (ticket <= 0) return ADFL_E_ARG;
  const Job* job = reinterpret_cast<const Job*>(ticket);
  return job->done.load(std::memory_order_acquire) == job->parts ? 1 : 0;
}

int adfl_host_copy_wait(int64_t ticket) {
  if (ticket <= 0) return ADFL_E_ARG;
  Job* job = reinterpret_cast<Job*>(ticket);
  const int st = Pool::get().wait(job);
  delete job;
  return st;
}

}  // extern "C"
