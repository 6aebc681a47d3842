// host_copy.cpp — parallel host staging copies (include/adfl_host.h): a persistent pool of std::threads
// that splits a list of memcpys into equal byte ranges. Used by the host-resident channel path to gather a
// CPU state dict into the pinned bucket and to scatter payloads back into per-tensor storage.

#include <emmintrin.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "adfl_host.h"
#include "adfl_slq.h"

namespace {

constexpr int kMaxThreads = 16;
constexpr int64_t kMinBytesPerThread = 256 << 10;  // below this, extra threads cost more than they copy

struct Job {
  bool stream;  // ADFL_HOST_COPY_STREAM
  void* const* dsts;
  const void* const* srcs;
  const int64_t* nbytes;
  int64_t n;
  const int64_t* prefix;  // prefix[k] = bytes before piece k; prefix[n] = total
  int parts;
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
      if (j.stream && take >= kStreamBytes)
        stream_copy(d, s, (size_t)take);
      else
        std::memcpy(d, s, (size_t)take);
      lo += take;
    }
    ++k;
  }
}

void run_part(const Job& j, int p) {
  const int64_t total = j.prefix[j.n];
  const int64_t lo = total * p / j.parts, hi = total * (p + 1) / j.parts;
  copy_range(j, lo, hi);
  _mm_sfence();  // the streaming stores are visible before this part counts as done
}

class Pool {
 public:
  static Pool& get() {
    static Pool* pool = new Pool();  // never destroyed: worker threads outlive static destruction order
    return *pool;
  }

  int size() const { return (int)workers_.size() + 1; }

  void run(const Job& job) {
    std::unique_lock<std::mutex> call(call_mu_);  // one job at a time; concurrent callers queue here
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &job;
      next_ = 1;  // part 0 is the caller's
      done_ = 0;
      ++generation_;
    }
    cv_.notify_all();
    run_part(job, 0);
    int mine = 1, p;
    while ((p = claim()) >= 0) {
      run_part(job, p);
      ++mine;
    }
    std::unique_lock<std::mutex> lk(mu_);
    done_ += mine;
    done_cv_.wait(lk, [&] { return done_ == job.parts; });
    job_ = nullptr;
  }

 private:
  Pool() {
    unsigned hw = std::thread::hardware_concurrency();
    const int n = (int)std::min<unsigned>(hw ? hw : 4, kMaxThreads) - 1;
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
    for (auto& t : workers_) t.detach();
  }

  int claim() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!job_ || next_ >= job_->parts) return -1;
    return next_++;
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const Job* job;
      int p;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return generation_ != seen && job_ && next_ < job_->parts; });
        seen = generation_;
        job = job_;
        p = next_++;
      }
      for (;;) {
        run_part(*job, p);
        std::lock_guard<std::mutex> lk(mu_);
        ++done_;
        if (done_ == job->parts) done_cv_.notify_all();
        if (job_ != job || next_ >= job->parts) break;
        p = next_++;
      }
    }
  }

  std::vector<std::thread> workers_;
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const Job* job_ = nullptr;
  int next_ = 0, done_ = 0;
  uint64_t generation_ = 0;
};

}  // namespace

extern "C" {

int32_t adfl_host_threads(void) { return Pool::get().size(); }

int adfl_host_copy(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n, int32_t nthreads) {
  return adfl_host_copy_ex(dsts, srcs, nbytes, n, nthreads, 0);
}

int adfl_host_copy_ex(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n, int32_t nthreads,
                      int32_t flags) {
  if (n < 0 || (n > 0 && (!dsts || !srcs || !nbytes)) || (flags & ~ADFL_HOST_COPY_STREAM)) return ADFL_E_ARG;
  std::vector<int64_t> prefix((size_t)n + 1, 0);
  for (int64_t k = 0; k < n; ++k) {
    if (nbytes[k] < 0 || (nbytes[k] > 0 && (!dsts[k] || !srcs[k]))) return ADFL_E_ARG;
    prefix[k + 1] = prefix[k] + nbytes[k];
  }
  const int64_t total = prefix[n];
  if (total == 0) return ADFL_OK;
  Pool& pool = Pool::get();
  int parts = nthreads > 0 ? std::min<int>(nthreads, pool.size()) : pool.size();
  parts = (int)std::max<int64_t>(1, std::min<int64_t>(parts, total / kMinBytesPerThread));
  Job job{(flags & ADFL_HOST_COPY_STREAM) != 0, dsts, srcs, nbytes, n, prefix.data(), parts};
  if (parts == 1) {
    run_part(job, 0);
    return ADFL_OK;
  }
  pool.run(job);
  return ADFL_OK;
}

}  // extern "C"
