// Minimal cooperative-launch program (no torch, no ADFL library) for the round-2 finding that
// `rocprofv3 --kernel-trace` over the C3 bench with the cooperative bucketed encode died with SIGSEGV in
// the process exit path. It launches one plain kernel and one kernel through hipLaunchCooperativeKernel
// (grid sized to the co-resident capacity, like the product's coop encode did), checks both results and
// returns 0. Run it plain and under rocprofv3: a crash only under the profiler, after "ok", puts the fault
// in the profiler's teardown, not in the cooperative launch or in libadfl_slq.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/coop_repro tools/coop_repro.hip
//   ./tools/coop_repro [reps] [plain]      (plain: the control, ordinary launches only)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                         \
    }                                                                                   \
  } while (0)

__global__ void k_plain(int* out) { out[blockIdx.x * blockDim.x + threadIdx.x] = (int)blockIdx.x; }

// Every block adds its index to a per-launch counter; no block waits on another (the launch mode alone is
// under test, not a grid barrier).
__global__ void k_coop(int* out, unsigned* counter) {
  out[blockIdx.x * blockDim.x + threadIdx.x] = (int)blockIdx.x + 1;
  if (threadIdx.x == 0) atomicAdd(counter, blockIdx.x);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  const bool coop_launch = !(argc > 2 && std::strcmp(argv[2], "plain") == 0);
  int dev = 0, coop = 0, per_cu = 0;
  hipDeviceProp_t prop;
  CHECK(hipGetDevice(&dev));
  CHECK(hipGetDeviceProperties(&prop, dev));
  CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
  const int block = 256;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_coop), block, 0));
  const int grid = per_cu * prop.multiProcessorCount;
  std::printf("device %s, %d CUs, cooperative launch %d, %d blocks/CU -> grid %d\n", prop.gcnArchName,
              prop.multiProcessorCount, coop, per_cu, grid);
  int* d_out = nullptr;
  unsigned* d_cnt = nullptr;
  CHECK(hipMalloc(&d_out, (size_t)grid * block * sizeof(int)));
  CHECK(hipMalloc(&d_cnt, sizeof(unsigned)));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  std::vector<int> h((size_t)grid * block);
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_plain, dim3(grid), dim3(block), 0, s, d_out);
    CHECK(hipGetLastError());
    CHECK(hipMemsetAsync(d_cnt, 0, sizeof(unsigned), s));
    void* args[] = {&d_out, &d_cnt};
    if (coop_launch) {
      CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop), dim3(grid), dim3(block), args, 0, s));
    } else {
      hipLaunchKernelGGL(k_coop, dim3(grid), dim3(block), 0, s, d_out, d_cnt);
      CHECK(hipGetLastError());
    }
    CHECK(hipStreamSynchronize(s));
    unsigned cnt = 0;
    CHECK(hipMemcpy(&cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(h.data(), d_out, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    const unsigned want = (unsigned)((long long)grid * (grid - 1) / 2);
    for (size_t i = 0; i < h.size(); ++i)
      if (h[i] != (int)(i / block) + 1) {
        std::fprintf(stderr, "rep %d: out[%zu] = %d\n", r, i, h[i]);
        return 1;
      }
    if (cnt != want) {
      std::fprintf(stderr, "rep %d: counter %u, want %u\n", r, cnt, want);
      return 1;
    }
  }
  CHECK(hipStreamDestroy(s));
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_cnt));
  std::printf("ok: %d reps of plain + %s launches\n", reps, coop_launch ? "cooperative" : "plain (control)");
  std::fflush(stdout);
  return 0;
}
