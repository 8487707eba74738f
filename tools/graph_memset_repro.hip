// Stand-alone check of hipMemsetAsync captured into a graph (no library code): the count-slab
// zeroing of the rollout graphs, replayed.  A buffer of 3 x 256 u64 (the library's slabs at 4
// capacity classes) is zeroed on the host side, the graph [memset(buf, 0) -> k kernels] is launched,
// and the buffer must read back all zero after every replay.  Variants: kernels after the memset
// (0 / 1 / 6, each with a 512-B argument struct like the step kernels' KParams), the replay stream
// (the null stream or a created one), and what runs between replays (direct memsets, pageable copies,
// kernels, other host calls overwriting the stack the capture ran on).
//   hipcc --offload-arch=gfx950 -O2 tools/graph_memset_repro.hip -o tools/bin/graph_memset_repro
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
      std::exit(2);                                                                        \
    }                                                                                      \
  } while (0)

struct Big {
  double v[64];
};

__global__ void k_touch(Big b, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = out[i] * 0.5 + b.v[i & 63];
}

// capture [memset(buf, 0) -> nk kernels] in its own stack frame (as the library's capture_graph does)
static hipGraphExec_t capture(hipStream_t cap, unsigned long long* buf, size_t words, int nk, const Big& b,
                              double* other) {
  hipGraph_t g;
  hipGraphExec_t ex;
  CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
  CK(hipMemsetAsync(buf, 0, words * 8, cap));
  for (int k = 0; k < nk; ++k) hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, cap, b, other, 1 << 20);
  CK(hipStreamEndCapture(cap, &g));
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  CK(hipGraphDestroy(g));
  CK(hipGraphUpload(ex, cap));
  return ex;
}

// overwrite the stack below the caller's frame with non-zero words (stack addresses), as the
// library's other host calls do between two replays
__attribute__((noinline)) static unsigned long long scribble() {
  volatile unsigned long long a[8192];
  for (int k = 0; k < 8192; ++k) a[k] = (unsigned long long)(uintptr_t)&a[k];
  return a[77];
}

int main() {
  const size_t words = 3 * 256;
  unsigned long long* buf = nullptr;
  double* other = nullptr;
  CK(hipMalloc(&buf, words * 8));
  CK(hipMalloc(&other, (1 << 20) * sizeof(double)));
  CK(hipMemset(other, 0, (1 << 20) * sizeof(double)));
  hipStream_t cap, mine;
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&mine, hipStreamNonBlocking));
  Big b{};
  for (int i = 0; i < 64; ++i) b.v[i] = i;
  int bad_total = 0;
  for (int inter : {0, 1, 2, 4, 7, 8, 15})
  for (int nk : {0, 1, 6}) {
    for (int on_null : {1, 0}) {
      hipStream_t ls = on_null ? (hipStream_t)0 : mine;
      hipGraphExec_t ex = capture(cap, buf, words, nk, b, other);
      std::printf("between replays %s%s%s%s, kernels after the memset %d, replay stream %s: non-zero words after each launch:",
                  inter & 1 ? "[memset]" : "", inter & 2 ? "[H2D copy]" : "", inter & 4 ? "[kernel]" : "",
                  inter & 8 ? "[stack overwritten]" : "", nk, on_null ? "null" : "created");
      for (int rep = 0; rep < 4; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipMemset(buf, 0, words * 8));
        CK(hipDeviceSynchronize());
        if (inter & 1) CK(hipMemsetAsync(other, 0x5a, 4096, ls));  // direct memsets between replays
        if (inter & 2) {  // small pageable host-to-device copies between replays
          unsigned long long stage[64];
          for (int k = 0; k < 64; ++k) stage[k] = (unsigned long long)(uintptr_t)&stage[k];  // stack addresses
          CK(hipMemcpyAsync(other + 4096, stage, sizeof(stage), hipMemcpyHostToDevice, ls));
        }
        if (inter & 4) hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, ls, b, other, 1 << 20);
        if (inter & 8) bad_total += scribble() == 0 ? 1 : 0;
        CK(hipGraphLaunch(ex, ls));
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(words);
        CK(hipMemcpy(h.data(), buf, words * 8, hipMemcpyDeviceToHost));
        int nz = 0;
        unsigned long long first = 0;
        for (auto v : h)
          if (v) {
            if (!nz) first = v;
            ++nz;
          }
        bad_total += nz;
        std::printf(" %d", nz);
        if (nz) std::printf(" (first 0x%llx)", first);
      }
      std::printf("\n");
      CK(hipGraphExecDestroy(ex));
    }
  }
  std::printf("%s\n", bad_total ? "REPRODUCED: a captured memset node wrote non-zero words" : "memset nodes clean");
  return 0;
}
