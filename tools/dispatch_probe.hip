// In-stream cost of an early-exit kernel by grid shape: 200 back-to-back launches between two HIP
// events, each kernel loading one flag and returning (the greedy select's "nothing to do" stage).
// Build: hipcc --offload-arch=gfx950 -O3 tools/dispatch_probe.hip -o tools/bin/dispatch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_exit(const int* flag, int* sink) {
  if (flag[0]) return;
  sink[blockIdx.x] = threadIdx.x;
}

int main() {
  int *flag, *sink;
  hipMalloc(&flag, 4);
  hipMalloc(&sink, 1 << 20);
  const int one = 1;
  hipMemcpy(flag, &one, 4, hipMemcpyHostToDevice);
  hipStream_t st;
  hipStreamCreate(&st);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int shapes[][2] = {{1, 64}, {64, 256}, {64, 1024}, {256, 256}, {256, 512}, {256, 1024}, {1024, 256}, {1024, 1024}};
  for (auto& s : shapes) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a, st);
      for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_exit, dim3(s[0]), dim3(s[1]), 0, st, flag, sink);
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("grid %5d x %5d threads (%6d waves): %.2f us per early-exit kernel\n", s[0], s[1],
                      s[0] * s[1] / 64, ms * 1000.f / 200.f);
    }
  }
  return 0;
}
