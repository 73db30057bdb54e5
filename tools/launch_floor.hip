// Launch-floor probe: per-kernel time of a dependent chain of tiny kernels (eager and hipGraph replay, on a
// created non-blocking stream and on the null stream), and of a kernel with a 192-byte argument struct.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct Big {
  const float* p[16];
  int v[16];
};

__global__ void empty_kernel(float* p) {
  if (p && threadIdx.x == 1023) p[0] = 1.f;
}
__global__ void big_kernel(Big b) {
  if (b.v[3] == 12345 && threadIdx.x == 1023) ((float*)b.p[0])[0] = 1.f;
}
__global__ void lds_kernel(float* p) {
  __shared__ float red[4][16][16];
  red[threadIdx.x >> 6][(threadIdx.x >> 4) & 3][threadIdx.x & 15] = threadIdx.x;
  __syncthreads();
  if (p && red[0][0][threadIdx.x & 15] == -1.f) p[0] = 1.f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  const int N = 700;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  Big big{};
  for (int kind = 0; kind < 3; ++kind) {
    for (int ns = 0; ns < 2; ++ns) {
      hipStream_t ls = ns ? (hipStream_t)0 : s;
      auto launch = [&](hipStream_t st) {
        if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, st, nullptr);
        else if (kind == 1) hipLaunchKernelGGL(big_kernel, dim3(256), dim3(256), 0, st, big);
        else hipLaunchKernelGGL(lds_kernel, dim3(256), dim3(256), 0, st, nullptr);
      };
      for (int i = 0; i < N; ++i) launch(ls);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, ls));
      for (int i = 0; i < N; ++i) launch(ls);
      CK(hipEventRecord(e1, ls));
      CK(hipEventSynchronize(e1));
      float ms_e;
      CK(hipEventElapsedTime(&ms_e, e0, e1));
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
      for (int i = 0; i < N; ++i) launch(s);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, ls));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, ls));
      for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(ge, ls));
      CK(hipEventRecord(e1, ls));
      CK(hipEventSynchronize(e1));
      float ms_g;
      CK(hipEventElapsedTime(&ms_g, e0, e1));
      printf("%-10s %-12s eager %.2f us/kernel   graph %.2f us/kernel\n", kind == 0 ? "empty" : kind == 1 ? "big-args" : "lds+bar",
             ns ? "null stream" : "own stream", 1e3 * ms_e / N, 1e3 * ms_g / (3 * N));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
