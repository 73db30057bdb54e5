// Latency probe: one wave times (shader clock) a first load, a store, a second load on the same page and a load on
// a fresh page, each waited with s_waitcnt; run standalone and right after a kernel that wrote the buffer.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lat_probe.hip -o tools/lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lat(float* p, float* q, unsigned long long* out) {
  if (threadIdx.x) return;
  unsigned long long t[6];
  t[0] = __builtin_amdgcn_s_memtime();
  float v = __builtin_nontemporal_load(p);
  __builtin_amdgcn_s_waitcnt(0);
  t[1] = __builtin_amdgcn_s_memtime();
  q[0] = v + 1.f;
  __builtin_amdgcn_s_waitcnt(0);
  t[2] = __builtin_amdgcn_s_memtime();
  float v2 = *(volatile float*)(p + 64);
  __builtin_amdgcn_s_waitcnt(0);
  t[3] = __builtin_amdgcn_s_memtime();
  float v3 = *(volatile float*)(p + (4 << 20));
  __builtin_amdgcn_s_waitcnt(0);
  t[4] = __builtin_amdgcn_s_memtime();
  float v4 = *(volatile float*)(p + 64);
  __builtin_amdgcn_s_waitcnt(0);
  t[5] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 5; ++i) out[i] = t[i + 1] - t[i];
  if (v2 + v3 + v4 == 1234.5f) q[1] = 0.f;
}
__global__ void k_write(float* p, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = 1.f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
int main() {
  float *p, *q;
  unsigned long long* out;
  CK(hipMalloc(&p, 64 << 20));
  CK(hipMalloc(&q, 1 << 20));
  CK(hipMallocManaged(&out, 64));
  CK(hipMemset(p, 0, 64 << 20));
  for (int r = 0; r < 8; ++r) {
    const bool after_write = r & 1;
    if (after_write) hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, 0, p, 1L << 20);
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, p, q, out);
    CK(hipDeviceSynchronize());
    printf("%-22s first load %llu, store %llu, same-page load %llu, fresh-page load %llu, re-load %llu cycles\n",
           after_write ? "after a writer kernel" : "standalone", out[0], out[1], out[2], out[3], out[4]);
  }
  return 0;
}
