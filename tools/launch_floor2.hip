// Launch-floor probe 2: per-node time of a 700-node hipGraph chain, varying what the reverse sweep's chain differs
// in from launch_floor.hip's empty kernel: grid size, alternating kernels, a kernel that writes, a big kernel body
// that returns early, and L2 state (a 64 MB read before every replay).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/launch_floor2.hip -o tools/launch_floor2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_empty(float* p, int flag) {
  if (flag == 12345 && threadIdx.x == 1023) p[0] = 1.f;
}
__global__ __launch_bounds__(256) void k_empty2(float* p, int flag) {
  if (flag == 12346 && threadIdx.x == 1023) p[0] = 2.f;
}
// writes 16 B per thread (512 blocks -> 2 MB)
__global__ __launch_bounds__(256) void k_write(float* p, int flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  reinterpret_cast<float4*>(p)[i] = make_float4(flag, 1, 2, 3);
}
// reads 16 B per thread
__global__ __launch_bounds__(256) void k_read(float* p, int flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  float4 v = reinterpret_cast<const float4*>(p)[i];
  if (v.x == 1234.5f && flag) p[0] = v.y;
}
// ~200 dependent VALU ops, LDS round trip and barrier, no global memory
__global__ __launch_bounds__(256) void k_valu(float* p, int flag) {
  __shared__ float red[256];
  float v = threadIdx.x * 0.5f;
#pragma unroll 1
  for (int i = 0; i < 200; ++i) v = v * 0.999f + 0.5f;
  red[threadIdx.x] = v;
  __syncthreads();
  v = red[(threadIdx.x + 1) & 255];
  if (v == 1234.5f && flag) p[0] = v;
}
// one dependent 16-B load of the previous node's output, one 16-B store (a minimal stage)
__global__ __launch_bounds__(256) void k_stage(float* p, int flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int src = flag & 7, dst = (flag + 1) & 7;
  float4 v = reinterpret_cast<const float4*>(p + src * (1 << 19))[i];
  v.x += 1.f;
  reinterpret_cast<float4*>(p + dst * (1 << 19))[i] = v;
}
// the same with src / dst fixed by the caller (no dependency on the previous node when src != previous dst)
__global__ __launch_bounds__(256) void k_copy(const float* src, float* dst) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  float4 v = reinterpret_cast<const float4*>(src)[i];
  v.x += 1.f;
  reinterpret_cast<float4*>(dst)[i] = v;
}
// k_copy that also records (shader clock, 100 MHz real time) at its start and end in block 0, lane 0 of wave 0
__global__ __launch_bounds__(256) void k_copy_clk(const float* src, float* dst, unsigned long long* clk) {
  unsigned long long c0 = 0, r0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  float4 v = reinterpret_cast<const float4*>(src)[i];
  v.x += 1.f;
  reinterpret_cast<float4*>(dst)[i] = v;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[0] = c1 - c0;
    clk[1] = r1 - r0;
  }
}
__global__ void k_fill(const float4* src, long n, float4* dst) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float4 v = src[i];
    acc.x += v.x;
  }
  if (acc.x == 1234.5f) dst[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  const int N = 700;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float* buf;
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMemset(buf, 0, 64 << 20));
  float* big;
  const long nbig = (256L << 20) / 16;
  CK(hipMalloc(&big, 256L << 20));
  CK(hipMemset(big, 0, 256L << 20));
  const char* names[] = {"empty 256 blk", "empty 512 blk", "empty 128 blk", "alternate 2 kernels 512", "write 2MB 512 blk",
                         "read 2MB 512 blk", "write+read chain 512", "empty 512, L2 filled 256MB before", "valu+lds+barrier 512", "load->store stage 512",
                         "load->store stage 128", "copy fixed src, 8 dst 512", "copy dependent, odd offset 512",
                         "copy fixed src, fixed dst 512", "copy dependent 512 EAGER"};
  unsigned long long* clk;
  CK(hipMallocManaged(&clk, 64));
  for (int rep = 0; rep < 3; ++rep) {
    for (int i = 0; i < (rep == 2 ? 5000 : 700); ++i)
      hipLaunchKernelGGL(k_copy_clk, dim3(512), dim3(256), 0, s, buf + (i & 7) * (1 << 19), buf + ((i + 1) & 7) * (1 << 19), clk);
    CK(hipStreamSynchronize(s));
    printf("copy_clk block0 wave0: %llu shader cycles in %llu x 10 ns -> %.0f MHz\n", clk[0], clk[1],
           clk[1] ? 100.0 * clk[0] / clk[1] : 0.0);
  }
  for (int kind = 0; kind < 15; ++kind) {
    auto launch = [&](hipStream_t st, int i) {
      switch (kind) {
        case 0: hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, st, buf, i); break;
        case 1: case 7: hipLaunchKernelGGL(k_empty, dim3(512), dim3(256), 0, st, buf, i); break;
        case 2: hipLaunchKernelGGL(k_empty, dim3(128), dim3(256), 0, st, buf, i); break;
        case 3:
          if (i & 1) hipLaunchKernelGGL(k_empty2, dim3(512), dim3(256), 0, st, buf, i);
          else hipLaunchKernelGGL(k_empty, dim3(512), dim3(256), 0, st, buf, i);
          break;
        case 4: hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, st, buf + (i % 8) * (1 << 19), i); break;
        case 5: hipLaunchKernelGGL(k_read, dim3(512), dim3(256), 0, st, buf + (i % 8) * (1 << 19), 0); break;
        case 6:
          if (i & 1) hipLaunchKernelGGL(k_read, dim3(512), dim3(256), 0, st, buf + (i % 8) * (1 << 19), 0);
          else hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, st, buf + ((i + 1) % 8) * (1 << 19), i);
          break;
        case 8: hipLaunchKernelGGL(k_valu, dim3(512), dim3(256), 0, st, buf, i); break;
        case 9: hipLaunchKernelGGL(k_stage, dim3(512), dim3(256), 0, st, buf, i); break;
        case 10: hipLaunchKernelGGL(k_stage, dim3(128), dim3(256), 0, st, buf, i); break;
        case 11: hipLaunchKernelGGL(k_copy, dim3(512), dim3(256), 0, st, buf, buf + (1 + (i & 7)) * (1 << 20)); break;
        case 12: case 14:
          hipLaunchKernelGGL(k_copy, dim3(512), dim3(256), 0, st, buf + (i & 7) * ((1 << 19) + 4096),
                             buf + ((i + 1) & 7) * ((1 << 19) + 4096)); break;
        case 13: hipLaunchKernelGGL(k_copy, dim3(512), dim3(256), 0, st, buf, buf + (1 << 22)); break;
      }
    };
    if (kind == 14) {
      for (int i = 0; i < N; ++i) launch(s, i);
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < N; ++i) launch(s, i);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-36s eager %.2f us/node\n", names[kind], 1e3 * ms / N);
      continue;
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < N; ++i) launch(s, i);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      if (kind == 7) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (const float4*)big, nbig, (float4*)buf);
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-36s graph %.2f us/node\n", names[kind], 1e3 * best / N);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
