// smallc_bench.hip — A/B the output-layer (to-RGB) kernels at the CIFAR-10 B=128 shape (256 ch @ 32x32
// -> 3 ch, k3 s1 p1): the dgrad (fp32 mask / sign-bit mask, fp32 / limb output) and the two-stage
// forward, timed in one process.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DDAMC_GEMM_NO_C_API tools/smallc_bench.hip -o tools/smallc_bench
#include <cmath>
#include <cstdio>
#include <cstring>
#include <type_traits>
#include <vector>

#include "../diffusion-amortized-mcmc_amd/csrc/gemm.hip"
#include "../diffusion-amortized-mcmc_amd/csrc/generator.hip"
#include "../diffusion-amortized-mcmc_amd/csrc/wgrad.hip"

namespace damc_prof {
bool enabled() { return false; }
int begin(const char*, double, hipStream_t) { return -1; }
void end(int, hipStream_t) {}
}  // namespace damc_prof
int damc_launch_posterior_update(const damc_ebm_t*, float*, const float*, int, long, int, int, double, int,
                                 const float*, uint64_t, uint64_t, uint64_t, float*, hipStream_t) {
  return 0;
}

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e = (x);                                                                   \
    if (e != hipSuccess) {                                                                \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);        \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

static float* rnd(size_t n, unsigned seed) {
  std::vector<float> h(n);
  unsigned s = seed;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
  }
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

// store-path probes: the dgrad's 201 MB limb output written with zeros, (0) one 16-B store per thread over the whole
// buffer, (1) the MFMA kernel's persistent 16-pixel units (768 x 256 threads), 24 contiguous 16-B stores per lane
__global__ void store_flat_probe(uint4* o, long n16) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) o[i] = uint4{0u, 0u, 0u, 0u};
}
__global__ __launch_bounds__(256) void store_unit_probe(unsigned char* o, int units, int rowb) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int un = blockIdx.x * 4 + wave; un < units; un += gridDim.x * 4) {
    uint4* d = reinterpret_cast<uint4*>(o + (long)un * 16 * rowb);
    for (int j = lane; j < 16 * rowb / 16; j += 64) d[j] = uint4{0u, 0u, 0u, 0u};
  }
}

int main() {
  const int B = 128, C = 256, H = 32;
  const long npix = (long)B * H * H;
  damc_layer_t L{};
  L.kind = DAMC_LAYER_SMALLC;
  L.cin = C; L.cout = 3; L.k = 3; L.stride = 1; L.pad = 1; L.hin = L.win = L.hout = L.wout = H;
  L.act = DAMC_ACT_TANH;
  float* wt = rnd((size_t)C * 3 * 9, 1);
  float *wf, *wb;
  CK(hipMalloc(&wf, C * 27 * 4));
  CK(hipMalloc(&wb, 32 * C * 4));
  L.w_fwd = wf; L.w_bwd = wb;
  L.bias = rnd(3, 2);
  CK((hipError_t)damc_pack_generator_layer(&L, wt, wf, wb, nullptr));
  float* h = rnd(npix * C, 3);
  float* x = rnd(npix * 3, 4);
  float* delta = rnd(npix * 3, 5);
  float* pbuf;
  CK(hipMalloc(&pbuf, npix * 32 * 4));
  unsigned short* h3;
  CK(hipMalloc(&h3, npix * C * 6));
  unsigned char* bits;
  CK(hipMalloc(&bits, npix * C / 8));
  CK(hipMemset(bits, 0x5a, npix * C / 8));
  float* hcopy;
  CK(hipMalloc(&hcopy, npix * C * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto fn) {
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      fn();
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < 20; ++k) fn();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms / 20);
    }
    printf("%-40s %8.1f us  %6.2f TB/s\n", name, best * 1e3, bytes / (best * 1e-3) / 1e12);
  };
  const double act = (double)npix * C * 4;
  timeit("fwd two-stage", act, [&] {
    smallc_fwd(L, h, B, x, 100.f, delta, nullptr, nullptr, pbuf, s);
  });
  {  // the output projection: limb engine vs the LDS-staged fp32-MFMA kernel
    float* pb2;
    CK(hipMalloc(&pb2, npix * 32 * 4));
    const int g1 = (int)((npix + 127) / 128);
    hipLaunchKernelGGL((smallc_proj_lds_kernel<1>), dim3(g1), dim3(256), 0, s, h, npix, C, L.w_bwd, pbuf);
    hipLaunchKernelGGL(smallc_proj_x3_kernel, dim3(768), dim3(256), 0, s, h, npix, L.w_bwd, pb2);
    CK(hipStreamSynchronize(s));
    std::vector<float> p1(npix * 32), p2(npix * 32);
    CK(hipMemcpy(p1.data(), pbuf, p1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(p2.data(), pb2, p2.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0, md = 0;
    for (size_t i = 0; i < p1.size(); ++i) {
      mx = std::max(mx, (double)std::fabs(p1[i]));
      md = std::max(md, (double)std::fabs(p1[i] - p2[i]));
    }
    printf("proj x3 vs fp32: max |diff| %.3e, max |value| %.3e (rel %.2e)\n", md, mx, md / mx);
    timeit("proj fp32-MFMA (LDS)", act, [&] {
      hipLaunchKernelGGL((smallc_proj_lds_kernel<1>), dim3(g1), dim3(256), 0, s, h, npix, C, L.w_bwd, pbuf);
    });
    for (int pg : {256, 512, 768, 1024}) {
      char nm2[64];
      snprintf(nm2, sizeof(nm2), "proj limb engine grid %d", pg);
      timeit(nm2, act, [&] {
        hipLaunchKernelGGL(smallc_proj_x3_kernel, dim3(pg), dim3(256), 0, s, h, npix, L.w_bwd, pb2);
      });
    }
  }
  timeit("dgrad fp32 mask, fp32 out", 2 * act, [&] {
    smallc_dgrad(L, hcopy, B, delta, DAMC_ACT_LRELU, 0.2f, nullptr, nullptr, s);
  });
  timeit("dgrad fp32 mask, limb out", act * 2.5, [&] {
    smallc_dgrad(L, h, B, delta, DAMC_ACT_LRELU, 0.2f, h3, nullptr, s);
  });
  timeit("dgrad bit mask, limb out", act * 1.5 + act / 32, [&] {
    smallc_dgrad(L, h, B, delta, DAMC_ACT_LRELU, 0.2f, h3, bits, s);
  });
  // limb-output dgrad geometry sweep (rows per block R, pixels in flight per wave UNR) and the write floor
  timeit("write floor: hipMemset of the limb out", act * 1.5, [&] { CK(hipMemsetAsync(h3, 0, npix * C * 6, s)); });
  auto k3 = [&](int R, auto unr, auto pf) {
    constexpr int U = decltype(unr)::value;
    constexpr bool PFv = decltype(pf)::value;
    const dim3 grid((unsigned)((H + R - 1) / R), (unsigned)B);
    const size_t sm = sizeof(float) * (R + 2) * (H + 2) * 4;
    hipLaunchKernelGGL((smallc_dgrad_k3_kernel<3, U, PFv>), grid, dim3(256), sm, s, h, H, H, C, R, L.w_fwd, delta,
                       (int)DAMC_ACT_LRELU, 0.2f, h3, bits);
  };
  timeit("store probe: flat 16-B stores", act * 1.5, [&] {
    const long n16 = npix * C * 6 / 16;
    hipLaunchKernelGGL(store_flat_probe, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<uint4*>(h3), n16);
  });
  timeit("store probe: 16-pixel units, 768 blocks", act * 1.5, [&] {
    hipLaunchKernelGGL(store_unit_probe, dim3(768), dim3(256), 0, s, reinterpret_cast<unsigned char*>(h3),
                       (int)(npix / 16), C * 6);
  });
  timeit("store probe: 16-pixel units, 2048 blocks", act * 1.5, [&] {
    hipLaunchKernelGGL(store_unit_probe, dim3(2048), dim3(256), 0, s, reinterpret_cast<unsigned char*>(h3),
                       (int)(npix / 16), C * 6);
  });
  char nm[64];
  for (int R : {4, 8, 16}) {
    snprintf(nm, sizeof(nm), "k3 bits->limbs R=%d UNR=4", R);
    timeit(nm, act * 1.5 + act / 32, [&] { k3(R, std::integral_constant<int, 4>(), std::false_type()); });
    snprintf(nm, sizeof(nm), "k3 bits->limbs R=%d UNR=4 PF", R);
    timeit(nm, act * 1.5 + act / 32, [&] { k3(R, std::integral_constant<int, 4>(), std::true_type()); });
    snprintf(nm, sizeof(nm), "k3 bits->limbs R=%d UNR=2 PF", R);
    timeit(nm, act * 1.5 + act / 32, [&] { k3(R, std::integral_constant<int, 2>(), std::true_type()); });
  }
  // the limb-engine (MFMA) form vs the VALU form: same inputs, max |difference| relative to max |value| of the
  // decoded limbs
  {
    unsigned short* h3b;
    CK(hipMalloc(&h3b, npix * C * 6));
    CK(hipMemset(h3, 0, npix * C * 6));
    CK(hipMemset(h3b, 0, npix * C * 6));
    const dim3 grid((unsigned)(H / 8), (unsigned)B);
    hipLaunchKernelGGL((smallc_dgrad_k3_kernel<3, 4, true>), grid, dim3(256), sizeof(float) * 10 * (H + 2) * 4, s, h,
                       H, H, C, 8, L.w_fwd, delta, (int)DAMC_ACT_LRELU, 0.2f, h3, bits);
    CK((hipError_t)launch_smallc_dgrad_k3_mfma(L, B, delta, 0.2f, h3b, bits, s));
    CK(hipStreamSynchronize(s));
    std::vector<unsigned short> a((size_t)npix * C * 3), bb((size_t)npix * C * 3);
    CK(hipMemcpy(a.data(), h3, a.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(bb.data(), h3b, bb.size() * 2, hipMemcpyDeviceToHost));
    auto bf = [](unsigned short u) { unsigned v = (unsigned)u << 16; float f; memcpy(&f, &v, 4); return f; };
    double mx = 0, md = 0;
    for (size_t oc = 0; oc < (size_t)npix * C / 8; ++oc)
      for (int e = 0; e < 8; ++e) {
        const size_t base = oc * 24 + e;
        const double va = (double)bf(a[base]) + bf(a[base + 8]) + bf(a[base + 16]);
        const double vb = (double)bf(bb[base]) + bf(bb[base + 8]) + bf(bb[base + 16]);
        mx = std::max(mx, std::fabs(va));
        md = std::max(md, std::fabs(va - vb));
      }
    printf("mfma vs valu dgrad: max |diff| %.3e, max |value| %.3e (rel %.2e)\n", md, mx, md / mx);
    timeit("k3 bits->limbs MFMA", act * 1.5 + act / 32, [&] {
      CK((hipError_t)launch_smallc_dgrad_k3_mfma(L, B, delta, 0.2f, h3b, bits, s));
    });
    const int units = (int)(npix / 16);
    for (int pg : {256, 512, 1024, 2048})
      for (int pr : {0, 1, 2, 3}) {
        snprintf(nm, sizeof(nm), "k3 MFMA grid %d probe %d", pg, pr);
        timeit(nm, act * 1.5, [&] {
          hipLaunchKernelGGL((smallc_dgrad_k3_mfma_kernel<3, 4>), dim3(std::min(units, pg)), dim3(256), 0, s,
                             (int)npix, H, H, L.w_fwd, delta, 0.2f, h3b, bits, pr);
        });
      }
  }
  CK(hipGetLastError());
  return 0;
}
