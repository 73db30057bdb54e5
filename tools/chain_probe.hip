// chain_probe.hip — per-block cost of the reverse sweep's chain kernel: each of the 7 block launches of step 0
// replayed 700 times from a graph (dependent launches, same buffers), with parts switched off (ChainArgs.dbg).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast-honor-pragmas -DDAMC_GEMM_NO_C_API \
//        tools/chain_probe.hip -o tools/chain_probe
#include <cstdio>
#include <vector>

#include "../diffusion-amortized-mcmc_amd/csrc/gemm.hip"
#include "../diffusion-amortized-mcmc_amd/csrc/denoiser.hip"

namespace damc_prof {
bool enabled() { return false; }
int begin(const char*, double, hipStream_t) { return -1; }
void end(int, hipStream_t) {}
}  // namespace damc_prof

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);               \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

static float* rnd(size_t n, unsigned seed, float scale) {
  std::vector<float> h(n);
  unsigned s = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = (((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f) * scale;
  }
  float* d = nullptr;
  if (hipMalloc(&d, n * 4) != hipSuccess) return nullptr;
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  return d;
}

int main(int argc, char** argv) {
  const int nz = 128, w = 128, nt = 128, nx = 1024, B = argc > 1 ? atoi(argv[1]) : 128, n = 100;
  damc_denoiser_t d{};
  d.nz = nz;
  d.ntemb = nt;
  d.nxemb = nx;
  d.residual = 1;
  const int din[7] = {2 * nz, w, 2 * w, 2 * w, 4 * w, 4 * w, 2 * w};
  const int dout[7] = {w, 2 * w, 2 * w, 2 * w, 2 * w, w, nz};
  unsigned seed = 1;
  d.bmat = rnd((size_t)nz * nz / 2, seed++, 1.f);
  d.tw1 = rnd((size_t)nt * nt, seed++, 0.08f);
  d.tb1 = rnd(nt, seed++, 0.08f);
  d.tw2 = rnd((size_t)nt * nt, seed++, 0.08f);
  d.tb2 = rnd(nt, seed++, 0.08f);
  for (int j = 0; j < 7; ++j) {
    damc_csq_block_t& b = d.blocks[j];
    b.din = din[j];
    b.dout = dout[j];
    const float si = 1.f / sqrtf((float)din[j]), so = 1.f / sqrtf((float)dout[j]);
    b.wl = rnd((size_t)dout[j] * din[j], seed++, si);
    b.bl = rnd(dout[j], seed++, si);
    b.ws = rnd((size_t)dout[j] * din[j], seed++, si);
    b.bs = rnd(dout[j], seed++, si);
    b.wg = rnd((size_t)dout[j] * dout[j], seed++, so);
    b.bg = rnd(dout[j], seed++, so);
    b.wb = rnd((size_t)dout[j] * dout[j], seed++, so);
    d.wctx[j] = rnd((size_t)dout[j] * (nt + nx), seed++, 0.03f);
    d.bctx[j] = rnd(dout[j], seed++, 0.03f);
  }
  float* xemb = rnd((size_t)B * nx, seed++, 1.f);
  float* zt = rnd((size_t)B * nz, seed++, 1.f);
  float* temb = rnd((size_t)n * nt, seed++, 1.f);
  std::vector<float> coef(6 * n);
  for (int k = 0; k < n; ++k) {
    float* c = &coef[6 * k];
    c[0] = 1.2f; c[1] = 0.7f; c[2] = 0.9f; c[3] = 0.1f; c[4] = 0.05f; c[5] = k == n - 1 ? 1.f : 0.f;
  }
  const size_t wsb = damc_sweep_workspace_bytes(&d, B, n);
  void* ws = nullptr;
  CK(hipMalloc(&ws, wsb));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int rc = damc_reverse_sweep(&d, xemb, zt, B, n, temb, coef.data(), 1, nullptr, 7, 0, nullptr, 0, ws, wsb, s);
  if (rc) { printf("sweep rc %d\n", rc); return 1; }
  CK(hipStreamSynchronize(s));
  SweepWs W;
  carve(&d, B, n, reinterpret_cast<char*>(ws), &W);
  std::vector<Launch> ls;
  chain_launches(&d, W, B, n, coef.data(), ls);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 700;
  auto time_graph = [&](const std::vector<Launch>& seq, float* us) -> int {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (const Launch& L : seq) launch_one(L, s);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    *us = 1e3f * ms / (3 * seq.size());
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
  };
  float us;
  if (time_graph(ls, &us)) return 1;
  printf("B=%d whole chain (7 x %d launches): %.2f us per launch = %.1f us per step\n", B, n, us, 7 * us);
  const int dbgs[] = {0, 3, 8, 31, 255, 255 + 256, 512};
  for (int j = 0; j < 7; ++j) {
    printf("block %d (din %d dout %d, %u WGs):", j, din[j], dout[j], ls[j].grid);
    for (int dbg : dbgs) {
      std::vector<Launch> seq(R, ls[j + 7 * (j == 6 ? 0 : 0)]);
      for (Launch& L : seq) L.a.dbg = dbg;
      if (time_graph(seq, &us)) return 1;
      printf("  dbg%d %.2f", dbg, us);
    }
    printf("  us\n");
  }
  return 0;
}
