// gemm_bench.hip — A/B the implicit-GEMM tile configurations on the four CIFAR-10 B=128 generator
// convolutions (upconv fwd L2/L3, upconv dgrad L3/L2), interleaved in one process (guide §5.4 r24).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DDAMC_GEMM_NO_C_API tools/gemm_bench.hip -o gemm_bench
#ifndef KMCHK
#define KMCHK 0
#endif
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../diffusion-amortized-mcmc_amd/csrc/gemm.hip"

namespace damc_prof {
bool enabled() { return false; }
int begin(const char*, double, hipStream_t) { return -1; }
void end(int, hipStream_t) {}
}  // namespace damc_prof

using namespace damc;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                             \
    }                                                                      \
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

struct Proj {
  const char* name;
  GemmArgs a;
  int zdim;
  double flops;
};

struct Shape {
  const char* name;
  GemmArgs a;
  bool phase;
  double flops;
  float* bt;  // weights transposed per phase to [n][k] for the K-major engine
  unsigned short* a3 = nullptr;  // limb-engine operands (x3 layout)
  unsigned short* b3 = nullptr;
  unsigned short* b3n = nullptr;  // the same with odd X3_NEGK-blocks negated (GemmArgs::b_negblk)
  unsigned short* b3c = nullptr;  // slice-major (channel-major K walk, V & 8) with sign blocks
};

static unsigned short* split_dev(const float* d, size_t n) {
  unsigned short* y;
  CK(hipMalloc(&y, n * 6));
  if (launch_split_x3(d, (long)n, y, 0) != 0) {
    printf("split failed\n");
    exit(1);
  }
  CK(hipDeviceSynchronize());
  return y;
}

template <int V, int NEG = 0>
static void run_x3(const Shape& sh, hipStream_t s) {
  GemmArgs a = sh.a;
  a.A3 = sh.a3;
  a.B3 = (V & 8) ? sh.b3c : (NEG ? sh.b3n : sh.b3);
  a.b_negblk = (V & 8) ? 1 : NEG;
  a.b_zstride = (long)a.N * a.K;
  if (sh.phase)
    launch_x3_t<EPI_BIAS_ACT, O_PHASE, V>(a, 4, s);
  else
    launch_x3_t<EPI_MASK, O_DENSE, V>(a, 1, s);
}

static std::vector<float> to_host(const float* d, size_t n) {
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
  return h;
}

// fp64 reference of sampled outputs; returns {max, mean} of |c - ref| / (sum_k |a b| + |bias|)
static void ref_check(const Shape& sh, int B, const std::vector<float>& hA, const std::vector<float>& hB,
                      const std::vector<float>& hbias, const std::vector<float>& hmask, const std::vector<float>& hc,
                      double* emax, double* emean, double* ebias) {
  const GemmArgs& a = sh.a;
  const int hwq = a.Hq * a.Wq;
  unsigned st = 12345;
  double mx = 0, sm = 0, sb = 0;
  const int NS = 384;
  for (int t = 0; t < NS; ++t) {
    st = st * 1664525u + 1013904223u;
    const int m = (int)((st >> 4) % (unsigned)a.M);
    st = st * 1664525u + 1013904223u;
    const int n = (int)((st >> 4) % (unsigned)a.N);
    st = st * 1664525u + 1013904223u;
    const int z = sh.phase ? (int)((st >> 4) % 4u) : 0;
    const int py = z >> 1, px = z & 1;
    const int pdy = sh.phase ? 1 - py : a.pad_y, pdx = sh.phase ? 1 - px : a.pad_x;
    const int b = m / hwq, r = m % hwq, qy = r / a.Wq, qx = r % a.Wq;
    double sum = 0, asum = 0;
    for (int k = 0; k < a.K; ++k) {
      const int tap = k / a.Cg, ci = k % a.Cg, ky = tap / a.kw, kx = tap % a.kw;
      const int iy = qy * a.stride - pdy + ky, ix = qx * a.stride - pdx + kx;
      if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
      const double av = hA[((size_t)(b * a.Hin + iy) * a.Win + ix) * a.Cg + ci];
      const double bv = hB[(size_t)z * a.K * a.N + (size_t)k * a.N + n];
      sum += av * bv;
      asum += std::fabs(av * bv);
    }
    size_t idx;
    double v;
    if (sh.phase) {
      idx = (((size_t)b * a.Hout + 2 * qy + py) * a.Wout + 2 * qx + px) * a.ldc + n;
      v = sum + hbias[n % a.bias_mod];
      asum += std::fabs((double)hbias[n % a.bias_mod]);
      v = v > 0 ? v : 0.2 * v;
    } else {
      idx = (size_t)m * a.ldc + n;
      v = sum * (hmask[idx] > 0.f ? 1.0 : 0.2);
    }
    const double e = std::fabs(hc[idx] - v) / asum;
    mx = std::max(mx, e);
    sm += e;
    sb += (hc[idx] - v) / asum;
  }
  (void)B;
  *emax = mx;
  *emean = sm / NS;
  *ebias = sb / NS;
}

// per-phase transpose of B[K][N] (ldb = N) into Bt[N][K]
static float* transpose_b(const float* dB, int nz, int K, int N) {
  std::vector<float> h((size_t)nz * K * N), t((size_t)nz * K * N);
  CK(hipMemcpy(h.data(), dB, h.size() * 4, hipMemcpyDeviceToHost));
  for (int z = 0; z < nz; ++z)
    for (int k = 0; k < K; ++k)
      for (int n = 0; n < N; ++n) t[((size_t)z * N + n) * K + k] = h[((size_t)z * K + k) * N + n];
  float* d;
  CK(hipMalloc(&d, t.size() * 4));
  CK(hipMemcpy(d, t.data(), t.size() * 4, hipMemcpyHostToDevice));
  return d;
}

template <int PIPE, int DBG = 0>
void run_km(const Shape& sh, hipStream_t s) {
  static_assert(PIPE >= 0 && PIPE <= 5, "pipe");
  GemmArgs a = sh.a;
  a.B = sh.bt;
  a.b_kmajor = 1;
  a.ldb = a.K;
  a.b_zstride = (long)a.N * a.K;
  if (sh.phase)
    launch_km_t<EPI_BIAS_ACT, O_PHASE, PIPE, DBG>(a, 4, s);
  else
    launch_km_t<EPI_MASK, O_DENSE, PIPE, DBG>(a, 1, s);
}

template <int BK, int OCC, int MT, int SCHED>
void run(const Shape& sh, hipStream_t s) {
  if (sh.phase)
    launch_t<A_CONV, EPI_BIAS_ACT, O_PHASE, true, BK, OCC, MT, SCHED>(sh.a, 4, s);
  else
    launch_t<A_CONV, EPI_MASK, O_DENSE, true, BK, OCC, MT, SCHED>(sh.a, 1, s);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 128;
  const int ngf = 128;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  // activations (NHWC) and packed weights for the CIFAR generator
  float* h1 = rnd((size_t)B * 8 * 8 * 8 * ngf, 1);
  float* h2 = rnd((size_t)B * 16 * 16 * 4 * ngf, 2);
  float* h3 = rnd((size_t)B * 32 * 32 * 2 * ngf, 3);
  float* d3 = rnd((size_t)B * 32 * 32 * 2 * ngf, 4);
  float* d2 = rnd((size_t)B * 16 * 16 * 4 * ngf, 5);
  float* w2 = rnd((size_t)16 * 8 * ngf * 4 * ngf, 6);
  float* w3 = rnd((size_t)16 * 4 * ngf * 2 * ngf, 7);
  float* o1 = rnd((size_t)B * 8 * 8 * 8 * ngf, 8);
  float* o2 = rnd((size_t)B * 16 * 16 * 4 * ngf, 9);
  float* o3 = rnd((size_t)B * 32 * 32 * 2 * ngf, 10);
  float* bias = rnd(1024, 11);
  std::vector<Shape> shapes;
  std::vector<Proj> projs;
  auto up = [&](const char* nm, float* in, int H, int cin, int cout, float* w, float* out) {
    GemmArgs a;
    a.A = in; a.Hin = H; a.Win = H; a.Cg = cin; a.Hq = H; a.Wq = H; a.kw = 2; a.stride = 1;
    a.B = w; a.ldb = cout; a.b_zstride = 4L * cin * cout; a.C = out; a.ldc = cout;
    a.M = B * H * H; a.N = cout; a.K = 4 * cin; a.Hout = 2 * H; a.Wout = 2 * H;
    a.bias = bias; a.bias_mod = cout; a.act = DAMC_ACT_LRELU; a.slope = 0.2f;
    shapes.push_back({nm, a, true, 2.0 * B * 4 * H * H * (double)cout * 4 * cin, transpose_b(w, 4, 4 * cin, cout)});
  };
  auto dg = [&](const char* nm, float* din, int Hout, int cout, int cin, float* w, float* out) {
    GemmArgs a;
    a.A = din; a.Hin = Hout; a.Win = Hout; a.Cg = cout; a.Hq = Hout / 2; a.Wq = Hout / 2; a.kw = 4; a.stride = 2;
    a.pad_y = 1; a.pad_x = 1; a.B = w; a.ldb = cin; a.C = out; a.ldc = cin;
    a.M = B * (Hout / 2) * (Hout / 2); a.N = cin; a.K = 16 * cout; a.k_per_z = a.K;
    a.mask = out; a.mask_act = DAMC_ACT_LRELU; a.mask_slope = 0.2f;
    shapes.push_back({nm, a, false, 2.0 * a.M * (double)a.N * a.K, transpose_b(w, 1, a.K, a.N)});
  };
  // PROJ (first layer, 1x1 input): fwd M=B, N=8*8*8ngf, K=nz=128 ; dgrad split-K 256 slices of 256
  const int nz = 128, NP = 8 * 8 * 8 * ngf;
  float* zin = rnd((size_t)B * nz, 12);
  float* wpf = rnd((size_t)NP * nz, 13);
  {
    GemmArgs a;
    a.A = zin; a.Cg = nz; a.B = wpf; a.ldb = nz; a.C = o1; a.ldc = NP; a.M = B; a.N = NP; a.K = nz; a.k_per_z = nz;
    a.bias = bias; a.bias_mod = 8 * ngf; a.act = DAMC_ACT_LRELU; a.slope = 0.2f;
    projs.push_back({"proj fwd 128x65536x128", a, 1, 2.0 * B * (double)NP * nz});
    GemmArgs d;
    d.A = o1; d.Cg = NP; d.B = wpf; d.ldb = NP; d.C = h2; d.ldc = nz; d.c_zstride = (long)B * nz; d.M = B; d.N = nz;
    d.K = NP; d.k_per_z = 256;
    projs.push_back({"proj dgrad 128x128x65536/256", d, NP / 256, 2.0 * B * (double)NP * nz});
  }
  up("L2 fwd  8->16 1024->512", h1, 8, 8 * ngf, 4 * ngf, w2, o2);
  up("L3 fwd 16->32  512->256", h2, 16, 4 * ngf, 2 * ngf, w3, o3);
  dg("L3 dgrad 32->16 256->512", d3, 32, 2 * ngf, 4 * ngf, w3, o2);
  dg("L2 dgrad 16->8  512->1024", d2, 16, 4 * ngf, 8 * ngf, w2, o1);

  typedef void (*RunFn)(const Shape&, hipStream_t);
  struct V { const char* name; RunFn fn; };
  for (Shape& sh : shapes) {
    const GemmArgs& a = sh.a;
    const size_t na = (size_t)(a.M / (a.Hq * a.Wq)) * a.Hin * a.Win * a.Cg;
    sh.a3 = split_dev(a.A, na);
    sh.b3 = split_dev(sh.bt, (size_t)(sh.phase ? 4 : 1) * a.N * a.K);
    const size_t nb = (size_t)(sh.phase ? 4 : 1) * a.N * a.K;
    CK(hipMalloc(&sh.b3n, nb * 6));
    CK(hipMalloc(&sh.b3c, nb * 6));
    if (launch_split_x3_cmaj(sh.bt, (long)nb, a.K, a.Cg, 32, sh.b3c, 0) != 0) {
      printf("split failed\n");
      exit(1);
    }
    if (launch_split_x3_negblk(sh.bt, (long)nb, a.K, sh.b3n, 0) != 0) {
      printf("split failed\n");
      exit(1);
    }
    CK(hipDeviceSynchronize());
  }
  // "eq" mode: bitwise equality of the F32A kernel against the default, unsplit and split-K (register slabs), with the
  // library's epilogue operands (sign-bit mask for the dgrads, sign-bit output for the forwards, limb copy of C)
  if (argc > 2 && !strcmp(argv[2], "eq")) {
    float* slab;
    const long slabn = 1L << 28;
    CK(hipMalloc(&slab, slabn * 4));
    for (size_t si = 0; si < shapes.size(); ++si) {
      const Shape& sh = shapes[si];
      const GemmArgs& a0 = sh.a;
      const size_t nout = sh.phase ? (size_t)B * a0.Hout * a0.Wout * a0.ldc : (size_t)a0.M * a0.ldc;
      float* mk = rnd(nout, 99);
      std::vector<float> hm = to_host(mk, nout);
      std::vector<unsigned char> bits(nout / 8, 0);
      for (size_t i = 0; i < nout; ++i)
        if (hm[i] > 0.f) bits[i / 8] |= (unsigned char)(1u << (i % 8));
      unsigned char* dbits;
      CK(hipMalloc(&dbits, nout / 8));
      CK(hipMemcpy(dbits, bits.data(), nout / 8, hipMemcpyHostToDevice));
      std::vector<float> outs[6];
      std::vector<unsigned char> sgns[6];
      for (int v = 0; v < 6; ++v) {
        const bool f32a = (v & 1) || v >= 4, split = (v & 2) || v >= 4;
        unsetenv("DAMC_X3_KSPLIT_BPW");
        unsetenv("DAMC_X3_KSLAB_REG");
        if (v == 4) setenv("DAMC_X3_KSPLIT_BPW", "1", 1);
        if (v == 5) setenv("DAMC_X3_KSLAB_REG", "0", 1);
        GemmArgs a = a0;
        float* c;
        unsigned char* sg;
        CK(hipMalloc(&c, nout * 4));
        CK(hipMalloc(&sg, nout / 8));
        CK(hipMemset(c, 0, nout * 4));
        CK(hipMemset(sg, 0, nout / 8));
        a.C = c;
        a.A3 = sh.a3;
        a.B3 = sh.b3n;
        a.b_negblk = 1;
        a.b_zstride = (long)a.N * a.K;
        a.a_f32 = f32a;
        if (split) {
          a.kslab = slab;
          a.kslab_floats = slabn;
        }
        if (sh.phase) {
          a.sgn = sg;
          if (f32a) launch_x3_t<EPI_BIAS_ACT, O_PHASE, 261 | X3_F32A>(a, 4, s);
          else launch_x3_t<EPI_BIAS_ACT, O_PHASE, 261>(a, 4, s);
        } else {
          a.mask = nullptr;
          a.mask_sgn = dbits;
          if (f32a) launch_x3_t<EPI_MASK, O_DENSE, 261 | X3_F32A>(a, 1, s);
          else launch_x3_t<EPI_MASK, O_DENSE, 261>(a, 1, s);
        }
        CK(hipStreamSynchronize(s));
        outs[v] = to_host(c, nout);
        sgns[v].resize(nout / 8);
        CK(hipMemcpy(sgns[v].data(), sg, nout / 8, hipMemcpyDeviceToHost));
        CK(hipFree(c));
        CK(hipFree(sg));
      }
      printf("eq B=%d %-28s", B, sh.name);
      const char* nm[6] = {"v261", "f32a", "v261 split", "f32a split", "f32a split bpw1", "f32a split rowmajor"};
      for (int v = 1; v < 6; ++v) {
        size_t nd = 0, first = (size_t)-1;
        for (size_t i = 0; i < nout; ++i)
          if (memcmp(&outs[v][i], &outs[0][i], 4)) {
            if (first == (size_t)-1) first = i;
            ++nd;
          }
        printf("  [%s: %zu differ%s%s]", nm[v], nd, sh.phase && memcmp(sgns[v].data(), sgns[0].data(), nout / 8) ? ", sign bits differ" : "",
               nd ? "" : "");
        if (nd) printf(" (first %zu: %.9g vs %.9g)", first, outs[v][first], outs[0][first]);
        if (nd && v == 3 && !sh.phase) {  // dgrad (O_DENSE, row = m): differing count per (wave_d, ij) of the 256x128 tile
          std::vector<int> h(8 * 16, 0);
          for (size_t i = 0; i < nout; ++i)
            if (memcmp(&outs[v][i], &outs[0][i], 4)) {
              const int m = (int)(i / a0.ldc) % 256, n = (int)(i % a0.ldc) % 128;
              h[((m / 64) * 2 + n / 64) * 16 + ((m % 64) / 16) * 4 + (n % 64) / 16]++;
            }
          printf("\n   per (wave_d, ij):");
          for (int k = 0; k < 128; ++k)
            if (h[k]) printf(" %d/%d:%d", k / 16, k % 16, h[k]);
          printf("\n");
        }
      }
      printf("\n");
      CK(hipFree(mk));
      CK(hipFree(dbits));
    }
    return 0;
  }
  // timing probes beside the default: 512 = no DMA after the first tile, 1024 = fragment reads of the first tile only,
  // 4096 = DMA from one L2-hot 64 KB window
  V vars[] = {{"v261", run_x3<261, 1>}, {"f32a", run_x3<261 | X3_F32A, 1>}, {"wide", run_x3<261 | 524288, 1>}};
  const int NV = sizeof(vars) / sizeof(vars[0]);
  // accuracy against an fp64 reference on sampled outputs (normalised by sum |a b|)
  {
    std::vector<float> hbias = to_host(bias, 1024);
    for (size_t si = 0; si < shapes.size(); ++si) {
      const Shape& sh = shapes[si];
      const GemmArgs& a0 = sh.a;
      const size_t na = (size_t)(a0.M / (a0.Hq * a0.Wq)) * a0.Hin * a0.Win * a0.Cg;
      const size_t nout = sh.phase ? (size_t)B * a0.Hout * a0.Wout * a0.ldc : (size_t)a0.M * a0.ldc;
      std::vector<float> hA = to_host(a0.A, na), hB = to_host(a0.B, (size_t)(sh.phase ? 4 : 1) * a0.K * a0.N);
      float *c, *mk = rnd(nout, 99);
      CK(hipMalloc(&c, nout * 4));
      std::vector<float> hmask = to_host(mk, nout);
      printf("accuracy %-28s", sh.name);
      std::vector<float> h0;
      for (int v = 0; v < NV; ++v) {
        Shape s2 = sh;
        s2.a.C = c;
        s2.a.mask = mk;
        CK(hipMemset(c, 0, nout * 4));
        vars[v].fn(s2, s);
        CK(hipStreamSynchronize(s));
        std::vector<float> hc = to_host(c, nout);
        if (v == 0) h0 = hc;
        else printf("  [%s bitwise v0: %s]", vars[v].name, memcmp(h0.data(), hc.data(), nout * 4) ? "NO" : "yes");
        double emax, emean, ebias;
        ref_check(sh, B, hA, hB, hbias, hmask, hc, &emax, &emean, &ebias);
        printf("  %s max %.2e mean %.2e bias %+.1e", vars[v].name, emax, emean, ebias);
      }
      printf("   (|c - fp64| / sum|ab|)\n");
      CK(hipFree(c));
      CK(hipFree(mk));
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int rounds = 5, reps = 10;
  std::vector<std::vector<float>> best(shapes.size(), std::vector<float>(NV, 1e30f));
  for (int r = 0; r < rounds; ++r)
    for (size_t si = 0; si < shapes.size(); ++si)
      for (int v = 0; v < NV; ++v) {
        vars[v].fn(shapes[si], s);  // warm
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < reps; ++k) vars[v].fn(shapes[si], s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        if (ms < best[si][v]) best[si][v] = ms;
      }
  CK(hipGetLastError());
  // sustained load (the bench's regime: the chip lowers its clock under minutes of MFMA work, MI355X_MICROARCH.md
  // DVFS give-back): per shape, variants alternate in blocks of 100 back-to-back launches, 6 blocks each after 100
  // warm-up launches; mean of the variant's blocks
  std::vector<std::vector<double>> sus(shapes.size(), std::vector<double>(NV, 0.0));
  for (size_t si = 0; si < shapes.size(); ++si) {
    for (int k = 0; k < 100; ++k) vars[0].fn(shapes[si], s);
    for (int blk = 0; blk < 6; ++blk)
      for (int v = 0; v < NV; ++v) {
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < 100; ++k) vars[v].fn(shapes[si], s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        sus[si][v] += ms / 100 / 6;
      }
  }
  printf("B=%d  sustained (6 x 100 launches, alternating) mean ms\n", B);
  for (size_t si = 0; si < shapes.size(); ++si) {
    printf("%-28s", shapes[si].name);
    for (int v = 0; v < NV; ++v)
      printf("  %s %.3f (%.1f)", vars[v].name, sus[si][v], shapes[si].flops / (sus[si][v] * 1e-3) / 1e12);
    printf("\n");
  }
  printf("B=%d  best-of-%d ms (TFLOP/s)\n", B, rounds);
  for (size_t si = 0; si < shapes.size(); ++si) {
    printf("%-28s", shapes[si].name);
    for (int v = 0; v < NV; ++v)
      printf("  %s %.3f (%.1f)", vars[v].name, best[si][v], shapes[si].flops / (best[si][v] * 1e-3) / 1e12);
    printf("\n");
  }
  // the first layer on the limb engine as the library runs it (z limbs . W limbs as a 1x1 conv, bias + LReLU, fp32 +
  // limb outputs, sign bits), both block layouts
  {
    GemmArgs a;
    a.A = zin; a.Cg = nz; a.Hin = a.Win = a.Hq = a.Wq = 1; a.kw = 1; a.stride = 1;
    a.A3 = split_dev(zin, (size_t)B * nz);
    a.B3 = split_dev(wpf, (size_t)NP * nz);
    a.b_negblk = 1;
    a.C = o1; a.ldc = NP; a.M = B; a.N = NP; a.K = nz; a.k_per_z = nz;
    a.bias = bias; a.bias_mod = 8 * ngf; a.act = DAMC_ACT_LRELU; a.slope = 0.2f;
    CK(hipMalloc(&a.C3, (size_t)B * NP * 6));
    CK(hipMalloc(&a.sgn, (size_t)B * NP / 8));
    float* c2;
    CK(hipMalloc(&c2, (size_t)B * NP * 4));
    GemmArgs a2 = a;
    a2.C = c2;
    launch_x3_t<EPI_BIAS_ACT, O_DENSE, 261>(a, 1, s);
    launch_x3_t<EPI_BIAS_ACT, O_DENSE, 261 | 524288>(a2, 1, s);
    CK(hipStreamSynchronize(s));
    std::vector<float> r1 = to_host(o1, (size_t)B * NP), r2 = to_host(c2, (size_t)B * NP);
    printf("proj fwd x3: wide bitwise default: %s\n", memcmp(r1.data(), r2.data(), r1.size() * 4) ? "NO" : "yes");
    float b1 = 1e30f, b2 = 1e30f;
    for (int r = 0; r < rounds; ++r) {
      for (int v = 0; v < 2; ++v) {
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < reps; ++k) {
          if (v == 0) launch_x3_t<EPI_BIAS_ACT, O_DENSE, 261>(a, 1, s);
          else launch_x3_t<EPI_BIAS_ACT, O_DENSE, 261 | 524288>(a, 1, s);
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (v == 0 ? b1 : b2) = std::min(v == 0 ? b1 : b2, ms / reps);
      }
    }
    printf("proj fwd x3 128x65536x128      v261 %.4f ms  wide %.4f ms\n", b1, b2);
  }
  for (const Proj& pr : projs) {
    float best = 1e30f;
    for (int r = 0; r < rounds; ++r) {
      if (pr.zdim == 1) launch_km_t<EPI_BIAS_ACT, O_DENSE>(pr.a, 1, s);
      else launch_km_t<EPI_STORE, O_DENSE>(pr.a, pr.zdim, s);
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < reps; ++k) {
        if (pr.zdim == 1) launch_km_t<EPI_BIAS_ACT, O_DENSE>(pr.a, 1, s);
        else launch_km_t<EPI_STORE, O_DENSE>(pr.a, pr.zdim, s);
      }
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms / reps);
    }
    printf("%-28s  KM/p3 %.4f ms (%.1f TFLOP/s)\n", pr.name, best, pr.flops / (best * 1e-3) / 1e12);
  }
  return 0;
}
