// mfma_bias.hip — statistical bias of one v_mfma_f32_16x16x32_bf16 (C = 0 and C = random) on random
// bf16 operands: mean and rms of (mfma - exact) in units of 2^-24 * max|product| of the output's 32 products
// build: hipcc -O2 --offload-arch=gfx950 tools/mfma_bias.hip -o tools/mfma_bias
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// one MFMA per wave; A [trial][16][32], B [trial][32][16], C [trial][16][16] fp32 in/out
__global__ void k(const float* A, const float* B, float* C, int trials, float sg) {
  const int t = blockIdx.x;
  if (t >= trials) return;
  const int lane = threadIdx.x;
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    const int kk = 8 * (lane >> 4) + e;
    a[e] = (__bf16)(sg * A[(long)t * 512 + (lane & 15) * 32 + kk]);
    b[e] = (__bf16)B[(long)t * 512 + kk * 16 + (lane & 15)];
  }
  f32x4 c;
  for (int r = 0; r < 4; ++r) c[r] = sg * C[(long)t * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)];
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(long)t * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)] = sg * c[r];
}

// the same with v_mfma_f32_16x16x4_f32 (fp32 operands, 4 products): A [trial][16][4], B [trial][4][16]
__global__ void k4(const float* A, const float* B, float* C, int trials, float sg) {
  const int t = blockIdx.x;
  if (t >= trials) return;
  const int lane = threadIdx.x;
  const float a = sg * A[(long)t * 512 + (lane & 15) * 32 + (lane >> 4)];
  const float b = B[(long)t * 512 + (lane >> 4) * 16 + (lane & 15)];
  f32x4 c;
  for (int r = 0; r < 4; ++r) c[r] = sg * C[(long)t * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)];
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(long)t * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)] = sg * c[r];
}

static float bf(float x) {  // RNE to bf16
  unsigned u;
  memcpy(&u, &x, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  u &= 0xFFFF0000u;
  float y;
  memcpy(&y, &u, 4);
  return y;
}

int main() {
  const int trials = 4096;
  std::vector<float> A(trials * 512), B(trials * 512), C(trials * 256), C0;
  srand(1);
  auto nrm = [] { double u1 = (rand() + 1.0) / (RAND_MAX + 2.0), u2 = rand() / (RAND_MAX + 1.0);
                  return (float)(sqrt(-2 * log(u1)) * cos(6.283185307179586 * u2)); };
  for (auto& v : A) v = bf(nrm());
  for (auto& v : B) v = bf(nrm());
  float *dA, *dB, *dC;
  hipMalloc(&dA, A.size() * 4);
  hipMalloc(&dB, B.size() * 4);
  hipMalloc(&dC, C.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 12; ++mode) {
    const bool f32 = mode >= 6;
    const int kdep = f32 ? 4 : 32;
    if (mode == 6)
      for (auto& v : A) v = nrm();  // full fp32 operands for the fp32 MFMA
    const float sg = mode % 6 >= 3 ? -1.f : 1.f;
    srand(7 + mode % 3);
    for (auto& v : C) v = mode % 3 == 0 ? 0.f : (mode % 3 == 1 ? 8.f * nrm() : 0.01f * nrm());
    C0 = C;
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    if (mode == 6) hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    if (f32)
      hipLaunchKernelGGL(k4, dim3(trials), dim3(64), 0, 0, dA, dB, dC, trials, sg);
    else
      hipLaunchKernelGGL(k, dim3(trials), dim3(64), 0, 0, dA, dB, dC, trials, sg);
    hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
    double sum = 0, sq = 0, sgn = 0, sum_rne = 0, sq_rne = 0;
    long n = 0;
    for (int t = 0; t < trials; ++t)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double ex = C0[t * 256 + i * 16 + j], mx = fabs(ex);
          for (int kk = 0; kk < kdep; ++kk) {
            const double p = (double)A[t * 512 + i * 32 + kk] * B[t * 512 + kk * 16 + j];
            ex += p;
            mx = fmax(mx, fabs(p));
          }
          const double u = ldexp(mx, -24);
          const double e = (C[t * 256 + i * 16 + j] - ex) / u;
          const double er = ((double)(float)ex - ex) / u;
          sum += e;
          sq += e * e;
          sgn += (ex > 0 ? e : -e);
          sum_rne += er;
          sq_rne += er * er;
          ++n;
        }
    printf("%s %s C %-12s: mfma error mean %+.3f rms %.3f  (sign-relative mean %+.3f)   fp32-rne of exact: mean %+.3f rms %.3f"
           "   [units 2^-24 max|term|]\n", f32 ? "f32 16x16x4 " : "bf16 16x16x32", sg > 0 ? "+" : "-(-A B - C)", mode % 3 == 0 ? "= 0" : (mode % 3 == 1 ? "~ 8 N(0,1)" : "~ .01 N(0,1)"), sum / n,
           sqrt(sq / n), sgn / n, sum_rne / n, sqrt(sq_rne / n));
  }
  return 0;
}
