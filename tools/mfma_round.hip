// mfma_round.hip — how v_mfma_f32_16x16x32_bf16 / v_mfma_f32_16x16x4_f32 round when the products' sum is added to
// the accumulator: C = 1.0 plus a product sum of +-f ulp(1.0) for several fractions f; prints the results in ulps of
// 1.0 next to round-to-nearest-even (tools/diag_chain.py: coherent dgrad errors)
// build: hipcc -O2 --offload-arch=gfx950 tools/mfma_round.hip -o tools/mfma_round
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* prod, int nf, float* out_bf, float* out_f32, float c0) {
  const int lane = threadIdx.x;
  for (int t = 0; t < nf; ++t) {
    // one product per MFMA in row 0 / col 0: A[0][0] = p (bf16-exact), B[0][0] = 1, all else 0
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) { a[e] = (__bf16)0.f; b[e] = (__bf16)0.f; }
    // 16x16x32 A fragment: lane = row (lane & 15), k octet = lane >> 4
    if (lane == 0) { a[0] = (__bf16)prod[t]; b[0] = (__bf16)1.f; }
    f32x4 c = {c0, c0, c0, c0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    if (lane == 0) out_bf[t] = c[0];
    float fa = lane == 0 ? prod[t] : 0.f, fb = lane == 0 ? 1.f : 0.f;
    f32x4 d = {c0, c0, c0, c0};
    d = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, d, 0, 0, 0);
    if (lane == 0) out_f32[t] = d[0];
  }
}

// 32 products in one MFMA: big (at k = 0) plus 31 copies of small, C = c0; row 0 / col 0
__global__ void k32(float big, const float* small, int nf, float* out, float c0) {
  const int lane = threadIdx.x;
  for (int t = 0; t < nf; ++t) {
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
      const int kk = 8 * (lane >> 4) + e;
      const bool r0 = (lane & 15) == 0;
      a[e] = (__bf16)(r0 ? (kk == 0 ? big : small[t]) : 0.f);
      b[e] = (__bf16)(r0 ? 1.f : 0.f);
    }
    f32x4 c = {c0, c0, c0, c0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    if (lane == 0) out[t] = c[0];
  }
}

int main() {
  const float ulp = std::ldexp(1.f, -23);
  const float fr[] = {0.25f, 0.5f, 0.75f, 1.5f, -0.25f, -0.5f, -0.75f, -1.5f, 0.125f, -0.125f};
  const int nf = sizeof(fr) / sizeof(fr[0]);
  float h[nf];
  for (int i = 0; i < nf; ++i) h[i] = fr[i] * ulp;
  float *dp, *db, *df;
  hipMalloc(&dp, sizeof h);
  hipMalloc(&db, sizeof h);
  hipMalloc(&df, sizeof h);
  hipMemcpy(dp, h, sizeof h, hipMemcpyHostToDevice);
  for (float c0 : {1.0f, -1.0f}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dp, nf, db, df, c0);
    float rb[nf], rf[nf];
    hipMemcpy(rb, db, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(rf, df, sizeof h, hipMemcpyDeviceToHost);
    for (int i = 0; i < nf; ++i) {
      const float rne = c0 + h[i];
      printf("C=%+.0f  product %+6.3f ulp:  bf16 mfma %+7.3f  f32 mfma %+7.3f  rne %+7.3f (ulps from C)\n", c0, fr[i],
             (rb[i] - c0) / ulp, (rf[i] - c0) / ulp, (rne - c0) / ulp);
    }
  }
  // small products in ulps of 1.0 (bf16-exact values)
  const float sf[] = {0.25f, 0.375f, -0.25f, -0.375f, 0.5f, -0.5f, 0.0625f, -0.0625f};
  const int ns = sizeof(sf) / sizeof(sf[0]);
  float hs[ns];
  for (int i = 0; i < ns; ++i) hs[i] = sf[i] * ulp;
  hipMemcpy(dp, hs, sizeof hs, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    const float big = mode == 0 ? 1.f : 0.f, c0 = mode == 0 ? 0.f : 1.f;
    hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, big, dp, ns, db, c0);
    float r[ns];
    hipMemcpy(r, db, sizeof hs, hipMemcpyDeviceToHost);
    for (int i = 0; i < ns; ++i) {
      const double exact = 1.0 + 31.0 * hs[i] + (mode == 1 ? hs[i] : 0.0);
      printf("%s + %s x %+7.4f ulp: mfma %+8.3f ulps, exact %+8.3f, rne %+8.3f\n", mode == 0 ? "product 1.0" : "C = 1.0",
             mode == 0 ? "31" : "32", sf[i], (r[i] - 1.f) / ulp, (exact - 1.0) / ulp, ((float)exact - 1.f) / ulp);
    }
  }
  return 0;
}
