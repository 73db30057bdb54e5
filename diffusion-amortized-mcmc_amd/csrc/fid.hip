// fid.hip — FID sufficient statistics on the device (workspace/src/MCMC.py:130-176, whose
// pfw.fid reduces Inception pool features to a mean and a covariance before the Frechet distance).
//
// A sample stream of n feature rows f (fp32, (n, d)) is reduced to s1 = sum f (d) and s2 = sum f f^T (d, d) in
// fp64, accumulated across calls; on multi-GPU runs the three tensors are summed over the ranks with one RCCL
// all_reduce (damc.fid), then damc_fid_mean_cov gives mu = s1 / n and sigma = (s2 - n mu mu^T) / (n - 1)
// (np.cov's unbiased estimate).  The Frechet distance itself needs sqrtm(sigma1 sigma2) of a 2048 x 2048
// non-symmetric product; like the reference (pytorch-fid's scipy.linalg.sqrtm) it runs on the host.
//
// s2 kernel: one 64 x 64 tile of s2 per workgroup (only tiles on or above the diagonal; the mirror tile is
// written from the same registers), 256 threads each owning 4 x 4 outputs, the 32-row slices of both column
// panels staged in LDS as fp64.  Work per 2048-wide call: d^2 n FMA, i.e. 4.2 GFLOP fp64 for n = 500.
#include "common.h"

namespace {

constexpr int FT = 64;   // tile edge
constexpr int FR = 32;   // rows per LDS slice

__global__ __launch_bounds__(256) void fid_s2_kernel(const float* __restrict__ f, int n, int d, double* __restrict__ s2) {
  // upper-triangular tile index -> (ti, tj), ti <= tj
  const int nt = (d + FT - 1) / FT;
  int t = blockIdx.x, ti = 0;
  while (t >= nt - ti) {
    t -= nt - ti;
    ++ti;
  }
  const int tj = ti + t;
  const int i0 = ti * FT, j0 = tj * FT;
  __shared__ double a[FR][FT + 1];
  __shared__ double b[FR][FT + 1];
  const int tid = threadIdx.x;
  const int ty = tid >> 4, tx = tid & 15;  // outputs rows i0 + 4 ty + {0..3}, cols j0 + 4 tx + {0..3}
  double acc[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0;
  for (int r0 = 0; r0 < n; r0 += FR) {
    for (int e = tid; e < FR * FT; e += 256) {
      const int r = e / FT, c = e - r * FT;
      const bool rok = r0 + r < n;
      a[r][c] = (rok && i0 + c < d) ? (double)f[(long)(r0 + r) * d + i0 + c] : 0.0;
      b[r][c] = (rok && j0 + c < d) ? (double)f[(long)(r0 + r) * d + j0 + c] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < FR; ++r) {
      double av[4], bv[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) av[p] = a[r][4 * ty + p];
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[q] = b[r][4 * tx + q];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][q] = fma(av[p], bv[q], acc[p][q]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = i0 + 4 * ty + p, j = j0 + 4 * tx + q;
      if (i < d && j < d) {
        s2[(long)i * d + j] += acc[p][q];
        if (ti != tj) s2[(long)j * d + i] += acc[p][q];  // mirror tile (never overlaps another block's)
      }
    }
}

__global__ void fid_s1_kernel(const float* __restrict__ f, int n, int d, double* __restrict__ s1) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d) return;
  double acc = 0.0;
  for (int r = 0; r < n; ++r) acc += (double)f[(long)r * d + j];  // row order: deterministic
  s1[j] += acc;
}

__global__ void fid_mean_cov_kernel(const double* __restrict__ s1, const double* __restrict__ s2, double n, int d,
                                    double* __restrict__ mu, double* __restrict__ sigma) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)d * d) return;
  const int i = (int)(idx / d), j = (int)(idx - (long)i * d);
  // the product in (min, max) index order, so sigma is exactly symmetric like s2
  const double a = s1[min(i, j)] / n, b = s1[max(i, j)] / n;
  sigma[idx] = (s2[idx] - n * a * b) / (n - 1.0);
  if (j == 0) mu[i] = s1[i] / n;
}

}  // namespace

extern "C" int damc_fid_accumulate(const float* feats, int n, int d, double* s1, double* s2, void* stream) {
  if (!feats || !s1 || !s2 || n < 0 || d <= 0) return DAMC_ERR_ARG;
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int nt = (d + FT - 1) / FT;
  hipLaunchKernelGGL(fid_s2_kernel, dim3(nt * (nt + 1) / 2), dim3(256), 0, s, feats, n, d, s2);
  hipLaunchKernelGGL(fid_s1_kernel, dim3((d + 255) / 256), dim3(256), 0, s, feats, n, d, s1);
  return (int)hipGetLastError();
}

extern "C" int damc_fid_mean_cov(const double* s1, const double* s2, double n, int d, double* mu, double* sigma,
                                 void* stream) {
  if (!s1 || !s2 || !mu || !sigma || d <= 0 || !(n > 1.0)) return DAMC_ERR_ARG;
  const long dd = (long)d * d;
  hipLaunchKernelGGL(fid_mean_cov_kernel, dim3((unsigned)((dd + 255) / 256)), dim3(256), 0, as_stream(stream), s1, s2,
                     n, d, mu, sigma);
  return (int)hipGetLastError();
}
