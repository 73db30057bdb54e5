// encoder.hip — the amortizer's image encoder Encoder_* (workspace/src/diffusion_net.py:227-413):
// [Conv2d -> InstanceNorm2d(affine, eps=1e-5) -> LeakyReLU(0.2)]* -> Conv2d, on NHWC activations.
// Convolutions run on the fp32 MFMA implicit-GEMM engine (gemm.hip); InstanceNorm statistics are
// per (sample, channel) Welford partials merged with Chan's formula (wave shuffles + LDS), then
// one fused normalise + affine + LeakyReLU pass in place.
#include <algorithm>

#include "gemm.h"
#include "wgrad.h"

namespace {

// (Cout,Cin,k,k) -> [(ky,kx,ci)][co], or [co][(ky,kx,ci)] for the K-major engine (km)
__global__ void pack_conv_kernel(const float* w, int cout, int cin, int k, int km, float* wp) {
  const long n = (long)cout * cin * k * k;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  long t = i;
  const int kx = (int)(t % k);
  t /= k;
  const int ky = (int)(t % k);
  t /= k;
  const int ci = (int)(t % cin);
  const int co = (int)(t / cin);
  const long kk = ((long)ky * k + kx) * cin + ci;
  if (km)
    wp[(long)co * k * k * cin + kk] = w[i];
  else
    wp[kk * cout + co] = w[i];
}

__global__ void nchw_to_nhwc_kernel(const float* x, int B, int C, int HW, float* y) {
  const long n = (long)B * C * HW;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // i enumerates the NHWC output
  const int c = (int)(i % C);
  const long t = i / C;
  const int p = (int)(t % HW);
  const int b = (int)(t / HW);
  y[i] = x[((long)b * C + c) * HW + p];
}

struct Wf {
  float n, mean, m2;
};
__device__ __forceinline__ Wf wmerge(Wf a, Wf b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float d = b.mean - a.mean;
  const float fb = b.n / n;
  Wf r;
  r.n = n;
  r.mean = a.mean + d * fb;
  r.m2 = a.m2 + b.m2 + d * d * a.n * fb;
  return r;
}

// grid: (B * ceil(C/64), S); block 256 = 64 channels x 4 pixel lanes
__global__ __launch_bounds__(256) void in_stats_kernel(const float* y, int B, int HW, int C, int S, float* part) {
  const int cg = (C + 63) / 64;
  const int b = blockIdx.x / cg, c = (blockIdx.x % cg) * 64 + (threadIdx.x & 63);
  const int prow = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const int p0 = (int)((long)HW * s / S), p1 = (int)((long)HW * (s + 1) / S);
  Wf w{0.f, 0.f, 0.f};
  if (c < C) {
    for (int p = p0 + prow; p < p1; p += 4) {
      const float v = y[((long)b * HW + p) * C + c];
      w.n += 1.f;
      const float d = v - w.mean;
      w.mean += d / w.n;
      w.m2 += d * (v - w.mean);
    }
  }
  __shared__ Wf red[4][64];
  red[prow][threadIdx.x & 63] = w;
  __syncthreads();
  if (prow == 0 && c < C) {
    Wf a = red[0][threadIdx.x];
    for (int r = 1; r < 4; ++r) a = wmerge(a, red[r][threadIdx.x]);
    float* o = part + (((long)b * C + c) * S + s) * 3;
    o[0] = a.n;
    o[1] = a.mean;
    o[2] = a.m2;
  }
}

// grid: (B * ceil(C/64), P); merges the S partials of its 64 channels, then normalises its pixels
__global__ __launch_bounds__(256) void in_apply_kernel(float* y, int B, int HW, int C, int S, const float* part,
                                                       const float* gamma, const float* beta, float eps, float slope) {
  const int cg = (C + 63) / 64;
  const int b = blockIdx.x / cg, c = (blockIdx.x % cg) * 64 + (threadIdx.x & 63);
  const int prow = threadIdx.x >> 6;
  __shared__ float sc[64], sh[64];
  if (prow == 0) {
    float scale = 0.f, shift = 0.f;
    if (c < C) {
      const float* pp = part + ((long)b * C + c) * S * 3;
      Wf a{pp[0], pp[1], pp[2]};
      for (int s = 1; s < S; ++s) a = wmerge(a, Wf{pp[3 * s], pp[3 * s + 1], pp[3 * s + 2]});
      const float var = a.m2 / a.n;  // biased, as InstanceNorm2d
      const float rstd = 1.f / sqrtf(var + eps);
      scale = rstd * gamma[c];
      shift = beta[c] - a.mean * scale;
    }
    sc[threadIdx.x] = scale;
    sh[threadIdx.x] = shift;
  }
  __syncthreads();
  if (c >= C) return;
  const float scl = sc[threadIdx.x & 63], shf = sh[threadIdx.x & 63];
  const int P = gridDim.y;
  const int p0 = (int)((long)HW * blockIdx.y / P), p1 = (int)((long)HW * (blockIdx.y + 1) / P);
  for (int p = p0 + prow; p < p1; p += 4) {
    float* q = y + ((long)b * HW + p) * C + c;
    const float v = fmaf(*q, scl, shf);
    *q = v > 0.f ? v : v * slope;
  }
}

// pixel splits of the statistics pass: <= 64 pixels per split (the Welford chain of a thread is serial),
// merged with Chan's formula
int in_splits(int hw) {
  int s = hw / 64;
  return s < 1 ? 1 : (s > 64 ? 64 : s);
}

// split-K slices for a K-major conv whose output tiles would not fill the chip (the encoder's deeper
// layers: 64 / 8 tiles at B=128), each slice >= 8 K tiles; 1 = no split
int conv_split(long M, int N, int K) {
  const long tiles = ((M + 127) / 128) * ((N + 127) / 128);
  if (tiles >= 192 || K < 512) return 1;
  const long s = std::min<long>((256 + tiles - 1) / tiles, K / 256);
  return (int)std::max<long>(1, s);
}

// y[m][n] = sum of the S slabs [S][M][N] + bias[n], fixed order
__global__ __launch_bounds__(256) void conv_slab_sum_kernel(const float* __restrict__ slabs, int S, long M, int N,
                                                            const float* __restrict__ bias, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  float acc = 0.f;
  for (int z = 0; z < S; ++z) acc += slabs[(long)z * M * N + i];
  if (bias) acc += bias[i % N];
  y[i] = acc;
}

}  // namespace

extern "C" int damc_pack_conv2d(const float* w, int cout, int cin, int k, float* wp, void* stream) {
  if (!w || !wp || cout <= 0 || cin <= 0 || k <= 0) return DAMC_ERR_ARG;
  const long n = (long)cout * cin * k * k;
  hipLaunchKernelGGL(pack_conv_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), w, cout, cin,
                     k, (int)damc::conv_kmajor_ok(cin), wp);
  return (int)hipGetLastError();
}

extern "C" int damc_nchw_to_nhwc(const float* x, int B, int C, int HW, float* y, void* stream) {
  if (!x || !y || B <= 0 || C <= 0 || HW <= 0) return DAMC_ERR_ARG;
  const long n = (long)B * C * HW;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), x, B, C,
                     HW, y);
  return (int)hipGetLastError();
}

extern "C" size_t damc_conv2d_workspace_floats(int B, int hin, int win, int cin, int cout, int k, int stride,
                                               int pad) {
  if (B <= 0 || cin <= 0 || cout <= 0 || k <= 0 || stride <= 0) return 0;
  const int hout = (hin + 2 * pad - k) / stride + 1, wout = (win + 2 * pad - k) / stride + 1;
  if (hout <= 0 || wout <= 0 || !damc::conv_kmajor_ok(cin)) return 0;
  const long M = (long)B * hout * wout;
  const int S = conv_split(M, cout, k * k * cin);
  return S > 1 ? (size_t)S * M * cout : 0;
}

extern "C" int damc_conv2d_nhwc(const float* x, int B, int hin, int win, int cin, const float* wp, const float* bias,
                                int cout, int k, int stride, int pad, float* y, float* workspace,
                                size_t workspace_floats, void* stream) {
  if (!x || !wp || !y || B <= 0) return DAMC_ERR_ARG;
  const int hout = (hin + 2 * pad - k) / stride + 1, wout = (win + 2 * pad - k) / stride + 1;
  if (hout <= 0 || wout <= 0) return DAMC_ERR_ARG;
  damc::GemmArgs a;
  a.A = x;
  a.Hin = hin;
  a.Win = win;
  a.Cg = cin;
  a.Hq = hout;
  a.Wq = wout;
  a.kw = k;
  a.stride = stride;
  a.pad_y = pad;
  a.pad_x = pad;
  a.B = wp;
  a.b_kmajor = damc::conv_kmajor_ok(cin);
  a.ldb = a.b_kmajor ? (long)k * k * cin : cout;
  a.C = y;
  a.ldc = cout;
  a.M = B * hout * wout;
  a.N = cout;
  a.K = k * k * cin;
  a.k_per_z = a.K;
  a.bias = bias;
  a.bias_mod = cout;
  a.act = DAMC_ACT_NONE;
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * a.M * (double)cout * a.K;
  int S = a.b_kmajor ? conv_split(a.M, cout, a.K) : 1;
  if (S > 1 && workspace && workspace_floats >= (size_t)S * a.M * cout) {
    // split K over S slices (multiples of the engine's 32-deep K tile, so no tile straddles a tap)
    a.k_per_z = (a.K / 32 + S - 1) / S * 32;
    S = (a.K + a.k_per_z - 1) / a.k_per_z;
    a.C = workspace;
    a.c_zstride = (long)a.M * cout;
    a.bias = nullptr;
    int rc = damc::launch_gemm(a, damc::A_CONV, damc::EPI_STORE, damc::O_DENSE, S, "enc_conv", flops, s);
    if (rc) return rc;
    const long n = (long)a.M * cout;
    hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       (const float*)workspace, S, (long)a.M, cout, bias, y);
    return (int)hipGetLastError();
  }
  return damc::launch_gemm(a, damc::A_CONV, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "enc_conv", flops, s);
}

extern "C" size_t damc_instnorm_workspace_floats(int B, int hw, int c) {
  return (size_t)B * c * in_splits(hw) * 3;
}

extern "C" int damc_instnorm_lrelu_nhwc(float* y, int B, int hw, int c, const float* gamma, const float* beta,
                                        float eps, float slope, float* ws, void* stream) {
  if (!y || !gamma || !beta || !ws || B <= 0 || hw <= 0 || c <= 0) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  const int S = in_splits(hw);
  const int cg = (c + 63) / 64;
  ProfScope ps("instnorm", 0.0, s);
  hipLaunchKernelGGL(in_stats_kernel, dim3(B * cg, S), dim3(256), 0, s, y, B, hw, c, S, ws);
  const int P = std::max(1, std::min(64, hw / 256));
  hipLaunchKernelGGL(in_apply_kernel, dim3(B * cg, P), dim3(256), 0, s, y, B, hw, c, S, ws, gamma, beta, eps, slope);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ training (Q update)
// InstanceNorm2d(affine) + LeakyReLU for the encoder's training forward/backward: the conv output y is kept,
// h = lrelu(IN(y)) goes to its own buffer and (mean, rstd) per (sample, channel) are saved.  The backward
// of a = gamma * (y - mean) * rstd + beta, h = lrelu(a) (biased variance, as InstanceNorm2d):
//   dA = dh * lrelu'(a);  dy = rstd * gamma * (dA - mean_p(dA) - xhat * mean_p(dA * xhat))
// with per-(sample, channel) sums over pixels taken in S splits and merged in fixed order.
namespace {

__global__ __launch_bounds__(256) void in_apply_train_kernel(const float* y, int B, int HW, int C, int S,
                                                             const float* part, const float* gamma,
                                                             const float* beta, float eps, float slope, float* h,
                                                             float* stats) {
  const int cg = (C + 63) / 64;
  const int b = blockIdx.x / cg, c = (blockIdx.x % cg) * 64 + (threadIdx.x & 63);
  const int prow = threadIdx.x >> 6;
  __shared__ float sc[64], sh[64];
  if (prow == 0) {
    float scale = 0.f, shift = 0.f;
    if (c < C) {
      const float* pp = part + ((long)b * C + c) * S * 3;
      Wf a{pp[0], pp[1], pp[2]};
      for (int s = 1; s < S; ++s) a = wmerge(a, Wf{pp[3 * s], pp[3 * s + 1], pp[3 * s + 2]});
      const float var = a.m2 / a.n;
      const float rstd = 1.f / sqrtf(var + eps);
      scale = rstd;
      shift = a.mean;
      if (blockIdx.y == 0) {
        stats[((long)b * C + c) * 2] = a.mean;
        stats[((long)b * C + c) * 2 + 1] = rstd;
      }
    }
    sc[threadIdx.x] = scale;
    sh[threadIdx.x] = shift;
  }
  __syncthreads();
  if (c >= C) return;
  // a = ((y - mean) * rstd) * gamma + beta, InstanceNorm's own order: the fused y * scale + shift form of
  // the inference pass loses low bits when |mean| >> std, and the backward's LReLU' reads the sign of a
  const float rstd = sc[threadIdx.x & 63], mean = sh[threadIdx.x & 63], g = gamma[c], bt = beta[c];
  const int P = gridDim.y;
  const int p0 = (int)((long)HW * blockIdx.y / P), p1 = (int)((long)HW * (blockIdx.y + 1) / P);
  for (int p = p0 + prow; p < p1; p += 4) {
    const long o = ((long)b * HW + p) * C + c;
    const float v = __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(y[o], mean), rstd), g), bt);
    h[o] = v > 0.f ? v : v * slope;
  }
}

// pass 1: per (b, c, split) partial sums {sum dA, sum dA * xhat}
__global__ __launch_bounds__(256) void in_bwd_sums_kernel(const float* y, const float* stats, const float* dh, int B,
                                                          int HW, int C, int S, const float* gamma, const float* beta,
                                                          float slope, float* part) {
  const int cg = (C + 63) / 64;
  const int b = blockIdx.x / cg, c = (blockIdx.x % cg) * 64 + (threadIdx.x & 63);
  const int prow = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const int p0 = (int)((long)HW * s / S), p1 = (int)((long)HW * (s + 1) / S);
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    const float mean = stats[((long)b * C + c) * 2], rstd = stats[((long)b * C + c) * 2 + 1];
    const float g = gamma[c], bt = beta[c];
    for (int p = p0 + prow; p < p1; p += 4) {
      const long o = ((long)b * HW + p) * C + c;
      const float xh = __fmul_rn(__fsub_rn(y[o], mean), rstd);
      const float a = __fadd_rn(__fmul_rn(xh, g), bt);  // the forward's a, bit for bit
      const float dA = a > 0.f ? dh[o] : dh[o] * slope;
      s1 += dA;
      s2 += dA * xh;
    }
  }
  __shared__ float r1[4][64], r2[4][64];
  r1[prow][threadIdx.x & 63] = s1;
  r2[prow][threadIdx.x & 63] = s2;
  __syncthreads();
  if (prow == 0 && c < C) {
    const int l = threadIdx.x;
    float* o = part + (((long)b * C + c) * S + s) * 2;
    o[0] = ((r1[0][l] + r1[1][l]) + r1[2][l]) + r1[3][l];
    o[1] = ((r2[0][l] + r2[1][l]) + r2[2][l]) + r2[3][l];
  }
}

// pass 2: merge the S partials (fixed order), write dy; totals per (b, c) go to bc (B x C x 2) for dgamma/dbeta
__global__ __launch_bounds__(256) void in_bwd_apply_kernel(const float* y, const float* stats, const float* dh, int B,
                                                           int HW, int C, int S, const float* gamma,
                                                           const float* beta, float slope, const float* part,
                                                           float* dy, float* bc) {
  const int cg = (C + 63) / 64;
  const int b = blockIdx.x / cg, c = (blockIdx.x % cg) * 64 + (threadIdx.x & 63);
  const int prow = threadIdx.x >> 6;
  if (c >= C) return;
  const float* pp = part + ((long)b * C + c) * S * 2;
  float t1 = 0.f, t2 = 0.f;
  for (int s = 0; s < S; ++s) {
    t1 += pp[2 * s];
    t2 += pp[2 * s + 1];
  }
  if (blockIdx.y == 0 && prow == 0) {  // bc [b][2][C]: dgamma rows (sum dA * xhat), then dbeta rows (sum dA)
    bc[((long)b * 2) * C + c] = t2;
    bc[((long)b * 2 + 1) * C + c] = t1;
  }
  const float mean = stats[((long)b * C + c) * 2], rstd = stats[((long)b * C + c) * 2 + 1];
  const float g = gamma[c], bt = beta[c];
  const float scl = rstd * g;
  const float m1 = t1 / (float)HW, m2 = t2 / (float)HW;
  const int P = gridDim.y;
  const int p0 = (int)((long)HW * blockIdx.y / P), p1 = (int)((long)HW * (blockIdx.y + 1) / P);
  for (int p = p0 + prow; p < p1; p += 4) {
    const long o = ((long)b * HW + p) * C + c;
    const float xh = __fmul_rn(__fsub_rn(y[o], mean), rstd);
    const float a = __fadd_rn(__fmul_rn(xh, g), bt);
    const float dA = a > 0.f ? dh[o] : dh[o] * slope;
    dy[o] = scl * (dA - m1 - xh * m2);
  }
}

}  // namespace

extern "C" int damc_instnorm_lrelu_train_nhwc(const float* y, int B, int hw, int c, const float* gamma,
                                              const float* beta, float eps, float slope, float* h, float* stats,
                                              float* ws, void* stream) {
  if (!y || !h || !stats || !gamma || !beta || !ws || B <= 0 || hw <= 0 || c <= 0) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  const int S = in_splits(hw);
  const int cg = (c + 63) / 64;
  ProfScope ps("instnorm", 0.0, s);
  hipLaunchKernelGGL(in_stats_kernel, dim3(B * cg, S), dim3(256), 0, s, y, B, hw, c, S, ws);
  const int P = std::max(1, std::min(64, hw / 256));
  hipLaunchKernelGGL(in_apply_train_kernel, dim3(B * cg, P), dim3(256), 0, s, y, B, hw, c, S, ws, gamma, beta, eps,
                     slope, h, stats);
  return (int)hipGetLastError();
}

extern "C" size_t damc_instnorm_bwd_workspace_floats(int B, int hw, int c) {
  if (B <= 0 || hw <= 0 || c <= 0) return 0;
  return (size_t)B * c * in_splits(hw) * 2 + (size_t)B * c * 2 + damc::colsum_tmp_floats(B, c);
}

extern "C" int damc_instnorm_lrelu_backward_nhwc(const float* y, const float* stats, const float* dh, int B, int hw,
                                                 int c, const float* gamma, const float* beta, float slope, float* dy,
                                                 float* dgamma, float* dbeta, float* ws, void* stream) {
  if (!y || !stats || !dh || !dy || !gamma || !beta || !ws || B <= 0 || hw <= 0 || c <= 0) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  const int S = in_splits(hw);
  const int cg = (c + 63) / 64;
  float* part = ws;
  float* bc = part + (size_t)B * c * S * 2;
  float* tmp = bc + (size_t)B * c * 2;
  ProfScope ps("instnorm_bwd", 0.0, s);
  hipLaunchKernelGGL(in_bwd_sums_kernel, dim3(B * cg, S), dim3(256), 0, s, y, stats, dh, B, hw, c, S, gamma, beta,
                     slope, part);
  const int P = std::max(1, std::min(64, hw / 256));
  hipLaunchKernelGGL(in_bwd_apply_kernel, dim3(B * cg, P), dim3(256), 0, s, y, stats, dh, B, hw, c, S, gamma, beta,
                     slope, (const float*)part, dy, bc);
  DAMC_LAUNCH_CHECK();
  // dgamma = sum_b bc[b][0][c], dbeta = sum_b bc[b][1][c]: fixed-order column sums over the B rows
  if (dgamma) {
    int rc = damc::launch_colsum(bc, B, c, 2L * c, dgamma, tmp, s);
    if (rc) return rc;
  }
  if (dbeta) {
    int rc = damc::launch_colsum(bc + c, B, c, 2L * c, dbeta, tmp, s);
    if (rc) return rc;
  }
  return 0;
}

// ---- the whole encoder forward in one call (damc_q_encoder_fwd): NCHW -> NHWC, then per layer the conv
// (split-K slabs when its tiles would not fill the chip) and InstanceNorm + LeakyReLU in place; two
// ping-pong activation buffers, the last conv writes xemb directly
namespace {
struct EncShapes {
  int h[DAMC_MAX_ENC_LAYERS + 1], w[DAMC_MAX_ENC_LAYERS + 1];
  size_t act_max = 0, slab_max = 0, in_max = 0;
};
bool enc_shapes(const damc_encoder_t* e, int B, EncShapes* sh) {
  if (!e || B <= 0 || e->n_layers < 1 || e->n_layers > DAMC_MAX_ENC_LAYERS || e->nc <= 0 || e->h <= 0 || e->w <= 0)
    return false;
  sh->h[0] = e->h;
  sh->w[0] = e->w;
  int c = e->nc;
  sh->act_max = (size_t)B * e->h * e->w * e->nc;
  for (int i = 0; i < e->n_layers; ++i) {
    const damc_enc_layer_t& L = e->layers[i];
    if (L.cin != c || L.cout <= 0 || L.k <= 0 || L.stride <= 0 || L.pad < 0 || !L.w_packed) return false;
    if ((L.in_gamma == nullptr) != (L.in_beta == nullptr)) return false;
    const int ho = (sh->h[i] + 2 * L.pad - L.k) / L.stride + 1, wo = (sh->w[i] + 2 * L.pad - L.k) / L.stride + 1;
    if (ho <= 0 || wo <= 0) return false;
    sh->h[i + 1] = ho;
    sh->w[i + 1] = wo;
    if (i + 1 < e->n_layers) sh->act_max = std::max(sh->act_max, (size_t)B * ho * wo * L.cout);
    sh->slab_max = std::max(sh->slab_max,
                            damc_conv2d_workspace_floats(B, sh->h[i], sh->w[i], L.cin, L.cout, L.k, L.stride, L.pad));
    if (L.in_gamma) sh->in_max = std::max(sh->in_max, damc_instnorm_workspace_floats(B, ho * wo, L.cout));
    c = L.cout;
  }
  return true;
}
size_t round256(size_t b) { return (b + 255) / 256 * 256; }
}  // namespace

extern "C" size_t damc_q_encoder_workspace_bytes(const damc_encoder_t* e, int B) {
  EncShapes sh;
  if (!enc_shapes(e, B, &sh)) return 0;
  return 2 * round256(sh.act_max * 4) + round256(std::max<size_t>(sh.slab_max, 1) * 4) +
         round256(std::max<size_t>(sh.in_max, 1) * 4);
}

extern "C" int damc_q_encoder_fwd(const damc_encoder_t* e, const float* x, int B, float* xemb, void* wsp, size_t wsb,
                                  void* stream) {
  EncShapes sh;
  if (!x || !xemb || !enc_shapes(e, B, &sh)) return DAMC_ERR_ARG;
  const int n = e->n_layers;
  if (sh.h[n] != 1 || sh.w[n] != 1) return DAMC_ERR_UNSUPPORTED;  // NHWC flatten == NCHW flatten only at 1 x 1
  if (!wsp || wsb < damc_q_encoder_workspace_bytes(e, B)) return DAMC_ERR_WORKSPACE;
  char* base = reinterpret_cast<char*>(wsp);
  float* buf[2] = {reinterpret_cast<float*>(base), reinterpret_cast<float*>(base + round256(sh.act_max * 4))};
  float* slabs = reinterpret_cast<float*>(base + 2 * round256(sh.act_max * 4));
  float* inws = reinterpret_cast<float*>(base + 2 * round256(sh.act_max * 4) +
                                         round256(std::max<size_t>(sh.slab_max, 1) * 4));
  int rc;
  if ((rc = damc_nchw_to_nhwc(x, B, e->nc, e->h * e->w, buf[0], stream))) return rc;
  for (int i = 0; i < n; ++i) {
    const damc_enc_layer_t& L = e->layers[i];
    float* out = (i + 1 == n) ? xemb : buf[(i + 1) & 1];
    const size_t nsl = damc_conv2d_workspace_floats(B, sh.h[i], sh.w[i], L.cin, L.cout, L.k, L.stride, L.pad);
    if ((rc = damc_conv2d_nhwc(buf[i & 1], B, sh.h[i], sh.w[i], L.cin, L.w_packed, L.bias, L.cout, L.k, L.stride,
                               L.pad, out, nsl ? slabs : nullptr, nsl, stream)))
      return rc;
    if (L.in_gamma &&
        (rc = damc_instnorm_lrelu_nhwc(out, B, sh.h[i + 1] * sh.w[i + 1], L.cout, L.in_gamma, L.in_beta, L.in_eps,
                                       L.slope, inws, stream)))
      return rc;
  }
  return 0;
}
