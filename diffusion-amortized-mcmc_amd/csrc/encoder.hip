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
    // four loads in flight, then their updates in pixel order (the same Welford chain as one at a time)
    int p = p0 + prow;
    for (; p + 12 < p1; p += 16) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = y[((long)b * HW + p + 4 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        w.n += 1.f;
        const float d = v[u] - w.mean;
        w.mean += d / w.n;
        w.m2 += d * (v[u] - w.mean);
      }
    }
    for (; p < p1; p += 4) {
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

// (scale, shift) of every (sample, channel) from the S statistics partials, merged once (in_apply_kernel's merge,
// same order): ss [B][2][C]
// one wave per (sample, channel): lane s loads strip s (one coalesced 12-B record per lane; S <= 64), and the strips
// merge as a fixed pairwise tree over lanes (strides 1, 2, 4, ...; an empty lane is an exact identity of wmerge).
// Round 5's one-thread-per-(sample, channel) left fold issued S dependent merges behind S scattered loads: 22 us per
// CelebA-HQ B=8 layer for 1024 threads (profiles/r06/enc_hq_b8_dispatches.txt).  The tree depends on S alone, which
// depends on the map size alone (in_splits), so a batch sharded over ranks merges exactly as the whole batch.
__global__ __launch_bounds__(256) void in_merge_kernel(const float* __restrict__ part, int B, int C, int S,
                                                       const float* gamma, const float* beta, float eps,
                                                       float* __restrict__ ss) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= B * C) return;  // wave-uniform
  const int b = i / C, c = i - b * C;
  Wf a{0.f, 0.f, 0.f};
  if (lane < S) {
    const float* pp = part + ((long)i * S + lane) * 3;
    a = Wf{pp[0], pp[1], pp[2]};
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const Wf o{__shfl_down(a.n, off), __shfl_down(a.mean, off), __shfl_down(a.m2, off)};
    if ((lane & (2 * off - 1)) == 0) a = wmerge(a, o);
  }
  if (lane != 0) return;
  const float var = a.m2 / a.n;
  const float rstd = 1.f / sqrtf(var + eps);
  const float scale = rstd * gamma[c];
  ss[(long)b * 2 * C + c] = scale;
  ss[(long)b * 2 * C + C + c] = beta[c] - a.mean * scale;
}

// the norm statistics of the 256-pixel strips (GemmArgs::in_part's partition and arithmetic: damc::strip256_stats)
// from the stored conv output, for a conv whose launch could not take them in its epilogue (split-K at a small batch):
// grid (HW / 256 strips, B, ceil(C / 128)), 512 threads; part as in_stats_kernel's with S = HW / 256
__global__ __launch_bounds__(512) void in_strip_stats_kernel(const float* __restrict__ y, int HW, int C, float* part) {
  __shared__ float red[1024];
  const int sp = blockIdx.x, b = blockIdx.y, c0 = blockIdx.z * 128, tid = threadIdx.x;
  const int S = HW >> 8;
  float st[3];
  damc::strip256_stats(y + ((long)b * HW + 256L * sp) * C + c0, C, tid, c0 + (tid & 127) < C, red, st);
  if (tid < 128 && c0 + tid < C) {
    float* o = part + (((long)b * C + c0 + tid) * S + sp) * 3;
    o[0] = st[0];
    o[1] = st[1];
    o[2] = st[2];
  }
}

// in_apply_x3_kernel's fp32 in-place form one channel quad per thread (round 6, late): the same fmaf and LReLU per
// element, and every load / store instruction covers 1 KB without gaps (the octet form's pair of 16-B accesses per
// lane half-covers two 2 KB spans)
__global__ __launch_bounds__(256) void in_apply_f32_kernel(float* y, long n4, int HW, int C,
                                                           const float* __restrict__ ss, float slope) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int C4 = C / 4;
  const long pix = i / C4;
  const int c0 = (int)(i - pix * C4) * 4;
  const int b = (int)(pix / HW);
  const float* sc = ss + (long)b * 2 * C + c0;
  f32x4 v = *reinterpret_cast<const f32x4*>(y + 4 * i);
  const f32x4 a = *reinterpret_cast<const f32x4*>(sc), h = *reinterpret_cast<const f32x4*>(sc + C);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float t = fmaf(v[e], a[e], h[e]);
    v[e] = t > 0.f ? t : t * slope;
  }
  *reinterpret_cast<f32x4*>(y + 4 * i) = v;
}

// the normalise + affine + LeakyReLU of in_apply_kernel (same fmaf), written as the next convolution's limbs (x3
// octets) instead of fp32 in place: the limb engine reads nothing else.  One thread per (pixel, channel octet).
// y32 != NULL: fp32 in place instead (y32 == y; every thread rewrites only the octet it read), for a next conv that
// stages its input as fp32 (gemm.hip X3_F32A)
__global__ __launch_bounds__(256) void in_apply_x3_kernel(const float* y, long n8, int HW, int C,
                                                          const float* __restrict__ ss, float slope,
                                                          unsigned short* __restrict__ y3, float* y32) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int C8 = C / 8;
  const long pix = i / C8;
  const int c0 = (int)(i - pix * C8) * 8;
  const int b = (int)(pix / HW);
  const float* sc = ss + (long)b * 2 * C + c0;
  const f32x4 v0 = *reinterpret_cast<const f32x4*>(y + 8 * i), v1 = *reinterpret_cast<const f32x4*>(y + 8 * i + 4);
  const f32x4 a0 = *reinterpret_cast<const f32x4*>(sc), a1 = *reinterpret_cast<const f32x4*>(sc + 4);
  const f32x4 h0 = *reinterpret_cast<const f32x4*>(sc + C), h1 = *reinterpret_cast<const f32x4*>(sc + C + 4);
  float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  const float sa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const float sb[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t = fmaf(v[e], sa[e], sb[e]);
    v[e] = t > 0.f ? t : t * slope;
  }
  if (y32) {
    *reinterpret_cast<f32x4*>(y32 + 8 * i) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(y32 + 8 * i + 4) = f32x4{v[4], v[5], v[6], v[7]};
  } else {
    damc::store_x3_octet(v, y3 + 24 * i);
  }
}

// ---- the first layer (Conv2d k3 s1 p1 on the nc <= 4 image channels, then InstanceNorm + LeakyReLU) in two passes
// that recompute the convolution (9 nc MACs per output) instead of storing it: pass 1 its per-(sample, channel)
// statistics, pass 2 the normalised activation as the next convolution's limbs.  The conv output, the largest
// tensor of the encoder (1 GB at CelebA-HQ B=64), never reaches HBM.  A block = R image rows of one sample, the
// (R+2) x (W+2) x CIN input window staged in LDS (read from the caller's NCHW image).  A wave owns one channel
// octet at a time (its 8 x 9 CIN weights wave-uniform: scalar loads, no LDS traffic) and its lanes own pixels, whose
// 9 CIN window values are read from LDS once for the 8 channels.  Both passes evaluate y with conv3_octet (fixed tap
// order, one fmaf chain per channel), so the statistics describe exactly the values pass 2 normalises.
// PX horizontally adjacent pixels (x .. x + PX - 1 of row r) x one channel octet: the window values of the run are read
// once (3 x (PX + 2) x CIN instead of PX x 9 CIN) and each weight pair once per run; every output keeps the same fmaf
// chain (tap order, from 0, then + bias), so PX changes no value
template <int CIN, int PX>
__device__ __forceinline__ void conv3_octet(const float* __restrict__ win, int ld, int r, int x,
                                            const float* __restrict__ wl, int C, int c0, const float* __restrict__ bl,
                                            float (&y)[PX][8]) {
  float xv[3][PX + 2][CIN];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int cx = 0; cx < PX + 2; ++cx)
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci) xv[ky][cx][ci] = win[((r + ky) * ld + x + cx) * CIN + ci];
  float acc[PX][8];
#pragma unroll
  for (int px = 0; px < PX; ++px)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[px][e] = 0.f;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci) {  // wl: the LDS copy of damc_pack_conv2d's [(ky, kx, ci)][co] (a wave-uniform
        const int t = (ky * 3 + kx) * CIN + ci;  // address: broadcast reads)
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(wl + t * C + c0);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(wl + t * C + c0 + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int px = 0; px < PX; ++px)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[px][e] = fmaf(wv[e], xv[ky][px + kx][ci], acc[px][e]);
      }
  }
#pragma unroll
  for (int px = 0; px < PX; ++px)
#pragma unroll
    for (int e = 0; e < 8; ++e) y[px][e] = acc[px][e] + bl[c0 + e];
}
// the strip's input window: rows r0-1 .. r0+R of sample b, columns -1 .. W, zero outside, [row][col][ci] in LDS
template <int CIN>
__device__ __forceinline__ void conv3_stage(const float* __restrict__ x, int b, int H, int W, int r0, int R, float* win) {
  // element i = (rr CIN + ci) ld + cc: lanes run along one channel row of x (coalesced), 8 unconditional loads (clamped
  // addresses, zeroed by select) in flight per thread before the LDS writes.  Round 5's loop took one element at a
  // time and its load -> ds_write chain paid a full HBM latency per element: with 2 workgroups per CU it was the
  // first layer's cost (40 us of CelebA-HQ B=8's stats pass)
  const int ld = W + 2, n = (R + 2) * ld * CIN;
  const float* xb = x + (long)b * CIN * H * W;
  for (int i0 = threadIdx.x; i0 < n; i0 += 8 * blockDim.x) {
    float v[8];
    int dst[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = min(i0 + j * (int)blockDim.x, n - 1);
      const int q = i / ld, cc = i - q * ld, rr = q / CIN, ci = q - rr * CIN;
      const int iy = r0 - 1 + rr, ix = cc - 1;
      const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
      const float t = xb[((long)ci * H + min(max(iy, 0), H - 1)) * W + min(max(ix, 0), W - 1)];
      v[j] = ok ? t : 0.f;
      dst[j] = (rr * ld + cc) * CIN + ci;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i0 + j * (int)blockDim.x < n) win[dst[j]] = v[j];
  }
}

// pass 1: grid (B, S strips of R rows); wave w takes octets w, w+4, ...; each lane a Welford chain over its pixels per
// channel (runs of PX pixels, W % PX == 0), then the 64 lanes merged (Chan, fixed butterfly order); part [B][C][S][3]
// as in_stats_kernel's
template <int CIN, int PX>
__global__ __launch_bounds__(256) void conv3_stats_kernel(const float* __restrict__ x, int H, int W, int C, int R,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float sm3[];  // [9 CIN][C] weights, [C] bias, then the window
  const int b = blockIdx.x, s = blockIdx.y, S = gridDim.y, r0 = s * R, rows = min(R, H - r0);
  float* wl = sm3;
  float* bl = wl + 9 * CIN * C;
  float* win = bl + C;
  for (int i = threadIdx.x; i < 9 * CIN * C; i += blockDim.x) wl[i] = w[i];
  for (int i = threadIdx.x; i < C; i += blockDim.x) bl[i] = bias ? bias[i] : 0.f;
  conv3_stage<CIN>(x, b, H, W, r0, R, win);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, npix = rows * W;
  for (int o = wave; o < C / 8; o += 4) {
    const int c0 = __builtin_amdgcn_readfirstlane(o * 8);
    Wf a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = Wf{0.f, 0.f, 0.f};
    float n = 0.f;
#pragma unroll 1
    for (int p = lane * PX; p < npix; p += 64 * PX) {
      // the weights are re-read from LDS per run (broadcast reads); held in registers across the loop they took
      // 216 VGPRs and left one wave per SIMD
      asm volatile("" ::: "memory");
      const int r = p / W, xx = p - r * W;
      float y[PX][8];
      conv3_octet<CIN, PX>(win, W + 2, r, xx, wl, C, c0, bl, y);
#pragma unroll
      for (int px = 0; px < PX; ++px) {
        n += 1.f;
        const float inv = 1.f / n;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = y[px][e] - a[e].mean;
          a[e].mean += d * inv;
          a[e].m2 += d * (y[px][e] - a[e].mean);
          a[e].n = n;
        }
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const Wf t{__shfl_xor(a[e].n, off), __shfl_xor(a[e].mean, off), __shfl_xor(a[e].m2, off)};
        a[e] = (lane & off) ? wmerge(t, a[e]) : wmerge(a[e], t);  // both partners form the same (lower, upper) merge
      }
    if (lane < 8) {
      Wf t = a[0];
#pragma unroll
      for (int e = 1; e < 8; ++e)
        if (lane == e) t = a[e];
      float* op = part + (((long)b * C + c0 + lane) * S + s) * 3;
      op[0] = t.n;
      op[1] = t.mean;
      op[2] = t.m2;
    }
  }
}

// pass 2: grid (B, S strips); wave w takes octets w, w+4, ..., lanes pixels; writes the limbs of lrelu(IN(y)), or the
// fp32 values (NHWC) at y32 for an F32A next conv
template <int CIN, int PX>
__global__ __launch_bounds__(256) void conv3_apply_x3_kernel(const float* __restrict__ x, int H, int W, int C, int R,
                                                             const float* __restrict__ w, const float* __restrict__ bias,
                                                             const float* __restrict__ ss, float slope,
                                                             unsigned short* __restrict__ y3, float* __restrict__ y32) {
  extern __shared__ __attribute__((aligned(16))) float sm3[];  // [9 CIN][C] weights, [C] bias, then the window
  const int b = blockIdx.x, s = blockIdx.y, r0 = s * R, rows = min(R, H - r0);
  float* wl = sm3;
  float* bl = wl + 9 * CIN * C;
  float* win = bl + C;
  for (int i = threadIdx.x; i < 9 * CIN * C; i += blockDim.x) wl[i] = w[i];
  for (int i = threadIdx.x; i < C; i += blockDim.x) bl[i] = bias ? bias[i] : 0.f;
  conv3_stage<CIN>(x, b, H, W, r0, R, win);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, npix = rows * W;
  const float* sb = ss + (long)b * 2 * C;
  for (int o = wave; o < C / 8; o += 4) {
    const int c0 = __builtin_amdgcn_readfirstlane(o * 8);
#pragma unroll 1
    for (int p = lane * PX; p < npix; p += 64 * PX) {
      asm volatile("" ::: "memory");  // weights re-read from LDS per run (see conv3_stats_kernel)
      const int r = p / W, xx = p - r * W;
      float y[PX][8];
      conv3_octet<CIN, PX>(win, W + 2, r, xx, wl, C, c0, bl, y);
#pragma unroll
      for (int px = 0; px < PX; ++px) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = fmaf(y[px][e], sb[c0 + e], sb[C + c0 + e]);
          v[e] = t > 0.f ? t : t * slope;
        }
        const long off = (((long)b * H + r0 + r) * W + xx + px) * C + c0;
        if (y32) {
          *reinterpret_cast<f32x4*>(y32 + off) = f32x4{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<f32x4*>(y32 + off + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          damc::store_x3_octet(v, y3 + 3 * off);
        }
      }
    }
  }
}

// ---- the first layer on the limb MFMA (round 6; DAMC_ENC_FIRST_MFMA=0 keeps the fmaf-chain passes above): the k3 conv
// on CIN <= 3 channels has K = 9 CIN <= 32, one K tile of v_mfma_f32_16x16x32_bf16.  A 16-pixel group's im2col rows
// (k = (ky 3 + kx) CIN + ci, zero past 9 CIN) come from the LDS window, each value split into its three RNE bf16 limbs
// (the GEMM engine's split3), the weights' limbs ([(ky, kx, ci)][co], damc_pack_conv2d's layout) sit in registers, and
// every output is the six limb products summed smallest first into fp32 (the limb engine's arithmetic: error at or
// below the fp32-MFMA engine's), plus the bias.  Pass 1 (STATS) runs a Welford chain per lane
// and channel over the lane's pixels (4 per group), merged over the lanes of a channel (butterfly) and the 4 waves
// (fixed order) into part [B][C][S][3] as conv3_stats_kernel does; pass 2 recomputes y with the same code (so the
// statistics describe exactly the values it normalises), applies lrelu(y scale + shift) and writes the NHWC activation
// as fp32 for an F32A next conv, or as its limbs.  Wave w takes the strip's 16-pixel groups w, w + 4, ...; W % 16 == 0.
typedef __bf16 c3b8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void c3_split8(const float (&v)[8], c3b8& h, c3b8& m, c3b8& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 b0 = (__bf16)v[e];
    const float r1 = sub_rn(v[e], (float)b0);
    const __bf16 b1 = (__bf16)r1;
    h[e] = b0;
    m[e] = b1;
    l[e] = (__bf16)sub_rn(r1, (float)b1);
  }
}
// the window as its three RNE bf16 limb planes (c3_split8's split, done once per window value instead of once per
// im2col use: each value feeds 9 CIN taps)
template <int CIN>
__device__ __forceinline__ void conv3_stage_limbs(const float* __restrict__ x, int b, int H, int W, int r0, int R,
                                                  __bf16* wh, __bf16* wm, __bf16* wl) {
  // element (q = rr CIN + ci, cc) of the flattened (R + 2) CIN x (W + 2) window; a thread's elements step by blockDim
  // (q and cc advanced incrementally: no division per element), 8 loads in flight; slots past the end repeat the last
  // element (the same value to the same address), so the loads and LDS stores run unconditionally
  const int ld = W + 2, nq = (R + 2) * CIN, n = nq * ld, dq = blockDim.x / ld, dc = blockDim.x - dq * ld;
  const float* xb = x + (long)b * CIN * H * W;
  int q = threadIdx.x / ld, cc = threadIdx.x - q * ld;
  for (int i0 = 0; i0 < n; i0 += 8 * blockDim.x) {
    float v[8];
    int dst[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int past = q >= nq;
      const int qc = past ? nq - 1 : q, ccc = past ? ld - 1 : cc;
      const int rr = qc / CIN, ci = qc - rr * CIN, iy = r0 - 1 + rr, ix = ccc - 1;
      const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const float t = xb[(unsigned)((ci * H + min(max(iy, 0), H - 1)) * W + min(max(ix, 0), W - 1))];
      v[j] = ok ? t : 0.f;
      dst[j] = (rr * ld + ccc) * CIN + ci;
      cc += dc;
      const int wr = cc >= ld;
      cc -= ld & -wr;
      q += dq + wr;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const __bf16 b0 = (__bf16)v[j];
      const float r1 = sub_rn(v[j], (float)b0);
      const __bf16 b1 = (__bf16)r1;
      wh[dst[j]] = b0;
      wm[dst[j]] = b1;
      wl[dst[j]] = (__bf16)sub_rn(r1, (float)b1);
    }
  }
}
template <int CIN, int NT, bool STATS>
__global__ __launch_bounds__(256) void conv3_mfma_kernel(const float* __restrict__ x, int H, int W, int C, int R,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         float* __restrict__ part, const float* __restrict__ ss,
                                                         float slope, float* __restrict__ y32,
                                                         unsigned short* __restrict__ y3) {
  static_assert(9 * CIN <= 32 && NT * 16 <= 128, "one K tile, at most 128 channels");
  extern __shared__ __attribute__((aligned(16))) __bf16 c3win[];  // the (R+2) x (W+2) x CIN window's 3 limb planes
  __shared__ Wf c3red[4][NT * 16];
  constexpr int OLD = NT * 16 + 4;  // the output staging tile's row stride (floats)
  __shared__ __attribute__((aligned(16))) float c3out[STATS ? 1 : 4][16][OLD];
  const int b = blockIdx.x, s = blockIdx.y, S = gridDim.y, r0 = s * R, rows = min(R, H - r0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n = lane & 15, kq = lane >> 4;
  const int pst = (R + 2) * (W + 2) * CIN;  // the limb planes' stride (elements)
  conv3_stage_limbs<CIN>(x, b, H, W, r0, R, c3win, c3win + pst, c3win + 2 * pst);
  // the weights' limbs: tile t, lane (channel 16 t + n, k-octet kq)
  c3b8 wb[NT][3];
  float bl[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * kq + e;
      v[e] = k < 9 * CIN ? w[(long)k * C + 16 * t + n] : 0.f;
    }
    c3_split8(v, wb[t][0], wb[t][1], wb[t][2]);
    bl[t] = bias ? bias[16 * t + n] : 0.f;
  }
  // the lane's im2col offsets within the window for its pixel n and k-octet: tap (ky, kx) and ci of k = 8 kq + e; a
  // k >= 9 CIN reads the pixel's own first value (any finite value: its weight limbs are zero, so the products are)
  int koff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * kq + e, tap = k / CIN, ci = k - tap * CIN;
    koff[e] = n * CIN + (k < 9 * CIN ? ((tap / 3) * (W + 2) + tap % 3) * CIN + ci : 0);
  }
  __syncthreads();
  const int ngrp = rows * W / 16;
  Wf a[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) a[t] = Wf{0.f, 0.f, 0.f};
  float nn = 0.f;
  float scl[NT], shf[NT];  // lrelu(acc scl + shf): the bias folded into the shift
  if constexpr (!STATS) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      scl[t] = ss[(long)b * 2 * C + 16 * t + n];
      shf[t] = fmaf(bl[t], scl[t], ss[(long)b * 2 * C + C + 16 * t + n]);
    }
  }
  for (int g = wave; g < ngrp; g += 4) {
    // A: pixel m = 16 g + (lane & 15) of the strip (one row: W % 16 == 0, so the group's row and first column are
    // wave-uniform), k-octet kq
    const int p0 = __builtin_amdgcn_readfirstlane(16 * g), r = p0 / W;
    const int base = (r * (W + 2) + p0 - r * W) * CIN;
    c3b8 ah, am, al;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = base + koff[e];
      ah[e] = c3win[idx];
      am[e] = c3win[pst + idx];
      al[e] = c3win[2 * pst + idx];
    }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wb[t][0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, wb[t][1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wb[t][2], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, wb[t][0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wb[t][1], c, 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wb[t][0], c, 0, 0, 0);
    }
    // lane (n, kq) holds y[pixel 16 g + 4 kq + i][channel 16 t + n], i = 0..3
    if constexpr (STATS) {
      // the lane's 4 values of channel 16 t + n as one chunk (its mean and m2 about it) merged into the lane's chain
      // (Chan's update, one division per group; round 5 ran a Welford step per value).  The chain runs on acc, the
      // bias joins the mean after the loop (y = acc + bias has acc's m2)
      const float nb = nn + 4.f, f = 4.f / nb, cw = nn * f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float mb = ((acc[t][0] + acc[t][1]) + (acc[t][2] + acc[t][3])) * 0.25f;
        const float d0 = acc[t][0] - mb, d1 = acc[t][1] - mb, d2 = acc[t][2] - mb, d3 = acc[t][3] - mb;
        const float q = fmaf(d3, d3, fmaf(d2, d2, fmaf(d1, d1, d0 * d0)));
        const float dl = mb - a[t].mean;
        a[t].mean = fmaf(dl, f, a[t].mean);
        a[t].m2 = fmaf(dl * dl, cw, a[t].m2 + q);
      }
      nn = nb;
    } else {
      // through the wave's LDS tile to whole channel octets per lane: 16-B fp32 stores, or the limbs
      // (damc::store_x3_octet, the F32A conv's in-register split), so both output forms carry the same values
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float tt = fmaf(acc[t][i], scl[t], shf[t]);
          c3out[wave][4 * kq + i][16 * t + n] = fmaxf(tt, tt * slope);  // lrelu for 0 <= slope <= 1 (host-checked)
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const long obase = (((long)b * H + r0 + r) * W + p0 - r * W) * C;  // wave-uniform
      if (y32) {
        // the group's 16 pixels x C channels are one contiguous run of the NHWC output: lane l of store j writes its
        // 16 B at float 4 (l + 64 j), so every store instruction covers 1 KB without gaps (round 6, late: the octet
        // form wrote two half-covered 2 KB spans per pair of stores)
#pragma unroll
        for (int it = 0; it < 16 * NT * 16 / 256; ++it) {
          const int j = lane + 64 * it, pp = j / (4 * NT), c4 = j - pp * (4 * NT);
          *reinterpret_cast<f32x4*>(y32 + obase + 4 * j) = *reinterpret_cast<const f32x4*>(&c3out[wave][pp][4 * c4]);
        }
      } else {
#pragma unroll
        for (int it = 0; it < 2 * NT * 16 / 64; ++it) {  // 16 pixels x NT * 2 octets
          const int id = lane + 64 * it, pp = id / (2 * NT), oc = id - pp * (2 * NT);
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = c3out[wave][pp][8 * oc + e];
          damc::store_x3_octet(v, y3 + 3 * (obase + (pp * (16 * NT) + 8 * oc)));  // C == 16 NT
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // the tile is rewritten by the wave's next group
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  if constexpr (STATS) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      a[t].n = nn;
      a[t].mean += bl[t];
    }
    // the four lanes of a channel (kq = 0..3), then the waves in order
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const Wf o{__shfl_xor(a[t].n, off), __shfl_xor(a[t].mean, off), __shfl_xor(a[t].m2, off)};
        a[t] = (lane & off) ? wmerge(o, a[t]) : wmerge(a[t], o);
      }
    if (kq == 0)
#pragma unroll
      for (int t = 0; t < NT; ++t) c3red[wave][16 * t + n] = a[t];
    __syncthreads();
    for (int c = threadIdx.x; c < NT * 16; c += 256) {
      Wf m = c3red[0][c];
#pragma unroll
      for (int v = 1; v < 4; ++v) m = wmerge(m, c3red[v][c]);
      float* op = part + (((long)b * C + c) * S + s) * 3;
      op[0] = m.n;
      op[1] = m.mean;
      op[2] = m.m2;
    }
  }
}

// wave reduce-scatter of N per-lane values: halving exchanges (N/2 + N/4 + ... shuffles instead of 6 N), then a plain
// butterfly over the lanes left sharing a channel; every lane returns the wave total of channel ch (fixed order)
template <int N>
__device__ __forceinline__ float wave_rsum(const float (&v)[N], int lane, int off, int& ch, int stop = 1) {
  if constexpr (N == 1) {
    float s = v[0];
    for (; off >= stop; off >>= 1) s += __shfl_xor(s, off);
    return s;
  } else {
    constexpr int H = N / 2;
    const bool hi = (lane & off) != 0;
    float nv[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float keep = hi ? v[H + i] : v[i], send = hi ? v[i] : v[H + i];
      nv[i] = keep + __shfl_xor(send, off);
    }
    ch = 2 * ch + (hi ? 1 : 0);
    return wave_rsum<H>(nv, lane, off >> 1, ch, stop);
  }
}

// The same layer in ONE pass when a sample has at most 1024 pixels (32 x 32: CIFAR-10, SVHN) and W % 4 == 0:
// grid (B, C / 16), 512 threads = 2 channel octets (one per group of 4 waves, so weights are wave-uniform) x 256
// 4-pixel row runs (1024 threads capped the kernel at 128 VGPRs and it spilled).  Each thread evaluates its 4 pixels x 8 channels with conv3_octet's arithmetic (same fmaf chain,
// so the same y; each weight read once per 4 pixels, each window value once per run), the workgroup sums them per
// channel (wave reduce-scatter, then the channel's 4 wave sums in a fixed order) for the mean, then sums
// (y - mean)^2 for the variance (two passes over registers), and writes lrelu(IN(y)) as the next convolution's limbs.
// The statistics pass, the Welford partials, the merge kernel and the recomputing second pass all drop out.
// 1-D grid: workgroup (b, C / 16 chunk) for the first nconv = B * C / 16, then the per-call limb packing of the
// limb layers' weights (pk, pack_conv_x3_block) as extra workgroups of the same launch, so the two fill the chip
// together (a separate packing launch, or one on a forked stream, costs its own ramp / the event hand-offs)
template <int CIN>
__global__ __launch_bounds__(512) void conv3_in_fused_kernel(const float* __restrict__ x, int H, int W, int C,
                                                              const float* __restrict__ w, const float* __restrict__ bias,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float eps, float slope,
                                                              unsigned short* __restrict__ y3, float* __restrict__ y32,
                                                              int nconv, damc::PackConvList pk) {
  extern __shared__ __attribute__((aligned(16))) float smf[];  // [9 CIN][16] weights, [8][8] sums, [2][16], window
  if ((int)blockIdx.x >= nconv) {  // workgroup-uniform
    damc::pack_conv_x3_block(pk, (int)blockIdx.x - nconv, threadIdx.x, 512, smf);
    return;
  }
  float* wl = smf;
  float* red = wl + 9 * CIN * 16;
  float* st = red + 8 * 8;
  float* win = st + 32;
  const int ncb = C / 16, b = blockIdx.x / ncb, c0 = (blockIdx.x - b * ncb) * 16, tid = threadIdx.x, lane = tid & 63,
            wave = tid >> 6;
  const int HW = H * W, cg = wave >> 2, run = tid & 255;  // channels c0 + 8 cg .. + 7; pixels 4 run .. + 3
  for (int i = tid; i < 9 * CIN * 16; i += 512) wl[i] = w[(i >> 4) * C + c0 + (i & 15)];
  conv3_stage<CIN>(x, b, H, W, 0, H, win);
  __syncthreads();
  const int p0 = 4 * run, r = p0 / W, x0 = p0 - r * W;
  const bool ok = p0 < HW;
  float y[4][8];
  {
    float acc[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
#pragma unroll 1
    for (int ky = 0; ky < 3; ++ky) {  // rolled: unrolled, the compiler hoisted every window and weight load and spilled
      float xr[CIN][6];  // the window row's 6 columns x0 - 1 .. x0 + 4 (padded coordinates x0 .. x0 + 5)
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
        for (int c = 0; c < 6; ++c) xr[ci][c] = ok ? win[((r + ky) * (W + 2) + x0 + c) * CIN + ci] : 0.f;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          const int t = (ky * 3 + kx) * CIN + ci;  // conv3_octet's tap order
          const f32x4 w0 = *reinterpret_cast<const f32x4*>(wl + t * 16 + 8 * cg);
          const f32x4 w1 = *reinterpret_cast<const f32x4*>(wl + t * 16 + 8 * cg + 4);
          const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[k][e] = fmaf(wv[e], xr[ci][k + kx], acc[k][e]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) y[k][e] = ok ? acc[k][e] + (bias ? bias[c0 + 8 * cg + e] : 0.f) : 0.f;
  }
  // per-channel workgroup sum of v[e] (channel c0 + 8 cg + e) into st[k * 16 + ...]
  auto block_sum = [&](const float (&v)[8], int k) {
    int ch = 0;
    const float t = wave_rsum<8>(v, lane, 32, ch);
    if ((lane & 7) == 0) red[wave * 8 + ch] = t;
    __syncthreads();
    if (tid < 16) {
      const int g = tid >> 3, e = tid & 7;  // channel 8 g + e: waves 4 g .. 4 g + 3
      st[k * 16 + tid] = ((red[(4 * g) * 8 + e] + red[(4 * g + 1) * 8 + e]) + red[(4 * g + 2) * 8 + e]) +
                         red[(4 * g + 3) * 8 + e];
    }
    __syncthreads();
  };
  const float inv_n = 1.f / (float)HW;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = ((y[0][e] + y[1][e]) + y[2][e]) + y[3][e];
  block_sum(v, 0);
  float mean[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = st[8 * cg + e] * inv_n;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = y[k][e] - mean[e];
      q = ok ? fmaf(d, d, q) : q;
    }
    v[e] = q;
  }
  block_sum(v, 1);
  if (!ok) return;
  float scl[8], shf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {  // in_merge_kernel's scale / shift form
    const int c = c0 + 8 * cg + e;
    scl[e] = (1.f / sqrtf(st[16 + 8 * cg + e] * inv_n + eps)) * gamma[c];
    shf[e] = beta[c] - mean[e] * scl[e];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float u = fmaf(y[k][e], scl[e], shf[e]);
      t[e] = u > 0.f ? u : u * slope;
    }
    const long off = ((long)b * HW + p0 + k) * C + c0 + 8 * cg;
    if (y32) {  // fp32 NHWC for an F32A next conv
      *reinterpret_cast<f32x4*>(y32 + off) = f32x4{t[0], t[1], t[2], t[3]};
      *reinterpret_cast<f32x4*>(y32 + off + 4) = f32x4{t[4], t[5], t[6], t[7]};
    } else {
      damc::store_x3_octet(t, y3 + 3 * off);
    }
  }
}

// InstanceNorm + LeakyReLU of a stored conv output (NHWC fp32) to the next convolution's limbs in ONE kernel when a
// sample has <= 256 pixels (the encoder's k4 s2 layers at 32x32 input): grid (B, C / 32), 256 threads = 64 pixel slots
// x 4 channel octets, NIT = ceil(HW / 64) pixels per thread held in registers.  Sum, then sum of squared deviations
// (two passes over registers; wave reduce-scatter + fixed-order wave sums), then in_merge_kernel's scale / shift and
// in_apply_x3_kernel's normalise + LReLU + limb store.  Replaces in_stats + in_merge + in_apply_x3 (one read of the
// activation instead of two, one launch instead of three).
template <int NIT>
// y32 != NULL: the result leaves as fp32 NHWC at y32 instead of limbs (the next conv stages it as fp32, gemm.hip
// X3_F32A); y32 may be y itself (every thread writes only the elements it read, after both block sums); chw: fp32 in
// CHW order per sample instead (the dense head's input; y32 must then be another buffer)
// slab != NULL: y was not written; the conv's ks split-K slabs (register layout of the 256 x 128 limb tiles, as
// x3_ksplit_reduce_tile_kernel reads them, sstride4 f32x4 per slab, ntn 128-channel tiles) are summed here in the
// reduce's order from 0, then the conv bias added: the reduce + epilogue's arithmetic, so the values are bitwise C's
__global__ __launch_bounds__(256) void in_fused_x3_kernel(const float* y, int HW, int C,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          float eps, float slope, unsigned short* __restrict__ y3,
                                                          float* y32, const float* __restrict__ slab, int ks, int ntn,
                                                          long sstride4, const float* __restrict__ cbias, int chw) {
  __shared__ float red[4][32];
  __shared__ float st[2][32];
  const int b = blockIdx.x, c0 = blockIdx.y * 32, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pr = tid >> 2, q = tid & 3;
  float v[NIT][8];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int p = pr + 64 * it;
    if (p < HW && slab) {
      const long m = (long)b * HW + p;
      const int n = c0 + 8 * q, rm = (int)(m & 255), rn = n & 127;
      const long tile = (m >> 8) * ntn + (n >> 7);
      const int wv = (rm >> 6) * 2 + (rn >> 6), ij = ((rm & 63) >> 4) * 4 + ((rn & 63) >> 4);
      const long base = ((tile * 8 + wv) * 16 + ij) * 64 + ((rm & 15) >> 2) * 16 + (rn & 15);  // f32x4 of element 0
      const int r = rm & 3;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[it][e] = 0.f;
      int sl = 0;
      for (; sl + 2 <= ks; sl += 2) {  // two slabs' 16 loads in flight, then their adds in slab order
        const float* s0 = slab + ((long)sl * sstride4 + base) * 4 + r;
        const float* s1 = s0 + sstride4 * 4;
        float t0[8], t1[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          t0[e] = s0[4 * e];
          t1[e] = s1[4 * e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[it][e] += t0[e];
          v[it][e] += t1[e];
        }
      }
      for (; sl < ks; ++sl) {
        const float* src = slab + ((long)sl * sstride4 + base) * 4 + r;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[it][e] += src[4 * e];
      }
      if (cbias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[it][e] += cbias[n + e];
      }
    } else if (p < HW) {
      const float* src = y + ((long)b * HW + p) * C + c0 + 8 * q;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(src), a1 = *reinterpret_cast<const f32x4*>(src + 4);
      v[it][0] = a0.x; v[it][1] = a0.y; v[it][2] = a0.z; v[it][3] = a0.w;
      v[it][4] = a1.x; v[it][5] = a1.y; v[it][6] = a1.z; v[it][7] = a1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[it][e] = 0.f;
    }
  }
  // per-channel workgroup sum of t[e] (channel c0 + 8 q + e) into st[k]
  auto block_sum = [&](const float (&t)[8], int k) {
    int ch = 0;
    const float w = wave_rsum<8>(t, lane, 32, ch, 4);  // lanes of one octet q differ in bits 2..5
    if ((lane & 4) == 0) red[wave][8 * q + ch] = w;
    __syncthreads();
    if (tid < 32) st[k][tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    __syncthreads();
  };
  const float inv_n = 1.f / (float)HW;
  float t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    t[e] = v[0][e];
#pragma unroll
    for (int it = 1; it < NIT; ++it) t[e] += v[it][e];
  }
  block_sum(t, 0);
  float mean[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = st[0][8 * q + e] * inv_n;
    t[e] = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const float d = v[it][e] - mean[e];
      t[e] = (pr + 64 * it < HW) ? fmaf(d, d, t[e]) : t[e];
    }
  }
  block_sum(t, 1);
  float scl[8], shf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + 8 * q + e;
    scl[e] = (1.f / sqrtf(st[1][8 * q + e] * inv_n + eps)) * gamma[c];
    shf[e] = beta[c] - mean[e] * scl[e];
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int p = pr + 64 * it;
    if (p >= HW) continue;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float u = fmaf(v[it][e], scl[e], shf[e]);
      o[e] = u > 0.f ? u : u * slope;
    }
    const long off = ((long)b * HW + p) * C + c0 + 8 * q;
    if (y32 && chw) {  // fp32 CHW (the dense head's rows, enc_head_x3_kernel); y32 is then not y
#pragma unroll
      for (int e = 0; e < 8; ++e) y32[((long)b * C + c0 + 8 * q + e) * HW + p] = o[e];
    } else if (y32) {
      *reinterpret_cast<f32x4*>(y32 + off) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(y32 + off + 4) = f32x4{o[4], o[5], o[6], o[7]};
    } else {
      damc::store_x3_octet(o, y3 + 3 * off);
    }
  }
}

// The encoder's last conv when it covers its whole input (k x k, stride 1, no padding, on a k x k map: every Encoder_*,
// diffusion_net.py:258-260): a Linear of the sample's CHW-flattened activation on the PyTorch weight itself, rows
// [cout][cin k k].  The limb product of the limb engine (three RNE bf16 limbs per operand, six MFMAs per K tile, one
// fp32 accumulation block per 512 k with the weight negated on odd blocks) without the limb copy of the weight: both
// operands are read as fp32 and split into limbs once per workgroup on their way into LDS.  One workgroup = 128 rows x
// 64 columns x one 512-k sign block; 8 waves of 32 x 32.  The block's sum (sign restored, exact) goes to its slab;
// enc_head_reduce_kernel adds the slabs in order and the bias.  Replaces the packing of the weight's limbs (84 MB of
// traffic at nemb = 1024) and a 64 x 128-tile limb GEMM over it.
typedef __bf16 hb8 __attribute__((ext_vector_type(8)));
constexpr int HD_BM = 128, HD_BN = 64, HD_KT = 32, HD_NEGK = 512, HD_THREADS = 512;
constexpr int HD_ROWS = HD_BM + HD_BN;                           // LDS rows per limb plane (A rows, then B rows)
constexpr size_t HD_LDS = 2 * 3 * HD_ROWS * 4 * sizeof(hb8);     // two K tiles x three limb planes: 72 KB

// 16-B slot of (row, octet q) in a limb plane of 64-B rows.  ds_read_b128 serves a wave in four groups of 16 lanes
// (MI355X_MICROARCH.md, LDS): a fragment read's group holds rows m, m + 12 (octet q) and m + 4, m + 8 (octet q ^ 1) of
// each m % 4 class; the octet swizzle by (row >> 2) & 3 (0 -> 0, 1 -> 2, 2 -> 3, 3 -> 1) gives the 16 lanes of every
// group 16 distinct slots mod 16, i.e. all 64 banks once
__device__ __forceinline__ int hd_slot(int row, int q) {
  return row * 4 + (q ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3));
}
// the engine's RNE limb split of 8 values times sg (exact: a sign)
__device__ __forceinline__ void hd_split(const f32x4 (&x)[2], float sg, hb8& h, hb8& m, hb8& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float v = sg * x[e >> 2][e & 3];
    const __bf16 b0 = (__bf16)v;
    const float r1 = sub_rn(v, (float)b0);
    const __bf16 b1 = (__bf16)r1;
    h[e] = b0;
    m[e] = b1;
    l[e] = (__bf16)sub_rn(r1, (float)b1);
  }
}

typedef __bf16 hb4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void hd_split4(const f32x4& x, float sg, hb4& h, hb4& m, hb4& l) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float v = sg * x[e];
    const __bf16 b0 = (__bf16)v;
    const float r1 = sub_rn(v, (float)b0);
    const __bf16 b1 = (__bf16)r1;
    h[e] = b0;
    m[e] = b1;
    l[e] = (__bf16)sub_rn(r1, (float)b1);
  }
}

// grid N / 64 * K / 512 * ceil(M / 128) (1-D); A [M][K] fp32 (CHW rows), W [N][K]; slab [K / 512][M][N].  PD K tiles
// of global loads in flight per thread (register stages; the K loop is unrolled so every stage index is static): at
// one workgroup per CU no other wave covers a tile's load latency
template <int PD>
__global__ __launch_bounds__(HD_THREADS) void enc_head_x3_kernel(const float* __restrict__ A,
                                                                 const float* __restrict__ W, int M, int N, int K,
                                                                 float* __restrict__ slab, int xcd) {
  extern __shared__ __attribute__((aligned(16))) hb8 hl[];  // [2 K tiles][3 limbs][HD_ROWS][4 slots]
  constexpr int NT = HD_NEGK / HD_KT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware tile order: workgroup L runs on XCD L % 8 (round-robin dispatch), so tile u = (L % 8) * (T / 8) + L / 8
  // gives each XCD a contiguous run of tiles, n fastest: a sign block's 128 x 512 A block is fetched into one XCD's
  // L2 (2 blocks per XCD at CIFAR B=128) instead of all eight
  const int T = gridDim.x, L = blockIdx.x;
  const int u = ((T & 7) || !xcd) ? L : (L & 7) * (T >> 3) + (L >> 3);
  const int nn = N / HD_BN, nkb = K / HD_NEGK, rem = u % (nn * nkb);
  const int n0 = (rem % nn) * HD_BN, kb = rem / nn, r0 = (u / (nn * nkb)) * HD_BM;
  const float sg = (kb & 1) ? -1.f : 1.f;
  // staging: thread = (row fr, octet fq) of the A tile and (row br, half octet bh) of the B tile: every thread issues
  // the same loads (no branch, so the waits can count outstanding loads per stage); rows past M (a partial last row
  // block) load row M - 1 again: an MFMA output row reads only its own A row, and those rows are never stored
  const int fr = tid >> 2, fq = tid & 3, br = tid >> 3, bh = tid & 7;
  const float* ap = A + (long)min(r0 + fr, M - 1) * K + (long)kb * HD_NEGK + 8 * fq;
  const float* bp = W + (long)(n0 + br) * K + (long)kb * HD_NEGK + 4 * bh;
  f32x4 pa[PD][2], pb[PD];
  auto gload = [&](int t, int st) {
    pa[st][0] = *reinterpret_cast<const f32x4*>(ap + t * HD_KT);
    pa[st][1] = *reinterpret_cast<const f32x4*>(ap + t * HD_KT + 4);
    pb[st] = *reinterpret_cast<const f32x4*>(bp + t * HD_KT);
  };
  auto lstore = [&](int buf, int st) {
    hb8* p = hl + buf * 3 * HD_ROWS * 4;
    hb8 h, m, l;
    hd_split(pa[st], 1.f, h, m, l);
    const int s = hd_slot(fr, fq);
    p[s] = h;
    p[HD_ROWS * 4 + s] = m;
    p[2 * HD_ROWS * 4 + s] = l;
    hb4 h4, m4, l4;
    hd_split4(pb[st], sg, h4, m4, l4);
    hb4* p4 = reinterpret_cast<hb4*>(p);
    const int s4 = 2 * hd_slot(HD_BM + br, bh >> 1) + (bh & 1);
    p4[s4] = h4;
    p4[2 * HD_ROWS * 4 + s4] = m4;
    p4[4 * HD_ROWS * 4 + s4] = l4;
  };
  const int wr = wave & 3, wc = wave >> 2, m = lane & 15, q = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < PD && st < NT; ++st) gload(st, st);
  lstore(0, 0);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    // stage t % PD held tile t, in LDS since the end of the last iteration: it takes tile t + PD
    if (t + PD < NT) gload(t + PD, t % PD);
    const hb8* p = hl + (t & 1) * 3 * HD_ROWS * 4;
    hb8 fa[2][3], fb[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int l = 0; l < 3; ++l) {
        fa[i][l] = p[l * HD_ROWS * 4 + hd_slot(32 * wr + 16 * i + m, q)];
        fb[i][l] = p[l * HD_ROWS * 4 + hd_slot(HD_BM + 32 * wc + 16 * i + m, q)];
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
      }
    if (t + 1 < NT) lstore((t + 1) & 1, (t + 1) % PD);
    __syncthreads();
  }
  float* sl = slab + (long)kb * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 32 * wr + 16 * i + 4 * q + r, col = n0 + 32 * wc + 16 * j + m;
        if (row < M) sl[(long)row * N + col] = sg * acc[i][j][r];
      }
}

// out[m][n] = (((slab 0 + slab 1) + ...) + slab nblk-1) + bias[n]   (N % 4 == 0)
// 64-thread workgroups: 512 of them at CIFAR B=128 (256-thread groups left half the CUs without one)
__global__ __launch_bounds__(64) void enc_head_reduce_kernel(const float* __restrict__ slab, int nblk, long mn4, int N,
                                                             const float* __restrict__ bias, float* __restrict__ out) {
  const long i = (long)blockIdx.x * 64 + threadIdx.x;
  if (i >= mn4) return;
  const f32x4* s = reinterpret_cast<const f32x4*>(slab);
  f32x4 v = s[i];
  int kb = 1;
  for (; kb + 8 <= nblk; kb += 8) {  // eight slabs' loads in flight, then their adds in order
    f32x4 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = s[(long)(kb + u) * mn4 + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  for (; kb < nblk; ++kb) v += s[(long)kb * mn4 + i];
  if (bias) {
    const int n = (int)((4 * i) % N);
    v += f32x4{bias[n], bias[n + 1], bias[n + 2], bias[n + 3]};
  }
  reinterpret_cast<f32x4*>(out)[i] = v;
}

}  // namespace

namespace damc {
int launch_dense_head_x3(const float* a, const float* w, const float* bias, int M, int N, int K, float* slab,
                         size_t slab_floats, float* out, hipStream_t s) {
  if (!a || !w || !slab || !out || M <= 0 || N <= 0 || N % HD_BN != 0 || K <= 0 || K % HD_NEGK != 0 ||
      (uintptr_t)a % 16 || (uintptr_t)w % 16 || (uintptr_t)slab % 16 || (uintptr_t)out % 16)
    return DAMC_ERR_UNSUPPORTED;
  const int nblk = K / HD_NEGK;
  if (slab_floats < (size_t)nblk * M * N) return DAMC_ERR_WORKSPACE;
  static const bool lds_ok = [] {
    return hipFuncSetAttribute((const void*)enc_head_x3_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)HD_LDS) == hipSuccess &&
           hipFuncSetAttribute((const void*)enc_head_x3_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)HD_LDS) == hipSuccess;
  }();
  if (!lds_ok) return DAMC_ERR_UNSUPPORTED;
  ProfScope ps("enc_head", 2.0 * M * (double)K * N * 6, s);
  const long nwg = (long)(N / HD_BN) * nblk * ((M + HD_BM - 1) / HD_BM);
  if (nwg > 0x7fffffffL) return DAMC_ERR_UNSUPPORTED;
  const dim3 g((unsigned)nwg);
  const char* pd = getenv("DAMC_ENC_HEAD_PD");  // (read per call) 1: one K tile of loads in flight (A/B)
  const char* xe = getenv("DAMC_ENC_HEAD_XCD");  // (read per call) 0: tiles in launch order (A/B)
  const int xcd = !(xe && xe[0] == '0');
  if (pd && pd[0] == '1')
    hipLaunchKernelGGL(enc_head_x3_kernel<1>, g, dim3(HD_THREADS), HD_LDS, s, a, w, M, N, K, slab, xcd);
  else
    hipLaunchKernelGGL(enc_head_x3_kernel<4>, g, dim3(HD_THREADS), HD_LDS, s, a, w, M, N, K, slab, xcd);
  const long mn4 = (long)M * N / 4;
  hipLaunchKernelGGL(enc_head_reduce_kernel, dim3((unsigned)((mn4 + 63) / 64)), dim3(64), 0, s, slab, nblk, mn4, N,
                     bias, out);
  return (int)hipGetLastError();
}
}  // namespace damc

namespace {

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
  if (dgamma && dbeta) return damc::launch_colsum2(bc, B, 2 * c, 2L * c, dgamma, dbeta, c, tmp, s);
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

// ---- the whole encoder forward in one call (damc_q_encoder_fwd): NCHW -> NHWC, then per layer the conv and
// InstanceNorm + LeakyReLU in place; two ping-pong activation buffers, the last conv writes xemb directly.
// Convolutions with cin % 32 == 0 (all but the first 3x3 at the reference's nif) run on the limb engine
// (gemm_x3_kernel, A_CONV gather with stride / pad, bias epilogue; split-K into the sign blocks when the grid would
// not fill the chip): the input activation is split into limbs per call, the weights' limb copy comes from the
// caller (damc_pack_conv2d_x3) or is split into the workspace.  The rest on the fp32 MFMA engine.
namespace {
struct EncShapes {
  int h[DAMC_MAX_ENC_LAYERS + 1], w[DAMC_MAX_ENC_LAYERS + 1];
  size_t act_max = 0, slab_max = 0, in_max = 0;
  size_t a3_max = 0, w3_max = 0, ks_max = 0;  // limb engine: activation limbs, weight limbs, split-K slabs
  size_t wsrc_off[DAMC_MAX_ENC_LAYERS] = {}, wsrc_bytes = 0;  // the limb operands packed from w_src (workspace)
  bool limb[DAMC_MAX_ENC_LAYERS] = {};
  bool first_fused = false;  // layer 0 as conv3_stats + conv3_apply_x3 (no stored conv output, no NHWC copy)
  int first_rows = 1, first_strips = 1;
  bool head_geom = false;  // the last conv fits enc_head_x3_kernel (its slabs are in ks_max)
};
size_t round256(size_t b) { return (b + 255) / 256 * 256; }

bool enc_limb_layer(const damc_encoder_t* e, const damc_enc_layer_t& L) {
  return e->engine == DAMC_ENGINE_LIMB && damc::conv_kmajor_ok(L.cin) && L.cout % 8 == 0 && L.k * L.k <= 32;
}
bool enc_shapes(const damc_encoder_t* e, int B, EncShapes* sh) {
  if (!e || B <= 0 || e->n_layers < 1 || e->n_layers > DAMC_MAX_ENC_LAYERS || e->nc <= 0 || e->h <= 0 || e->w <= 0)
    return false;
  if (e->engine != DAMC_ENGINE_LIMB && e->engine != DAMC_ENGINE_FP32) return false;
  sh->h[0] = e->h;
  sh->w[0] = e->w;
  int c = e->nc;
  sh->act_max = (size_t)B * e->h * e->w * e->nc;
  for (int i = 0; i < e->n_layers; ++i) {
    const damc_enc_layer_t& L = e->layers[i];
    if (L.cin != c || L.cout <= 0 || L.k <= 0 || L.stride <= 0 || L.pad < 0) return false;
    if ((L.in_gamma == nullptr) != (L.in_beta == nullptr)) return false;
    const int ho = (sh->h[i] + 2 * L.pad - L.k) / L.stride + 1, wo = (sh->w[i] + 2 * L.pad - L.k) / L.stride + 1;
    if (ho <= 0 || wo <= 0) return false;
    sh->h[i + 1] = ho;
    sh->w[i + 1] = wo;
    if (i + 1 < e->n_layers) sh->act_max = std::max(sh->act_max, (size_t)B * ho * wo * L.cout);
    sh->limb[i] = enc_limb_layer(e, L);
    if (!L.w_packed && !(sh->limb[i] && (L.w_x3 || L.w_src))) return false;  // the engine's weight operand
    if (L.w_src && (!sh->limb[i] || L.w_x3 || (uintptr_t)L.w_src % 16 != 0)) return false;
    if (sh->limb[i]) {
      const long M = (long)B * ho * wo, K = (long)L.k * L.k * L.cin;
      sh->a3_max = std::max(sh->a3_max, (size_t)B * sh->h[i] * sh->w[i] * L.cin * 6);
      if (L.w_src) {
        sh->wsrc_off[i] = sh->wsrc_bytes;
        sh->wsrc_bytes += round256((size_t)L.cout * K * 6);
      } else if (!L.w_x3) {
        sh->w3_max = std::max(sh->w3_max, (size_t)L.cout * K * 6);
      }
      sh->ks_max = std::max(sh->ks_max, (size_t)damc::x3_ksplit_floats((int)M, L.cout, (int)K, 1));
    } else {
      sh->slab_max = std::max(sh->slab_max,
                              damc_conv2d_workspace_floats(B, sh->h[i], sh->w[i], L.cin, L.cout, L.k, L.stride, L.pad));
    }
    if (L.in_gamma)
      sh->in_max = std::max(sh->in_max, damc_instnorm_workspace_floats(B, ho * wo, L.cout) + (size_t)B * L.cout * 2);
    c = L.cout;
  }
  const damc_enc_layer_t& F0 = e->layers[0];
  sh->first_fused = e->n_layers > 1 && sh->limb[1] && F0.k == 3 && F0.stride == 1 && F0.pad == 1 &&
                    (F0.cin == 1 || F0.cin == 3 || F0.cin == 4) && F0.cout % 64 == 0 && F0.cout <= 512 &&
                    F0.in_gamma && F0.w_packed && !damc::conv_kmajor_ok(F0.cin) && e->w <= 1024;
  if (sh->first_fused) {
    // strips per sample from the sample's shape alone, never the batch (each strip's lanes merge their statistics once,
    // a butterfly per channel octet, and in_merge_kernel merges the strips in a fixed tree: the strip partition sets the
    // rounding, so a batch sharded over ranks must keep the whole batch's partition to reproduce its xemb bit for bit;
    // round 5 took ~1024 / B strips, and 8 x B=8 CelebA-HQ shards differed from B=64 in every row,
    // tests/test_gpu_strong_scaling.py): ~512 pixels per strip, at most 64 strips, at least 128 pixels per strip
    const int want = std::max(1, std::min(64, e->h * e->w / 512));
    sh->first_rows = std::max((e->h + want - 1) / want, (128 + e->w - 1) / e->w);
    sh->first_strips = (e->h + sh->first_rows - 1) / sh->first_rows;
    sh->in_max = std::max(sh->in_max, (size_t)B * F0.cout * (sh->first_strips * 3 + 2));
    sh->a3_max = std::max(sh->a3_max, (size_t)B * e->h * e->w * F0.cout * 6);
  }
  // the dense head: the last conv covers its k x k input, reads the PyTorch weight (w_src), and the norm before it is
  // the one-pass kernel (which then writes the head's CHW rows)
  const int nl = e->n_layers - 1;
  const damc_enc_layer_t& LH = e->layers[nl];
  const long KH = (long)LH.cin * LH.k * LH.k;
  sh->head_geom = nl >= 2 && sh->limb[nl] && LH.w_src && LH.stride == 1 && LH.pad == 0 && sh->h[nl] == LH.k &&
                  sh->w[nl] == LH.k && LH.cout % HD_BN == 0 && KH % HD_NEGK == 0 && e->layers[nl - 1].in_gamma &&
                  e->layers[nl - 1].cout % 32 == 0;
  if (sh->head_geom) sh->ks_max = std::max(sh->ks_max, (size_t)(KH / HD_NEGK) * B * LH.cout);
  return true;
}

// y (B, ho, wo, cout) NHWC = conv(x3 limbs of x) + bias on the limb engine
// af32 != NULL: the input as fp32 NHWC, staged as fp32 and split into limbs in registers (X3_F32A; bitwise the limb
// input a3 = the RNE limbs of af32)
int enc_conv_x3(const unsigned short* a3, const float* af32, int B, int hin, int win, const damc_enc_layer_t& L,
                const void* w3, float* y, float* kslab, size_t kslab_floats, int* defer, hipStream_t s,
                float* in_part = nullptr, int* in_done = nullptr) {
  const int hout = (hin + 2 * L.pad - L.k) / L.stride + 1, wout = (win + 2 * L.pad - L.k) / L.stride + 1;
  damc::GemmArgs a;
  if (af32) {
    a.A = af32;
    a.a_f32 = 1;
  } else {
    a.A3 = a3;
  }
  a.Hin = hin;
  a.Win = win;
  a.Cg = L.cin;
  a.Hq = hout;
  a.Wq = wout;
  a.kw = L.k;
  a.stride = L.stride;
  a.pad_y = L.pad;
  a.pad_x = L.pad;
  a.B3 = static_cast<const unsigned short*>(w3);
  a.b_negblk = 1;  // damc::launch_split_x3_conv's layout (sign-alternating blocks)
  a.C = y;
  a.ldc = L.cout;
  a.M = B * hout * wout;
  a.N = L.cout;
  a.K = L.k * L.k * L.cin;
  a.k_per_z = a.K;
  a.bias = L.bias;
  a.bias_mod = L.cout;
  a.act = DAMC_ACT_NONE;
  a.kslab = kslab;
  a.kslab_floats = (long)kslab_floats;
  a.ksplit_deferred = defer;
  a.kwalk = damc::x3_conv_walk(L.k, L.cin);  // the weight operand's K order (every packer of it reads the same rule)
  if (in_part) {  // the norm's statistics in the epilogue where the launch allows (GemmArgs::in_part)
    a.in_part = in_part;
    a.in_hw = hout * wout;
    a.in_S = hout * wout / 256;
    a.in_done = in_done;
  }
  return damc::launch_gemm(a, damc::A_CONV, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "enc_conv",
                           2.0 * a.M * (double)L.cout * a.K, s);
}
}  // namespace

extern "C" int damc_x3_sign_block(void) { return damc::X3_NEGK; }

extern "C" int damc_x3_conv_walk(int k, int cin) { return damc::x3_conv_walk(k, cin); }

extern "C" size_t damc_conv2d_x3_bytes(int cout, int cin, int k) {
  if (cout <= 0 || cin <= 0 || k <= 0 || !damc::conv_kmajor_ok(cin) || cout % 8 != 0 || k * k > 32) return 0;
  return (size_t)cout * k * k * cin * 6;
}

extern "C" int damc_pack_conv2d_x3(const float* w, int cout, int cin, int k, void* w_x3, void* stream) {
  if (!w || !w_x3 || !damc_conv2d_x3_bytes(cout, cin, k)) return DAMC_ERR_ARG;
  return damc::launch_pack_conv_x3(w, cout, cin, k, static_cast<unsigned short*>(w_x3), as_stream(stream));
}

// one Conv2d + bias on the limb engine for the Q update's encoder forward (the training path keeps every conv output,
// so it runs the convs one by one): k4 s2 p1 layers stage their fp32 NHWC input directly (X3_F32A), other shapes split
// it into limbs in the workspace first; split-K slabs in the workspace where the output tiles would not fill the chip
extern "C" size_t damc_conv2d_x3_workspace_bytes(int B, int hin, int win, int cin, int cout, int k, int stride,
                                                 int pad) {
  if (B <= 0 || hin <= 0 || win <= 0 || stride <= 0 || pad < 0 || !damc_conv2d_x3_bytes(cout, cin, k)) return 0;
  const int hout = (hin + 2 * pad - k) / stride + 1, wout = (win + 2 * pad - k) / stride + 1;
  if (hout <= 0 || wout <= 0) return 0;
  const bool f32a = k == 4 && stride == 2 && pad == 1;
  const size_t a3 = f32a ? 0 : round256((size_t)B * hin * win * cin * 6);
  return a3 + round256((size_t)std::max<long>(damc::x3_ksplit_floats(B * hout * wout, cout, k * k * cin, 1), 1) * 4);
}

extern "C" int damc_conv2d_x3_nhwc(const float* x, int B, int hin, int win, int cin, const void* w_x3,
                                   const float* bias, int cout, int k, int stride, int pad, float* y, void* wsp,
                                   size_t wsb, void* stream) {
  const size_t need = damc_conv2d_x3_workspace_bytes(B, hin, win, cin, cout, k, stride, pad);
  if (!x || !w_x3 || !y || !need) return DAMC_ERR_ARG;
  if (!wsp || wsb < need) return DAMC_ERR_WORKSPACE;
  hipStream_t s = as_stream(stream);
  damc_enc_layer_t L{};
  L.cin = cin;
  L.cout = cout;
  L.k = k;
  L.stride = stride;
  L.pad = pad;
  L.bias = bias;
  const bool f32a = k == 4 && stride == 2 && pad == 1;
  char* base = static_cast<char*>(wsp);
  unsigned short* a3 = nullptr;
  size_t off = 0;
  if (!f32a) {
    a3 = reinterpret_cast<unsigned short*>(base);
    off = round256((size_t)B * hin * win * cin * 6);
    const int rc = damc::launch_split_x3(x, (long)B * hin * win * cin, a3, s);
    if (rc) return rc;
  }
  return enc_conv_x3(a3, f32a ? x : nullptr, B, hin, win, L, w_x3, y, reinterpret_cast<float*>(base + off),
                     (wsb - off) / 4, nullptr, s);
}

extern "C" size_t damc_q_encoder_workspace_bytes(const damc_encoder_t* e, int B) {
  EncShapes sh;
  if (!enc_shapes(e, B, &sh)) return 0;
  return 2 * round256(sh.act_max * 4) + round256(std::max<size_t>(sh.slab_max, 1) * 4) +
         round256(std::max<size_t>(sh.in_max, 1) * 4) + round256(sh.a3_max) + round256(sh.w3_max) +
         round256(sh.ks_max * 4) + sh.wsrc_bytes + 256;  // + the packing's status word (DAMC_ENC_PACK_CHECK)
}

extern "C" int damc_q_encoder_fwd(const damc_encoder_t* e, const float* x, int B, float* xemb, void* wsp, size_t wsb,
                                  void* stream) {
  EncShapes sh;
  if (!x || !xemb || !enc_shapes(e, B, &sh)) return DAMC_ERR_ARG;
  const int n = e->n_layers;
  if (sh.h[n] != 1 || sh.w[n] != 1) return DAMC_ERR_UNSUPPORTED;  // NHWC flatten == NCHW flatten only at 1 x 1
  if (!wsp || wsb < damc_q_encoder_workspace_bytes(e, B)) return DAMC_ERR_WORKSPACE;
  char* base = reinterpret_cast<char*>(wsp);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base + off;
    off += round256(bytes);
    return p;
  };
  float* buf[2];
  buf[0] = reinterpret_cast<float*>(take(sh.act_max * 4));
  buf[1] = reinterpret_cast<float*>(take(sh.act_max * 4));
  float* slabs = reinterpret_cast<float*>(take(std::max<size_t>(sh.slab_max, 1) * 4));
  float* inws = reinterpret_cast<float*>(take(std::max<size_t>(sh.in_max, 1) * 4));
  unsigned short* a3 = reinterpret_cast<unsigned short*>(take(sh.a3_max));
  unsigned short* w3 = reinterpret_cast<unsigned short*>(take(sh.w3_max));
  float* kslab = reinterpret_cast<float*>(take(sh.ks_max * 4));
  char* wsrc = sh.wsrc_bytes ? take(sh.wsrc_bytes) : nullptr;
  int* pack_err = reinterpret_cast<int*>(take(256));
  hipStream_t s = as_stream(stream);
  int rc;
  // DAMC_ENC_PACK_CHECK=1 (read per call; tests, never timed work): the packing workgroups report any workgroup outside
  // their list in a status word the call zeroes first and reads back at its end (one host sync), returning
  // DAMC_ERR_UNSUPPORTED if it was set
  const char* pc = getenv("DAMC_ENC_PACK_CHECK");
  const bool pack_check = pc && pc[0] == '1';
  if (pack_check && (rc = (int)hipMemsetAsync(pack_err, 0, sizeof(int), s))) return rc;
  const char* io = getenv("DAMC_ENC_IN_ONEPASS");  // (read per call) 0: the three-kernel norm below
  // the last conv as the dense head (enc_head_x3_kernel) where it fits; DAMC_ENC_HEAD=0 (read per call): on the limb
  // GEMM over its packed weight limbs
  const char* hde = getenv("DAMC_ENC_HEAD");
  const bool head = sh.head_geom && !(hde && hde[0] == '0') && !(io && io[0] == '0') && (uintptr_t)xemb % 16 == 0;
  // the w_src layers' limb operands, all in one launch: as extra workgroups of the one-pass first layer when it runs
  // (conv3_in_fused_kernel), else on their own before it
  damc::PackConvList pl{};
  if (wsrc) {
    for (int i = 0; i < n; ++i) {
      const damc_enc_layer_t& L = e->layers[i];
      if (!L.w_src || (head && i == n - 1)) continue;  // (the head reads the fp32 weight itself)
      unsigned short* y = reinterpret_cast<unsigned short*>(wsrc + sh.wsrc_off[i]);
      if (pl.n < 8 && damc::pack_conv_x3_many_ok(L.w_src, L.cin, L.k)) {
        pl.w[pl.n] = L.w_src;
        pl.y[pl.n] = y;
        pl.cin[pl.n] = L.cin;
        pl.taps[pl.n] = L.k * L.k;
        pl.blk0[++pl.n] = L.cout;
      } else if ((rc = damc::launch_pack_conv_x3(L.w_src, L.cout, L.cin, L.k, y, s))) {
        return rc;
      }
    }
    if (pl.n && damc::pack_conv_x3_many_prep(pl)) return DAMC_ERR_UNSUPPORTED;
    pl.err = pack_check ? pack_err : nullptr;
  }
  bool pl_done = pl.n == 0;
  bool a3_ready = false;  // a3 holds the limbs of the current layer's input (written by the previous layer's norm)
  bool in32 = false;      // or the previous layer's norm left it as fp32 NHWC in buf[i & 1] for an F32A conv
  // the k4 s2 p1 limb convs stage their input as fp32 (X3_F32A) where the norm before them can write fp32 (the
  // one-pass kernels); DAMC_ENC_F32A=0 (read per call): limbs throughout
  const char* fe = getenv("DAMC_ENC_F32A");
  const bool f32a_on = !(fe && fe[0] == '0');
  auto f32a_layer = [&](int i) {
    const damc_enc_layer_t& L = e->layers[i];
    return f32a_on && i < n && sh.limb[i] && L.k == 4 && L.stride == 2 && L.pad == 1;
  };
  int i0 = 0;
  if (sh.first_fused) {  // layer 0: conv3 + InstanceNorm + LeakyReLU straight to layer 1's limbs
    const damc_enc_layer_t& L = e->layers[0];
    const int H = e->h, W = e->w, C = L.cout, R = sh.first_rows, S = sh.first_strips;
    const size_t sm = ((size_t)(R + 2) * (W + 2) * L.cin + (size_t)9 * L.cin * C + C) * sizeof(float);
    if (sm > 65536) return DAMC_ERR_UNSUPPORTED;
    float* ssb = inws + (size_t)B * C * S * 3;
    ProfScope ps("enc_first", 2.0 * B * H * W * (double)C * 9 * L.cin * 2, s);
    // one pass (conv3_in_fused_kernel) when a sample fits 1024 threads x <= 4 pixels; DAMC_ENC_FIRST_ONEPASS=0 (read
    // per call) keeps the two recomputing passes
    const char* op = getenv("DAMC_ENC_FIRST_ONEPASS");
    const size_t sm1 = ((size_t)(H + 2) * (W + 2) * L.cin + (size_t)9 * L.cin * 16 + 8 * 8 + 32) * sizeof(float);
    // (a sample of at most 1024 pixels; CelebA-64 and larger keep the two passes)
    const bool one = !(op && op[0] == '0') && H * W <= 1024 && W % 4 == 0 && C % 16 == 0 && sm1 <= 65536;
    if (!one && !pl_done) {
      if ((rc = damc::launch_pack_conv_x3_many(pl, s))) return rc;
      pl_done = true;
    }
    const int nconv = B * (C / 16), npk = pl_done ? 0 : pl.blk0[pl.n];
    float* y32 = f32a_layer(1) ? buf[1] : nullptr;
    const size_t smp = std::max(sm1, pl_done ? (size_t)0 : (size_t)pl.lds);
#define DAMC_C1(CIN_)                                                                                               \
  if (one && L.cin == CIN_) {                                                                                       \
    hipLaunchKernelGGL((conv3_in_fused_kernel<CIN_>), dim3(nconv + npk), dim3(512), smp, s, x, H, W, C, L.w_packed,  \
                       L.bias, L.in_gamma, L.in_beta, L.in_eps, L.slope, a3, y32, nconv, pl);                       \
    pl_done = true;                                                                                                 \
  }
    DAMC_C1(1) DAMC_C1(3) DAMC_C1(4)
#undef DAMC_C1
#define DAMC_C3(CIN_, PX_, PA_)                                                                                     \
  if (!one && !mf && L.cin == CIN_ && px == PX_) {                                                                  \
    hipLaunchKernelGGL((conv3_stats_kernel<CIN_, PX_>), dim3(B, S), dim3(256), sm, s, x, H, W, C, R, L.w_packed,     \
                       L.bias, inws);                                                                               \
    hipLaunchKernelGGL(in_merge_kernel, dim3((B * C + 3) / 4), dim3(256), 0, s, inws, B, C, S, L.in_gamma,        \
                       L.in_beta, L.in_eps, ssb);                                                                   \
    hipLaunchKernelGGL((conv3_apply_x3_kernel<CIN_, PA_>), dim3(B, S), dim3(256), sm, s, x, H, W, C, R, L.w_packed,  \
                       L.bias, ssb, L.slope, a3, y32);                                                              \
  }
    // round 6: both passes on the limb MFMA (conv3_mfma_kernel; CelebA-HQ B=64 first layer 0.87 -> see DESIGN.md) where
    // K = 9 CIN fits one K tile, C is 64 or 128, rows are whole 16-pixel groups and the next conv stages fp32;
    // DAMC_ENC_FIRST_MFMA=0 (read per call) keeps the fmaf-chain passes below
    const char* fmf = getenv("DAMC_ENC_FIRST_MFMA");
    const size_t smw = 3 * (size_t)(R + 2) * (W + 2) * L.cin * sizeof(__bf16);  // + ~11 KB static
    const bool mf = !one && !(fmf && fmf[0] == '0') && (L.cin == 1 || L.cin == 3) && (C == 64 || C == 128) &&
                    W % 16 == 0 && smw <= 49152 && L.slope >= 0.f && L.slope <= 1.f;
#define DAMC_C3M(CIN_, NT_)                                                                                          \
  if (mf && L.cin == CIN_ && C == 16 * NT_) {                                                                        \
    hipLaunchKernelGGL((conv3_mfma_kernel<CIN_, NT_, true>), dim3(B, S), dim3(256), smw, s, x, H, W, C, R, L.w_packed,\
                       L.bias, inws, nullptr, 0.f, nullptr, nullptr);                                                \
    hipLaunchKernelGGL(in_merge_kernel, dim3((B * C + 3) / 4), dim3(256), 0, s, inws, B, C, S, L.in_gamma,        \
                       L.in_beta, L.in_eps, ssb);                                                                   \
    hipLaunchKernelGGL((conv3_mfma_kernel<CIN_, NT_, false>), dim3(B, S), dim3(256), smw, s, x, H, W, C, R,           \
                       L.w_packed, L.bias, nullptr, ssb, L.slope, y32, a3);                                          \
  }
    DAMC_C3M(1, 4) DAMC_C3M(3, 4) DAMC_C3M(1, 8) DAMC_C3M(3, 8)
#undef DAMC_C3M
    // runs of 4 pixels per lane in the statistics pass (the apply pass keeps one: its 2- and 4-pixel forms took 256 VGPRs)
    // where the rows allow it (DAMC_ENC_FIRST_PX=1, read per call: one pixel per lane)
    const char* fpx = getenv("DAMC_ENC_FIRST_PX");
    const int px = (W % 4 == 0 && !(fpx && fpx[0] == '1')) ? 4 : 1;
    DAMC_C3(1, 1, 1) DAMC_C3(3, 1, 1) DAMC_C3(4, 1, 1) DAMC_C3(1, 4, 1) DAMC_C3(3, 4, 1) DAMC_C3(4, 4, 1)
#undef DAMC_C3
    DAMC_LAUNCH_CHECK();
    in32 = y32 != nullptr;
    a3_ready = !in32;
    i0 = 1;
  } else if ((rc = damc_nchw_to_nhwc(x, B, e->nc, e->h * e->w, buf[0], stream))) {
    return rc;
  }
  if (!pl_done && (rc = damc::launch_pack_conv_x3_many(pl, s))) return rc;
  const char* isl = getenv("DAMC_ENC_IN_SLABS");   // (read per call) 0: the split-K reduce kernel writes C first
  for (int i = i0; i < n; ++i) {
    const damc_enc_layer_t& L = e->layers[i];
    float* out = (i + 1 == n) ? xemb : buf[(i + 1) & 1];
    const int hw = sh.h[i + 1] * sh.w[i + 1];
    if (head && i == n - 1) {  // its CHW rows are in buf[(i + 1) & 1] (written by the norm before it)
      if ((rc = damc::launch_dense_head_x3(buf[(i + 1) & 1], L.w_src, L.bias, B, L.cout, L.cin * L.k * L.k, kslab,
                                           sh.ks_max, xemb, s)))
        return rc;
      continue;
    }
    // the norm after this conv is the one-pass kernel; it then also sums the conv's split-K slabs itself
    const bool in1 = L.in_gamma && i + 1 < n && sh.limb[i + 1] && L.cout % 32 == 0 && hw <= 256 && !(io && io[0] == '0');
    // the three-kernel norm on 256-pixel strips, its statistics taken in the conv's epilogue (round 6; GemmArgs::in_part;
    // in_strip_stats_kernel where the conv ran split): the stats pass's read of the conv output is gone (CelebA-HQ
    // B=64: 537 + 268 + 67 MB).  DAMC_ENC_IN_STRIP=0 (read per call) keeps in_stats_kernel's partition
    const char* istr = getenv("DAMC_ENC_IN_STRIP");
    const bool strip = L.in_gamma && !in1 && i + 1 < n && sh.limb[i + 1] && L.cout % 8 == 0 && sh.limb[i] &&
                       hw % 256 == 0 && hw / 256 <= 64 && !(istr && istr[0] == '0');
    int strip_done = 1;
    int ks_def = 0;
    if (sh.limb[i]) {
      if (!a3_ready && !in32) {
        const long na = (long)B * sh.h[i] * sh.w[i] * L.cin;
        if ((rc = damc::launch_split_x3(buf[i & 1], na, a3, s))) return rc;
      }
      const void* wl = L.w_x3 ? L.w_x3 : L.w_src ? static_cast<const void*>(wsrc + sh.wsrc_off[i]) : nullptr;
      if (!wl) {  // the limb copy from the fp32 packing
        const int K = L.k * L.k * L.cin;
        if ((rc = damc::x3_conv_walk(L.k, L.cin)
                      ? damc::launch_split_x3_walk(L.w_packed, (long)L.cout * K, K, L.cin, w3, s)
                      : damc::launch_split_x3_conv(L.w_packed, (long)L.cout * K, K, L.cin, w3, s)))
          return rc;
        wl = w3;
      }
      if ((rc = enc_conv_x3(a3, in32 ? buf[i & 1] : nullptr, B, sh.h[i], sh.w[i], L, wl, out, kslab, sh.ks_max,
                            (in1 && !(isl && isl[0] == '0')) ? &ks_def : nullptr, s, strip ? inws : nullptr,
                            strip ? &strip_done : nullptr)))
        return rc;
    } else {
      const size_t nsl = damc_conv2d_workspace_floats(B, sh.h[i], sh.w[i], L.cin, L.cout, L.k, L.stride, L.pad);
      if ((rc = damc_conv2d_nhwc(buf[i & 1], B, sh.h[i], sh.w[i], L.cin, L.w_packed, L.bias, L.cout, L.k, L.stride,
                                 L.pad, out, nsl ? slabs : nullptr, nsl, stream)))
        return rc;
    }
    a3_ready = false;
    in32 = false;
    if (!L.in_gamma) continue;
    if (in1) {
      ProfScope ps("instnorm", 0.0, s);
      const dim3 g(B, L.cout / 32);
      // in place: the next conv's fp32 input; before the head: its CHW rows, into this layer's (consumed) input buffer
      const int chw = head && i + 2 == n;
      float* y32 = chw ? buf[i & 1] : f32a_layer(i + 1) ? out : nullptr;
      const int ntn = (L.cout + 127) / 128;
      const long sstride4 = (long)((B * hw + 255) / 256) * ntn * (256 * 128 / 4);
      const float* sl = ks_def > 0 ? kslab : nullptr;
      if (hw <= 64)
        hipLaunchKernelGGL(in_fused_x3_kernel<1>, g, dim3(256), 0, s, out, hw, L.cout, L.in_gamma, L.in_beta, L.in_eps,
                           L.slope, a3, y32, sl, ks_def, ntn, sstride4, L.bias, chw);
      else if (hw <= 128)
        hipLaunchKernelGGL(in_fused_x3_kernel<2>, g, dim3(256), 0, s, out, hw, L.cout, L.in_gamma, L.in_beta, L.in_eps,
                           L.slope, a3, y32, sl, ks_def, ntn, sstride4, L.bias, chw);
      else
        hipLaunchKernelGGL(in_fused_x3_kernel<4>, g, dim3(256), 0, s, out, hw, L.cout, L.in_gamma, L.in_beta, L.in_eps,
                           L.slope, a3, y32, sl, ks_def, ntn, sstride4, L.bias, chw);
      DAMC_LAUNCH_CHECK();
      in32 = y32 != nullptr;
      a3_ready = !in32;
    } else if (i + 1 < n && sh.limb[i + 1] && L.cout % 8 == 0) {  // the norm writes the next convolution's limbs
      const int S = strip ? hw / 256 : in_splits(hw), cg = (L.cout + 63) / 64;
      float* ssb = inws + (size_t)B * L.cout * S * 3;
      ProfScope ps("instnorm", 0.0, s);
      if (!strip)
        hipLaunchKernelGGL(in_stats_kernel, dim3(B * cg, S), dim3(256), 0, s, out, B, hw, L.cout, S, inws);
      else if (!strip_done)
        hipLaunchKernelGGL(in_strip_stats_kernel, dim3(S, B, (L.cout + 127) / 128), dim3(512), 0, s, out, hw, L.cout,
                           inws);
      hipLaunchKernelGGL(in_merge_kernel, dim3((B * L.cout + 3) / 4), dim3(256), 0, s, inws, B, L.cout, S,
                         L.in_gamma, L.in_beta, L.in_eps, ssb);
      const long n8 = (long)B * hw * (L.cout / 8);
      float* y32 = f32a_layer(i + 1) ? out : nullptr;  // in place: the next conv's fp32 input
      if (y32) {
        const long n4 = 2 * n8;
        hipLaunchKernelGGL(in_apply_f32_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, out, n4, hw,
                           L.cout, ssb, L.slope);
      } else {
        hipLaunchKernelGGL(in_apply_x3_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, out, n8, hw,
                           L.cout, ssb, L.slope, a3, y32);
      }
      DAMC_LAUNCH_CHECK();
      in32 = y32 != nullptr;
      a3_ready = !in32;
    } else if ((rc = damc_instnorm_lrelu_nhwc(out, B, hw, L.cout, L.in_gamma, L.in_beta, L.in_eps, L.slope, inws,
                                              stream))) {
      return rc;
    }
  }
  if (pack_check) {
    int flag = 0;
    if ((rc = (int)hipMemcpyAsync(&flag, pack_err, sizeof(int), hipMemcpyDeviceToHost, s))) return rc;
    if ((rc = (int)hipStreamSynchronize(s))) return rc;
    if (flag) return DAMC_ERR_UNSUPPORTED;
  }
  return 0;
}

