// generator.hip — ConvTranspose generator forward + input-gradient (J_G^T) and the posterior
// Langevin loop (sample_langevin_post_z_with_prior, workspace/src/MCMC.py:48-74).
//
// Layout in HBM: every hidden activation is NHWC fp32 (channels contiguous = the GEMM K axis);
// the caller's x / x_hat stay NCHW.  Per step:
//   fwd : PROJ (GEMM z.W, bias+lrelu)  ->  UP2 x n (4-phase implicit GEMM, bias+lrelu)
//         -> SMALLC (to-RGB conv, tanh, residual delta = (x_hat - x)/s^2 * (1 - x_hat^2))
//   bwd : SMALLC dgrad * lrelu'  ->  UP2 dgrad (stride-2 conv implicit GEMM) * lrelu'
//         -> PROJ dgrad (split-K GEMM into slabs)  ->  fused EBM grad + slab sum + z update
// dgrad outputs overwrite the activation they are masked with (same thread reads h, writes dh).
#include <cstdlib>
#include <mutex>
#include <vector>

#include "gemm.h"
#include "wgrad.h"

using damc::GemmArgs;

int damc_launch_posterior_update(const damc_ebm_t* e, float* z, const float* slabs, int nslab, long slab_stride, int B,
                                 int nz, double step, int with_noise, const float* noise, uint64_t seed,
                                 uint64_t step_idx, uint64_t chain_base, float* diag, hipStream_t s,
                                 unsigned short* z3 = nullptr, bool* wrote_z3 = nullptr);
bool damc_posterior_update_fusable(const damc_ebm_t* e, int nz);

namespace {

// ------------------------------------------------------------------------------ packing
// PROJ: w (Cin,Cout,k,k) -> fwd [ci][(oy,ox,co)], bwd [(oy,ox,co)][ci]
__global__ void pack_proj_kernel(const float* w, int cin, int cout, int k, float* wf, float* wb) {
  const long n = (long)cin * cout * k * k;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // i enumerates torch layout
  long t = i;
  const int kx = (int)(t % k);
  t /= k;
  const int ky = (int)(t % k);
  t /= k;
  const int co = (int)(t % cout);
  const int ci = (int)(t / cout);
  const long col = ((long)ky * k + kx) * cout + co;
  const float v = w[i];
  wf[(long)ci * ((long)k * k * cout) + col] = v;
  wb[col * cin + ci] = v;
}
// UP2 (k4 s2 p1): fwd [phase(py,px)][ty][tx][ci][co] = W[ci][co][3-py-2ty][3-px-2tx];
//                 bwd [ky][kx][co][ci] = W[ci][co][ky][kx]
// or, for the K-major engine (conv_kmajor_ok of the gathered channel count), the same matrices
// transposed to [n][k]: fwd [phase][co][ty][tx][ci], bwd [ci][ky][kx][co]
__global__ void pack_up2_kernel(const float* w, int cin, int cout, int km_f, int km_b, float* wf, float* wb) {
  const long n = (long)cin * cout * 16;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  long t = i;
  const int kx = (int)(t % 4);
  t /= 4;
  const int ky = (int)(t % 4);
  t /= 4;
  const int co = (int)(t % cout);
  const int ci = (int)(t / cout);
  const float v = w[i];
  // ky = 3 - py - 2 ty  ->  py = (3 - ky) & 1, ty = (3 - ky - py) / 2
  const int py = (3 - ky) & 1, ty = (3 - ky - py) >> 1;
  const int px = (3 - kx) & 1, tx = (3 - kx - px) >> 1;
  const int phase = py * 2 + px;
  if (km_f)
    wf[(((long)phase * cout + co) * 4 + ty * 2 + tx) * cin + ci] = v;
  else
    wf[((((long)phase * 2 + ty) * 2 + tx) * cin + ci) * cout + co] = v;
  if (km_b)
    wb[(((long)ci * 4 + ky) * 4 + kx) * cout + co] = v;
  else
    wb[(((long)ky * 4 + kx) * cout + co) * cin + ci] = v;
}
// SMALLC: fwd [ky][kx][ci][co]; bwd (the two-stage projection) [(ky*k+kx)*cout + co][ci] (rows padded
// to a multiple of 32 with zeros by the caller's memset)
__global__ void pack_smallc_kernel(const float* w, int cin, int cout, int k, float* wf, float* wb) {
  const long n = (long)cin * cout * k * k;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  long t = i;
  const int kx = (int)(t % k);
  t /= k;
  const int ky = (int)(t % k);
  t /= k;
  const int co = (int)(t % cout);
  const int ci = (int)(t / cout);
  wf[(((long)ky * k + kx) * cin + ci) * cout + co] = w[i];
  if (wb) wb[((long)(ky * k + kx) * cout + co) * cin + ci] = w[i];
}
// LINEAR: w (out,in): fwd = W^T (in,out), bwd = W (out,in)
__global__ void pack_linear_kernel(const float* w, int in, int out, float* wf, float* wb) {
  const long n = (long)in * out;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long o = i / in, c = i - o * in;
  wf[c * out + o] = w[i];
  wb[i] = w[i];
}

// ---------------------------------------------------------------- small-Cout output layer
// One wave per output pixel, lanes across input channels; weights staged once per
// workgroup in LDS as [tap][ci][co] and the grid strides over pixels.
template <int NC>
__global__ __launch_bounds__(256) void smallc_fwd_kernel(const float* h, int B, int Hin, int Win, int Cin, int k,
                                                         int stride, int pad, int Hout, int Wout, const float* wpk,
                                                         const float* bias, const float* x, float inv_s2,
                                                         float* delta, float* xhat, float* sqerr_sum) {
  extern __shared__ __attribute__((aligned(16))) float wl[];
  const int nw = k * k * Cin * NC;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) wl[i] = wpk[i];
  __shared__ float red[4];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long npix = (long)B * Hout * Wout;
  float sq_local = 0.f;
  for (long pix = (long)blockIdx.x * 4 + wave; pix < npix; pix += (long)gridDim.x * 4) {
    const int b = (int)(pix / ((long)Hout * Wout));
    const int rem = (int)(pix - (long)b * Hout * Wout);
    const int oy = rem / Wout, ox = rem - oy * Wout;
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.f;
    for (int ky = 0; ky < k; ++ky) {
      const int ty = oy + pad - ky;
      if (ty < 0 || ty % stride) continue;
      const int iy = ty / stride;
      if (iy >= Hin) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int tx = ox + pad - kx;
        if (tx < 0 || tx % stride) continue;
        const int ix = tx / stride;
        if (ix >= Win) continue;
        const float* hp = h + (((long)b * Hin + iy) * Win + ix) * Cin;
        const float* wp = wl + (ky * k + kx) * Cin * NC;
        for (int ci = lane; ci < Cin; ci += 64) {
          const float hv = hp[ci];
#pragma unroll
          for (int c = 0; c < NC; ++c) acc[c] = fmaf(hv, wp[ci * NC + c], acc[c]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = wave_sum(acc[c]);
    if (lane < NC) {
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c == lane) a = acc[c];
      a += bias ? bias[lane] : 0.f;
      const float t = tanhf(a);
      const long nchw = (((long)b * NC + lane) * Hout + oy) * Wout + ox;
      if (xhat) xhat[nchw] = t;
      if (delta) {
        const float r = t - x[nchw];
        delta[pix * NC + lane] = r * inv_s2 * (1.f - t * t);
        sq_local += r * r;
      }
    }
  }
  if (sqerr_sum) {
    sq_local = wave_sum(sq_local);
    if (lane == 0) red[wave] = sq_local;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(sqerr_sum, (red[0] + red[1] + red[2] + red[3]) * (0.5f * inv_s2));
  }
}

// dh[b,iy,ix,ci] = lrelu'(h) * sum_{ky,kx,co} delta[b, iy*s-p+ky, ix*s-p+kx, co] W[ci][co][ky][kx]
// written in place over h.
template <int NC>
__global__ __launch_bounds__(256) void smallc_dgrad_kernel(float* h, int B, int Hin, int Win, int Cin, int k,
                                                           int stride, int pad, int Hout, int Wout, const float* wpk,
                                                           const float* delta, int mask_act, float mask_slope) {
  extern __shared__ __attribute__((aligned(16))) float wl[];
  const int nw = k * k * Cin * NC;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) wl[i] = wpk[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long npix = (long)B * Hin * Win;
  for (long pix = (long)blockIdx.x * 4 + wave; pix < npix; pix += (long)gridDim.x * 4) {
    const int b = (int)(pix / ((long)Hin * Win));
    const int rem = (int)(pix - (long)b * Hin * Win);
    const int iy = rem / Win, ix = rem - iy * Win;
    float* hp = h + pix * Cin;
    for (int ci0 = 0; ci0 < Cin; ci0 += 64) {
      const int ci = ci0 + lane;
      float acc = 0.f;
      for (int ky = 0; ky < k; ++ky) {
        const int oy = iy * stride - pad + ky;
        if (oy < 0 || oy >= Hout) continue;
        for (int kx = 0; kx < k; ++kx) {
          const int ox = ix * stride - pad + kx;
          if (ox < 0 || ox >= Wout) continue;
          const float* dp = delta + (((long)b * Hout + oy) * Wout + ox) * NC;
          if (ci < Cin) {
            const float* wp = wl + ((ky * k + kx) * Cin + ci) * NC;
#pragma unroll
            for (int c = 0; c < NC; ++c) acc = fmaf(dp[c], wp[c], acc);
          }
        }
      }
      if (ci < Cin) hp[ci] = acc * act_grad_from_out(hp[ci], mask_act, mask_slope);
    }
  }
}

// ---- register-resident variants (the BASELINE shapes): a group of G = Cin/CH lanes owns one pixel,
// lane g holds channels [g*CH, g*CH+CH) and ALL their weights (K*K*CH*NC floats) in VGPRs for the
// whole launch; activations move as float4/float2 channel vectors (one coalesced 16*G-byte row per
// group), the NC partial dots are reduced across the group with xor-shuffles.
template <int CH>
struct VecT;
template <>
struct VecT<4> {
  typedef f32x4 T;
};
template <>
struct VecT<2> {
  typedef float __attribute__((ext_vector_type(2))) T;
};

template <int NC, int K, int S, int CH>
__global__ __launch_bounds__(256) void smallc_fwd_reg_kernel(const float* __restrict__ h, int B, int Hin, int Win,
                                                             int Cin, int pad, int Hout, int Wout,
                                                             const float* __restrict__ wpk,
                                                             const float* __restrict__ bias, const float* x,
                                                             float inv_s2, float* delta, float* xhat,
                                                             float* sqerr_sum) {
  typedef typename VecT<CH>::T V;
  __shared__ float red[4];
  const int G = Cin / CH, P = 64 / G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane % G, sub = lane / G;
  const int ci0 = g * CH;
  float w[K * K][CH][NC];
#pragma unroll
  for (int t = 0; t < K * K; ++t)
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int o = 0; o < NC; ++o) w[t][c][o] = wpk[((long)t * Cin + ci0 + c) * NC + o];
  float bo[NC];
#pragma unroll
  for (int o = 0; o < NC; ++o) bo[o] = bias ? bias[o] : 0.f;
  const long npix = (long)B * Hout * Wout;
  float sq_local = 0.f;
  const long step = (long)gridDim.x * 4 * P;
  for (long pix0 = ((long)blockIdx.x * 4 + wave) * P; pix0 < npix; pix0 += step) {
    const long pix = pix0 + sub;
    const bool live = pix < npix;
    const long pp = live ? pix : 0;
    const int b = (int)(pp / ((long)Hout * Wout));
    const int rem = (int)(pp - (long)b * Hout * Wout);
    const int oy = rem / Wout, ox = rem - oy * Wout;
    static_assert(S == 1, "stride-2 output layers use smallc_fwd_s2_kernel");
    // all K*K taps are loaded unconditionally (border taps clamped + zero-weighted) so the loads
    // issue back to back instead of serialising their latency behind per-tap branches
    V hv[K * K];
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy + pad - ky;
      const int iyc = min(max(iy, 0), Hin - 1);
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int ix = ox + pad - kx;
        const int ixc = min(max(ix, 0), Win - 1);
        hv[ky * K + kx] = *reinterpret_cast<const V*>(h + (((long)b * Hin + iyc) * Win + ixc) * Cin + ci0);
        const float m = (iy == iyc && ix == ixc) ? 1.f : 0.f;
        hv[ky * K + kx] *= m;
      }
    }
    float acc[NC];
#pragma unroll
    for (int o = 0; o < NC; ++o) acc[o] = 0.f;
#pragma unroll
    for (int t = 0; t < K * K; ++t)
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int o = 0; o < NC; ++o) acc[o] = fmaf(hv[t][c], w[t][c][o], acc[o]);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1)
      if (off < G)
#pragma unroll
        for (int o = 0; o < NC; ++o) acc[o] += __shfl_xor(acc[o], off, 64);
    if (g == 0 && live) {
#pragma unroll
      for (int o = 0; o < NC; ++o) {
        const float t = tanhf(acc[o] + bo[o]);
        const long nchw = (((long)b * NC + o) * Hout + oy) * Wout + ox;
        if (xhat) xhat[nchw] = t;
        if (delta) {
          const float r = t - x[nchw];
          delta[pix * NC + o] = r * inv_s2 * (1.f - t * t);
          sq_local += r * r;
        }
      }
    }
  }
  if (sqerr_sum) {
    sq_local = wave_sum(sq_local);
    if (lane == 0) red[wave] = sq_local;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(sqerr_sum, (red[0] + red[1] + red[2] + red[3]) * (0.5f * inv_s2));
  }
}

// k4 s2 p1 forward: a pixel group owns the output QUAD (2qy+py, 2qx+px), py,px in {0,1}, whose 16
// taps are exactly the 3x3 input neighbourhood (qy+dy, qx+dx) with ky = 1 + py - 2dy (0..3), so each
// input vector is loaded once and every tap index is a compile-time constant.
template <int NC, int CH>
__global__ __launch_bounds__(256) void smallc_fwd_s2_kernel(const float* __restrict__ h, int B, int Hin, int Win,
                                                            int Cin, const float* __restrict__ wpk,
                                                            const float* __restrict__ bias, const float* x,
                                                            float inv_s2, float* delta, float* xhat,
                                                            float* sqerr_sum) {
  typedef typename VecT<CH>::T V;
  constexpr int K = 4;
  __shared__ float red[4];
  const int G = Cin / CH, P = 64 / G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane % G, sub = lane / G;
  const int ci0 = g * CH;
  const int Hout = 2 * Hin, Wout = 2 * Win;
  float w[K * K][CH][NC];
#pragma unroll
  for (int t = 0; t < K * K; ++t)
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int o = 0; o < NC; ++o) w[t][c][o] = wpk[((long)t * Cin + ci0 + c) * NC + o];
  float bo[NC];
#pragma unroll
  for (int o = 0; o < NC; ++o) bo[o] = bias ? bias[o] : 0.f;
  const long nq = (long)B * Hin * Win;
  float sq_local = 0.f;
  const long step = (long)gridDim.x * 4 * P;
  for (long q0 = ((long)blockIdx.x * 4 + wave) * P; q0 < nq; q0 += step) {
    const long q = q0 + sub;
    const bool live = q < nq;
    const long qq = live ? q : 0;
    const int b = (int)(qq / ((long)Hin * Win));
    const int rem = (int)(qq - (long)b * Hin * Win);
    const int qy = rem / Win, qx = rem - qy * Win;
    V hv[3][3];
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int iy = qy + dy, iyc = min(max(iy, 0), Hin - 1);
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int ix = qx + dx, ixc = min(max(ix, 0), Win - 1);
        V v = *reinterpret_cast<const V*>(h + (((long)b * Hin + iyc) * Win + ixc) * Cin + ci0);
        v *= (iy == iyc && ix == ixc) ? 1.f : 0.f;
        hv[dy + 1][dx + 1] = v;
      }
    }
    float acc[2][2][NC];
#pragma unroll
    for (int py = 0; py < 2; ++py)
#pragma unroll
      for (int px = 0; px < 2; ++px) {
#pragma unroll
        for (int o = 0; o < NC; ++o) acc[py][px][o] = 0.f;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
          const int ky = 1 + py - 2 * dy;
          if (ky < 0 || ky > 3) continue;  // compile-time
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) {
            const int kx = 1 + px - 2 * dx;
            if (kx < 0 || kx > 3) continue;
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
              for (int o = 0; o < NC; ++o)
                acc[py][px][o] = fmaf(hv[dy + 1][dx + 1][c], w[ky * K + kx][c][o], acc[py][px][o]);
          }
        }
      }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1)
      if (off < G)
#pragma unroll
        for (int py = 0; py < 2; ++py)
#pragma unroll
          for (int px = 0; px < 2; ++px)
#pragma unroll
            for (int o = 0; o < NC; ++o) acc[py][px][o] += __shfl_xor(acc[py][px][o], off, 64);
    if (g == 0 && live) {
#pragma unroll
      for (int py = 0; py < 2; ++py)
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          const int oy = 2 * qy + py, ox = 2 * qx + px;
          const long pix = ((long)b * Hout + oy) * Wout + ox;
#pragma unroll
          for (int o = 0; o < NC; ++o) {
            const float t = tanhf(acc[py][px][o] + bo[o]);
            const long nchw = (((long)b * NC + o) * Hout + oy) * Wout + ox;
            if (xhat) xhat[nchw] = t;
            if (delta) {
              const float r = t - x[nchw];
              delta[pix * NC + o] = r * inv_s2 * (1.f - t * t);
              sq_local += r * r;
            }
          }
        }
    }
  }
  if (sqerr_sum) {
    sq_local = wave_sum(sq_local);
    if (lane == 0) red[wave] = sq_local;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(sqerr_sum, (red[0] + red[1] + red[2] + red[3]) * (0.5f * inv_s2));
  }
}

template <int NC, int K, int S, int CH>
__global__ __launch_bounds__(256) void smallc_dgrad_reg_kernel(float* h, int B, int Hin, int Win, int Cin, int pad,
                                                               int Hout, int Wout, const float* __restrict__ wpk,
                                                               const float* __restrict__ delta, int mask_act,
                                                               float mask_slope, unsigned short* __restrict__ h3) {
  typedef typename VecT<CH>::T V;
  const int G = Cin / CH, P = 64 / G;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane % G, sub = lane / G;
  const int ci0 = g * CH;
  float w[K * K][CH][NC];
#pragma unroll
  for (int t = 0; t < K * K; ++t)
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int o = 0; o < NC; ++o) w[t][c][o] = wpk[((long)t * Cin + ci0 + c) * NC + o];
  const long npix = (long)B * Hin * Win;
  const long step = (long)gridDim.x * 4 * P;
  for (long pix0 = ((long)blockIdx.x * 4 + wave) * P; pix0 < npix; pix0 += step) {
    const long pix = pix0 + sub;
    if (pix >= npix) continue;
    const int b = (int)(pix / ((long)Hin * Win));
    const int rem = (int)(pix - (long)b * Hin * Win);
    const int iy = rem / Win, ix = rem - iy * Win;
    V* hp = reinterpret_cast<V*>(h + pix * Cin + ci0);
    V hv = *hp;  // issued first: its latency overlaps the delta gathers
    float d[K * K][NC];
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int oy = iy * S - pad + ky;
      const int oyc = min(max(oy, 0), Hout - 1);
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int ox = ix * S - pad + kx;
        const int oxc = min(max(ox, 0), Wout - 1);
        const float* dp = delta + (((long)b * Hout + oyc) * Wout + oxc) * NC;
        const float m = (oy == oyc && ox == oxc) ? 1.f : 0.f;
#pragma unroll
        for (int o = 0; o < NC; ++o) d[ky * K + kx][o] = dp[o] * m;
      }
    }
    float acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = 0.f;
#pragma unroll
    for (int t = 0; t < K * K; ++t)
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int o = 0; o < NC; ++o) acc[c] = fmaf(d[t][o], w[t][c][o], acc[c]);
#pragma unroll
    for (int c = 0; c < CH; ++c) hv[c] = acc[c] * act_grad_from_out(hv[c], mask_act, mask_slope);
    if (h3) {
      // limbs only (the limb engine reads this gradient); h keeps the activation.  x3 layout:
      // pixel row of 3*Cin bf16, channel octet o at 24 o, limb l at + 8 l
      unsigned short* q = h3 + pix * 3 * Cin + (ci0 >> 3) * 24 + (ci0 & 7);
      typedef unsigned short U __attribute__((ext_vector_type(CH)));
      U lh, lm, ll;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const __bf16 b0 = (__bf16)hv[c];
        const float r1 = sub_rn(hv[c], (float)b0);
        const __bf16 b1 = (__bf16)r1;
        const __bf16 b2 = (__bf16)(sub_rn(r1, (float)b1));
        lh[c] = __builtin_bit_cast(unsigned short, b0);
        lm[c] = __builtin_bit_cast(unsigned short, b1);
        ll[c] = __builtin_bit_cast(unsigned short, b2);
      }
      *reinterpret_cast<U*>(q) = lh;
      *reinterpret_cast<U*>(q + 8) = lm;
      *reinterpret_cast<U*>(q + 16) = ll;
    } else {
      *hp = hv;
    }
  }
}

// k3 s1 p1 output-layer dgrad (CIFAR-10): a block owns R input rows of one image and stages the
// (R+2) x (W+2) x NC delta window (zero border) in LDS once, so the 9 taps read LDS broadcasts instead
// of per-pixel global gathers; lanes own 4 channels of a pixel and each wave walks its pixels UNR at a
// time (UNR activation loads in flight).  Output: the masked gradient as fp32 in place, or (h3) as x3
// limbs only, lane pairs exchanging halves so every store is a whole 16-B limb octet.
template <int NC, int UNR, bool PF = false>
__global__ __launch_bounds__(256) void smallc_dgrad_k3_kernel(float* __restrict__ h, int Hin, int Win, int Cin,
                                                              int R, const float* __restrict__ wpk,
                                                              const float* __restrict__ delta, int mask_act,
                                                              float mask_slope, unsigned short* __restrict__ h3,
                                                              const unsigned char* __restrict__ hbits) {
  extern __shared__ __attribute__((aligned(16))) float dl[];  // [(R+2)][(Win+2)][4]
  __shared__ __attribute__((aligned(16))) unsigned char stg_all[4][UNR * 1536];  // per-wave x3 staging
  constexpr int K = 3, CH = 4;
  const int G = Cin / CH, P = 64 / G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned char* stg = stg_all[wave];
  const int g = lane % G, sub = lane / G;
  const int ci0 = g * CH;
  const int b = blockIdx.y, y0 = blockIdx.x * R;
  const int rows = min(R, Hin - y0);
  const int W2 = Win + 2;
  // delta window rows y0-1 .. y0+rows (output pixel (oy, ox) at [oy - y0 + 1][ox + 1])
  // window cells padded to 4 floats: one ds_read_b128 broadcast per tap
  for (int i = threadIdx.x; i < (R + 2) * W2 * 4; i += 256) {
    const int o = i & 3, c = (i >> 2) % W2, r = (i >> 2) / W2;
    const int oy = y0 - 1 + r, ox = c - 1;
    dl[i] = (o < NC && oy >= 0 && oy < Hin && ox >= 0 && ox < Win && r < rows + 2)
                ? delta[(((long)b * Hin + oy) * Win + ox) * NC + o]
                : 0.f;
  }
  float w[K * K][CH][NC];
#pragma unroll
  for (int t = 0; t < K * K; ++t)
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int o = 0; o < NC; ++o) w[t][c][o] = wpk[((long)t * Cin + ci0 + c) * NC + o];
  __syncthreads();
  const int npix = rows * Win;
  const long pbase = ((long)b * Hin + y0) * Win;
  // PF (sign-bit masks): the next iteration's mask nibbles are loaded while this one computes
  unsigned mbn[UNR];
  if (PF && hbits) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pl = wave * P * UNR + u * P + sub;
      mbn[u] = pl < npix ? (hbits[((pbase + pl) * Cin + ci0) >> 3] >> (ci0 & 4)) & 15u : 0u;
    }
  }
  for (int p0 = wave * P * UNR; p0 < npix; p0 += 4 * P * UNR) {
    // the LReLU' mask source: the fp32 activation, or (hbits) its sign bits (nibble of this lane's 4 channels)
    f32x4 hv[UNR];
    unsigned mb[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pl = p0 + u * P + sub;
      if (PF && hbits) {
        mb[u] = mbn[u];
        const int pn = pl + 4 * P * UNR;
        mbn[u] = pn < npix ? (hbits[((pbase + pn) * Cin + ci0) >> 3] >> (ci0 & 4)) & 15u : 0u;
        hv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else if (hbits) {
        mb[u] = pl < npix ? (hbits[((pbase + pl) * Cin + ci0) >> 3] >> (ci0 & 4)) & 15u : 0u;
        hv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        mb[u] = 0u;
        hv[u] = pl < npix ? *reinterpret_cast<const f32x4*>(h + (pbase + pl) * Cin + ci0) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pl = p0 + u * P + sub;
      if (p0 + u * P >= npix) break;  // wave-uniform (the flush below stores only the valid pixels)
      const int iy = pl / Win, ix = pl - iy * Win;
      float acc[CH] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          // output pixel (iy - 1 + ky, ix - 1 + kx) -> window [iy + ky][ix + kx]
          const f32x4 dv = *reinterpret_cast<const f32x4*>(dl + ((min(iy, rows - 1) + ky) * W2 + ix + kx) * 4);
#pragma unroll
          for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int o = 0; o < NC; ++o) acc[c] = fmaf(dv[o], w[ky * K + kx][c][o], acc[c]);
        }
      float v[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c)
        v[c] = acc[c] * (hbits ? (((mb[u] >> c) & 1u) ? 1.f : mask_slope) : act_grad_from_out(hv[u][c], mask_act, mask_slope));
      const bool live = pl < npix;
      const long pix = pbase + pl;
      if (!h3) {
        if (live) *reinterpret_cast<f32x4*>(h + pix * Cin + ci0) = f32x4{v[0], v[1], v[2], v[3]};
        continue;
      }
      // limbs of the 4 channels (2 per dword) into this wave's LDS image of the iteration's x3 rows
      unsigned lh[2], lm[2], ll[2];
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        unsigned short hh[2], mm[2], lo[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float x = v[2 * c2 + e];
          const __bf16 b0 = (__bf16)x;
          const float r1 = sub_rn(x, (float)b0);
          const __bf16 b1 = (__bf16)r1;
          hh[e] = __builtin_bit_cast(unsigned short, b0);
          mm[e] = __builtin_bit_cast(unsigned short, b1);
          lo[e] = __builtin_bit_cast(unsigned short, (__bf16)(sub_rn(r1, (float)b1)));
        }
        lh[c2] = hh[0] | ((unsigned)hh[1] << 16);
        lm[c2] = mm[0] | ((unsigned)mm[1] << 16);
        ll[c2] = lo[0] | ((unsigned)lo[1] << 16);
      }
      typedef unsigned u2 __attribute__((ext_vector_type(2)));
      unsigned char* q = stg + (u * P + sub) * 6 * Cin + (ci0 >> 3) * 48 + (ci0 & 4) * 2;
      *reinterpret_cast<u2*>(q) = u2{lh[0], lh[1]};
      *reinterpret_cast<u2*>(q + 16) = u2{lm[0], lm[1]};
      *reinterpret_cast<u2*>(q + 32) = u2{ll[0], ll[1]};
    }
    if (h3) {
      // the iteration's UNR*P consecutive pixels are one contiguous x3 span: 16-B chunks, 1 KiB per
      // wave-instruction
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int nv = (int)min((long)UNR * P, (long)npix - p0);
      const int nchunk = nv * 3 * Cin / 8;
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
      u4* dst = reinterpret_cast<u4*>(h3 + (pbase + p0) * 3 * Cin);
      for (int c = lane; c < nchunk; c += 64) dst[c] = reinterpret_cast<const u4*>(stg)[c];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// k3 s1 p1 output-layer dgrad on the limb engine (sign-bit mask in, x3 limbs out).  Per 16 pixels it is the product
// dh^T (Cin x 16) = W^T (Cin x 9 NC) . D (9 NC x 16), D = the pixels' 3x3 delta windows (k = tap NC + o, zero past
// 9 NC <= 32 and outside the image): one 16x16x32 tile per 16 channels, six bf16 limb products each (fp32-accurate,
// as gemm_x3_kernel; the accumulation order differs from the VALU form's fmaf chain, not the accuracy).
// A workgroup's NG waves share a 16-pixel unit, wave w taking channels 64 w .. 64 w + 63 (four tiles): its W^T limb
// fragments (12 registers) are loaded once, the unit's D fragment and sign bits are loaded one unit ahead, and the
// unit's 16 x 384 B of limbs leave through a per-wave LDS image as whole 16-B chunks.  Output lane l holds channels
// 16 i + 4 (l >> 4) + r of pixel l & 15, so the LReLU' nibble of the sign bits applies directly.
// F32O (round 4): the gradient leaves as fp32 NHWC (4 B per element: the next dgrad stages its A operand as fp32,
// gemm.hip X3_F32A) through a per-wave image of 272-B pixel rows (8 rows of a ds_write_b128 group on 8 distinct
// 4-bank groups), 4 wave-instructions of 16-B stores per unit; the values are the limb form's before its split.
// KT x KT taps at stride ST (round 4: also the k4 s2 p1 output layer of the 64x64 / 256x256 generators, whose K =
// 16 NC = 48 runs as two 32-deep k steps per limb product, both in one accumulation chain; pixel y's window is
// delta rows ST y - 1 .. ST y - 1 + KT - 1)
template <int NC, int NG, bool F32O = false, int KT = 3, int ST = 1>
__global__ __launch_bounds__(64 * NG) void smallc_dgrad_k3_mfma_kernel(int npix, int Hin, int Win,
                                                                      const float* __restrict__ wpk,
                                                                      const float* __restrict__ delta,
                                                                      float mask_slope, void* __restrict__ outp,
                                                                      const unsigned char* __restrict__ hbits,
                                                                      int probe = 0) {
  // probe (tools/smallc_bench.hip only, wrong results): 1 no delta / sign-bit loads, 2 no output stores
  constexpr int KK = KT * KT * NC, KS = (KK + 31) / 32;  // k values of a pixel's window, 32-deep k steps
  static_assert(KS <= 2, "at most two k steps");
  const int Hout = ST * Hin, Wout = ST * Win;
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  constexpr int Cin = 64 * NG;
  // per-wave output image, pixel rows padded 384 -> 392 B (98 dwords): the 16 lanes of a ds_write_b64 group (16
  // pixels) then cover all 32 banks (at 384 B they all hit one: 16-way; at 400 B, 2-way); rows are 8-B aligned, so the
  // copy-out reads 8 B at a time
  constexpr int SROW = 392;
  __shared__ __attribute__((aligned(16))) unsigned char stg_all[NG][16 * SROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, m = lane & 15;
  unsigned char* const stg = stg_all[wave];
  // this wave's W^T limb fragments: tile t = channels 64 w + 16 t + m (rows), k = 8 q .. 8 q + 7
  bf16x8_t wa[KS][4][3];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ch = 64 * wave + 16 * t + m;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 32 * ks + 8 * q + e, tp = k / NC, o = k - tp * NC;
        const float v = k < KK ? wpk[((long)tp * Cin + ch) * NC + o] : 0.f;
        const __bf16 b0 = (__bf16)v;
        const float r1 = sub_rn(v, (float)b0);
        const __bf16 b1 = (__bf16)r1;
        wa[ks][t][0][e] = b0;
        wa[ks][t][1][e] = b1;
        wa[ks][t][2][e] = (__bf16)(sub_rn(r1, (float)b1));
      }
    }
  const int hw = Hin * Win;
  const int units = (npix + 15) >> 4;
  // every global access is a buffer access whose out-of-range offset reads zero / drops the store, so no load or store
  // sits in a branch (a store in a divergent branch made the compiler wait vmcnt(0) for it at every unit)
  const __amdgpu_buffer_rsrc_t rd =
      __builtin_amdgcn_make_buffer_rsrc((void*)delta, (short)0, npix * ST * ST * NC * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)hbits, (short)0, npix * (Cin / 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc(outp, (short)0, npix * (F32O ? 4 : 6) * Cin, 0x00020000);
  constexpr int OOB = 0x7FFFFFF0;
  // the unit's loads: D's column for this lane's pixel (k = 8 q .. 8 q + 7) and the pixel's 8 sign-bit bytes of this
  // wave's 64 channels
  float dv[KS][8];
  unsigned mw0 = 0u, mw1 = 0u;
  auto load_unit = [&](int un) {
    const int pix = un * 16 + m;
    const bool live = un < units && pix < npix && !(probe & 1);
    const int b = live ? pix / hw : 0, rem = live ? pix - b * hw : 0;
    const int y = rem / Win, x = rem - y * Win;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 32 * ks + 8 * q + e, tp = k / NC, o = k - tp * NC;
        const int yy = ST * y + tp / KT - 1, xx = ST * x + tp % KT - 1;
        const bool ok = live && k < KK && (unsigned)yy < (unsigned)Hout && (unsigned)xx < (unsigned)Wout;
        dv[ks][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rd, ok ? ((((b * Hout + yy) * Wout + xx) * NC + o) * 4) : OOB, 0, 0));
      }
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    const u2 t = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(rb, live ? pix * (Cin / 8) + 8 * wave : OOB,
                                                                             0, 0));
    mw0 = t[0];
    mw1 = t[1];
  };
  int un = blockIdx.x;
  load_unit(un);
  const int nsh = 8 * (q >> 1) + 4 * (q & 1);
  for (; un < units; un += gridDim.x) {
    bf16x8_t d0[KS], d1[KS], d2[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const __bf16 b0 = (__bf16)dv[ks][e];
        const float r1 = sub_rn(dv[ks][e], (float)b0);
        const __bf16 b1 = (__bf16)r1;
        d0[ks][e] = b0;
        d1[ks][e] = b1;
        d2[ks][e] = (__bf16)(sub_rn(r1, (float)b1));
      }
    const unsigned m0w = mw0, m1w = mw1;
    load_unit(un + gridDim.x);  // the next unit's loads land under this one's MFMAs and stores
    f32x4 c[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) c[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the four tiles' six-MFMA chains interleaved (independent accumulators), smallest limb products first, each
    // limb product over the k steps in order
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][t][2], d0[ks], c[t], 0, 0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][t][1], d1[ks], c[t], 0, 0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][t][0], d2[ks], c[t], 0, 0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][t][1], d0[ks], c[t], 0, 0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][t][0], d1[ks], c[t], 0, 0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][t][0], d0[ks], c[t], 0, 0, 0);
    if constexpr (F32O) {
      constexpr int FROW = 272;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const unsigned nib = ((t < 2 ? m0w : m1w) >> (16 * (t & 1) + nsh)) & 15u;
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = c[t][r] * (((nib >> r) & 1u) ? 1.f : mask_slope);
        *reinterpret_cast<f32x4*>(stg + m * FROW + (16 * t + 4 * q) * 4) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cidx = lane + 64 * j, px = cidx >> 4, w = cidx & 15;
        const u4 v = *reinterpret_cast<const u4*>(stg + px * FROW + w * 16);
        const bool ok = un * 16 + px < npix && !(probe & 2);
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, ok ? ((un * 16 + px) * Cin + wave * 64) * 4 + w * 16 : OOB, 0, 0);
      }
    } else {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      // channels 64 w + 16 t + 4 q .. + 3: byte 2 t + (q >> 1) of the wave's 8, nibble q & 1
      const unsigned nib = ((t < 2 ? m0w : m1w) >> (16 * (t & 1) + nsh)) & 15u;
      unsigned short lh[4], lm[4], ll[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = c[t][r] * (((nib >> r) & 1u) ? 1.f : mask_slope);
        const __bf16 b0 = (__bf16)v;
        const float r1 = sub_rn(v, (float)b0);
        const __bf16 b1 = (__bf16)r1;
        lh[r] = __builtin_bit_cast(unsigned short, b0);
        lm[r] = __builtin_bit_cast(unsigned short, b1);
        ll[r] = __builtin_bit_cast(unsigned short, (__bf16)(sub_rn(r1, (float)b1)));
      }
      // image [16 pixels][8 octets x 48 B]: this lane's 4 channels at octet 2 t + (q >> 1), half q & 1
      typedef unsigned u2 __attribute__((ext_vector_type(2)));
      unsigned char* sp = stg + m * SROW + (2 * t + (q >> 1)) * 48 + (q & 1) * 8;
      *reinterpret_cast<u2*>(sp) = u2{lh[0] | ((unsigned)lh[1] << 16), lh[2] | ((unsigned)lh[3] << 16)};
      *reinterpret_cast<u2*>(sp + 16) = u2{lm[0] | ((unsigned)lm[1] << 16), lm[2] | ((unsigned)lm[3] << 16)};
      *reinterpret_cast<u2*>(sp + 32) = u2{ll[0] | ((unsigned)ll[1] << 16), ll[2] | ((unsigned)ll[3] << 16)};
    }
    // the unit's 16 x 384 B of this wave's channels leave as whole 16-B chunks (6 wave-instructions)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int cidx = lane + 64 * j, px = cidx / 24, w = cidx - px * 24;
      const u2 lo = *reinterpret_cast<const u2*>(stg + px * SROW + w * 16);
      const u2 hi = *reinterpret_cast<const u2*>(stg + px * SROW + w * 16 + 8);
      const bool ok = un * 16 + px < npix && !(probe & 2);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, u4{lo[0], lo[1], hi[0], hi[1]}), ro,
                                             ok ? (un * 16 + px) * 6 * Cin + wave * 384 + w * 16 : OOB, 0, 0);
    }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// the limb-engine form applies to the Langevin path's output layer: sign bits in, limbs out, Cin = 128 or 256
bool smallc_k3_mfma_ok(const damc_layer_t& L) { return L.cin == 128 || L.cin == 256; }
// ... and to the k4 s2 p1 output layer (round 4), Cin = 64, 128 or 256 (the caller checks the layer's geometry)
bool smallc_s2_mfma_cin(const damc_layer_t& L) { return L.cin == 64 || L.cin == 128 || L.cin == 256; }

int launch_smallc_dgrad_k3_mfma(const damc_layer_t& L, int B, const float* delta, float mask_slope,
                                unsigned short* h3, const unsigned char* hbits, hipStream_t s, float* out32 = nullptr) {
  // the kernel addresses its operands through 32-bit buffer offsets: batches whose gradient image would reach 2^31
  // bytes (CelebA-HQ from B = 342 with limbs out, CIFAR from B = 2731) run in per-sample-aligned chunks (pixels never
  // interact across samples, so the chunking changes no result)
  const long hw = (long)L.hin * L.win;
  const long per_sample = hw * L.cin * (out32 ? 4 : 6);
  if (per_sample >= 2147483647L - 16) return DAMC_ERR_UNSUPPORTED;
  const int bc = (int)std::min<long>(B, (2147483647L - 16) / per_sample);
  // persistent grid: 1024 workgroups (CelebA-HQ B=64 step 8.03 / 8.06 -> 7.77 / 7.89 ms against 512, CIFAR B=128 within
  // noise; profiles/r04/smallc_dgrad_grid_ab.txt); DAMC_SMALLC_DGRAD_GRID pins it (A/B)
  static const int gmax = [] {
    const char* e = getenv("DAMC_SMALLC_DGRAD_GRID");
    return e ? atoi(e) : 1024;
  }();
  const int ng = L.cin / 64;
  for (int b0 = 0; b0 < B; b0 += bc) {
    const int npix = (int)(std::min(bc, B - b0) * hw);
    const int units = (npix + 15) / 16;
    const int grid = std::max(1, std::min(units, gmax));
    const float* dl = delta + (long)b0 * L.hout * L.wout * L.cout;
    const unsigned char* hb = hbits + (long)b0 * hw * (L.cin / 8);
    float* o32 = out32 ? out32 + (long)b0 * hw * L.cin : nullptr;
    unsigned short* o3 = h3 ? h3 + (long)b0 * hw * L.cin * 3 : nullptr;
#define SDM(NC_, NG_, KT_, ST_)                                                                                    \
  if (o32)                                                                                                         \
    hipLaunchKernelGGL((smallc_dgrad_k3_mfma_kernel<NC_, NG_, true, KT_, ST_>), dim3(grid), dim3(64 * NG_), 0, s,    \
                       npix, L.hin, L.win, L.w_fwd, dl, mask_slope, (void*)o32, hb);                                \
  else                                                                                                             \
    hipLaunchKernelGGL((smallc_dgrad_k3_mfma_kernel<NC_, NG_, false, KT_, ST_>), dim3(grid), dim3(64 * NG_), 0, s,   \
                       npix, L.hin, L.win, L.w_fwd, dl, mask_slope, (void*)o3, hb)
    if (L.k == 4) {
      if (L.cout == 3 && ng == 4) SDM(3, 4, 4, 2);
      else if (L.cout == 3 && ng == 2) SDM(3, 2, 4, 2);
      else if (L.cout == 3) SDM(3, 1, 4, 2);
      else if (ng == 4) SDM(1, 4, 4, 2);
      else if (ng == 2) SDM(1, 2, 4, 2);
      else SDM(1, 1, 4, 2);
    } else {
      if (L.cout == 3 && ng == 4) SDM(3, 4, 3, 1);
      else if (L.cout == 3) SDM(3, 2, 3, 1);
      else if (ng == 4) SDM(1, 4, 3, 1);
      else SDM(1, 2, 3, 1);
    }
#undef SDM
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  return 0;
}

bool smallc_reg_ok(const damc_layer_t& L) {
  if (L.cout != 1 && L.cout != 3) return false;
  if (!((L.k == 3 && L.stride == 1) || (L.k == 4 && L.stride == 2))) return false;
  const int CH = L.k == 3 ? 4 : 2;
  if (L.cin % CH) return false;
  const int G = L.cin / CH;
  return G <= 64 && (64 % G) == 0;
}

// dispatch of a register-resident instantiation (caller checked smallc_reg_ok)
template <int NC>
bool smallc_reg_dispatch(bool fwd, const damc_layer_t& L, const float* h_in, float* h_out, int B, const float* x,
                         float inv_s2, float* delta, const float* delta_in, float* xhat, float* sqerr, int mask_act,
                         float mask_slope, hipStream_t s, unsigned short* h3 = nullptr) {
  const int CH = L.k == 3 ? 4 : 2;
  if (!((L.k == 3 && L.stride == 1) || (L.k == 4 && L.stride == 2))) return false;
  if (L.cin % CH) return false;
  const int G = L.cin / CH;
  if (G > 64 || (64 % G)) return false;
  const int P = 64 / G;
  const long npix = (fwd && L.k == 3) ? (long)B * L.hout * L.wout : (long)B * L.hin * L.win;
  const int grid = (int)std::max<long>(1, std::min<long>((npix + 4L * P - 1) / (4L * P), 1024));
  if (fwd) {
    if (L.k == 3)
      hipLaunchKernelGGL((smallc_fwd_reg_kernel<NC, 3, 1, 4>), dim3(grid), dim3(256), 0, s, h_in, B, L.hin, L.win,
                         L.cin, L.pad, L.hout, L.wout, L.w_fwd, L.bias, x, inv_s2, delta, xhat, sqerr);
    else
      hipLaunchKernelGGL((smallc_fwd_s2_kernel<NC, 2>), dim3(grid), dim3(256), 0, s, h_in, B, L.hin, L.win, L.cin,
                         L.w_fwd, L.bias, x, inv_s2, delta, xhat, sqerr);
  } else {
    if (L.k == 3)
      hipLaunchKernelGGL((smallc_dgrad_reg_kernel<NC, 3, 1, 4>), dim3(grid), dim3(256), 0, s, h_out, B, L.hin,
                         L.win, L.cin, L.pad, L.hout, L.wout, L.w_fwd, delta_in, mask_act, mask_slope, h3);
    else
      hipLaunchKernelGGL((smallc_dgrad_reg_kernel<NC, 4, 2, 2>), dim3(grid), dim3(256), 0, s, h_out, B, L.hin,
                         L.win, L.cin, L.pad, L.hout, L.wout, L.w_fwd, delta_in, mask_act, mask_slope, h3);
  }
  return true;
}

// ---- two-stage output-layer forward -------------------------------------------------------
// Stage 1 (MFMA): per INPUT pixel p the per-tap projections P[p][n], n = (ky*K + kx)*NC + co,
//   P = h (npix x Cin) . Wp^T,  Wp packed [NTILE*32][Cin] (rows n >= K*K*NC are zero).
// A wave owns 32 pixels x 32 columns per 32-column tile (v_mfma_f32_32x32x2_f32).  Operands come
// straight from L2 as float4: lane (i = l&31, h = l>>5) loads h[p_i][8j + 4h .. +3] and
// Wp[n_i][8j + 4h .. +3]; element t of those feeds k-step 4j + t, i.e. half h covers
// k = 8j + 4h + t — the same bijection of k for A and B, so the sum is unchanged.
template <int NTILE>
__global__ __launch_bounds__(256) void smallc_proj_kernel(const float* __restrict__ h, long npix, int Cin,
                                                          const float* __restrict__ wp, float* __restrict__ P) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long p0 = ((long)blockIdx.x * 4 + wave) * 32;
  if (p0 >= npix) return;
  const int i = lane & 31, hh = lane >> 5;
  const long pi = min(p0 + i, npix - 1);
  const float* hrow = h + pi * Cin + 4 * hh;
  f32x16 acc[NTILE];
#pragma unroll
  for (int t = 0; t < NTILE; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const float* wrow[NTILE];
#pragma unroll
  for (int t = 0; t < NTILE; ++t) wrow[t] = wp + (long)(32 * t + i) * Cin + 4 * hh;
#pragma unroll 8
  for (int j = 0; j < Cin; j += 8) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(hrow + j);
    f32x4 b[NTILE];
#pragma unroll
    for (int t = 0; t < NTILE; ++t) b[t] = *reinterpret_cast<const f32x4*>(wrow[t] + j);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int t = 0; t < NTILE; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], b[t][e], acc[t], 0, 0, 0);
  }
  // C layout: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  const int ldp = NTILE * 32;
#pragma unroll
  for (int t = 0; t < NTILE; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long p = p0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (p < npix) P[p * ldp + 32 * t + i] = acc[t][r];
    }
}

// The same products in the same k order, with each wave's 32 pixels (one contiguous NHWC block) staged through LDS
// 64 channels at a time: whole 256-B row spans per load instruction instead of 32 B of 32 rows, the next chunk's
// loads in flight under the current chunk's MFMAs.  Row stride 68 floats: conflict-free ds_read_b128 fragments.
constexpr int PJ_KC = 64, PJ_RS = PJ_KC + 4;
template <int NTILE>
__global__ __launch_bounds__(256) void smallc_proj_lds_kernel(const float* __restrict__ h, long npix, int Cin,
                                                              const float* __restrict__ wp, float* __restrict__ P) {
  __shared__ __attribute__((aligned(16))) float st[4][32 * PJ_RS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long p0 = ((long)blockIdx.x * 4 + wave) * 32;
  const int i = lane & 31, hh = lane >> 5;
  float* ls = st[wave];
  f32x16 acc[NTILE];
#pragma unroll
  for (int t = 0; t < NTILE; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const float* wrow[NTILE];
#pragma unroll
  for (int t = 0; t < NTILE; ++t) wrow[t] = wp + (long)(32 * t + i) * Cin + 4 * hh;
  // staging: load q of a chunk covers rows 4q + lane/16, float4 lane%16 of the row's 64 channels
  f32x4 g[8];
  auto gload = [&](int c0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = 4 * q + (lane >> 4);
      const long pr = min(p0 + row, npix - 1);
      g[q] = *reinterpret_cast<const f32x4*>(h + pr * Cin + c0 + 4 * (lane & 15));
    }
  };
  gload(0);
  for (int c0 = 0; c0 < Cin; c0 += PJ_KC) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q)
      *reinterpret_cast<f32x4*>(ls + (4 * q + (lane >> 4)) * PJ_RS + 4 * (lane & 15)) = g[q];
    __syncthreads();
    if (c0 + PJ_KC < Cin) gload(c0 + PJ_KC);
#pragma unroll
    for (int j = 0; j < PJ_KC; j += 8) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(ls + i * PJ_RS + j + 4 * hh);
      f32x4 b[NTILE];
#pragma unroll
      for (int t = 0; t < NTILE; ++t) b[t] = *reinterpret_cast<const f32x4*>(wrow[t] + c0 + j);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < NTILE; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], b[t][e], acc[t], 0, 0, 0);
    }
  }
  const int ldp = NTILE * 32;
#pragma unroll
  for (int t = 0; t < NTILE; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long p = p0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (p < npix) P[p * ldp + 32 * t + i] = acc[t][r];
    }
}

// The same projection on the limb engine (round 3): per 32-deep k step a lane loads its pixel's 8 channels (2 x 16 B)
// and splits them into bf16 limbs; Wp's limb fragments for the 32 columns (2 tiles x 8 k steps x 3 limbs) are staged in
// LDS once per workgroup.  A wave owns 32 pixels (two 16-row tiles) x 32 columns; six limb-product MFMAs per tile pair
// and k step (fp32-accurate, gemm_x3_kernel's products; the sum order differs from the fp32-MFMA kernel's).  Cin = 256.
__global__ __launch_bounds__(256) void smallc_proj_x3_kernel(const float* __restrict__ h, long npix,
                                                             const float* __restrict__ wp, float* __restrict__ P) {
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  constexpr int Cin = 256, KS = Cin / 32;
  __shared__ __attribute__((aligned(16))) bf16x8_t wfr[2][KS][3][64];  // [N tile][k step][limb][lane]: 48 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, q = lane >> 4;
  // Wp (32 x Cin, row n = tap * NC + co) as B fragments: lane (col n = 16 t + m, k-group q) holds k = 8 q .. 8 q + 7
  for (int u = tid; u < 2 * KS * 64; u += 256) {
    const int t = u / (KS * 64), ks = (u / 64) % KS, l = u & 63;
    // k permutation shared with the A loads below: fragment element e of k-group q is k = 4 q + e (e < 4) or
    // 16 + 4 q + e - 4, so each of a lane's two 16-B activation loads is a quarter of one contiguous 64-B span
    const float* src = wp + (long)(16 * t + (l & 15)) * Cin + 32 * ks + 4 * (l >> 4);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(src), v1 = *reinterpret_cast<const f32x4*>(src + 16);
    const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    bf16x8_t hb, mb, lb;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const __bf16 b0 = (__bf16)v[e];
      const float r1 = sub_rn(v[e], (float)b0);
      const __bf16 b1 = (__bf16)r1;
      hb[e] = b0;
      mb[e] = b1;
      lb[e] = (__bf16)(sub_rn(r1, (float)b1));
    }
    wfr[t][ks][0][l] = hb;
    wfr[t][ks][1][l] = mb;
    wfr[t][ks][2][l] = lb;
  }
  __syncthreads();
  // persistent: the Wp fragments are staged once per workgroup, each wave then walks 32-pixel tasks
  for (long p0 = ((long)blockIdx.x * 4 + wave) * 32; p0 < npix; p0 += (long)gridDim.x * 128) {
  f32x4 acc[2][2];  // [pixel tile][column tile]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* hrow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) hrow[i] = h + min(p0 + 16 * i + m, npix - 1) * Cin + 4 * q;
  // the pixels' channels two k steps ahead (4 x 16 B per lane and step in flight)
  f32x4 ga[KS][2][2];
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ga[ks][i][0] = *reinterpret_cast<const f32x4*>(hrow[i] + 32 * ks);
      ga[ks][i][1] = *reinterpret_cast<const f32x4*>(hrow[i] + 32 * ks + 16);
    }
  };
  gload(0);
  gload(1);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8_t a[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float v[8] = {ga[ks][i][0][0], ga[ks][i][0][1], ga[ks][i][0][2], ga[ks][i][0][3],
                          ga[ks][i][1][0], ga[ks][i][1][1], ga[ks][i][1][2], ga[ks][i][1][3]};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const __bf16 b0 = (__bf16)v[e];
        const float r1 = sub_rn(v[e], (float)b0);
        const __bf16 b1 = (__bf16)r1;
        a[i][0][e] = b0;
        a[i][1][e] = b1;
        a[i][2][e] = (__bf16)(sub_rn(r1, (float)b1));
      }
    }
    if (ks + 2 < KS) gload(ks + 2);  // lands under this and the next step's MFMAs
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16x8_t b0 = wfr[j][ks][0][lane], b1 = wfr[j][ks][1][lane], b2 = wfr[j][ks][2][lane];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b2, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b1, c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b0, c, 0, 0, 0);
      }
    }
  }
  // C layout (16x16): col = lane & 15, rows 4 q + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long p = p0 + 16 * i + 4 * q + r;
        if (p < npix) P[p * 32 + 16 * j + m] = acc[i][j][r];
      }
  }
}

// Stage 2: out[b,oy,ox,co] = bias + sum over the valid taps of P[input pixel][tap*NC + co], then tanh,
// x_hat (NCHW) and the residual delta = (x_hat - x)/s^2 * (1 - x_hat^2) (NHWC).  One thread per output pixel.
template <int NC, int K, int S>
__global__ __launch_bounds__(256) void smallc_gather_kernel(const float* __restrict__ P, const float* __restrict__ P1,
                                                            int ldp, int B, int Hin, int Win, int pad, int Hout, int Wout,
                                                            const float* __restrict__ bias, const float* x,
                                                            float inv_s2, float* delta, float* xhat,
                                                            float* sqerr_sum) {
  __shared__ float red[4];
  const long npix = (long)B * Hout * Wout;
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float sq = 0.f;
  if (pix < npix) {
    const int b = (int)(pix / ((long)Hout * Wout));
    const int rem = (int)(pix - (long)b * Hout * Wout);
    const int oy = rem / Wout, ox = rem - oy * Wout;
    float acc[NC];
#pragma unroll
    for (int o = 0; o < NC; ++o) acc[o] = bias ? bias[o] : 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int ty = oy + pad - ky;
      if (ty < 0 || (S == 2 && (ty & 1))) continue;
      const int iy = ty / S;
      if (iy >= Hin) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int tx = ox + pad - kx;
        if (tx < 0 || (S == 2 && (tx & 1))) continue;
        const int ix = tx / S;
        if (ix >= Win) continue;
        const long po = (((long)b * Hin + iy) * Win + ix) * ldp + (ky * K + kx) * NC;
#pragma unroll
        for (int o = 0; o < NC; ++o) acc[o] += P1 ? P[po + o] + P1[po + o] : P[po + o];  // chunk partials in order
      }
    }
#pragma unroll
    for (int o = 0; o < NC; ++o) {
      const float t = tanhf(acc[o]);
      const long nchw = (((long)b * NC + o) * Hout + oy) * Wout + ox;
      if (xhat) xhat[nchw] = t;
      if (delta) {
        const float r = t - x[nchw];
        delta[pix * NC + o] = r * inv_s2 * (1.f - t * t);
        sq += r * r;
      }
    }
  }
  if (sqerr_sum) {
    sq = wave_sum(sq);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = red[0];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) t += red[w];
      atomicAdd(sqerr_sum, t * (0.5f * inv_s2));
    }
  }
}

// The k3 s1 gather through LDS: a workgroup takes R output rows of one sample, stages the R + 2 input rows' projection
// rows (9 NC taps each, the two chunk partials already added in order) with coalesced loads, then gathers from LDS with
// smallc_gather_kernel's arithmetic (same tap order, same adds), so the result is bitwise that kernel's.  The
// direct gather issued 27 (x 2 partials) scattered 4-B loads per output pixel: 36 us at CIFAR B=128.
template <int NC>
__global__ __launch_bounds__(256) void smallc_gather_lds_kernel(const float* __restrict__ P, const float* __restrict__ P1,
                                                                int ldp, int H, int W, int R,
                                                                const float* __restrict__ bias, const float* x,
                                                                float inv_s2, float* delta, float* xhat,
                                                                float* sqerr_sum) {
  constexpr int T = 9 * NC;
  extern __shared__ float pr[];  // [(R + 2) rows][W][T]
  __shared__ float red[4];
  const int b = blockIdx.x, r0 = blockIdx.y * R, rows = min(R, H - r0);
  const int n = (rows + 2) * W * T;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int rr = i / (W * T), rem = i - rr * (W * T), px = rem / T, t = rem - px * T;
    const int iy = r0 - 1 + rr;
    if (iy < 0 || iy >= H) continue;
    const long po = (((long)b * H + iy) * W + px) * ldp + t;
    pr[i] = P1 ? P[po] + P1[po] : P[po];
  }
  __syncthreads();
  float sq = 0.f;
  for (int p = threadIdx.x; p < rows * W; p += 256) {
    const int oy = r0 + p / W, ox = p - (p / W) * W;
    float acc[NC];
#pragma unroll
    for (int o = 0; o < NC; ++o) acc[o] = bias ? bias[o] : 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy + 1 - ky;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox + 1 - kx;
        if (ix < 0 || ix >= W) continue;
        const float* q = pr + ((iy - r0 + 1) * W + ix) * T + (ky * 3 + kx) * NC;
#pragma unroll
        for (int o = 0; o < NC; ++o) acc[o] += q[o];
      }
    }
    const long pix = ((long)b * H + oy) * W + ox;
#pragma unroll
    for (int o = 0; o < NC; ++o) {
      const float t = tanhf(acc[o]);
      const long nchw = (((long)b * NC + o) * H + oy) * W + ox;
      if (xhat) xhat[nchw] = t;
      if (delta) {
        const float rd = t - x[nchw];
        delta[pix * NC + o] = rd * inv_s2 * (1.f - t * t);
        sq += rd * rd;
      }
    }
  }
  if (sqerr_sum) {
    sq = wave_sum(sq);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = sq;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(sqerr_sum, (red[0] + red[1] + red[2] + red[3]) * (0.5f * inv_s2));
  }
}

// The k4 s2 p1 gather through LDS (round 4): a workgroup takes an R x CW tile of output pixels (R, CW even) of one
// sample; the R/2 + 2 x CW/2 + 2 input pixels its taps reach have their 16 NC projection values staged in LDS (the
// chunk partials already added in order), then smallc_gather_kernel's loops and adds run over LDS: bitwise that kernel.
template <int NC>
__global__ __launch_bounds__(256) void smallc_gather_s2_lds_kernel(const float* __restrict__ P,
                                                                   const float* __restrict__ P1, int ldp, int Hin,
                                                                   int Win, int R, int CW,
                                                                   const float* __restrict__ bias, const float* x,
                                                                   float inv_s2, float* delta, float* xhat,
                                                                   float* sqerr_sum) {
  constexpr int T = 16 * NC;
  extern __shared__ float pr[];  // [R/2 + 2][CW/2 + 2][T]
  __shared__ float red[4];
  const int Hout = 2 * Hin, Wout = 2 * Win;
  const int b = blockIdx.z, oy0 = blockIdx.y * R, ox0 = blockIdx.x * CW;
  const int IR = R / 2 + 2, IC = CW / 2 + 2, iy0 = oy0 / 2 - 1, ix0 = ox0 / 2 - 1;
  for (int i = threadIdx.x; i < IR * IC * T; i += 256) {
    const int rc = i / T, t = i - rc * T, r = rc / IC, c = rc - r * IC;
    const int iy = iy0 + r, ix = ix0 + c;
    if (iy < 0 || iy >= Hin || ix < 0 || ix >= Win) continue;
    const long po = (((long)b * Hin + iy) * Win + ix) * ldp + t;
    pr[i] = P1 ? P[po] + P1[po] : P[po];
  }
  __syncthreads();
  float sq = 0.f;
  for (int p = threadIdx.x; p < R * CW; p += 256) {
    const int oy = oy0 + p / CW, ox = ox0 + p % CW;
    if (oy >= Hout || ox >= Wout) continue;
    float acc[NC];
#pragma unroll
    for (int o = 0; o < NC; ++o) acc[o] = bias ? bias[o] : 0.f;
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) {
      const int ty = oy + 1 - ky;
      if (ty < 0 || (ty & 1)) continue;
      const int iy = ty / 2;
      if (iy >= Hin) continue;
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        const int tx = ox + 1 - kx;
        if (tx < 0 || (tx & 1)) continue;
        const int ix = tx / 2;
        if (ix >= Win) continue;
        const float* q = pr + ((iy - iy0) * IC + (ix - ix0)) * T + (ky * 4 + kx) * NC;
#pragma unroll
        for (int o = 0; o < NC; ++o) acc[o] += q[o];
      }
    }
    const long pix = ((long)b * Hout + oy) * Wout + ox;
#pragma unroll
    for (int o = 0; o < NC; ++o) {
      const float t = tanhf(acc[o]);
      const long nchw = (((long)b * NC + o) * Hout + oy) * Wout + ox;
      if (xhat) xhat[nchw] = t;
      if (delta) {
        const float rd = t - x[nchw];
        delta[pix * NC + o] = rd * inv_s2 * (1.f - t * t);
        sq += rd * rd;
      }
    }
  }
  if (sqerr_sum) {
    sq = wave_sum(sq);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = sq;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(sqerr_sum, (red[0] + red[1] + red[2] + red[3]) * (0.5f * inv_s2));
  }
}

int smallc_ntile(const damc_layer_t& L) { return (L.k * L.k * L.cout + 31) / 32; }

bool smallc_twostage_ok(const damc_layer_t& L) {
  if (L.cout != 1 && L.cout != 3) return false;
  if (!((L.k == 3 && L.stride == 1) || (L.k == 4 && L.stride == 2))) return false;
  return L.cin % 8 == 0 && smallc_ntile(L) <= 2 && L.w_bwd != nullptr;
}

// the projection on proj16 (gemm.hip launch_proj_rows; the arithmetic of the fused ConvT epilogue) applies
bool smallc_proj16_ok(const damc_layer_t& L) { return L.cin <= 256 && L.cin % 16 == 0 && smallc_ntile(L) <= 2; }

// p_ready: Pbuf already holds the projections (the layer before ran them in its epilogue, GemmArgs::proj_out)
int smallc_fwd_twostage(const damc_layer_t& L, const float* h, int B, const float* x, float inv_s2, float* delta,
                        float* xhat, float* sqerr, float* Pbuf, hipStream_t s, bool p_ready = false) {
  ProfScope ps("smallc_fwd", 2.0 * B * L.hout * L.wout * L.cout * L.cin * L.k * L.k / (L.stride * L.stride), s);
  const long npin = (long)B * L.hin * L.win;
  const int nt = smallc_ntile(L);
  // DAMC_SMALLC_PROJ16=0 (read per call): the round-3 projection kernels below instead of proj16's
  const char* p16 = getenv("DAMC_SMALLC_PROJ16");
  const bool use16 = !(p16 && p16[0] == '0') && smallc_proj16_ok(L);
  int rc = 0;
  if (p_ready) {
  } else if (use16) {
    if ((rc = damc::launch_proj_rows(h, npin, L.cin, L.w_bwd, L.cin, 32 * nt, Pbuf, npin * 32 * nt, s))) return rc;
  } else {
  const int g1 = (int)((npin + 127) / 128);
  // the LDS-staged kernel when Cin is whole 64-channel chunks (CIFAR B=128: 63.5 -> 51.3 us for projection + gather);
  // DAMC_SMALLC_PROJ_LDS=0 (read per call) selects the direct-load kernel
  const char* pe = getenv("DAMC_SMALLC_PROJ_LDS");
  const bool lds = !(pe && atoi(pe) == 0) && L.cin % PJ_KC == 0;
  // Cin = 256: the limb-engine projection, opt-in (DAMC_SMALLC_PROJ_X3=1, read per call).  Standalone it is 14 %
  // faster (31.3 vs 36.6 us, tools/smallc_bench.hip), but in the bench line, where h3 was just written by the layer
  // before, projection + gather took 60.6 us against 52.4 us for the LDS-staged fp32-MFMA kernel (same-box A/B,
  // profiles/r03/ab_output_proj.txt), so that stays the default
  const char* px3 = getenv("DAMC_SMALLC_PROJ_X3");
  if (nt == 1 && L.cin == 256 && px3 && px3[0] == '1')
    // one workgroup per CU measured fastest (CIFAR B=128: 31.3 us at 256 workgroups, 35.9 at 768, 38.4 at 1024;
    // the fp32-MFMA kernel 36.6; tools/smallc_bench.hip)
    {
      const char* pg = getenv("DAMC_SMALLC_PROJ_GRID");  // A/B of the persistent grid (read per call)
      const int gm = pg ? std::max(1, atoi(pg)) : 256;
      hipLaunchKernelGGL(smallc_proj_x3_kernel, dim3(std::min(g1, gm)), dim3(256), 0, s, h, npin, L.w_bwd, Pbuf);
    }
  else if (lds && nt == 1)
    hipLaunchKernelGGL((smallc_proj_lds_kernel<1>), dim3(g1), dim3(256), 0, s, h, npin, L.cin, L.w_bwd, Pbuf);
  else if (lds)
    hipLaunchKernelGGL((smallc_proj_lds_kernel<2>), dim3(g1), dim3(256), 0, s, h, npin, L.cin, L.w_bwd, Pbuf);
  else if (nt == 1)
    hipLaunchKernelGGL((smallc_proj_kernel<1>), dim3(g1), dim3(256), 0, s, h, npin, L.cin, L.w_bwd, Pbuf);
  else
    hipLaunchKernelGGL((smallc_proj_kernel<2>), dim3(g1), dim3(256), 0, s, h, npin, L.cin, L.w_bwd, Pbuf);
  }
  const long npout = (long)B * L.hout * L.wout;
  const int g2 = (int)((npout + 255) / 256);
  // the proj16 forms (proj_rows_kernel and the fused epilogues) leave one partial per 128-channel chunk
  const float* P1 = ((p_ready || use16) && L.cin > damc::PROJ_CHUNK) ? Pbuf + npin * 32 * nt : nullptr;
  // k3 s1 p1, the same grid in and out: the LDS-staged gather (bitwise); DAMC_SMALLC_GATHER_LDS=0 (read per call)
  // keeps the direct one
  const char* gl = getenv("DAMC_SMALLC_GATHER_LDS");
  // rows per workgroup: at most what 60 KB of LDS holds (with the 2 halo rows), spread evenly over the strips
  const int gRmax = L.wout > 0 ? std::min(L.hout, 15360 / (L.wout * 9 * L.cout) - 2) : 0;
  const int gR = gRmax > 0 ? (L.hout + (L.hout + gRmax - 1) / gRmax - 1) / ((L.hout + gRmax - 1) / gRmax) : 0;
  // (only where the strips fill the chip: at CIFAR B=16, 48 workgroups, it measured 10 us slower than the direct
  // gather; at B=128, 384 workgroups, 13 us faster; profiles/r04/gather_lds_ab.txt)
  if (!(gl && gl[0] == '0') && L.k == 3 && L.stride == 1 && L.pad == 1 && L.hin == L.hout && L.win == L.wout &&
      gR >= 4 && (long)B * ((L.hout + gR - 1) / gR) >= 256) {
    const size_t sm = (size_t)(gR + 2) * L.wout * 9 * L.cout * sizeof(float);
    const dim3 g(B, (L.hout + gR - 1) / gR);
    if (L.cout == 3)
      hipLaunchKernelGGL(smallc_gather_lds_kernel<3>, g, dim3(256), sm, s, Pbuf, P1, nt * 32, L.hout, L.wout, gR,
                         L.bias, x, inv_s2, delta, xhat, sqerr);
    else
      hipLaunchKernelGGL(smallc_gather_lds_kernel<1>, g, dim3(256), sm, s, Pbuf, P1, nt * 32, L.hout, L.wout, gR,
                         L.bias, x, inv_s2, delta, xhat, sqerr);
    return (int)hipGetLastError();
  }
  // k4 s2 p1: the LDS-staged gather over 16 x 32 output tiles (bitwise), where the tiles fill the chip
  if (!(gl && gl[0] == '0') && L.k == 4 && L.stride == 2 && L.pad == 1 && L.hout == 2 * L.hin &&
      L.wout == 2 * L.win && B <= 65535 && (long)B * ((L.hout + 15) / 16) * ((L.wout + 31) / 32) >= 256) {
    const int R2 = 16, CW2 = 32;
    const size_t sm = (size_t)(R2 / 2 + 2) * (CW2 / 2 + 2) * 16 * L.cout * sizeof(float);
    const dim3 g((L.wout + CW2 - 1) / CW2, (L.hout + R2 - 1) / R2, B);
    if (L.cout == 3)
      hipLaunchKernelGGL(smallc_gather_s2_lds_kernel<3>, g, dim3(256), sm, s, Pbuf, P1, nt * 32, L.hin, L.win, R2, CW2,
                         L.bias, x, inv_s2, delta, xhat, sqerr);
    else
      hipLaunchKernelGGL(smallc_gather_s2_lds_kernel<1>, g, dim3(256), sm, s, Pbuf, P1, nt * 32, L.hin, L.win, R2, CW2,
                         L.bias, x, inv_s2, delta, xhat, sqerr);
    return (int)hipGetLastError();
  }
  // one wave per workgroup where 256-thread workgroups would leave CUs idle (CIFAR B=16: 256 workgroups of 64 instead
  // of 64 of 256 -- a pixel's 54 scattered loads are latency-bound, so the CU count carries it); pixels are independent
  const int tpb = g2 < 512 ? 64 : 256;
  const int g2t = (int)((npout + tpb - 1) / tpb);
#define SG(NC_, K_, S_)                                                                                             \
  hipLaunchKernelGGL((smallc_gather_kernel<NC_, K_, S_>), dim3(g2t), dim3(tpb), 0, s, Pbuf, P1, nt * 32, B, L.hin,    \
                     L.win, L.pad, L.hout, L.wout, L.bias, x, inv_s2, delta, xhat, sqerr)
  if (L.cout == 3) {
    if (L.k == 3) SG(3, 3, 1); else SG(3, 4, 2);
  } else {
    if (L.k == 3) SG(1, 3, 1); else SG(1, 4, 2);
  }
#undef SG
  return (int)hipGetLastError();
}

int smallc_fwd(const damc_layer_t& L, const float* h, int B, const float* x, float inv_s2, float* delta, float* xhat,
               float* sqerr, float* Pbuf, hipStream_t s, bool p_ready = false) {
  if (Pbuf && smallc_twostage_ok(L))
    return smallc_fwd_twostage(L, h, B, x, inv_s2, delta, xhat, sqerr, Pbuf, s, p_ready);
  if (p_ready) return DAMC_ERR_ARG;
  if (smallc_reg_ok(L)) {
    ProfScope ps("smallc_fwd", 2.0 * B * L.hout * L.wout * L.cout * L.cin * L.k * L.k / (L.stride * L.stride), s);
    if (L.cout == 3)
      smallc_reg_dispatch<3>(true, L, h, nullptr, B, x, inv_s2, delta, nullptr, xhat, sqerr, 0, 0.f, s);
    else
      smallc_reg_dispatch<1>(true, L, h, nullptr, B, x, inv_s2, delta, nullptr, xhat, sqerr, 0, 0.f, s);
    return (int)hipGetLastError();
  }
  const size_t sm = (size_t)L.k * L.k * L.cin * L.cout * sizeof(float);
  const long npix = (long)B * L.hout * L.wout;
  const int grid = (int)std::min<long>((npix + 3) / 4, 2048);
  ProfScope ps("smallc_fwd", 2.0 * npix * L.cout * L.cin * L.k * L.k / (L.stride * L.stride), s);
#define SC(NC_)                                                                                              \
  hipLaunchKernelGGL((smallc_fwd_kernel<NC_>), dim3(grid), dim3(256), sm, s, h, B, L.hin, L.win, L.cin, L.k, \
                     L.stride, L.pad, L.hout, L.wout, L.w_fwd, L.bias, x, inv_s2, delta, xhat, sqerr)
  switch (L.cout) {
    case 1: SC(1); break;
    case 2: SC(2); break;
    case 3: SC(3); break;
    case 4: SC(4); break;
    default: return DAMC_ERR_UNSUPPORTED;
  }
#undef SC
  return (int)hipGetLastError();
}

// the register-resident dgrad can write its gradient as x3 limbs (channel groups never straddle an octet)
bool smallc_x3_ok(const damc_layer_t& L) { return smallc_reg_ok(L) && L.cin % 8 == 0; }

// k3 s1 p1 output layer handled by smallc_dgrad_k3_kernel (reads sign bits / writes limbs)
bool smallc_k3(const damc_layer_t& L) {
  return L.kind == DAMC_LAYER_SMALLC && L.k == 3 && L.stride == 1 && L.pad == 1 && L.hout == L.hin &&
         L.wout == L.win && (L.cout == 1 || L.cout == 3) && L.cin % 8 == 0 && L.cin / 4 <= 64 &&
         64 % (L.cin / 4) == 0;
}


// k4 s2 p1 output layer with the limb-engine dgrad (round 4): the layer before it writes sign bits for it
// (DAMC_SMALLC_S2_MFMA=0, read per call: the register-resident VALU dgrad with the fp32 activation as mask)
bool smallc_s2_mfma(const damc_layer_t& L) {
  const char* e = getenv("DAMC_SMALLC_S2_MFMA");
  return L.kind == DAMC_LAYER_SMALLC && L.k == 4 && L.stride == 2 && L.pad == 1 && L.hout == 2 * L.hin &&
         L.wout == 2 * L.win && (L.cout == 1 || L.cout == 3) && smallc_s2_mfma_cin(L) && !(e && e[0] == '0');
}

// f32_out (with sign bits, limb engine): the MFMA kernel writes the fp32 gradient into h instead of limbs into h3
int smallc_dgrad(const damc_layer_t& L, float* h, int B, const float* delta, int mask_act, float mask_slope,
                 unsigned short* h3, const unsigned char* hbits_in, hipStream_t s, bool f32_out = false) {
  if (h3 && !smallc_x3_ok(L)) return DAMC_ERR_ARG;
  if (hbits_in && (!(smallc_k3(L) || smallc_s2_mfma(L)) || mask_act != DAMC_ACT_LRELU)) return DAMC_ERR_ARG;
  if (smallc_s2_mfma(L) && hbits_in) {  // sign bits in, limbs or fp32 out, on the limb engine
    ProfScope ps("smallc_dgrad", 2.0 * B * L.hout * L.wout * L.cout * L.cin * L.k * L.k / 4, s);
    const bool fp32 = f32_out || !h3;  // the fp32 gradient into h (in place of the activation) when no limbs are asked
    return launch_smallc_dgrad_k3_mfma(L, B, delta, mask_slope, fp32 ? nullptr : h3, hbits_in, s, fp32 ? h : nullptr);
  }
  if (smallc_k3(L)) {
    ProfScope ps("smallc_dgrad", 2.0 * B * L.hout * L.wout * L.cout * L.cin * L.k * L.k, s);
    // the Langevin path (sign bits in, limbs out) on the limb engine; DAMC_SMALLC_DGRAD_MFMA=0 (read per call)
    // selects the VALU kernel below
    // (any batch: the MFMA kernel runs in batch chunks below 2^31 bytes)
    const char* mf = getenv("DAMC_SMALLC_DGRAD_MFMA");
    const bool use_mf = hbits_in && smallc_k3_mfma_ok(L) && !(mf && mf[0] == '0');
    if (f32_out && use_mf) return launch_smallc_dgrad_k3_mfma(L, B, delta, mask_slope, nullptr, hbits_in, s, h);
    if (f32_out) h3 = nullptr;  // the VALU kernel below writes the fp32 gradient into h when no limbs are asked
    if (h3 && use_mf) return launch_smallc_dgrad_k3_mfma(L, B, delta, mask_slope, h3, hbits_in, s);
    // 8 rows per block with the next mask nibbles prefetched: 66.4 us vs 69.9 (4 rows, no prefetch) at the
    // CIFAR B=128 shape (tools/smallc_bench.hip; 16 rows leave CUs idle: 115 us); fewer rows per block when the
    // batch would leave fewer than 256 blocks (B=16: 60 us at 8 rows, 64 blocks).  Pixels are independent, so
    // the row blocking never changes a result
    int R = 8;
    while (R > 1 && (long)((L.hin + R - 1) / R) * B < 256) R >>= 1;
    const dim3 grid((unsigned)((L.hin + R - 1) / R), (unsigned)B);
    const size_t sm = sizeof(float) * (R + 2) * (L.win + 2) * 4;
    if (L.cout == 3)
      hipLaunchKernelGGL((smallc_dgrad_k3_kernel<3, 4, true>), grid, dim3(256), sm, s, h, L.hin, L.win, L.cin, R,
                         L.w_fwd, delta, mask_act, mask_slope, h3, hbits_in);
    else
      hipLaunchKernelGGL((smallc_dgrad_k3_kernel<1, 4, true>), grid, dim3(256), sm, s, h, L.hin, L.win, L.cin, R,
                         L.w_fwd, delta, mask_act, mask_slope, h3, hbits_in);
    return (int)hipGetLastError();
  }
  if (smallc_reg_ok(L)) {
    ProfScope ps("smallc_dgrad", 2.0 * B * L.hout * L.wout * L.cout * L.cin * L.k * L.k / (L.stride * L.stride), s);
    if (L.cout == 3)
      smallc_reg_dispatch<3>(false, L, nullptr, h, B, nullptr, 0.f, nullptr, delta, nullptr, nullptr, mask_act,
                             mask_slope, s, h3);
    else
      smallc_reg_dispatch<1>(false, L, nullptr, h, B, nullptr, 0.f, nullptr, delta, nullptr, nullptr, mask_act,
                             mask_slope, s, h3);
    return (int)hipGetLastError();
  }
  const size_t sm = (size_t)L.k * L.k * L.cin * L.cout * sizeof(float);
  const long npix = (long)B * L.hin * L.win;
  const int grid = (int)std::min<long>((npix + 3) / 4, 2048);
  ProfScope ps("smallc_dgrad", 2.0 * npix * L.cout * L.cin * L.k * L.k / (L.stride * L.stride), s);
#define SD(NC_)                                                                                                \
  hipLaunchKernelGGL((smallc_dgrad_kernel<NC_>), dim3(grid), dim3(256), sm, s, h, B, L.hin, L.win, L.cin, L.k, \
                     L.stride, L.pad, L.hout, L.wout, L.w_fwd, delta, mask_act, mask_slope)
  switch (L.cout) {
    case 1: SD(1); break;
    case 2: SD(2); break;
    case 3: SD(3); break;
    case 4: SD(4); break;
    default: return DAMC_ERR_UNSUPPORTED;
  }
#undef SD
  return (int)hipGetLastError();
}

// fixed-order (deterministic) reduction of the split-K slabs: one thread per element, loads unrolled
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slabs, int nslab, long n,
                                                       float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f;
  int k = 0;
  for (; k + 8 <= nslab; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = slabs[(long)(k + u) * n + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; k < nslab; ++k) acc += slabs[(long)k * n + i];
  out[i] = acc;
}

// the same sums with 4x the parallelism: a block owns 64 outputs (16 float4) and splits the slabs over 16
// groups of 16 threads; a thread adds slabs g, g+16, g+32, ... in order (loads in flight together), then the
// 16 group sums are added in group order.  Fixed order per element, independent of n (so of the batch split).
__global__ __launch_bounds__(256) void slab_sum4_kernel(const float* __restrict__ slabs, int nslab, long n4,
                                                        float* __restrict__ out) {
  __shared__ f32x4 part[16][16];
  const int q = threadIdx.x & 15, g = threadIdx.x >> 4;
  const long i4 = (long)blockIdx.x * 16 + q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i4 < n4) {
    const f32x4* src = reinterpret_cast<const f32x4*>(slabs) + i4;
#pragma unroll 16
    for (int k = g; k < nslab; k += 16) acc += src[(long)k * n4];
  }
  part[g][q] = acc;
  __syncthreads();
  if (threadIdx.x < 16 && i4 < n4) {
    f32x4 t = part[0][q];
#pragma unroll
    for (int j = 1; j < 16; ++j) t += part[j][q];
    reinterpret_cast<f32x4*>(out)[i4] = t;
  }
}

int slab_sum(const float* slabs, int nslab, long n, float* out, hipStream_t s) {
  ProfScope ps("slab_sum", 0.0, s);
  if ((n & 3) == 0 && ((reinterpret_cast<uintptr_t>(slabs) | reinterpret_cast<uintptr_t>(out)) & 15) == 0) {
    const long n4 = n >> 2;
    hipLaunchKernelGGL(slab_sum4_kernel, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, s, slabs, nslab, n4, out);
  } else {
    hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slabs, nslab, n, out);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------- plan helpers
long act_floats(const damc_layer_t& L, int B) { return (long)B * L.hout * L.wout * L.cout; }

int validate(const damc_generator_t* g) {
  if (!g || g->n_layers < 1 || g->n_layers > DAMC_MAX_LAYERS) return DAMC_ERR_ARG;
  for (int i = 0; i < g->n_layers; ++i) {
    const damc_layer_t& L = g->layers[i];
    const bool last = i == g->n_layers - 1;
    switch (L.kind) {
      case DAMC_LAYER_PROJ:
        if (i != 0 || L.hin != 1 || L.win != 1 || L.stride != 1 || L.pad != 0 || L.hout != L.k) return DAMC_ERR_ARG;
        break;
      case DAMC_LAYER_UP2:
        if (i == 0 || last || L.k != 4 || L.stride != 2 || L.pad != 1 || L.hout != 2 * L.hin) return DAMC_ERR_ARG;
        break;
      case DAMC_LAYER_SMALLC:
        if (!last || i == 0 || L.cout > 4 || L.act != DAMC_ACT_TANH) return DAMC_ERR_ARG;
        break;
      case DAMC_LAYER_LINEAR:
        if (L.hin != 1 || L.hout != 1) return DAMC_ERR_ARG;
        break;
      default:
        return DAMC_ERR_ARG;
    }
    if (L.engine != DAMC_ENGINE_LIMB && L.engine != DAMC_ENGINE_FP32) return DAMC_ERR_ARG;
    if (i > 0) {
      const damc_layer_t& P = g->layers[i - 1];
      if (P.cout != L.cin || P.hout != L.hin || P.wout != L.win) return DAMC_ERR_ARG;
      if (P.engine != L.engine) return DAMC_ERR_ARG;  // one engine per generator
    }
    if (!last && L.act == DAMC_ACT_TANH) return DAMC_ERR_UNSUPPORTED;
  }
  const damc_layer_t& F = g->layers[g->n_layers - 1];
  if (F.kind == DAMC_LAYER_PROJ || F.kind == DAMC_LAYER_UP2) return DAMC_ERR_UNSUPPORTED;
  if (g->layers[0].cin != g->nz) return DAMC_ERR_ARG;
  return 0;
}

// split-K slices for the PROJ/LINEAR-first-layer dgrad: depends on K only (never on the batch),
// so per-chain results are bitwise identical for any sharding of the batch.
int proj_slices(long K) {
  long s = K / 256;
  if (s < 1) s = 1;
  if (s > 512) s = 512;
  return (int)s;
}
// slice length: a multiple of the K-major engine's K tile (depends on K only, never on the batch)
int proj_k_per(long K, int S) { return (int)(((K + S - 1) / S + 31) / 32 * 32); }

// Limb engine (gemm.hip, fp32-accurate bf16 MFMA) for the UP2 convolutions whose gathered channel
// count is a multiple of 32.  Packed weights and workspaces always carry the x3 copies such a layer
// can use; a descriptor whose layers say engine = DAMC_ENGINE_FP32 routes the launches to the fp32-MFMA
// K-major engine instead.  The choice travels in the descriptor (no process-global state), so two
// streams or threads may use different engines at once.
bool limb(const damc_layer_t& L) { return L.engine == DAMC_ENGINE_LIMB; }
bool x3_fwd_cap(const damc_layer_t& L) {
  return L.kind == DAMC_LAYER_UP2 && L.cin % damc::KM_BK == 0 && L.cout % 8 == 0;
}
bool x3_bwd_cap(const damc_layer_t& L) {
  return L.kind == DAMC_LAYER_UP2 && L.cout % damc::KM_BK == 0 && L.cin % 8 == 0;
}
bool x3_fwd(const damc_layer_t& L) { return limb(L) && x3_fwd_cap(L); }
// first layer z.W as a 1x1 convolution on the limb engine (z split into limbs per call)
bool x3_proj_cap(const damc_layer_t& L) {
  return L.kind == DAMC_LAYER_PROJ && L.cin % damc::KM_BK == 0 && L.cout % 8 == 0;
}
bool x3_proj(const damc_layer_t& L) { return limb(L) && x3_proj_cap(L); }
bool x3_bwd(const damc_layer_t& L) { return limb(L) && x3_bwd_cap(L); }
size_t up2_floats(const damc_layer_t& L) { return (size_t)L.cin * L.cout * 16; }
// the sign block of a UP2 layer's forward (K = 4 Cin per phase) and input-gradient (K = 16 Cout) limb weights
// (damc::x3_conv_negk: by shape, the same for the packing and every launch that reads it)
int up2_negk_fwd(const damc_layer_t& L) { return damc::x3_conv_negk((long)L.hin * L.win, L.cout, 4 * L.cin, 4); }
int up2_negk_bwd(const damc_layer_t& L) { return damc::x3_conv_negk((long)L.hin * L.win, L.cin, 16 * L.cout, 1); }
// x3 copy of a packed weight matrix, stored behind its fp32 packing (n floats, 16-B aligned)
const unsigned short* x3_of(const float* w, size_t n) { return reinterpret_cast<const unsigned short*>(w + n); }
// activation j needs an x3 copy when layer j+1 consumes it in the forward pass, or layer j consumes its
// gradient (stored in the same buffer) in the backward pass
bool h_needs_x3(const damc_generator_t* g, int j) {
  return (j + 1 < g->n_layers && x3_fwd_cap(g->layers[j + 1])) || (j >= 1 && x3_bwd_cap(g->layers[j]));
}

// Activation j as sign bits: its producer is a limb-engine epilogue with LReLU, and the kernel that
// masks the next gradient with it (limb dgrad of layer j+1, or the k3 output-layer dgrad) reads bits.
bool hbits_cap(const damc_generator_t* g, int j) {
  if (j + 1 >= g->n_layers) return false;
  const damc_layer_t& L = g->layers[j];
  const damc_layer_t& N = g->layers[j + 1];
  const bool prod = (j == 0) ? x3_proj_cap(L) : x3_fwd_cap(L);
  return prod && L.act == DAMC_ACT_LRELU && (x3_bwd_cap(N) || smallc_k3(N) || smallc_s2_mfma(N));
}
bool hbits(const damc_generator_t* g, int j) { return limb(g->layers[0]) && hbits_cap(g, j); }
// the fp32 activation j is stored unless sign bits carry the mask and the next layer's forward gathers
// limbs (the output layer's forward reads fp32)
bool h_f32(const damc_generator_t* g, int j) {
  return !(hbits(g, j) && j + 1 < g->n_layers && x3_fwd(g->layers[j + 1]));
}

struct Workspace {
  std::vector<float*> h;  // activations (NHWC), one per layer except the final one
  std::vector<unsigned char*> hb;  // sign bits of h (LReLU' masks) or nullptr
  std::vector<unsigned short*> h3;  // x3 limb copies of h (limb engine operands) or nullptr
  unsigned short* z3;               // x3 limbs of z (limb-engine first layer) or nullptr
  float* delta;           // final-layer pre-activation gradient (NHWC / row-major)
  float* slabs;           // split-K partial gradients
  float* glik;            // their fixed-order sum: grad of the likelihood term (B, nz)
  float* pbuf;            // per-tap projections of the output layer (two-stage forward)
  float* kslab;           // split-K slabs of the limb-engine convolutions at small batch (or nullptr)
  long kslab_floats;
  unsigned* kticket_mem;  // split-K fix-up counters and claims (2 damc::X3_KTICKETS words, with kslab)
  unsigned* kticket;      // = kticket_mem once this call has zeroed them (the posterior call), else nullptr
  unsigned kepoch;        // the call's fix-up launches so far (GemmArgs::kepoch_ctr)
  int nslab;
  size_t bytes;
};

__global__ void zero_u32_kernel(unsigned* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0u;
}

size_t carve(const damc_generator_t* g, int B, char* base, Workspace* w) {
  size_t off = 0;
  auto take = [&](long floats) -> float* {
    float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((size_t)floats * sizeof(float) + 255) / 256 * 256;
    return p;
  };
  if (w) {
    w->h.clear();
    w->h3.clear();
  }
  for (int i = 0; i + 1 < g->n_layers; ++i) {
    float* p = take(act_floats(g->layers[i], B));
    if (w) w->h.push_back(p);
  }
  for (int i = 0; i + 1 < g->n_layers; ++i) {
    unsigned short* p = nullptr;
    if (h_needs_x3(g, i)) p = reinterpret_cast<unsigned short*>(take(act_floats(g->layers[i], B) * 3 / 2));
    if (w) w->h3.push_back(p);
  }
  if (w) w->hb.clear();
  for (int i = 0; i + 1 < g->n_layers; ++i) {
    unsigned char* p = nullptr;
    if (hbits_cap(g, i)) p = reinterpret_cast<unsigned char*>(take(act_floats(g->layers[i], B) / 32 + 4));
    if (w) w->hb.push_back(p);
  }
  const damc_layer_t& F = g->layers[g->n_layers - 1];
  float* d = take(act_floats(F, B));
  const damc_layer_t& L0 = g->layers[0];
  const long K0 = (long)L0.hout * L0.wout * L0.cout;
  const int S = (g->n_layers == 1) ? 1 : proj_slices(K0);
  float* sl = take((long)S * B * g->nz);
  float* gl = take((long)B * g->nz);
  // the output layer's per-tap projections, one buffer per 128-channel chunk of its input (proj16's partials)
  float* pb = (F.kind == DAMC_LAYER_SMALLC)
                  ? take((long)B * F.hin * F.win * smallc_ntile(F) * 32 * ((F.cin + damc::PROJ_CHUNK - 1) / damc::PROJ_CHUNK))
                  : nullptr;
  unsigned short* z3 =
      x3_proj_cap(L0) ? reinterpret_cast<unsigned short*>(take((long)B * g->nz * 3 / 2 + 4)) : nullptr;
  // split-K slabs: the largest any UP2 forward / input gradient of this batch uses (damc::x3_ksplit)
  long ksf = 0;
  for (int i = 0; i < g->n_layers; ++i) {
    const damc_layer_t& L = g->layers[i];
    if (L.kind != DAMC_LAYER_UP2) continue;
    if (x3_fwd_cap(L))
      ksf = std::max(ksf, damc::x3_ksplit_floats(B * L.hin * L.win, L.cout, 4 * L.cin, 4, up2_negk_fwd(L)));
    if (x3_bwd_cap(L))
      ksf = std::max(ksf, damc::x3_ksplit_floats(B * L.hin * L.win, L.cin, 16 * L.cout, 1, up2_negk_bwd(L)));
  }
  float* ks = ksf ? take(ksf) : nullptr;
  unsigned* tk = ksf ? reinterpret_cast<unsigned*>(take(2 * damc::X3_KTICKETS)) : nullptr;
  if (w) {
    w->kslab = ks;
    w->kslab_floats = ksf;
    w->kticket_mem = tk;
    w->kticket = nullptr;
    w->kepoch = 0;
    w->z3 = z3;
    w->delta = d;
    w->slabs = sl;
    w->glik = gl;
    w->pbuf = pb;
    w->nslab = S;
    w->bytes = off;
  }
  return off;
}

double conv_flops(const damc_layer_t& L, int B) {
  // MACs of the transposed conv = outputs x Cin x (taps hitting each output)
  const double taps = (double)L.k * L.k / ((double)L.stride * L.stride);
  return 2.0 * B * (double)L.hout * L.wout * L.cout * L.cin * taps;
}

// forward of layers [0, n-1) into ws.h; returns 0 on success.  z3_ready: ws.z3 already holds z's limbs (the previous
// posterior update wrote them)
// f32a: limb-engine convolutions gather their input as fp32 (gemm.hip X3_F32A), so every activation is stored fp32
// and no limb copy is written
// proj: the last hidden layer's epilogue also runs the output layer's projection into ws.pbuf (proj_fusable)
int forward_hidden(const damc_generator_t* g, const float* z, int B, Workspace& ws, hipStream_t s,
                   bool z3_ready = false, bool f32a = false, bool proj = false) {
  for (int i = 0; i + 1 < g->n_layers; ++i) {
    const damc_layer_t& L = g->layers[i];
    GemmArgs a;
    a.bias = L.bias;
    a.bias_mod = L.cout;
    a.act = L.act;
    a.slope = L.slope;
    a.C = ws.h[i];
    int rc;
    bool wrote_x3 = false;  // the epilogue already wrote ws.h3[i]
    if (x3_proj(L) && i == 0) {
      // z . W on the limb engine: z -> limbs, 1x1 "convolution" against the x3 copy of the dgrad
      // packing [(oy,ox,co)][ci]; the epilogue writes the next layer's limbs too
      const int N = L.hout * L.wout * L.cout;
      if (!z3_ready) {
        ProfScope ps("split_x3", 0.0, s);
        if ((rc = damc::launch_split_x3(z, (long)B * L.cin, ws.z3, s))) return rc;
      }
      a.A = z;
      a.A3 = ws.z3;
      a.B3 = x3_of(L.w_bwd, (size_t)L.cin * N);
      a.b32k = L.w_bwd;  // the same weights as fp32 rows (the skinny kernel splits them in registers)
      a.b_negblk = 1;
      a.Cg = L.cin;
      a.ldc = N;
      a.M = B;
      a.N = N;
      a.K = L.cin;
      a.k_per_z = a.K;
      if (g->n_layers > 1 && x3_fwd(g->layers[1])) {
        if (!f32a) a.C3 = ws.h3[0];
        wrote_x3 = true;
      }
      if (hbits(g, 0)) a.sgn = ws.hb[0];
      if (!h_f32(g, 0) && !f32a) a.C = nullptr;
      rc = damc::launch_gemm(a, damc::A_CONV, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "proj_fwd",
                             2.0 * B * (double)N * L.cin, s);
    } else if (L.kind == DAMC_LAYER_PROJ && damc::conv_kmajor_ok(L.cin)) {
      // z . W as a 1x1 "convolution" on the K-major engine; its B operand [(oy,ox,co)][ci] is the
      // dgrad packing
      const int N = L.hout * L.wout * L.cout;
      a.A = (i == 0) ? z : ws.h[i - 1];
      a.Cg = L.cin;
      a.B = L.w_bwd;
      a.b_kmajor = 1;
      a.ldb = L.cin;
      a.ldc = N;
      a.M = B;
      a.N = N;
      a.K = L.cin;
      a.k_per_z = a.K;
      rc = damc::launch_gemm(a, damc::A_CONV, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "proj_fwd",
                             2.0 * B * (double)N * L.cin, s);
    } else if (L.kind == DAMC_LAYER_PROJ || L.kind == DAMC_LAYER_LINEAR) {
      const int N = L.hout * L.wout * L.cout;
      a.A = (i == 0) ? z : ws.h[i - 1];
      a.lda = L.cin;
      a.B = L.w_fwd;
      a.ldb = N;
      a.ldc = N;
      a.M = B;
      a.N = N;
      a.K = L.cin;
      a.k_per_z = a.K;
      // a first layer whose nz is no multiple of 32 (SVHN, CelebA-64: nz = 100): the small-GEMM kernel, one 16 x 16
      // tile per wave (SVHN B=64: 2048 waves; the tiled engine ran 64 workgroups for 29 us); chosen by shape, never by
      // batch, so sharded chains stay bitwise the whole batch's.  DAMC_PROJ_SMALL=0 (read per call): the tiled engine
      const char* eps_ = getenv("DAMC_PROJ_SMALL");
      rc = DAMC_ERR_UNSUPPORTED;
      if (L.kind == DAMC_LAYER_PROJ && !(eps_ && eps_[0] == '0')) {
        ProfScope ps("proj_fwd", 2.0 * B * (double)N * L.cin, s);
        rc = damc::launch_small_gemm(a.A, a.lda, a.B, a.ldb, L.bias, a.C, a.ldc, B, N, L.cin, s, L.cout, L.act,
                                     L.slope);
      }
      if (rc == DAMC_ERR_UNSUPPORTED)
        rc = damc::launch_gemm(a, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "proj_fwd",
                               2.0 * B * (double)N * L.cin, s);
    } else {  // UP2
      a.A = ws.h[i - 1];
      a.Hin = L.hin;
      a.Win = L.win;
      a.Cg = L.cin;
      a.Hq = L.hin;
      a.Wq = L.win;
      a.kw = 2;
      a.stride = 1;
      a.B = L.w_fwd;
      a.b_kmajor = damc::conv_kmajor_ok(L.cin);
      a.ldb = a.b_kmajor ? 4L * L.cin : L.cout;
      a.b_zstride = 4L * L.cin * L.cout;
      a.ldc = L.cout;
      a.M = B * L.hin * L.win;
      a.N = L.cout;
      a.K = 4 * L.cin;
      a.Hout = L.hout;
      a.Wout = L.wout;
      if (x3_fwd(L)) {
        if (f32a)
          a.a_f32 = 1;  // A = ws.h[i - 1] as fp32
        else
          a.A3 = ws.h3[i - 1];
        a.B3 = x3_of(L.w_fwd, up2_floats(L));
        a.b_negblk = 1;
        a.negk = up2_negk_fwd(L);
        if (i + 1 < g->n_layers && x3_fwd(g->layers[i + 1])) {  // the next layer's operand
          if (!f32a) a.C3 = ws.h3[i];
          wrote_x3 = true;
        }
        if (hbits(g, i)) a.sgn = ws.hb[i];
        if (!h_f32(g, i) && !f32a) a.C = nullptr;
        a.kslab = ws.kslab;  // split-K when the batch leaves the grid under-filled
        a.kslab_floats = ws.kslab_floats;
        a.kticket = ws.kticket;
        a.kepoch_ctr = &ws.kepoch;
        if (proj && i + 2 == g->n_layers) {  // the output layer's per-tap projections (smallc_fwd_twostage's stage 1)
          const damc_layer_t& F = g->layers[i + 1];
          a.proj_w = F.w_bwd;
          a.proj_ldw = F.cin;
          a.proj_np = 32 * smallc_ntile(F);
          a.proj_out = ws.pbuf;
          a.proj_pstride = (long)B * F.hin * F.win * a.proj_np;
          // the activation itself is not stored when its sign bits carry the output layer's dgrad mask (k3 output
          // layers, hbits); a k4 s2 output layer's dgrad reads the fp32 activation's sign
          a.proj_nostore = hbits(g, i) ? 1 : 0;
          if (!a.C) a.C = ws.h[i];
        }
      }
      rc = damc::launch_gemm(a, damc::A_CONV, damc::EPI_BIAS_ACT, damc::O_PHASE, 4, "upconv_fwd", conv_flops(L, B), s);
    }
    if (rc) return rc;
    if (i + 1 < g->n_layers && x3_fwd(g->layers[i + 1]) && !wrote_x3 && !f32a) {
      ProfScope ps("split_x3", 0.0, s);
      if ((rc = damc::launch_split_x3(ws.h[i], act_floats(L, B), ws.h3[i], s))) return rc;
    }
  }
  return 0;
}

// the output layer's projection can run in the epilogue of the ConvT before it (limb engine, k4 s2, every channel in
// one 128 x 256 tile)
bool proj_fusable(const damc_generator_t* g, const Workspace& ws) {
  const int n = g->n_layers;
  if (n < 3 || !ws.pbuf) return false;
  const damc_layer_t& F = g->layers[n - 1];
  const damc_layer_t& L = g->layers[n - 2];
  return F.kind == DAMC_LAYER_SMALLC && smallc_twostage_ok(F) && smallc_proj16_ok(F) && L.kind == DAMC_LAYER_UP2 &&
         x3_fwd(L) && L.cout == F.cin && F.w_bwd && (F.cin <= damc::PROJ_CHUNK || F.cin % damc::PROJ_CHUNK == 0);
}

// final layer forward: delta (+ optional x_hat NCHW / row-major) and |x_hat-x|^2/(2s^2) into sqerr
int forward_final(const damc_generator_t* g, int B, const float* z, const float* x, float inv_s2, Workspace& ws,
                  float* xhat, float* sqerr, bool want_delta, hipStream_t s, bool p_ready = false) {
  const int n = g->n_layers;
  const damc_layer_t& F = g->layers[n - 1];
  const float* hin = n >= 2 ? ws.h[n - 2] : z;
  if (F.kind == DAMC_LAYER_SMALLC)
    return smallc_fwd(F, hin, B, want_delta ? x : nullptr, inv_s2, want_delta ? ws.delta : nullptr, xhat, sqerr,
                      ws.pbuf, s, p_ready);
  // LINEAR final layer
  GemmArgs a;
  a.A = hin;
  a.lda = F.cin;
  a.B = F.w_fwd;
  a.ldb = F.cout;
  a.ldc = F.cout;
  a.M = B;
  a.N = F.cout;
  a.K = F.cin;
  a.k_per_z = a.K;
  a.bias = F.bias;
  a.bias_mod = F.cout;
  a.act = F.act;
  a.slope = F.slope;
  if (want_delta) {
    a.C = ws.delta;
    a.xres = x;
    a.inv_s2 = inv_s2;
    a.xhat = xhat;
    a.sqerr = sqerr;
    int rc = damc::launch_gemm(a, damc::A_DENSE, damc::EPI_RESID, damc::O_DENSE, 1, "linear_out",
                               2.0 * B * (double)F.cout * F.cin, s);
    return rc;
  }
  a.C = xhat;
  return damc::launch_gemm(a, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "linear_out",
                           2.0 * B * (double)F.cout * F.cin, s);
}

// input gradient of layer i >= 1 from d (the gradient w.r.t. its pre-activation), masked with the
// activation derivative of layer i-1: the result (the pre-activation gradient of layer i-1) overwrites
// ws.h[i-1] and/or, when only a limb-engine dgrad reads it, ws.h3[i-1] (*x3_only = true)
// f32a: the gradients limb-engine dgrads read are stored fp32 (d_f32: the incoming d is fp32 even where a limb copy
// would have been read); *f32_out reports the form written
int dgrad_layer(const damc_generator_t* g, int B, Workspace& ws, int i, const float* d, bool* x3_only,
                hipStream_t s, bool f32a = false, bool d_f32 = false, bool* f32_out = nullptr) {
  if (f32_out) *f32_out = false;
  {
    const damc_layer_t& L = g->layers[i];
    const damc_layer_t& P = g->layers[i - 1];
    float* out = ws.h[i - 1];  // dgrad overwrites the activation it is masked with
    int rc;
    bool x3_out = false;  // the gradient went straight into its x3 copy
    if (L.kind == DAMC_LAYER_SMALLC) {
      const bool fo = f32a && x3_bwd(P) && hbits(g, i - 1) &&
                      ((smallc_k3(L) && smallc_k3_mfma_ok(L)) || smallc_s2_mfma(L));
      x3_out = !fo && x3_bwd(P) && smallc_x3_ok(L);
      rc = smallc_dgrad(L, out, B, d, P.act, P.slope, x3_out ? ws.h3[i - 1] : nullptr,
                        hbits(g, i - 1) ? ws.hb[i - 1] : nullptr, s, fo);
      if (fo && f32_out) *f32_out = true;
    } else if (L.kind == DAMC_LAYER_UP2) {
      const bool x3 = x3_bwd(L);
      GemmArgs a;
      a.A = d;
      a.Hin = L.hout;
      a.Win = L.wout;
      a.Cg = L.cout;
      a.Hq = L.hin;
      a.Wq = L.win;
      a.kw = 4;
      a.stride = 2;
      a.pad_y = 1;
      a.pad_x = 1;
      a.B = L.w_bwd;
      a.b_kmajor = damc::conv_kmajor_ok(L.cout);
      a.ldb = a.b_kmajor ? 16L * L.cout : L.cin;
      a.C = out;
      a.ldc = L.cin;
      a.M = B * L.hin * L.win;
      a.N = L.cin;
      a.K = 16 * L.cout;
      a.k_per_z = a.K;
      a.mask = out;
      a.mask_act = P.act;
      a.mask_slope = P.slope;
      if (x3) {
        if (d_f32)
          a.a_f32 = 1;  // A = d as fp32
        else
          a.A3 = ws.h3[i];
        a.B3 = x3_of(L.w_bwd, up2_floats(L));
        a.b_negblk = 1;
        a.negk = up2_negk_bwd(L);
        a.kslab = ws.kslab;
        a.kslab_floats = ws.kslab_floats;
        a.kticket = ws.kticket;
        a.kepoch_ctr = &ws.kepoch;
        if (hbits(g, i - 1)) {
          a.mask_sgn = ws.hb[i - 1];
          a.mask = nullptr;
        }
        if (x3_bwd(P) && f32a && hbits(g, i - 1)) {  // the next dgrad gathers this gradient as fp32
          if (f32_out) *f32_out = true;
        } else if (x3_bwd(P)) {  // only the next dgrad reads this gradient: limbs only, the fp32 activation stays
          a.C3 = ws.h3[i - 1];
          a.C = nullptr;
          x3_out = true;
        }
      }
      rc = damc::launch_gemm(a, damc::A_CONV, damc::EPI_MASK, damc::O_DENSE, 1, "upconv_dgrad", conv_flops(L, B), s);
    } else {  // LINEAR hidden/final
      GemmArgs a;
      a.A = d;
      a.lda = L.cout;
      a.B = L.w_bwd;
      a.ldb = L.cin;
      a.C = out;
      a.ldc = L.cin;
      a.M = B;
      a.N = L.cin;
      a.K = L.cout;
      a.k_per_z = a.K;
      a.mask = out;
      a.mask_act = P.act;
      a.mask_slope = P.slope;
      rc = damc::launch_gemm(a, damc::A_DENSE, damc::EPI_MASK, damc::O_DENSE, 1, "linear_dgrad",
                             2.0 * B * (double)L.cin * L.cout, s);
    }
    if (rc) return rc;
    if (x3_bwd(P) && !x3_out && !(f32_out && *f32_out)) {  // the next dgrad reads this gradient through the limb engine
      ProfScope ps("split_x3", 0.0, s);
      if ((rc = damc::launch_split_x3(out, act_floats(P, B), ws.h3[i - 1], s))) return rc;
    }
    *x3_only = x3_out;
  }
  return 0;
}

// first layer: dz = dA0 . W0^T  (split-K into slabs); d = the fp32 pre-activation gradient of layer 0
int dz_slabs(const damc_generator_t* g, int B, Workspace& ws, const float* d, hipStream_t s) {
  const damc_layer_t& L0 = g->layers[0];
  const long K = (long)L0.hout * L0.wout * L0.cout;
  GemmArgs a;
  a.A = d;
  a.lda = K;
  a.B = L0.w_bwd;
  a.ldb = L0.cin;
  const bool km = L0.kind == DAMC_LAYER_PROJ && damc::conv_kmajor_ok((int)K);
  if (km) {  // 1x1 "convolution" with Cg = K; B operand [ci][(oy,ox,co)] is the forward packing
    a.Cg = (int)K;
    a.B = L0.w_fwd;
    a.b_kmajor = 1;
    a.ldb = K;
  }
  a.C = ws.slabs;
  a.ldc = L0.cin;
  a.c_zstride = (long)B * L0.cin;
  a.M = B;
  a.N = L0.cin;
  a.K = (int)K;
  a.k_per_z = proj_k_per(K, ws.nslab);
  const int S = (int)((K + a.k_per_z - 1) / a.k_per_z);
  // slices beyond S (when rounding shrank the count) must contribute zeros
  if (S < ws.nslab) DAMC_CHECK(hipMemsetAsync(ws.slabs, 0, sizeof(float) * ws.nslab * (size_t)B * L0.cin, s));
  return damc::launch_gemm(a, km ? damc::A_CONV : damc::A_DENSE, damc::EPI_STORE, damc::O_DENSE, S, "proj_dgrad",
                           2.0 * B * (double)K * L0.cin, s);
}

// backward from ws.delta to the PROJ/first-layer split-K slabs (f32a: see dgrad_layer)
int backward(const damc_generator_t* g, int B, Workspace& ws, hipStream_t s, bool f32a = false) {
  const float* d = ws.delta;  // gradient w.r.t. the pre-activation of layer i (current)
  bool d_f32 = false;
  for (int i = g->n_layers - 1; i >= 1; --i) {
    bool x3_only = false, fo = false;
    int rc = dgrad_layer(g, B, ws, i, d, &x3_only, s, f32a, d_f32, &fo);
    if (rc) return rc;
    d = ws.h[i - 1];
    d_f32 = fo;
  }
  return dz_slabs(g, B, ws, d, s);
}

// ------------------------------------------------------------------ training backward (weight gradients)
// The G update of a training iteration (workspace/train_gen_recon.py:222-231): after the forward above,
// dL/dx_hat -> per-layer dL/dW, dL/db (and optionally dL/dz).  Layer i's weight gradient is taken before
// its input gradient overwrites the activation buffers it reads.  k4 s2 p1 and first-layer weight
// gradients run on the limb engine (gemm.hip O_WGRAD) over pixel-major transposes (wgrad.hip) of the layer
// input and of the pre-activation gradient, the latter split into the 4 output phases; batches are padded
// to Bp = a multiple of 32 samples with zeros.
struct TrainWs {
  unsigned short* tin;  // transposed layer input, x3 [Cin][pixels][Bp]
  unsigned short* tdl;  // transposed pre-activation gradient, x3 [phase][Cout][pixels][Bp]
  float* wslab;         // O_WGRAD split-K slabs
  float* part;          // bias partial sums / output-layer wgrad partials
  float* ctmp;          // column-sum scratch
};

int bp_of(int B) { return (B + 31) / 32 * 32; }

// split-K of a k4 s2 p1 weight gradient: >= 512 workgroups; slice length a multiple of 32 (depends on the
// shape and Bp only)
void up2_wgrad_split(const damc_layer_t& L, int Bp, int* S, int* kper) {
  const long M = 4L * L.cin, N = L.cout, K = (long)L.hin * L.win * Bp;
  const long base = ((M + 255) / 256) * ((N + 127) / 128) * 4;
  const long nkt = K / 32;
  long sl = std::max(1L, std::min(std::min((512 + base - 1) / base, 16L), nkt));
  const long kp = (nkt + sl - 1) / sl * 32;
  *kper = (int)kp;
  *S = (int)((K + kp - 1) / kp);
}

size_t carve_train(const damc_generator_t* g, int B, char* base, TrainWs* t) {
  const int Bp = bp_of(B);
  size_t tin = 0, tdl = 0, wslab = 0, part = 0, ctmp = 0;
  for (int i = 0; i < g->n_layers; ++i) {
    const damc_layer_t& L = g->layers[i];
    const size_t nb = Bp / 32;
    if (L.kind == DAMC_LAYER_UP2) {
      const size_t P = (size_t)L.hin * L.win;
      int S, kp;
      up2_wgrad_split(L, Bp, &S, &kp);
      tin = std::max(tin, (size_t)L.cin * P * Bp);
      tdl = std::max(tdl, 4 * (size_t)L.cout * P * Bp);
      wslab = std::max(wslab, 4 * (size_t)S * 4 * L.cin * L.cout);
      part = std::max(part, 4 * P * nb * L.cout);
      ctmp = std::max(ctmp, damc::colsum_tmp_floats((long)(4 * P * nb), L.cout));
    } else if (L.kind == DAMC_LAYER_PROJ) {
      const size_t Pd = (size_t)L.hout * L.wout;
      tin = std::max(tin, (size_t)L.cin * Bp);
      tdl = std::max(tdl, (size_t)L.cout * Pd * Bp);
      part = std::max(part, Pd * nb * L.cout);
      ctmp = std::max(ctmp, damc::colsum_tmp_floats((long)(Pd * nb), L.cout));
    } else if (L.kind == DAMC_LAYER_SMALLC) {
      part = std::max(part, damc::smallc_wgrad_part_floats(L, B));
      ctmp = std::max(ctmp, damc::smallc_wgrad_tmp_floats(L, B));
      ctmp = std::max(ctmp, damc::colsum_tmp_floats((long)B * L.hout * L.wout, L.cout));
    } else {
      ctmp = std::max(ctmp, damc::colsum_tmp_floats(B, L.cout));
    }
  }
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) / 256 * 256;
    return p;
  };
  char* p_tin = take(tin * 6);
  char* p_tdl = take(tdl * 6);
  char* p_ws = take(wslab * 4);
  char* p_part = take(part * 4);
  char* p_ct = take(ctmp * 4);
  if (t) {
    t->tin = reinterpret_cast<unsigned short*>(p_tin);
    t->tdl = reinterpret_cast<unsigned short*>(p_tdl);
    t->wslab = reinterpret_cast<float*>(p_ws);
    t->part = reinterpret_cast<float*>(p_part);
    t->ctmp = reinterpret_cast<float*>(p_ct);
  }
  return off;
}

int train_backward(const damc_generator_t* g, int B, const float* z, const float* xhat, const float* gx,
                   const damc_generator_grads_t* gr, float* gz, Workspace& ws, TrainWs& tw, hipStream_t s) {
  const int n = g->n_layers;
  const damc_layer_t& F = g->layers[n - 1];
  const int Bp = bp_of(B), nb = Bp / 32;
  int rc;
  {
    ProfScope ps("out_delta", 0.0, s);
    const int hw = F.kind == DAMC_LAYER_LINEAR ? 1 : F.hout * F.wout;
    if ((rc = damc::launch_out_delta(gx, xhat, B, F.cout, hw, F.act, ws.delta, s))) return rc;
  }
  const float* d = ws.delta;  // pre-activation gradient of layer i: fp32 ...
  bool d_x3 = false;          // ... or (when a limb dgrad wrote it) only the limbs in ws.h3[i]
  for (int i = n - 1; i >= 0; --i) {
    const damc_layer_t& L = g->layers[i];
    float* dW = gr->w[i];
    float* db = L.bias ? gr->b[i] : nullptr;
    const float* in32 = i ? ws.h[i - 1] : z;
    if (L.kind == DAMC_LAYER_SMALLC) {
      if (i == 0 || !h_f32(g, i - 1) || d_x3) return DAMC_ERR_UNSUPPORTED;
      if (dW && (rc = damc::launch_smallc_wgrad(L, in32, d, B, tw.part, tw.ctmp, dW, s))) return rc;
      if (db && (rc = damc::launch_colsum(d, (long)B * L.hout * L.wout, L.cout, L.cout, db, tw.ctmp, s))) return rc;
    } else if (L.kind == DAMC_LAYER_LINEAR) {
      if (d_x3 || (i > 0 && !h_f32(g, i - 1))) return DAMC_ERR_UNSUPPORTED;
      if (dW && (rc = damc::launch_linear_wgrad(d, in32, B, L.cout, L.cin, dW, s))) return rc;
      if (db && (rc = damc::launch_colsum(d, B, L.cout, L.cout, db, tw.ctmp, s))) return rc;
    } else {
      const bool up2 = L.kind == DAMC_LAYER_UP2;
      const int hq = up2 ? L.hin : 1, wq = up2 ? L.win : 1;
      const long P = (long)hq * wq;
      // layer input, pixel-major (the limbs the forward gathered, else fp32)
      const unsigned short* in3 = (up2 && x3_fwd(L)) ? ws.h3[i - 1] : nullptr;
      if (up2 && !in3 && !h_f32(g, i - 1)) return DAMC_ERR_UNSUPPORTED;
      if (dW && (rc = damc::launch_transpose_x3(in3 ? nullptr : in32, in3, B, hq, wq, L.cin, hq, wq, 1, 1, 0, 0, Bp,
                                                tw.tin, nullptr, s)))
        return rc;
      const float* d32 = d_x3 ? nullptr : d;
      const unsigned short* d3 = d_x3 ? ws.h3[i] : nullptr;
      if (up2) {  // the 4 output phases of the gradient, each on the input grid
        rc = damc::launch_transpose_x3_4ph(d32, d3, B, L.hout, L.wout, L.cout, L.hin, L.win, Bp, tw.tdl,
                                           (long)L.cout * P * Bp * 3, db ? tw.part : nullptr, (long)P * nb * L.cout, s);
        if (rc) return rc;
      } else {  // PROJ: rows (co, output pixel) = the PyTorch (Cin, Cout, k, k) column order
        rc = damc::launch_transpose_x3(d32, d3, B, L.hout, L.wout, L.cout, L.hout, L.wout, 1, 1, 0, 0, Bp, tw.tdl,
                                       db ? tw.part : nullptr, s);
        if (rc) return rc;
      }
      if (dW) {
        GemmArgs a;
        a.A3 = tw.tin;
        a.B3 = tw.tdl;
        a.Cg = L.cin;
        a.Hin = hq;
        a.Win = wq;
        a.K = (int)(P * Bp);
        a.wg_bp = Bp;
        if (up2) {
          int S, kp;
          up2_wgrad_split(L, Bp, &S, &kp);
          a.kw = 2;
          a.wg_phases = 4;
          a.M = 4 * L.cin;
          a.N = L.cout;
          a.ldc = L.cout;
          a.c_zstride = (long)a.M * a.N;
          a.b_zstride = (long)L.cout * a.K;
          a.k_per_z = kp;
          a.C = tw.wslab;
          if ((rc = damc::launch_wgrad_x3(a, S, "wgrad_up2", conv_flops(L, B), s))) return rc;
          if ((rc = damc::launch_up2_wgrad_reduce(tw.wslab, S, L.cin, L.cout, dW, s))) return rc;
        } else {
          a.kw = 1;
          a.wg_phases = 1;
          a.M = L.cin;
          a.N = L.cout * L.hout * L.wout;
          a.ldc = a.N;
          a.c_zstride = (long)a.M * a.N;
          a.k_per_z = a.K;
          a.C = dW;
          if ((rc = damc::launch_wgrad_x3(a, 1, "wgrad_proj", 2.0 * B * (double)a.M * a.N, s))) return rc;
        }
      }
      if (db) {
        const long rows = (up2 ? 4 * P : (long)L.hout * L.wout) * nb;
        if ((rc = damc::launch_colsum(tw.part, rows, L.cout, L.cout, db, tw.ctmp, s))) return rc;
      }
    }
    if (i >= 1) {
      bool x3o = false;
      if ((rc = dgrad_layer(g, B, ws, i, d, &x3o, s))) return rc;
      d = ws.h[i - 1];
      d_x3 = x3o;
    } else if (gz) {
      if (n < 2 || d_x3) return DAMC_ERR_UNSUPPORTED;
      if ((rc = dz_slabs(g, B, ws, d, s))) return rc;
      if ((rc = slab_sum(ws.slabs, ws.nslab, (long)B * g->nz, gz, s))) return rc;
    }
  }
  return 0;
}

}  // namespace

// =============================================================================== C ABI
extern "C" int damc_generator_layer_packed_sizes(const damc_layer_t* L, size_t* fwd, size_t* bwd) {
  if (!L || !fwd || !bwd) return DAMC_ERR_ARG;
  const size_t n = (size_t)L->cin * L->cout * (L->kind == DAMC_LAYER_LINEAR ? 1 : (size_t)L->k * L->k);
  switch (L->kind) {
    case DAMC_LAYER_UP2:
      // fp32 packing, then (limb engine) its x3 copy: 3 bf16 per element = 1.5 floats
      *fwd = n + (x3_fwd_cap(*L) ? n * 3 / 2 : 0);
      *bwd = n + (x3_bwd_cap(*L) ? n * 3 / 2 : 0);
      return 0;
    case DAMC_LAYER_PROJ:
      *fwd = n;
      *bwd = n + (x3_proj_cap(*L) ? n * 3 / 2 : 0);
      return 0;
    case DAMC_LAYER_LINEAR:
      *fwd = n;
      *bwd = n;
      return 0;
    case DAMC_LAYER_SMALLC:
      *fwd = n;
      *bwd = (size_t)smallc_ntile(*L) * 32 * L->cin;  // two-stage projection layout
      return 0;
  }
  return DAMC_ERR_ARG;
}

extern "C" int damc_x3_layer_sign_block(const damc_layer_t* L, int input_grad) {
  if (!L) return 0;
  if (input_grad) return x3_bwd_cap(*L) ? up2_negk_bwd(*L) : 0;
  return x3_fwd_cap(*L) ? up2_negk_fwd(*L) : 0;
}

extern "C" int damc_pack_generator_layer(const damc_layer_t* L, const float* w, float* wf, float* wb, void* stream) {
  if (!L || !w || !wf) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  const long n = (long)L->cin * L->cout * (L->kind == DAMC_LAYER_LINEAR ? 1 : (long)L->k * L->k);
  const dim3 grid((unsigned)((n + 255) / 256)), blk(256);
  // LDS-tiled packing (fp32 + limbs in one pass) unless DAMC_PACK_TILED=0 (the element-wise A/B; bitwise the same)
  const char* pt = getenv("DAMC_PACK_TILED");
  const bool tiled = !(pt && pt[0] == '0');
  switch (L->kind) {
    case DAMC_LAYER_PROJ:
      if (!wb) return DAMC_ERR_ARG;
      if (tiled) {
        const int rc = damc::launch_pack_proj_tiled(
            w, L->cin, L->cout, L->k * L->k, wf, wb,
            x3_proj_cap(*L) ? reinterpret_cast<unsigned short*>(wb + n) : nullptr, s);
        if (rc != 1) return rc;
      }
      hipLaunchKernelGGL(pack_proj_kernel, grid, blk, 0, s, w, L->cin, L->cout, L->k, wf, wb);
      if (x3_proj_cap(*L))
        DAMC_CHECK((hipError_t)damc::launch_split_x3_negblk(wb, n, L->cin, reinterpret_cast<unsigned short*>(wb + n), s));
      break;
    case DAMC_LAYER_UP2:
      if (!wb || L->k != 4) return DAMC_ERR_ARG;
      if (tiled) {
        const int rc = damc::launch_pack_up2_tiled(
            w, L->cin, L->cout, wf, x3_fwd_cap(*L) ? reinterpret_cast<unsigned short*>(wf + n) : nullptr, wb,
            x3_bwd_cap(*L) ? reinterpret_cast<unsigned short*>(wb + n) : nullptr, s, up2_negk_fwd(*L),
            up2_negk_bwd(*L));
        if (rc != 1) return rc;
      }
      hipLaunchKernelGGL(pack_up2_kernel, grid, blk, 0, s, w, L->cin, L->cout, (int)damc::conv_kmajor_ok(L->cin),
                         (int)damc::conv_kmajor_ok(L->cout), wf, wb);
      // x3 copies with sign-alternating K blocks (gemm.h GemmArgs::b_negblk): rows of 4 Cin (forward, per phase
      // and output channel) and 16 Cout (input gradient, per input channel)
      // (in the K order the limb-engine kernels walk: damc::launch_split_x3_conv)
      if (x3_fwd_cap(*L))
        DAMC_CHECK((hipError_t)damc::launch_split_x3_conv(wf, n, 4 * L->cin, L->cin, reinterpret_cast<unsigned short*>(wf + n), s,
                                                          up2_negk_fwd(*L)));
      if (x3_bwd_cap(*L))
        DAMC_CHECK((hipError_t)damc::launch_split_x3_conv(wb, n, 16 * L->cout, L->cout, reinterpret_cast<unsigned short*>(wb + n), s,
                                                          up2_negk_bwd(*L)));
      break;
    case DAMC_LAYER_SMALLC:
      if (wb) DAMC_CHECK(hipMemsetAsync(wb, 0, sizeof(float) * smallc_ntile(*L) * 32 * (size_t)L->cin, s));
      hipLaunchKernelGGL(pack_smallc_kernel, grid, blk, 0, s, w, L->cin, L->cout, L->k, wf, wb);
      break;
    case DAMC_LAYER_LINEAR:
      if (!wb) return DAMC_ERR_ARG;
      hipLaunchKernelGGL(pack_linear_kernel, grid, blk, 0, s, w, L->cin, L->cout, wf, wb);
      break;
    default:
      return DAMC_ERR_ARG;
  }
  return (int)hipGetLastError();
}

extern "C" size_t damc_posterior_workspace_bytes(const damc_generator_t* g, int B) {
  if (validate(g) || B <= 0) return 0;
  return carve(g, B, nullptr, nullptr);
}

static int setup_ws(const damc_generator_t* g, int B, void* wsp, size_t wsb, Workspace* ws) {
  int rc = validate(g);
  if (rc) return rc;
  if (B <= 0) return DAMC_ERR_ARG;
  const size_t need = carve(g, B, nullptr, nullptr);
  if (!wsp || wsb < need) return DAMC_ERR_WORKSPACE;
  carve(g, B, reinterpret_cast<char*>(wsp), ws);
  return 0;
}

extern "C" int damc_generator_forward(const damc_generator_t* g, const float* z, int B, float* xhat, void* wsp,
                                      size_t wsb, void* stream) {
  Workspace ws;
  int rc = setup_ws(g, B, wsp, wsb, &ws);
  if (rc) return rc;
  if (!z || !xhat) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  rc = forward_hidden(g, z, B, ws, s);
  if (rc) return rc;
  return forward_final(g, B, z, nullptr, 1.f, ws, xhat, nullptr, false, s);
}

extern "C" int damc_likelihood_grad(const damc_generator_t* g, const float* z, const float* x, int B, double sigma,
                                    float* grad, void* wsp, size_t wsb, void* stream) {
  Workspace ws;
  int rc = setup_ws(g, B, wsp, wsb, &ws);
  if (rc) return rc;
  if (!z || !x || !grad) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  const float inv_s2 = (float)(1.0 / (sigma * sigma));
  if ((rc = forward_hidden(g, z, B, ws, s))) return rc;
  if ((rc = forward_final(g, B, z, x, inv_s2, ws, nullptr, nullptr, true, s))) return rc;
  if (g->n_layers == 1) {
    // single layer: the delta is the gradient w.r.t. layer-0 pre-activation; dz = delta . W
    return DAMC_ERR_UNSUPPORTED;
  }
  if ((rc = backward(g, B, ws, s))) return rc;
  const long n = (long)B * g->nz;
  return slab_sum(ws.slabs, ws.nslab, n, grad, s);
}

// ---- per-op hooks for ONE k4 s2 p1 ConvTranspose2d layer (damc_convT_fwd / damc_convT_dgrad),
// NHWC activations, the same kernels and engine choice as inside the Langevin step
static bool up2_hook_ok(const damc_layer_t* L, int B) {
  return L && B > 0 && L->kind == DAMC_LAYER_UP2 && L->k == 4 && L->stride == 2 && L->pad == 1 && L->cin > 0 &&
         L->cout > 0 && L->hout == 2 * L->hin && L->wout == 2 * L->win && L->w_fwd && L->w_bwd;
}

extern "C" size_t damc_convT_workspace_bytes(const damc_layer_t* L, int B) {
  if (!up2_hook_ok(L, B)) return 0;
  const size_t in = (size_t)B * L->hin * L->win * L->cin, out = (size_t)B * L->hout * L->wout * L->cout;
  return (std::max(in, out) * 6 + 255) / 256 * 256;  // limb copy of the A operand
}

extern "C" int damc_convT_fwd(const damc_layer_t* L, const float* in, int B, float* out, void* wsp, size_t wsb,
                              void* stream) {
  if (!up2_hook_ok(L, B) || !in || !out) return DAMC_ERR_ARG;
  if (!wsp || wsb < damc_convT_workspace_bytes(L, B)) return DAMC_ERR_WORKSPACE;
  hipStream_t s = as_stream(stream);
  GemmArgs a;
  a.bias = L->bias;
  a.bias_mod = L->cout;
  a.act = L->act;
  a.slope = L->slope;
  a.C = out;
  a.A = in;
  a.Hin = L->hin;
  a.Win = L->win;
  a.Cg = L->cin;
  a.Hq = L->hin;
  a.Wq = L->win;
  a.kw = 2;
  a.stride = 1;
  a.B = L->w_fwd;
  a.b_kmajor = damc::conv_kmajor_ok(L->cin);
  a.ldb = a.b_kmajor ? 4L * L->cin : L->cout;
  a.b_zstride = 4L * L->cin * L->cout;
  a.ldc = L->cout;
  a.M = B * L->hin * L->win;
  a.N = L->cout;
  a.K = 4 * L->cin;
  a.Hout = L->hout;
  a.Wout = L->wout;
  int rc;
  if (x3_fwd(*L)) {
    unsigned short* a3 = reinterpret_cast<unsigned short*>(wsp);
    if ((rc = damc::launch_split_x3(in, (long)B * L->hin * L->win * L->cin, a3, s))) return rc;
    a.A3 = a3;
    a.B3 = x3_of(L->w_fwd, up2_floats(*L));
    a.b_negblk = 1;
    a.negk = up2_negk_fwd(*L);
  }
  return damc::launch_gemm(a, damc::A_CONV, damc::EPI_BIAS_ACT, damc::O_PHASE, 4, "upconv_fwd", conv_flops(*L, B), s);
}

extern "C" int damc_convT_dgrad(const damc_layer_t* L, const float* gout, int B, const float* mask_pre, int mask_act,
                                float mask_slope, float* gin, void* wsp, size_t wsb, void* stream) {
  if (!up2_hook_ok(L, B) || !gout || !gin) return DAMC_ERR_ARG;
  if (!wsp || wsb < damc_convT_workspace_bytes(L, B)) return DAMC_ERR_WORKSPACE;
  hipStream_t s = as_stream(stream);
  GemmArgs a;
  a.A = gout;
  a.Hin = L->hout;
  a.Win = L->wout;
  a.Cg = L->cout;
  a.Hq = L->hin;
  a.Wq = L->win;
  a.kw = 4;
  a.stride = 2;
  a.pad_y = 1;
  a.pad_x = 1;
  a.B = L->w_bwd;
  a.b_kmajor = damc::conv_kmajor_ok(L->cout);
  a.ldb = a.b_kmajor ? 16L * L->cout : L->cin;
  a.C = gin;
  a.ldc = L->cin;
  a.M = B * L->hin * L->win;
  a.N = L->cin;
  a.K = 16 * L->cout;
  a.k_per_z = a.K;
  a.mask = mask_pre;
  a.mask_act = mask_pre ? mask_act : DAMC_ACT_NONE;
  a.mask_slope = mask_slope;
  int rc;
  if (x3_bwd(*L)) {
    unsigned short* a3 = reinterpret_cast<unsigned short*>(wsp);
    if ((rc = damc::launch_split_x3(gout, (long)B * L->hout * L->wout * L->cout, a3, s))) return rc;
    a.A3 = a3;
    a.B3 = x3_of(L->w_bwd, up2_floats(*L));
    a.b_negblk = 1;
    a.negk = up2_negk_bwd(*L);
  }
  return damc::launch_gemm(a, damc::A_CONV, mask_pre ? damc::EPI_MASK : damc::EPI_STORE, damc::O_DENSE, 1,
                           "upconv_dgrad", conv_flops(*L, B), s);
}

extern "C" int damc_posterior_langevin(const damc_generator_t* g, const damc_ebm_t* ebm, float* z, const float* x,
                                       int B, int n_steps, double sigma, double step, int with_noise, const float* noise,
                                       uint64_t seed, uint64_t step_offset, uint64_t chain_base, float* diag,
                                       void* wsp, size_t wsb, void* stream) {
  Workspace ws;
  int rc = setup_ws(g, B, wsp, wsb, &ws);
  if (rc) return rc;
  if (!z || !x || n_steps < 0) return DAMC_ERR_ARG;
  if (g->n_layers < 2) return DAMC_ERR_UNSUPPORTED;
  if (ebm && (ebm->nz != g->nz || !ebm->w1t || !ebm->w2t)) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  if (diag) DAMC_CHECK(hipMemsetAsync(diag, 0, sizeof(float) * 4 * (size_t)n_steps, s));
  const float inv_s2 = (float)(1.0 / (sigma * sigma));
  // the register-resident update kernel sums the first layer's split-K slabs itself (slab_sum4's order) and writes
  // z's limbs for the next step's first layer; DAMC_POST_FUSE=0 (read per call) keeps the separate kernels
  const char* pf = getenv("DAMC_POST_FUSE");
  const bool fuse = !(pf && pf[0] == '0');
  // the limb-engine convolutions gather fp32 activations and gradients (gemm.hip X3_F32A), bitwise the limb-gathering
  // form; DAMC_X3_F32A=0 (read per call) gathers limbs (CIFAR B=128 bench 51.1K -> 56.1K z-steps/s, B=16 per-rank
  // step 0.625 -> 0.478 ms; profiles/r04/bench_f32a_ab.txt, step_f32a_ab.txt)
  const char* fa = getenv("DAMC_X3_F32A");
  const bool f32a = !(fa && fa[0] == '0');
  // DAMC_SMALLC_FUSE (read per call, default on): the last ConvT's epilogue runs the output layer's projection on both
  // paths: the F32A tile projects its own 128-channel chunk per N tile (the gather adds the chunks' partials), the
  // limb-gathering path (DAMC_X3_F32A=0) projects every channel in the 128 x 256 tile
  const char* sf = getenv("DAMC_SMALLC_FUSE");
  const bool proj = !(sf && sf[0] == '0') && proj_fusable(g, ws);
  const bool z3_use = x3_proj(g->layers[0]) && ws.z3;
  bool z3_ready = false;
  if (ws.kticket_mem && n_steps > 0) {
    // the split-K GEMMs' in-GEMM fix-up counters and claims (damc::GemmArgs::kticket): zeroed once per call by a kernel
    // (a stream-ordered node like any other under graph capture); the call's launches tag them with their epochs
    hipLaunchKernelGGL(zero_u32_kernel, dim3((2 * damc::X3_KTICKETS + 255) / 256), dim3(256), 0, s, ws.kticket_mem,
                       2 * damc::X3_KTICKETS);
    DAMC_LAUNCH_CHECK();
    ws.kticket = ws.kticket_mem;
  }
  for (int i = 0; i < n_steps; ++i) {
    float* dg = diag ? diag + 4 * i : nullptr;
    if ((rc = forward_hidden(g, z, B, ws, s, z3_ready, f32a, proj))) return rc;
    if ((rc = forward_final(g, B, z, x, inv_s2, ws, nullptr, dg ? dg + 1 : nullptr, true, s, proj))) return rc;
    if ((rc = backward(g, B, ws, s, f32a))) return rc;
    const float* nz_i = noise ? noise + (size_t)i * B * g->nz : nullptr;
    const long n = (long)B * g->nz;
    // fused only where slab_sum takes its slab_sum4 order (the order the update kernel reproduces)
    const bool f = fuse && damc_posterior_update_fusable(ebm, g->nz) && (n & 3) == 0 &&
                   ((reinterpret_cast<uintptr_t>(ws.slabs) | reinterpret_cast<uintptr_t>(ws.glik)) & 15) == 0;
    if (!f && (rc = slab_sum(ws.slabs, ws.nslab, n, ws.glik, s))) return rc;
    bool wrote = false;
    rc = damc_launch_posterior_update(ebm, z, f ? ws.slabs : ws.glik, f ? ws.nslab : 1, n, B, g->nz, step,
                                      with_noise, nz_i, seed, step_offset + i, chain_base, dg, s,
                                      (f && z3_use) ? ws.z3 : nullptr, &wrote);
    if (rc) return rc;
    z3_ready = wrote;
  }
  return 0;
}

// ------------------------------------------------------------------------------------ training (G update)
extern "C" size_t damc_generator_train_workspace_bytes(const damc_generator_t* g, int B) {
  if (validate(g) || B <= 0) return 0;
  return carve(g, B, nullptr, nullptr) + carve_train(g, B, nullptr, nullptr);
}

static int setup_train(const damc_generator_t* g, int B, void* wsp, size_t wsb, Workspace* ws, TrainWs* tw) {
  int rc = validate(g);
  if (rc) return rc;
  if (B <= 0) return DAMC_ERR_ARG;
  const size_t n0 = carve(g, B, nullptr, nullptr);
  const size_t n1 = carve_train(g, B, nullptr, nullptr);
  if (!wsp || wsb < n0 + n1) return DAMC_ERR_WORKSPACE;
  carve(g, B, reinterpret_cast<char*>(wsp), ws);
  carve_train(g, B, reinterpret_cast<char*>(wsp) + n0, tw);
  return 0;
}

// The engine a G-update forward ran on decides which buffers it filled (limbs + sign bits, or fp32
// activations), so the backward must run on the same one: train_forward records (batch, engine) per
// workspace and train_backward refuses a descriptor that disagrees (DAMC_ERR_ARG) instead of reading
// buffers the forward never wrote.  Keyed by the caller's workspace, so concurrent streams / threads with
// their own workspaces do not interfere.  The backward consumes the record: it overwrites activation buffers
// as it goes, so a second backward of one forward (retain_graph) is refused rather than run on clobbered
// inputs.  The table is a bounded ring: a forward that is never backpropagated holds one slot until 64 newer
// workspaces have been recorded.
static std::mutex g_train_mu;
constexpr int TRAIN_REC_SLOTS = 64;
static const void* g_train_ws[TRAIN_REC_SLOTS];
static long g_train_key[TRAIN_REC_SLOTS];
static int g_train_next = 0;
static long train_key(const damc_generator_t* g, int B) { return (long)B * 4 + g->layers[0].engine; }
static int train_rec_find(const void* wsp) {
  for (int i = 0; i < TRAIN_REC_SLOTS; ++i)
    if (g_train_ws[i] == wsp) return i;
  return -1;
}

extern "C" int damc_generator_train_forward(const damc_generator_t* g, const float* z, int B, float* xhat, void* wsp,
                                            size_t wsb, void* stream) {
  Workspace ws;
  TrainWs tw;
  int rc = setup_train(g, B, wsp, wsb, &ws, &tw);
  if (rc) return rc;
  if (!z || !xhat) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  if ((rc = forward_hidden(g, z, B, ws, s))) return rc;
  if ((rc = forward_final(g, B, z, nullptr, 1.f, ws, xhat, nullptr, false, s))) return rc;
  std::lock_guard<std::mutex> lk(g_train_mu);
  int i = train_rec_find(wsp);
  if (i < 0) {
    i = g_train_next;
    g_train_next = (g_train_next + 1) % TRAIN_REC_SLOTS;
    g_train_ws[i] = wsp;
  }
  g_train_key[i] = train_key(g, B);
  return 0;
}

extern "C" int damc_generator_train_backward(const damc_generator_t* g, const float* z, const float* xhat,
                                             const float* grad_xhat, int B, const damc_generator_grads_t* grads,
                                             float* grad_z, void* wsp, size_t wsb, void* stream) {
  Workspace ws;
  TrainWs tw;
  int rc = setup_train(g, B, wsp, wsb, &ws, &tw);
  if (rc) return rc;
  if (!z || !xhat || !grad_xhat || !grads) return DAMC_ERR_ARG;
  {
    std::lock_guard<std::mutex> lk(g_train_mu);
    const int i = train_rec_find(wsp);
    if (i < 0 || g_train_key[i] != train_key(g, B)) return DAMC_ERR_ARG;
    g_train_ws[i] = nullptr;
  }
  return train_backward(g, B, z, xhat, grad_xhat, grads, grad_z, ws, tw, as_stream(stream));
}
