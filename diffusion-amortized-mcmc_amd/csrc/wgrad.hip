// wgrad.hip — generator weight / bias gradients: the device side of the G update of a training iteration
// (workspace/train_gen_recon.py:222-231: x_hat = G(z); sum((x_hat - x)^2).mean().backward()).
//
// The k4 s2 p1 and first-layer weight gradients are GEMMs over pixels and samples; they run on the limb
// engine (gemm.hip, O_WGRAD) over PIXEL-MAJOR transposed operands written here: [channel][pixel][sample]
// with the sample index fastest, so a 32-deep K tile is 32 samples of one pixel and a filter tap is a
// pixel shift of a whole K tile (no per-element masks, 16-B aligned limb loads).  The output layer
// (Cout <= 4) has N = k*k*Cout <= 64 and reads one large activation once: a direct kernel with the
// gradient window in LDS and the Cin channels across threads.
#include <algorithm>

#include "gemm.h"
#include "wgrad.h"

namespace damc {

typedef __bf16 wg_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf16_bits_to_f32(unsigned short u) { return __uint_as_float((unsigned)u << 16); }

// ---------------------------------------------------------------------------------------- transpose
// grid (Hq*Wq, Bp/32, nph * ceil(C/64)), 256 threads: a 32-sample x 64-channel tile of one pixel through LDS.  nph = 4
// (round 5): the four output phases (py, px) = (ph >> 1, ph & 1) of a k4 s2 p1 layer in one launch (offsets oy + py,
// ox + px; phase ph writes dst + ph * dst_pstride and part + ph * part_pstride), instead of four launches
template <bool X3>
__global__ __launch_bounds__(256) void transpose_x3_kernel(const float* __restrict__ src32,
                                                           const unsigned short* __restrict__ src3, int B, int H,
                                                           int W, int C, int Wq, int sy, int sx, int oy, int ox,
                                                           int Bp, int P, unsigned short* __restrict__ dst,
                                                           float* __restrict__ part, int ncb, long dst_pstride,
                                                           long part_pstride) {
  __shared__ float tile[64][33];
  const int pq = blockIdx.x, nb = blockIdx.y, ph = blockIdx.z / ncb, cb = blockIdx.z - ph * ncb;
  oy += ph >> 1;
  ox += ph & 1;
  dst += ph * dst_pstride;
  if (part) part += ph * part_pstride;
  const int qy = pq / Wq, qx = pq - qy * Wq;
  const int y = sy * qy + oy, x = sx * qx + ox;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = tid + 256 * i;
    const int nl = e >> 6, cl = e & 63;
    const int n = nb * 32 + nl, c = cb * 64 + cl;
    float v = 0.f;
    if (n < B && c < C) {
      const long pix = ((long)n * H + y) * W + x;
      if (X3) {  // octet [limb][8]: the three limbs sum back to the fp32 value exactly
        const long o = (pix * C + (c & ~7)) * 3 + (c & 7);
        v = (bf16_bits_to_f32(src3[o]) + bf16_bits_to_f32(src3[o + 8])) + bf16_bits_to_f32(src3[o + 16]);
      } else {
        v = src32[pix * C + c];
      }
    }
    tile[cl][nl] = v;
  }
  __syncthreads();
  {
    const int cl = tid >> 2, oct = tid & 3;
    const int c = cb * 64 + cl;
    if (c < C) {
      wg_bf16x8 h, m, l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // RNE limb split, as the engine's own split (gemm.hip split3_octet)
        const float v = tile[cl][oct * 8 + e];
        const __bf16 b0 = (__bf16)v;
        const float r1 = sub_rn(v, (float)b0);
        const __bf16 b1 = (__bf16)r1;
        h[e] = b0;
        m[e] = b1;
        l[e] = (__bf16)(sub_rn(r1, (float)b1));
      }
      wg_bf16x8* o = reinterpret_cast<wg_bf16x8*>(dst + (((long)c * P + pq) * Bp + nb * 32 + oct * 8) * 3);
      o[0] = h;
      o[1] = m;
      o[2] = l;
    }
  }
  if (part && tid < 64) {
    const int c = cb * 64 + tid;
    if (c < C) {
      float sum = 0.f;
#pragma unroll 8
      for (int n = 0; n < 32; ++n) sum += tile[tid][n];
      part[((long)pq * (Bp / 32) + nb) * C + c] = sum;
    }
  }
}

int launch_transpose_x3(const float* src32, const unsigned short* src3, int B, int H, int W, int C, int Hq, int Wq,
                        int sy, int sx, int oy, int ox, int Bp, unsigned short* dst, float* part, hipStream_t s) {
  if ((!src32) == (!src3) || !dst || B <= 0 || C <= 0 || Hq <= 0 || Wq <= 0 || Bp < B || Bp % 32 != 0)
    return DAMC_ERR_ARG;
  if (src3 && C % 8 != 0) return DAMC_ERR_ARG;
  if ((uintptr_t)dst % 16 != 0) return DAMC_ERR_ARG;
  if (sy * (Hq - 1) + oy >= H || sx * (Wq - 1) + ox >= W || oy < 0 || ox < 0) return DAMC_ERR_ARG;
  const int ncb = (C + 63) / 64;
  const dim3 grid((unsigned)(Hq * Wq), (unsigned)(Bp / 32), (unsigned)ncb);
  ProfScope ps("wgrad_transpose", 0.0, s);
  if (src3)
    hipLaunchKernelGGL(transpose_x3_kernel<true>, grid, dim3(256), 0, s, nullptr, src3, B, H, W, C, Wq, sy, sx, oy,
                       ox, Bp, Hq * Wq, dst, part, ncb, 0L, 0L);
  else
    hipLaunchKernelGGL(transpose_x3_kernel<false>, grid, dim3(256), 0, s, src32, nullptr, B, H, W, C, Wq, sy, sx, oy,
                       ox, Bp, Hq * Wq, dst, part, ncb, 0L, 0L);
  return (int)hipGetLastError();
}

int launch_transpose_x3_4ph(const float* src32, const unsigned short* src3, int B, int H, int W, int C, int Hq, int Wq,
                            int Bp, unsigned short* dst, long dst_pstride, float* part, long part_pstride,
                            hipStream_t s) {
  if ((!src32) == (!src3) || !dst || B <= 0 || C <= 0 || Hq <= 0 || Wq <= 0 || Bp < B || Bp % 32 != 0)
    return DAMC_ERR_ARG;
  if (src3 && C % 8 != 0) return DAMC_ERR_ARG;
  if ((uintptr_t)dst % 16 != 0 || (dst_pstride * 2) % 16 != 0) return DAMC_ERR_ARG;
  if (2 * (Hq - 1) + 1 >= H || 2 * (Wq - 1) + 1 >= W) return DAMC_ERR_ARG;
  const int ncb = (C + 63) / 64;
  if (4L * ncb > 65535) return DAMC_ERR_UNSUPPORTED;
  const dim3 grid((unsigned)(Hq * Wq), (unsigned)(Bp / 32), (unsigned)(4 * ncb));
  ProfScope ps("wgrad_transpose", 0.0, s);
  if (src3)
    hipLaunchKernelGGL(transpose_x3_kernel<true>, grid, dim3(256), 0, s, nullptr, src3, B, H, W, C, Wq, 2, 2, 0, 0, Bp,
                       Hq * Wq, dst, part, ncb, dst_pstride, part_pstride);
  else
    hipLaunchKernelGGL(transpose_x3_kernel<false>, grid, dim3(256), 0, s, src32, nullptr, B, H, W, C, Wq, 2, 2, 0, 0,
                       Bp, Hq * Wq, dst, part, ncb, dst_pstride, part_pstride);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ k4 s2 p1 slab reduce
// each of the 16 taps a fixed-order sum over the split-K slices; tap (ky, kx) comes from phase (py, px) =
// ((ky+1)&1, (kx+1)&1) and GEMM row (ty, tx) with ky = 3 - py - 2 ty.  One workgroup per (ci, 16 consecutive co): thread (tap, co) sums its S slab values in order (16 co = one 64-B run
// per tap), the 16 x 16 results go through LDS and leave as the 1 KB contiguous run dW[ci][co0 .. co0 + 15][16 taps]
// (round 5: one thread per (ci, co) walking all 16 taps left the encoder's 64 -> 128 conv 8192 threads of 256 slab
// loads each, 62 us; same sums, same order)
__global__ __launch_bounds__(256) void up2_wgrad_reduce_kernel(const float* __restrict__ slabs, int S, int Cin,
                                                               int Cout, float* __restrict__ dW) {
  __shared__ float t16[16][17];
  const int ng = Cout / 16;
  const int ci = blockIdx.x / ng, co0 = (blockIdx.x - ci * ng) * 16;
  const int tap = threadIdx.x >> 4, cl = threadIdx.x & 15;
  const int ky = tap >> 2, kx = tap & 3;
  const long M = 4L * Cin;
  const int py = (ky + 1) & 1, ty = (3 - ky - py) >> 1;
  const int px = (kx + 1) & 1, tx = (3 - kx - px) >> 1;
  const int ph = py * 2 + px, t = ty * 2 + tx;
  const float* sp = slabs + ((long)ph * S * M + (long)t * Cin + ci) * Cout + co0 + cl;
  float acc = 0.f;
  for (int sl = 0; sl < S; ++sl) acc += sp[(long)sl * M * Cout];
  t16[cl][tap] = acc;
  __syncthreads();
  dW[((long)ci * Cout + co0) * 16 + threadIdx.x] = t16[threadIdx.x >> 4][threadIdx.x & 15];
}

// any Cout: one thread per (ci, co), all 16 taps
__global__ __launch_bounds__(256) void up2_wgrad_reduce_any_kernel(const float* __restrict__ slabs, int S, int Cin,
                                                                   int Cout, float* __restrict__ dW) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cin * Cout) return;
  const int ci = (int)(i / Cout), co = (int)(i - (long)ci * Cout);
  const long M = 4L * Cin;
#pragma unroll
  for (int tap = 0; tap < 16; ++tap) {
    const int ky = tap >> 2, kx = tap & 3;
    const int py = (ky + 1) & 1, ty = (3 - ky - py) >> 1;
    const int px = (kx + 1) & 1, tx = (3 - kx - px) >> 1;
    const int ph = py * 2 + px, t = ty * 2 + tx;
    const float* sp = slabs + ((long)ph * S * M + (long)t * Cin + ci) * Cout + co;
    float acc = 0.f;
    for (int sl = 0; sl < S; ++sl) acc += sp[(long)sl * M * Cout];
    dW[i * 16 + tap] = acc;
  }
}

int launch_up2_wgrad_reduce(const float* slabs, int S, int Cin, int Cout, float* dW, hipStream_t s) {
  if (!slabs || !dW || S < 1 || Cin <= 0 || Cout <= 0 || (uintptr_t)dW % 16 != 0) return DAMC_ERR_ARG;
  const long n = (long)Cin * Cout;
  ProfScope ps("wgrad_reduce", 0.0, s);
  if (Cout % 16 == 0)
    hipLaunchKernelGGL(up2_wgrad_reduce_kernel, dim3((unsigned)(n / 16)), dim3(256), 0, s, slabs, S, Cin, Cout, dW);
  else
    hipLaunchKernelGGL(up2_wgrad_reduce_any_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slabs, S, Cin,
                       Cout, dW);
  return (int)hipGetLastError();
}

// --------------------------------------------------------------------------------------- column sums
// grid (ceil(C/CL), row blocks), 256 threads = RL row lanes x CL channel lanes (CL = min(64, pow2 >= C)),
// each row lane summing every RL-th row of the block's range; the RL partials combine in a fixed tree
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, long R, int C, long ld, int CL,
                                                     long rows_per, float* __restrict__ out) {
  __shared__ float red[256];
  const int RL = 256 / CL;
  const int cl = threadIdx.x % CL, rl = threadIdx.x / CL;
  const int c = blockIdx.x * CL + cl;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = min(R, r0 + rows_per);
  float sum = 0.f;
  if (c < C)
    for (long r = r0 + rl; r < r1; r += RL) sum += X[r * ld + c];
  red[threadIdx.x] = sum;
  __syncthreads();
  for (int h = RL / 2; h > 0; h >>= 1) {
    if (rl < h) red[threadIdx.x] += red[threadIdx.x + h * CL];
    __syncthreads();
  }
  if (rl == 0 && c < C) out[(long)blockIdx.y * C + c] = red[cl];
}

// the same sums four channels per thread (C % 4 == 0, ld % 4 == 0, 16-B aligned): CL4 float4 lanes of 4 channels,
// 256 / CL4 row lanes (16 at C = 64 instead of 4), so both passes keep many more loads in flight per thread-row
// out2 (single pass only): float4 columns from split4 on go to out2 instead (two gradients sharing one row layout)
__global__ __launch_bounds__(256) void colsum4_kernel(const float* __restrict__ X, long R, int C4, long ld4, int CL4,
                                                      long rows_per, float* __restrict__ out,
                                                      float* __restrict__ out2 = nullptr, int split4 = 0) {
  __shared__ f32x4 red[256];
  const int RL = 256 / CL4;
  const int cl = threadIdx.x % CL4, rl = threadIdx.x / CL4;
  const int c4 = blockIdx.x * CL4 + cl;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = min(R, r0 + rows_per);
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  if (c4 < C4) {
    const f32x4* X4 = reinterpret_cast<const f32x4*>(X);
    for (long r = r0 + rl; r < r1; r += RL) sum += X4[r * ld4 + c4];
  }
  red[threadIdx.x] = sum;
  __syncthreads();
  for (int h = RL / 2; h > 0; h >>= 1) {
    if (rl < h) red[threadIdx.x] += red[threadIdx.x + h * CL4];
    __syncthreads();
  }
  if (rl == 0 && c4 < C4) {
    if (out2 && c4 >= split4)
      reinterpret_cast<f32x4*>(out2)[c4 - split4] = red[cl];
    else
      reinterpret_cast<f32x4*>(out)[(long)blockIdx.y * C4 + c4] = red[cl];
  }
}

static int colsum_lanes(int C) {
  int cl = 1;
  while (cl < C && cl < 64) cl <<= 1;
  return cl;
}
// row blocks of the first pass: <= 16 rows per thread, at most 1024 blocks (the second pass sums them); a single
// pass up to 8x that (a two-pass sum of a 128-row batch cost two launches for 32 loads per thread)
static long colsum_blocks(long R, int C) {
  const long per = 16L * (256 / colsum_lanes(C));
  return R <= 8 * per ? 1 : std::min<long>(1024, (R + per - 1) / per);
}
// float4 form: 256 row blocks at most (32 float4 rows per thread per pass at R = 131072, C = 64), one pass up to 32
// rows per thread
// at most 16 float4 lanes (64 channels) per workgroup: 16 row lanes, so a B = 128-row sum is 8 loads per thread across
// C / 64 workgroups (round 5: 64 lanes left 4 row lanes walking 32 rows each in ONE workgroup, 6-12 us per call for the
// Q update's 29 bias / InstanceNorm column sums)
static int colsum4_lanes(int C4) {
  int cl = 1;
  while (cl < C4 && cl < 16) cl <<= 1;
  return cl;
}
static long colsum4_blocks(long R, int C) {
  const long rl = 256 / colsum4_lanes(C / 4);
  return R <= 32 * rl ? 1 : std::min<long>(256, (R + 32 * rl - 1) / (32 * rl));
}

size_t colsum_tmp_floats(long R, int C) {
  return (size_t)std::max(colsum_blocks(R, C), colsum4_blocks(R, C)) * C;
}

int launch_colsum2(const float* X, long R, int C, long ld, float* out_lo, float* out_hi, int split, float* tmp,
                   hipStream_t s) {
  if (!X || !out_lo || !out_hi || split <= 0 || split >= C) return DAMC_ERR_ARG;
  const bool one = C % 4 == 0 && split % 4 == 0 && ld % 4 == 0 && colsum4_blocks(R, C) == 1 &&
                   ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(out_lo) |
                     reinterpret_cast<uintptr_t>(out_hi)) & 15) == 0;
  if (!one) {  // two column sums
    const int rc = launch_colsum(X, R, split, ld, out_lo, tmp, s);
    return rc ? rc : launch_colsum(X + split, R, C - split, ld, out_hi, tmp, s);
  }
  ProfScope ps("bias_grad", 0.0, s);
  const int C4 = C / 4, CL4 = colsum4_lanes(C4);
  hipLaunchKernelGGL(colsum4_kernel, dim3((unsigned)((C4 + CL4 - 1) / CL4), 1), dim3(256), 0, s, X, R, C4, ld / 4, CL4,
                     R, out_lo, out_hi, split / 4);
  return (int)hipGetLastError();
}

int launch_colsum(const float* X, long R, int C, long ld, float* out, float* tmp, hipStream_t s) {
  if (!X || !out || R <= 0 || C <= 0 || ld < C) return DAMC_ERR_ARG;
  ProfScope ps("bias_grad", 0.0, s);
  if (C % 4 == 0 && ld % 4 == 0 && ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(out) |
                                      reinterpret_cast<uintptr_t>(tmp)) & 15) == 0) {
    const int C4 = C / 4, CL4 = colsum4_lanes(C4);
    const long nrb = colsum4_blocks(R, C);
    const unsigned gx = (unsigned)((C4 + CL4 - 1) / CL4);
    if (nrb == 1) {
      hipLaunchKernelGGL(colsum4_kernel, dim3(gx, 1), dim3(256), 0, s, X, R, C4, ld / 4, CL4, R, out);
      return (int)hipGetLastError();
    }
    if (!tmp) return DAMC_ERR_ARG;
    const long per = (R + nrb - 1) / nrb;
    hipLaunchKernelGGL(colsum4_kernel, dim3(gx, (unsigned)nrb), dim3(256), 0, s, X, R, C4, ld / 4, CL4, per, tmp);
    hipLaunchKernelGGL(colsum4_kernel, dim3(gx, 1), dim3(256), 0, s, (const float*)tmp, nrb, C4, (long)C4, CL4, nrb,
                       out);
    return (int)hipGetLastError();
  }
  const int CL = colsum_lanes(C);
  const long nrb = colsum_blocks(R, C);
  const unsigned gx = (unsigned)((C + CL - 1) / CL);
  if (nrb == 1) {
    hipLaunchKernelGGL(colsum_kernel, dim3(gx, 1), dim3(256), 0, s, X, R, C, ld, CL, R, out);
    return (int)hipGetLastError();
  }
  if (!tmp) return DAMC_ERR_ARG;
  const long per = (R + nrb - 1) / nrb;
  hipLaunchKernelGGL(colsum_kernel, dim3(gx, (unsigned)nrb), dim3(256), 0, s, X, R, C, ld, CL, per, tmp);
  hipLaunchKernelGGL(colsum_kernel, dim3(gx, 1), dim3(256), 0, s, (const float*)tmp, nrb, C, (long)C, CL, nrb, out);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ output-layer wgrad
// grid (row blocks of R input rows, B): dw = the delta window [S(R-1)+K rows][Wd = S(Win-1)+K][NC] in LDS
// (zero outside the map); each thread owns input channels and accumulates all K*K*NC taps
template <int NC, int K>
__global__ __launch_bounds__(256) void smallc_wgrad_kernel(const float* __restrict__ h, const float* __restrict__ delta,
                                                           int Hin, int Win, int Cin, int S, int pad, int Hout,
                                                           int Wout, int R, int Wd, float* __restrict__ part) {
  extern __shared__ float dw[];
  const int rb = blockIdx.x, n = blockIdx.y, nrb = gridDim.x;
  const int iy0 = rb * R;
  const int rows = min(R, Hin - iy0);
  const int nrows = S * (R - 1) + K;
  const int oy0 = S * iy0 - pad;
  for (int i = threadIdx.x; i < nrows * Wd * NC; i += blockDim.x) {
    const int o = i % NC, rc = i / NC;
    const int r = rc / Wd, cc = rc - r * Wd;
    const int oy = oy0 + r, ox = cc - pad;
    float v = 0.f;
    if (oy >= 0 && oy < Hout && ox >= 0 && ox < Wout) v = delta[(((long)n * Hout + oy) * Wout + ox) * NC + o];
    dw[i] = v;
  }
  __syncthreads();
  constexpr int T = K * K * NC;
  for (int ci = threadIdx.x; ci < Cin; ci += blockDim.x) {
    float acc[T];
#pragma unroll
    for (int j = 0; j < T; ++j) acc[j] = 0.f;
    for (int yy = 0; yy < rows; ++yy) {
      const float* hr = h + ((long)n * Hin + iy0 + yy) * Win * Cin + ci;
      const float* wr = dw + (S * yy) * Wd * NC;
      int ix = 0;
      for (; ix + 4 <= Win; ix += 4) {  // four loads in flight, then their taps in order
        float hv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) hv[u] = hr[(long)(ix + u) * Cin];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float* w0 = wr + S * (ix + u) * NC;
#pragma unroll
          for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx)
#pragma unroll
              for (int o = 0; o < NC; ++o) acc[(ky * K + kx) * NC + o] += hv[u] * w0[(ky * Wd + kx) * NC + o];
        }
      }
      for (; ix < Win; ++ix) {
        const float hv = hr[(long)ix * Cin];
        const float* w0 = wr + S * ix * NC;
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
          for (int kx = 0; kx < K; ++kx)
#pragma unroll
            for (int o = 0; o < NC; ++o) acc[(ky * K + kx) * NC + o] += hv * w0[(ky * Wd + kx) * NC + o];
      }
    }
    // this block's partial, in the PyTorch (Cin, Cout, k, k) order: a column sum over blocks is dW
    float* pp = part + (long)(n * nrb + rb) * T * Cin + (long)ci * T;
#pragma unroll
    for (int o = 0; o < NC; ++o)
#pragma unroll
      for (int t = 0; t < K * K; ++t) pp[o * K * K + t] = acc[t * NC + o];
  }
}

// rows per block: >= 2048 blocks where the map allows (latency-bound loads), window within 40 KiB of LDS
static int smallc_rows(const damc_layer_t& L, int B) {
  int R = 8;
  const int Wd = L.stride * (L.win - 1) + L.k;
  while (R > 1 && ((size_t)(L.stride * (R - 1) + L.k) * Wd * L.cout * sizeof(float) > 40960 ||
                   (long)B * ((L.hin + R - 1) / R) < 2048))
    R /= 2;
  return R;
}

static long smallc_blocks(const damc_layer_t& L, int B) {
  const int R = smallc_rows(L, B);
  return (long)B * ((L.hin + R - 1) / R);
}

size_t smallc_wgrad_part_floats(const damc_layer_t& L, int B) {
  return (size_t)smallc_blocks(L, B) * L.k * L.k * L.cout * L.cin;
}

size_t smallc_wgrad_tmp_floats(const damc_layer_t& L, int B) {
  return colsum_tmp_floats(smallc_blocks(L, B), L.k * L.k * L.cout * L.cin);
}

int launch_smallc_wgrad(const damc_layer_t& L, const float* h, const float* delta, int B, float* part, float* tmp,
                        float* dW, hipStream_t s) {
  if (!h || !delta || !part || !dW || B <= 0) return DAMC_ERR_ARG;
  const int R = smallc_rows(L, B);
  const int Wd = L.stride * (L.win - 1) + L.k;
  const size_t sm = (size_t)(L.stride * (R - 1) + L.k) * Wd * L.cout * sizeof(float);
  if (sm > 65536) return DAMC_ERR_UNSUPPORTED;
  const int nrb = (L.hin + R - 1) / R;
  const dim3 grid((unsigned)nrb, (unsigned)B);
  const int T = L.k * L.k * L.cout;
  bool launched = false;
  {
    ProfScope ps("smallc_wgrad", 2.0 * B * L.hin * L.win * L.cin * L.k * L.k * L.cout, s);
#define SW(NC_, K_)                                                                                           \
  if (!launched && L.cout == NC_ && L.k == K_) {                                                              \
    hipLaunchKernelGGL((smallc_wgrad_kernel<NC_, K_>), grid, dim3(256), sm, s, h, delta, L.hin, L.win, L.cin, \
                       L.stride, L.pad, L.hout, L.wout, R, Wd, part);                                         \
    launched = true;                                                                                          \
  }
    SW(3, 3) SW(3, 4) SW(1, 3) SW(1, 4) SW(2, 3) SW(2, 4) SW(4, 3) SW(4, 4)
#undef SW
  }
  if (!launched) return DAMC_ERR_UNSUPPORTED;
  DAMC_LAUNCH_CHECK();
  return launch_colsum(part, (long)B * nrb, T * L.cin, (long)T * L.cin, dW, tmp, s);
}

// --------------------------------------------------------------------------------- output delta
__global__ __launch_bounds__(256) void out_delta_kernel(const float* __restrict__ g, const float* __restrict__ xhat,
                                                        int NC, int HW, long n, int act, float* __restrict__ delta) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long b = i / ((long)NC * HW);
  const long r = i - b * NC * HW;
  const int o = (int)(r / HW), p = (int)(r - (long)o * HW);
  float d = g[i];
  if (act == DAMC_ACT_TANH) {
    const float t = xhat[i];
    d = d * (1.f - t * t);
  }
  delta[(b * HW + p) * NC + o] = d;
}

int launch_out_delta(const float* g, const float* xhat, int B, int NC, int HW, int act, float* delta, hipStream_t s) {
  if (!g || !delta || B <= 0 || NC <= 0 || HW <= 0) return DAMC_ERR_ARG;
  if (act != DAMC_ACT_NONE && act != DAMC_ACT_TANH) return DAMC_ERR_UNSUPPORTED;
  if (act == DAMC_ACT_TANH && !xhat) return DAMC_ERR_ARG;
  const long n = (long)B * NC * HW;
  hipLaunchKernelGGL(out_delta_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, xhat, NC, HW, n, act,
                     delta);
  return (int)hipGetLastError();
}

// --------------------------------------------------------------------------------- Linear wgrad
__global__ __launch_bounds__(256) void linear_wgrad_kernel(const float* __restrict__ d, const float* __restrict__ h,
                                                           int B, int nout, int nin, float* __restrict__ dW) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)nout * nin) return;
  const int o = (int)(i / nin), k = (int)(i - (long)o * nin);
  float sum = 0.f;
  for (int n = 0; n < B; ++n) sum += d[(long)n * nout + o] * h[(long)n * nin + k];
  dW[i] = sum;
}

int launch_linear_wgrad(const float* d, const float* h, int B, int nout, int nin, float* dW, hipStream_t s) {
  if (!d || !h || !dW || B <= 0 || nout <= 0 || nin <= 0) return DAMC_ERR_ARG;
  const long n = (long)nout * nin;
  ProfScope ps("linear_wgrad", 2.0 * B * n, s);
  hipLaunchKernelGGL(linear_wgrad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, h, B, nout, nin, dW);
  return (int)hipGetLastError();
}

}  // namespace damc
