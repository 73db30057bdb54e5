// denoiser.hip — Diffusion_UnetA eps-prediction and the amortizer's latent reverse sweep
// (_netQ_U.forward, workspace/src/diffusion_net.py:585-622) on gfx950.
//
// A ConcatSquash block (diffusion_net.py:417-445) is
//     out = (x Wl^T + bl) * sigmoid(c Wg^T + bg) + c Wb^T + (x Ws^T + bs),   c = SiLU(Lc(SiLU(cat(temb, xemb))))
// and its ctx c depends on (step, row) only — never on zt.  So per call (not per step):
//   1. pack   : every weight from the caller's PyTorch layouts into the workspace (the nets train between calls);
//   2. ctx    : time MLP on the n sinusoidal embeddings (batch-invariant) and SiLU(xemb) . Wctx_x (step-invariant),
//               c[k][b] = SiLU(px[b] + qt[k]) for all n*B (step, row) pairs;
//   3. hyper  : per block one fp32-MFMA GEMM over the n*B rows, [gate | hyper bias] = [sigmoid(c Wg^T + bg) | c Wb^T]
//               (EPI_GATE).  51 % + 20 % of the reference's per-step MACs (ctx Linear, hyper Linears) leave the
//               dependent chain this way.
// What stays in the chain is x Wl^T and x Ws^T of the 7 blocks plus the reverse-step update: 7 dependent launches
// per step (block j+1 needs every column of block j for its rows).  They are kept short:
//   * one workgroup = 16 rows x 8 output columns of BOTH products (one 16 x 16 v_mfma_f32_16x16x4_f32 tile: 8 Wl
//     rows + 8 Ws rows of the packed weight), 4 waves splitting K in quarters; each lane's x and weight fragments
//     are f32x4 global loads issued together up front through the k-permutation of the MFMA steps (step s of
//     k-group g reads k = 16 g + 4 (lane >> 4) + s on both operands), so a launch costs one memory round trip;
//   * the epilogue operands (gate, hyper bias, biases, zt, the Philox draw) are fetched before the main loop;
//   * N tiles are the fastest grid index: with dout / 8 a multiple of 8 an N tile stays on one XCD for every step,
//     so each XCD keeps 1/8 of the chain's weights in its L2;
//   * the 7n launches are captured once into a HIP graph (cached per workspace / shape / schedule) and replayed:
//     eager launches cost the host ~3.5 us each, more than these kernels take on the GPU.
// The last block's epilogue applies eps = z + out, pred_x_from_eps and the reverse step with Philox noise in place.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "gemm.h"

namespace {

constexpr int CH_THREADS = 256;  // 4 waves, K split in quarters
constexpr int TM = 16;           // rows per workgroup
constexpr int TC = 8;            // output columns per workgroup (x 2 products)
constexpr int KG = 64;           // K padding granule: 4 waves x one 16-deep k-group
constexpr int CH_CHUNK = 8;      // k-groups whose loads a lane keeps in flight at once
constexpr int EMB_G = 8;         // in0: 16-deep k-groups of z (nz <= 128)

// per-call values read by the last block (device memory in the workspace, written before each sweep so a cached
// graph needs no new kernel arguments)
struct SweepCall {
  const float* noise;  // injected (n-1, B, nz) or null (Philox)
  float* eps_log;      // (eps_log_steps, B, nz) or null
  uint64_t seed, chain_base, step_offset;
  int with_noise, eps_log_steps;
};

struct ChainArgs {
  const float* srcA;  // block input = lrelu(cat(srcA, srcB), 0.01) (not in0)
  const float* srcB;
  int wa, wb;
  int emb;            // in0: input = [sin 2pi zB, cos 2pi zB, z]
  const float* z;     // (B, nz) current zt (the workspace copy)
  const float* bmat;  // B^T (nz/2, nz), packed per call
  int nz;
  int din, kp, dout, B;
  const float* w;     // [ntn][16][kp]: rows 0-7 Wl, 8-15 Ws of the tile's columns (zero-padded)
  const float* bls;   // [ntn][16]: bl, bs
  const float* gh;    // this step's rows: gate at gh[b * ldgh + n], hyper bias at gh[b * ldgh + dout + n]
  long ldgh;
  float* out;         // (B, dout)
  // last block
  int final_, residual, last, k, noisy_k;
  float c0, c1, c2, c3, c4;
  float* zt;          // == z
  const SweepCall* call;
  int dbg;  // timing experiments only (DAMC_CHAIN_DBG, wrong results): 1 no x loads, 2 no weight loads, 4 no MFMA,
            // 8 no epilogue prefetch, 16 no output stores; in0: 32 no sin/cos, 64 no B loads, 128 no zB MFMA
};

__host__ __device__ inline int kpad(int din) { return (din + KG - 1) / KG * KG; }
__host__ __device__ inline int emb_ld(int kp) { return kp + 8; }  // in0 LDS image row stride (floats)

// EMB: the in0 block (Fourier embedding, sin / cos with their large-argument path) is its own instantiation, so
// the six other blocks' kernels carry no scratch segment
template <bool EMB>
__global__ __launch_bounds__(CH_THREADS) void chain_kernel(ChainArgs a) {
  __shared__ __attribute__((aligned(16))) float red[4][TM][16];
  extern __shared__ __attribute__((aligned(16))) float embs[];  // in0: [TM][emb_ld(kp)]
  if (a.dbg & 512) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (a.dout + TC - 1) / TC;
  const int tn = blockIdx.x % ntn, tm = blockIdx.x / ntn;
  const int r0 = tm * TM, n0 = tn * TC;
  const int m = lane & 15, q = lane >> 4;

  // ---- epilogue operands first (independent of the main loop): thread (row er, column ec)
  const int er = tid >> 3, ec = tid & 7;
  const int erow = r0 + er, ecol = n0 + ec;
  const bool eok = tid < TM * TC && erow < a.B && ecol < a.dout;
  float gate = 0.f, hb = 0.f, bl = 0.f, bs = 0.f, zv = 0.f, xi = 0.f;
  const SweepCall* call = a.call;
  if (eok && !(a.dbg & 8)) {
    gate = a.gh[(long)erow * a.ldgh + ecol];
    hb = a.gh[(long)erow * a.ldgh + a.dout + ecol];
    bl = a.bls[tn * 16 + ec];
    bs = a.bls[tn * 16 + 8 + ec];
    if (a.final_) {
      zv = a.zt[(long)erow * a.nz + ecol];
      if (!a.last && call->with_noise) {
        if (call->noise) {
          xi = call->noise[((long)a.noisy_k * a.B + erow) * a.nz + ecol];
        } else {
          float n4[4];
          philox_normal4(call->seed, call->chain_base + erow, call->step_offset + a.noisy_k, (uint32_t)(ecol >> 2),
                         DAMC_STREAM_SWEEP, n4);
          xi = pick4(n4, ecol);
        }
      }
    }
  }

  // ---- in0: the Fourier input embedding of the 16 rows into LDS (zB on MFMA, wave w -> 16-column tiles w, w+4..)
  const int ld = emb_ld(a.kp);
  if (EMB) {
    const int nz = a.nz, half = nz >> 1;
    const int row = r0 + m;
    const bool rok = row < a.B;
    // all of a lane's z and B operands are loaded before the first MFMA (one memory round trip; nz <= 128)
    f32x4 zv4[EMB_G];
#pragma unroll
    for (int g = 0; g < EMB_G; ++g) {
      const int k = 16 * g + 4 * q;
      zv4[g] = (rok && k < nz) ? *reinterpret_cast<const f32x4*>(a.z + (long)row * nz + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int t = wave; t * 16 < half; t += 4) {
      const int col = t * 16 + m;
      const bool cok = col < half;
      f32x4 bv[EMB_G];  // a.bmat is B^T (half, nz): lane (m, q) reads B[16 g + 4 q + s][col] as one f32x4
#pragma unroll
      for (int g = 0; g < EMB_G; ++g) {
        const int k = 16 * g + 4 * q;
        bv[g] = (cok && k < nz && !(a.dbg & 64)) ? *reinterpret_cast<const f32x4*>(a.bmat + (long)col * nz + k)
                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (!(a.dbg & 128)) {
#pragma unroll
        for (int g = 0; g < EMB_G; ++g)
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(zv4[g][s], bv[g][s], acc, 0, 0, 0);
      }
      // sin / cos (2 pi zB) on the hardware units, whose argument is in revolutions: t = zB - rint(zB) is exact,
      // so the only rounding is the unit's (the reference rounds 2 pi zB to fp32 first, ~4e-6 rad at |zB| ~ 10;
      // both are below the spread of zB itself between summation orders)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 4 * q + r;
        if (cok) {
          const float t = acc[r] - rintf(acc[r]);
          const bool ok = r0 + rr < a.B;
          embs[rr * ld + col] = ok ? ((a.dbg & 32) ? t : __builtin_amdgcn_sinf(t)) : 0.f;
          embs[rr * ld + half + col] = ok ? ((a.dbg & 32) ? t : __builtin_amdgcn_cosf(t)) : 0.f;
        }
      }
    }
    // z itself from the registers that already hold it (wave 0: lane (m, q) has z[row m][16 g + 4 q + s]),
    // then zeros up to kp (no global loads here: a strided load loop would serialise its memory latencies)
    if (wave == 0) {
#pragma unroll
      for (int g = 0; g < EMB_G; ++g)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = 16 * g + 4 * q + s;
          if (k < nz) embs[m * ld + 2 * half + k] = zv4[g][s];
        }
    }
    for (int c = 2 * half + nz + tid; c < a.kp; c += CH_THREADS)
#pragma unroll
      for (int rr = 0; rr < TM; ++rr) embs[rr * ld + c] = 0.f;
    __syncthreads();
  }

  // ---- main loop: wave w covers k in [w kq, (w+1) kq) of the padded K
  const int kq = a.kp >> 2;
  const int ng = kq >> 4;
  const int kbase = wave * kq;
  const int xrow = r0 + m;
  const bool xok = xrow < a.B;
  const float* wrow = a.w + ((long)tn * 16 + m) * a.kp + kbase + 4 * q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int g0 = 0; g0 < ng; g0 += CH_CHUNK) {
    f32x4 xa[CH_CHUNK], wb[CH_CHUNK];
#pragma unroll
    for (int c = 0; c < CH_CHUNK; ++c) {
      const int g = g0 + c;
      const int k = kbase + 16 * g + 4 * q;
      f32x4 wv = {0.f, 0.f, 0.f, 0.f}, xv = {0.f, 0.f, 0.f, 0.f};
      if (g < ng) {
        if (!(a.dbg & 2)) wv = *reinterpret_cast<const f32x4*>(wrow + 16 * g);
        if (EMB) {
          xv = *reinterpret_cast<const f32x4*>(embs + m * ld + k);
        } else if (xok && k < a.din && !(a.dbg & 1)) {
          xv = k < a.wa ? *reinterpret_cast<const f32x4*>(a.srcA + (long)xrow * a.wa + k)
                        : *reinterpret_cast<const f32x4*>(a.srcB + (long)xrow * a.wb + (k - a.wa));
        }
      }
      wb[c] = wv;
      xa[c] = xv;
    }
#pragma unroll
    for (int c = 0; c < CH_CHUNK; ++c) {
      f32x4 x = xa[c];
      if (!EMB) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = x[e] > 0.f ? x[e] : 0.01f * x[e];
      }
      if (a.dbg & 4) {
        acc[0] += x[0] * wb[c][0] + x[1] * wb[c][1] + x[2] * wb[c][2] + x[3] * wb[c][3];
        continue;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s], wb[c][s], acc, 0, 0, 0);
    }
  }
  if (a.dbg & 256) {
    if (acc[0] == 12345.f) a.out[0] = acc[1];
    return;
  }
  // C layout 16x16x4: column = lane & 15 (0-7 Wl, 8-15 Ws), rows 4 (lane >> 4) + r
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][4 * q + r][m] = acc[r];
  __syncthreads();

  if (!eok) return;
  float l = 0.f, sk = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {  // fixed order: deterministic
    l += red[w][er][ec];
    sk += red[w][er][8 + ec];
  }
  // ConcatSquashLinearSkipCtx.forward: ret = layer(x) * gate + bias; ret + skip(x)
  const float o = ((l + bl) * gate + hb) + (sk + bs);
  if (!a.final_) {
    if (!(a.dbg & 16)) a.out[(long)erow * a.dout + ecol] = o;
    return;
  }
  // reverse step (diffusion_net.py:601-620): eps = z + out; pred = c0 (z - eps c1)
  const long zi = (long)erow * a.nz + ecol;
  const float eps = a.residual ? zv + o : o;
  if (call->eps_log && a.k < call->eps_log_steps) call->eps_log[(long)a.k * a.B * a.nz + zi] = eps;
  const float pred = mul_rn(a.c0, sub_rn(zv, mul_rn(eps, a.c1)));
  float zn;
  if (a.last) {
    zn = pred;
  } else {
    zn = add_rn(mul_rn(a.c2, zv), mul_rn(a.c3, pred));
    if (call->with_noise) zn = add_rn(zn, mul_rn(a.c4, xi));
  }
  a.zt[zi] = zn;
}

// ------------------------------------------------------------------------------------- per-call helpers
__global__ void silu_kernel(const float* x, long n, float* y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const float v = x[i];
    y[i] = v / (1.f + expf(-v));
  }
}

// c[k][b][s] = SiLU(px[b][s] + qt[k][s])
__global__ void ctx_kernel(const float* __restrict__ px, const float* __restrict__ qt, int B, int S, long total,
                           float* __restrict__ c) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long per = (long)B * S;
  const long k = i / per;
  const long r = i - k * per;
  const int s = (int)(r % S);
  const float u = px[r] + qt[k * S + s];
  c[i] = u / (1.f + expf(-u));
}

struct PackBlock {
  const float *wl, *bl, *ws, *bs, *wg, *bg, *wb, *wctx, *bctx;
  int din, dout, kp, coloff;
  float *w, *bls, *wgb, *bg2;
};
struct PackArgs {
  PackBlock b[7];
  int ntemb, nxemb, S;
  float *wctx_t, *wctx_x, *bctx;
};

// grid.y = block, grid.z = part: 0 chain weights [tile][16][kp] + biases, 1 [Wg^T | Wb^T] (dout, 2 dout) + [bg | 0],
// 2 the block's columns of Wctx_t (ntemb, S), Wctx_x (nxemb, S) and bctx (S)
__global__ void pack_denoiser_kernel(PackArgs pa) {
  const PackBlock& b = pa.b[blockIdx.y];
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.z == 0) {
    const int ntn = (b.dout + TC - 1) / TC;
    const long n = (long)ntn * 16 * b.kp;
    if (i < n) {
      const int k = (int)(i % b.kp);
      const long rr = i / b.kp;
      const int r = (int)(rr % 16), t = (int)(rr / 16);
      const int col = t * TC + (r & 7);
      float v = 0.f;
      if (col < b.dout && k < b.din) v = (r < 8 ? b.wl : b.ws)[(long)col * b.din + k];
      b.w[i] = v;
    }
    if (i < (long)ntn * 16) {
      const int r = (int)(i % 16), t = (int)(i / 16);
      const int col = t * TC + (r & 7);
      b.bls[i] = col < b.dout ? (r < 8 ? b.bl : b.bs)[col] : 0.f;
    }
  } else if (blockIdx.z == 1) {
    const long n = (long)b.dout * 2 * b.dout;
    if (i < n) {
      const int k = (int)(i / (2 * b.dout)), c = (int)(i % (2 * b.dout));
      b.wgb[i] = c < b.dout ? b.wg[(long)c * b.dout + k] : b.wb[(long)(c - b.dout) * b.dout + k];
    }
    if (i < 2 * b.dout) b.bg2[i] = i < b.dout ? b.bg[i] : 0.f;
  } else {
    const int kc = pa.ntemb + pa.nxemb;
    const long n = (long)kc * b.dout;
    if (i < n) {
      const int k = (int)(i / b.dout), c = (int)(i % b.dout);
      const float v = b.wctx[(long)c * kc + k];
      if (k < pa.ntemb) pa.wctx_t[(long)k * pa.S + b.coloff + c] = v;
      else pa.wctx_x[(long)(k - pa.ntemb) * pa.S + b.coloff + c] = v;
    }
    if (i < b.dout) pa.bctx[b.coloff + i] = b.bctx[i];
  }
}

// (rows, cols) -> (cols, rows)
__global__ void transpose_kernel(const float* in, int rows, int cols, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)rows * cols) return;
  const long r = i / cols, c = i - r * cols;
  out[c * rows + r] = in[i];
}

__global__ void sweep_setup_kernel(SweepCall c, SweepCall* dst, const float* zt, float* zw, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *dst = c;
  if (i < n) zw[i] = zt[i];
}

__global__ void copy_kernel(const float* src, float* dst, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

int sum_dout(const damc_denoiser_t* d) {
  int s = 0;
  for (int j = 0; j < 7; ++j) s += d->blocks[j].dout;
  return s;
}

struct SweepWs {
  float *w[7], *bls[7], *wgb[7], *bg2[7];
  float *wctx_t, *wctx_x, *bctx, *tw1t, *tw2t, *bmat;
  float *px, *qt, *t1, *t2, *xs, *cx, *gh, *z;
  float* outs[7];
  SweepCall* call;
  size_t bytes;
};

size_t carve(const damc_denoiser_t* d, int B, int n, char* base, SweepWs* w) {
  size_t off = 0;
  auto take = [&](long floats) -> float* {
    float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((size_t)floats * sizeof(float) + 255) / 256 * 256;
    return p;
  };
  const int S = sum_dout(d);
  const int nt = d->ntemb, nx = d->nxemb;
  SweepWs t;
  for (int j = 0; j < 7; ++j) {
    const damc_csq_block_t& b = d->blocks[j];
    const int ntn = (b.dout + TC - 1) / TC;
    t.w[j] = take((long)ntn * 16 * kpad(b.din));
    t.bls[j] = take((long)ntn * 16);
    t.wgb[j] = take((long)b.dout * 2 * b.dout);
    t.bg2[j] = take(2L * b.dout);
  }
  t.wctx_t = take((long)nt * S);
  t.wctx_x = take((long)nx * S);
  t.bctx = take(S);
  t.tw1t = take((long)nt * nt);
  t.tw2t = take((long)nt * nt);
  t.bmat = take((long)d->nz * (d->nz / 2));
  t.px = take((long)B * S);
  t.qt = take((long)n * S);
  t.t1 = take((long)n * nt);
  t.t2 = take((long)n * nt);
  t.xs = take((long)B * nx);
  t.cx = take((long)n * B * S);
  t.gh = take((long)n * B * 2 * S);
  t.z = take((long)B * d->nz);
  for (int j = 0; j < 7; ++j) t.outs[j] = take((long)B * d->blocks[j].dout);
  t.call = reinterpret_cast<SweepCall*>(take(64));
  t.bytes = off;
  if (w) *w = t;
  return off;
}

int validate(const damc_denoiser_t* d) {
  if (!d || d->nz <= 0 || (d->nz & 1) || d->ntemb <= 0 || d->nxemb <= 0) return DAMC_ERR_ARG;
  const int nz = d->nz;
  const int w = d->blocks[0].dout;
  // in0 in1 in2 mid out0 out1 out2 widths (Diffusion_UnetA with w = 32 * nf)
  const int din[7] = {2 * nz, w, 2 * w, 2 * w, 4 * w, 4 * w, 2 * w};
  const int dout[7] = {w, 2 * w, 2 * w, 2 * w, 2 * w, w, nz};
  if (!d->bmat || !d->tw1 || !d->tb1 || !d->tw2 || !d->tb2) return DAMC_ERR_ARG;
  for (int j = 0; j < 7; ++j) {
    const damc_csq_block_t& b = d->blocks[j];
    if (b.din != din[j] || b.dout != dout[j]) return DAMC_ERR_ARG;
    if (!b.wl || !b.bl || !b.ws || !b.bs || !b.wg || !b.bg || !b.wb || !d->wctx[j] || !d->bctx[j]) return DAMC_ERR_ARG;
    // float4 fragments / staging need every width % 4 == 0; the in0 LDS image must fit
    if ((b.din & 3) || (b.dout & 3) || (nz & 3)) return DAMC_ERR_UNSUPPORTED;
  }
  if (nz > 16 * EMB_G) return DAMC_ERR_UNSUPPORTED;
  return 0;
}

struct Launch {
  ChainArgs a;
  unsigned grid;
  size_t smem;
};

// the chain launches of one sweep (n steps from step index k0), in order
void chain_launches(const damc_denoiser_t* d, const SweepWs& w, int B, int n, const float* coef,
                    std::vector<Launch>& out) {
  const int S = sum_dout(d);
  int coloff[7];
  for (int j = 0, o = 0; j < 7; ++j) {
    coloff[j] = o;
    o += d->blocks[j].dout;
  }
  float* const* O = w.outs;
  const float* srcA[7] = {nullptr, O[0], O[1], O[2], O[3], O[4], O[5]};
  const float* srcB[7] = {nullptr, nullptr, nullptr, nullptr, O[2], O[1], O[0]};
  const int wa[7] = {0, d->blocks[0].dout, d->blocks[1].dout, d->blocks[2].dout, d->blocks[3].dout,
                     d->blocks[4].dout, d->blocks[5].dout};
  const int wbw[7] = {0, 0, 0, 0, d->blocks[2].dout, d->blocks[1].dout, d->blocks[0].dout};
  out.clear();
  static const int dbg = [] {
    const char* e = getenv("DAMC_CHAIN_DBG");
    return e ? atoi(e) : 0;
  }();
  int noisy_k = 0;
  for (int k = 0; k < n; ++k) {
    const float* c = coef + 6 * (size_t)k;
    const bool last = c[5] != 0.f;
    for (int j = 0; j < 7; ++j) {
      const damc_csq_block_t& b = d->blocks[j];
      Launch L;
      ChainArgs& a = L.a;
      memset(&a, 0, sizeof(a));
      a.srcA = srcA[j];
      a.srcB = srcB[j];
      a.wa = wa[j];
      a.wb = wbw[j];
      a.emb = j == 0;
      a.z = w.z;
      a.bmat = w.bmat;
      a.nz = d->nz;
      a.din = b.din;
      a.kp = kpad(b.din);
      a.dout = b.dout;
      a.B = B;
      a.w = w.w[j];
      a.bls = w.bls[j];
      a.gh = w.gh + (size_t)k * B * 2 * S + 2 * coloff[j];
      a.ldgh = 2L * S;
      a.out = O[j];
      a.final_ = j == 6;
      a.zt = w.z;
      a.call = w.call;
      a.dbg = dbg;
      if (a.final_) {
        a.residual = d->residual;
        a.last = last;
        a.k = k;
        a.noisy_k = noisy_k;
        a.c0 = c[0];
        a.c1 = c[1];
        a.c2 = c[2];
        a.c3 = c[3];
        a.c4 = c[4];
      }
      L.grid = (unsigned)(((b.dout + TC - 1) / TC) * ((B + TM - 1) / TM));
      L.smem = a.emb ? (size_t)TM * emb_ld(a.kp) * sizeof(float) : 0;
      out.push_back(L);
    }
    if (!last) ++noisy_k;
  }
}

void launch_one(const Launch& L, hipStream_t s) {
  if (L.a.emb) hipLaunchKernelGGL(chain_kernel<true>, dim3(L.grid), dim3(CH_THREADS), L.smem, s, L.a);
  else hipLaunchKernelGGL(chain_kernel<false>, dim3(L.grid), dim3(CH_THREADS), L.smem, s, L.a);
}

int launch_chain(const std::vector<Launch>& ls, hipStream_t s) {
  for (const Launch& L : ls) launch_one(L, s);
  return (int)hipGetLastError();
}

// ---- graph cache: the chain of one sweep depends only on workspace addresses, shapes and the schedule scalars
struct GraphEntry {
  int dev;
  const void* wsp;
  size_t wsb;
  int B, n;
  std::vector<char> key;  // shapes + schedule bytes
  hipGraph_t graph;
  hipGraphExec_t exec;
  unsigned long stamp;
};
std::mutex g_mu;
std::vector<GraphEntry> g_cache;
unsigned long g_clock = 0;
constexpr size_t kMaxGraphs = 16;

bool graphs_enabled() {
  static const bool on = [] {
    const char* e = getenv("DAMC_SWEEP_GRAPH");
    return !(e && e[0] == '0');
  }();
  return on;
}

std::vector<char> graph_key(const damc_denoiser_t* d, int n, const float* coef) {
  std::vector<char> k;
  auto put = [&](const void* p, size_t nb) { k.insert(k.end(), (const char*)p, (const char*)p + nb); };
  int dims[4] = {d->nz, d->ntemb, d->nxemb, d->residual};
  put(dims, sizeof(dims));
  for (int j = 0; j < 7; ++j) put(&d->blocks[j].din, 2 * sizeof(int));
  put(coef, sizeof(float) * 6 * (size_t)n);
  return k;
}

// replay (capturing on first use) the chain of a sweep; returns 0 or a hip error
int run_chain_graph(const damc_denoiser_t* d, const SweepWs& w, void* wsp, size_t wsb, int B, int n, const float* coef,
                    hipStream_t s) {
  int dev = 0;
  DAMC_CHECK(hipGetDevice(&dev));
  std::vector<char> key = graph_key(d, n, coef);
  std::lock_guard<std::mutex> lk(g_mu);
  for (GraphEntry& e : g_cache) {
    if (e.dev == dev && e.wsp == wsp && e.wsb == wsb && e.B == B && e.n == n && e.key == key) {
      e.stamp = ++g_clock;
      return (int)hipGraphLaunch(e.exec, s);
    }
  }
  std::vector<Launch> ls;
  chain_launches(d, w, B, n, coef, ls);
  hipStream_t cs;
  DAMC_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipError_t err = hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed);
  if (err == hipSuccess) {
    for (const Launch& L : ls) launch_one(L, cs);
    err = hipStreamEndCapture(cs, &graph);
  }
  if (err == hipSuccess) err = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipStreamDestroy(cs);
  if (err != hipSuccess) {
    if (graph) (void)hipGraphDestroy(graph);
    return (int)err;
  }
  if (g_cache.size() >= kMaxGraphs) {
    auto old = std::min_element(g_cache.begin(), g_cache.end(),
                                [](const GraphEntry& x, const GraphEntry& y) { return x.stamp < y.stamp; });
    (void)hipGraphExecDestroy(old->exec);
    (void)hipGraphDestroy(old->graph);
    g_cache.erase(old);
  }
  g_cache.push_back(GraphEntry{dev, wsp, wsb, B, n, std::move(key), graph, exec, ++g_clock});
  return (int)hipGraphLaunch(exec, s);
}

}  // namespace

extern "C" size_t damc_sweep_workspace_bytes(const damc_denoiser_t* d, int B, int n) {
  if (validate(d) || B <= 0 || n <= 0) return 0;
  return carve(d, B, n, nullptr, nullptr);
}

// step_offset: Philox step index of the first noisy step (a single-step call continues a sweep's noise stream)
static int reverse_sweep_impl(const damc_denoiser_t* d, const float* xemb, float* zt, int B, int n,
                              const float* temb_in, const float* coef, int with_noise, const float* noise,
                              uint64_t seed, uint64_t chain_base, float* eps_log, int eps_log_steps, void* wsp,
                              size_t wsb, void* stream, uint64_t step_offset, bool allow_graph) {
  int rc = validate(d);
  if (rc) return rc;
  if (!xemb || !zt || !temb_in || !coef || B <= 0 || n <= 0) return DAMC_ERR_ARG;
  const size_t need = carve(d, B, n, nullptr, nullptr);
  if (!wsp || wsb < need) return DAMC_ERR_WORKSPACE;
  SweepWs w;
  carve(d, B, n, reinterpret_cast<char*>(wsp), &w);
  hipStream_t s = as_stream(stream);
  const int S = sum_dout(d);
  const int nt = d->ntemb, nx = d->nxemb;
  int coloff[7];
  for (int j = 0, o = 0; j < 7; ++j) {
    coloff[j] = o;
    o += d->blocks[j].dout;
  }

  // ---- 1. pack the live weights
  {
    PackArgs pa;
    long maxn = 0;
    for (int j = 0; j < 7; ++j) {
      const damc_csq_block_t& b = d->blocks[j];
      PackBlock& p = pa.b[j];
      p.wl = b.wl;
      p.bl = b.bl;
      p.ws = b.ws;
      p.bs = b.bs;
      p.wg = b.wg;
      p.bg = b.bg;
      p.wb = b.wb;
      p.wctx = d->wctx[j];
      p.bctx = d->bctx[j];
      p.din = b.din;
      p.dout = b.dout;
      p.kp = kpad(b.din);
      p.coloff = coloff[j];
      p.w = w.w[j];
      p.bls = w.bls[j];
      p.wgb = w.wgb[j];
      p.bg2 = w.bg2[j];
      const long ntn = (b.dout + TC - 1) / TC;
      maxn = std::max({maxn, ntn * 16 * p.kp, 2L * b.dout * b.dout, (long)(nt + nx) * b.dout});
    }
    pa.ntemb = nt;
    pa.nxemb = nx;
    pa.S = S;
    pa.wctx_t = w.wctx_t;
    pa.wctx_x = w.wctx_x;
    pa.bctx = w.bctx;
    hipLaunchKernelGGL(pack_denoiser_kernel, dim3((unsigned)((maxn + 255) / 256), 7, 3), dim3(256), 0, s, pa);
    const long ntt = (long)nt * nt;
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((ntt + 255) / 256)), dim3(256), 0, s, d->tw1, nt, nt, w.tw1t);
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((ntt + 255) / 256)), dim3(256), 0, s, d->tw2, nt, nt, w.tw2t);
    const long nb = (long)d->nz * (d->nz / 2);
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, d->bmat, d->nz, d->nz / 2,
                       w.bmat);
    DAMC_LAUNCH_CHECK();
  }

  // ---- 2. ctx: time MLP (n rows), xemb part (B rows), c for every (step, row)
  {
    damc::GemmArgs g;
    g.M = n;
    g.N = nt;
    g.K = nt;
    g.k_per_z = nt;
    g.A = temb_in;
    g.lda = nt;
    g.B = w.tw1t;
    g.ldb = nt;
    g.C = w.t1;
    g.ldc = nt;
    g.bias = d->tb1;
    g.bias_mod = nt;
    g.act = DAMC_ACT_SILU;
    if ((rc = damc::launch_gemm(g, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "sweep_pre", 2.0 * n * nt * nt, s)))
      return rc;
    g.A = w.t1;
    g.B = w.tw2t;
    g.C = w.t2;
    g.bias = d->tb2;
    g.act = DAMC_ACT_SILU;  // the ctx Linear consumes SiLU(temb)
    if ((rc = damc::launch_gemm(g, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "sweep_pre", 2.0 * n * nt * nt, s)))
      return rc;
    g.A = w.t2;
    g.B = w.wctx_t;
    g.ldb = S;
    g.N = S;
    g.C = w.qt;
    g.ldc = S;
    g.bias = w.bctx;
    g.bias_mod = S;
    g.act = DAMC_ACT_NONE;
    if ((rc = damc::launch_gemm(g, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "sweep_pre", 2.0 * n * nt * S, s)))
      return rc;
    const long nxe = (long)B * nx;
    hipLaunchKernelGGL(silu_kernel, dim3((unsigned)((nxe + 255) / 256)), dim3(256), 0, s, xemb, nxe, w.xs);
    damc::GemmArgs h;
    h.M = B;
    h.N = S;
    h.K = nx;
    h.k_per_z = nx;
    h.A = w.xs;
    h.lda = nx;
    h.B = w.wctx_x;
    h.ldb = S;
    h.C = w.px;
    h.ldc = S;
    if ((rc = damc::launch_gemm(h, damc::A_DENSE, damc::EPI_STORE, damc::O_DENSE, 1, "sweep_pre", 2.0 * B * nx * S, s)))
      return rc;
    const long tot = (long)n * B * S;
    hipLaunchKernelGGL(ctx_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, w.px, w.qt, B, S, tot, w.cx);
    DAMC_LAUNCH_CHECK();
  }

  // ---- 3. every block's gate and hyper bias for every (step, row): [sigmoid(c Wg^T + bg) | c Wb^T]
  for (int j = 0; j < 7; ++j) {
    const int dout = d->blocks[j].dout;
    damc::GemmArgs g;
    g.M = n * B;
    g.N = 2 * dout;
    g.K = dout;
    g.k_per_z = dout;
    g.A = w.cx + coloff[j];
    g.lda = S;
    g.B = w.wgb[j];
    g.ldb = 2 * dout;
    g.C = w.gh + 2 * coloff[j];
    g.ldc = 2L * S;
    g.bias = w.bg2[j];
    g.bias_mod = 2 * dout;
    g.gate_cols = dout;
    if ((rc = damc::launch_gemm(g, damc::A_DENSE, damc::EPI_GATE, damc::O_DENSE, 1, "sweep_hyper",
                                2.0 * n * B * dout * 2.0 * dout, s)))
      return rc;
  }

  // ---- 4. the dependent chain
  SweepCall call;
  call.noise = (with_noise && noise) ? noise : nullptr;
  call.eps_log = eps_log;
  call.eps_log_steps = eps_log ? eps_log_steps : 0;
  call.seed = seed;
  call.chain_base = chain_base;
  call.step_offset = step_offset;
  call.with_noise = with_noise ? 1 : 0;
  const long nzb = (long)B * d->nz;
  hipLaunchKernelGGL(sweep_setup_kernel, dim3((unsigned)((nzb + 255) / 256)), dim3(256), 0, s, call, w.call, zt, w.z,
                     nzb);
  DAMC_LAUNCH_CHECK();
  double flops_step = 0;
  for (int j = 0; j < 7; ++j) flops_step += 2.0 * B * 2.0 * d->blocks[j].din * d->blocks[j].dout;
  {
    ProfScope ps("denoise_chain", flops_step * n, s);
    if (allow_graph && graphs_enabled()) {
      if ((rc = run_chain_graph(d, w, wsp, wsb, B, n, coef, s))) return rc;
    } else {
      std::vector<Launch> ls;
      chain_launches(d, w, B, n, coef, ls);
      if ((rc = launch_chain(ls, s))) return rc;
    }
  }
  hipLaunchKernelGGL(copy_kernel, dim3((unsigned)((nzb + 255) / 256)), dim3(256), 0, s, w.z, zt, nzb);
  return (int)hipGetLastError();
}

extern "C" int damc_reverse_sweep(const damc_denoiser_t* d, const float* xemb, float* zt, int B, int n,
                                  const float* temb_in, const float* coef, int with_noise, const float* noise,
                                  uint64_t seed, uint64_t chain_base, float* eps_log, int eps_log_steps,
                                  void* wsp, size_t wsb, void* stream) {
  return reverse_sweep_impl(d, xemb, zt, B, n, temb_in, coef, with_noise, noise, seed, chain_base, eps_log,
                            eps_log_steps, wsp, wsb, stream, 0, true);
}

// SURVEY.md §8b names
extern "C" int damc_q_reverse_sweep(const damc_denoiser_t* d, const float* xemb, float* zt, int B, int n,
                                    const float* temb_in, const float* coef, int with_noise, const float* noise,
                                    uint64_t seed, uint64_t chain_base, float* eps_log, int eps_log_steps,
                                    void* wsp, size_t wsb, void* stream) {
  return reverse_sweep_impl(d, xemb, zt, B, n, temb_in, coef, with_noise, noise, seed, chain_base, eps_log,
                            eps_log_steps, wsp, wsb, stream, 0, true);
}

extern "C" int damc_denoise_step(const damc_denoiser_t* d, const float* xemb, float* zt, int B, const float* temb_row,
                                 const float* coef_row, int with_noise, const float* noise, uint64_t seed,
                                 uint64_t noise_step, uint64_t chain_base, float* eps, void* wsp, size_t wsb,
                                 void* stream) {
  return reverse_sweep_impl(d, xemb, zt, B, 1, temb_row, coef_row, with_noise, noise, seed, chain_base, eps,
                            eps ? 1 : 0, wsp, wsb, stream, noise_step, false);
}
