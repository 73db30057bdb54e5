// denoiser.hip — Diffusion_UnetA eps-prediction and the amortizer's latent reverse sweep
// (_netQ_U.forward, workspace/src/diffusion_net.py:585-622) on gfx950.
//
// Per sweep (once):  SiLU(xemb) -> px = SiLU(xemb) . Wctx_x           (B, sum dout)   [step-invariant]
//                    time-MLP on the n sinusoidal embeddings -> qt = SiLU(temb) . Wctx_t + bctx
//                                                                      (n, sum dout)   [batch-invariant]
// Per step (7 launches): one fused ConcatSquash block kernel per block:
//     out = (x Wl + bl) * sigmoid(c Wg + bg) + c Wb + (x Ws + bs),   c = SiLU(px[b] + qt[k])
// with the block input x = lrelu(cat(prev, skip), 0.01) formed while staging (in0: the Fourier input
// embedding [sin 2pi zB, cos 2pi zB, z] is computed in the prologue), and the last block's epilogue
// applying eps = z + out, pred_x_from_eps and the reverse-step update with Philox noise in place.
// Block kernel: 4 waves, wave w owns one of the four products (l, s, g, b) for a 16 x 32 output
// tile on v_mfma_f32_16x16x4_f32; operands x / c are staged once per workgroup in LDS.
#include <vector>

#include "gemm.h"

namespace {

constexpr int TM = 16, TN = 32;

struct CsqArgs {
  const float* srcA;  // block input source 1 (B, wa)
  int wa;
  const float* srcB;  // concat source 2 (B, wb) or null
  int wb_;
  int emb_mode;       // 1: input = Fourier embedding of z (in0)
  const float* z;     // (B, nz) current zt
  const float* bmat;  // (nz, nz/2)
  int nz;
  int din, dout, B;
  const float *wl, *bl, *ws, *bs, *wg, *bg, *wb;
  const float* px;    // (B, ldpx) at this block's column offset
  int ldpx;
  const float* qt;    // (ldpx) row of this step at this block's column offset
  float* out;         // (B, dout)
  // final block (reverse step) epilogue
  int final_;
  int residual;
  float c0, c1, c2, c3, c4;
  int last;
  int with_noise;
  const float* noise;  // (B, nz) for this step or null
  uint64_t seed, chain_base, step;
  float* zt;           // updated in place (== z)
  float* eps_log;      // (B, nz) or null
};

__global__ __launch_bounds__(256) void csq_block_kernel(CsqArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int din = a.din, dout = a.dout;
  const int ldx = din + 2, ldcs = dout + 2;  // row strides = 2 (mod 32): conflict-free fragment reads
  float* xs = sm;                            // [TM][ldx]
  float* cs = xs + TM * ldx;                 // [TM][ldcs]
  float* red = cs + TM * ldcs;               // [4][TM][TN]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * TM, n0 = blockIdx.y * TN;

  // ---- stage x (block input) for the 16 rows
  if (a.emb_mode) {
    const int half = a.nz >> 1;
    const float two_pi = 6.28318548f;  // fp32(2*pi), as the reference's 2*np.pi*tensor
    for (int i = tid; i < TM * half; i += 256) {
      const int r = i / half, j = i - r * half;
      const int row = r0 + r;
      float s = 0.f;
      if (row < a.B) {
        const float* zr = a.z + (long)row * a.nz;
        for (int k = 0; k < a.nz; ++k) s = fmaf(zr[k], a.bmat[(long)k * half + j], s);
      }
      const float p = two_pi * s;
      xs[r * ldx + j] = row < a.B ? sinf(p) : 0.f;
      xs[r * ldx + half + j] = row < a.B ? cosf(p) : 0.f;
    }
    for (int i = tid; i < TM * a.nz; i += 256) {
      const int r = i / a.nz, k = i - r * a.nz;
      const int row = r0 + r;
      xs[r * ldx + 2 * half + k] = row < a.B ? a.z[(long)row * a.nz + k] : 0.f;
    }
  } else {
    for (int i = tid; i < TM * din; i += 256) {
      const int r = i / din, k = i - r * din;
      const int row = r0 + r;
      float v = 0.f;
      if (row < a.B) v = k < a.wa ? a.srcA[(long)row * a.wa + k] : a.srcB[(long)row * a.wb_ + (k - a.wa)];
      xs[r * ldx + k] = v > 0.f ? v : 0.01f * v;
    }
  }
  // ---- stage c = SiLU(px + qt)
  for (int i = tid; i < TM * dout; i += 256) {
    const int r = i / dout, n = i - r * dout;
    const int row = r0 + r;
    float v = 0.f;
    if (row < a.B) {
      const float u = a.px[(long)row * a.ldpx + n] + a.qt[n];
      v = u / (1.f + expf(-u));
    }
    cs[r * ldcs + n] = v;
  }
  __syncthreads();

  // ---- wave w: product w over its K; two 16x16 column tiles
  const float* As = (wave < 2) ? xs : cs;
  const int lda_s = (wave < 2) ? ldx : ldcs;
  const int K = (wave < 2) ? din : dout;
  const float* W = wave == 0 ? a.wl : wave == 1 ? a.ws : wave == 2 ? a.wg : a.wb;
  const int am = lane & 15, ak = lane >> 4;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int nA = n0 + am, nB = n0 + 16 + am;
  const bool okA = nA < dout, okB = nB < dout;
#pragma unroll 4
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + ak;
    const float av = As[am * lda_s + k];
    const float* wr = W + (long)k * dout;
    const float b0 = okA ? wr[nA] : 0.f;
    const float b1 = okB ? wr[nB] : 0.f;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc1, 0, 0, 0);
  }
  // C layout 16x16x4: col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (lane >> 4) * 4 + r;
    red[(wave * TM + row) * TN + (lane & 15)] = acc0[r];
    red[(wave * TM + row) * TN + 16 + (lane & 15)] = acc1[r];
  }
  __syncthreads();

  // ---- combine: out = (l + bl) * sigmoid(g + bg) + b + (s + bs)
  for (int i = tid; i < TM * TN; i += 256) {
    const int r = i / TN, c = i - r * TN;
    const int row = r0 + r, col = n0 + c;
    if (row >= a.B || col >= dout) continue;
    const float l = red[(0 * TM + r) * TN + c] + a.bl[col];
    const float s = red[(1 * TM + r) * TN + c] + a.bs[col];
    const float g = red[(2 * TM + r) * TN + c] + a.bg[col];
    const float bb = red[(3 * TM + r) * TN + c];
    const float gate = 1.f / (1.f + expf(-g));
    const float o = l * gate + bb + s;
    if (!a.final_) {
      a.out[(long)row * dout + col] = o;
      continue;
    }
    // reverse step (diffusion_net.py:601-620): eps = z + out; pred = c0 * (z - eps * c1)
    const long zi = (long)row * a.nz + col;
    const float zv = a.zt[zi];
    const float eps = a.residual ? zv + o : o;
    if (a.eps_log) a.eps_log[zi] = eps;
    const float pred = mul_rn(a.c0, sub_rn(zv, mul_rn(eps, a.c1)));
    float zn;
    if (a.last) {
      zn = pred;
    } else {
      zn = add_rn(mul_rn(a.c2, zv), mul_rn(a.c3, pred));
      if (a.with_noise) {
        float xi;
        if (a.noise) {
          xi = a.noise[zi];
        } else {
          float n4[4];
          philox_normal4(a.seed, a.chain_base + row, a.step, (uint32_t)(col >> 2), DAMC_STREAM_SWEEP, n4);
          xi = n4[col & 3];
        }
        zn = add_rn(zn, mul_rn(a.c4, xi));
      }
    }
    a.zt[zi] = zn;
  }
}

__global__ void silu_kernel(const float* x, long n, float* y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const float v = x[i];
    y[i] = v / (1.f + expf(-v));
  }
}

int sum_dout(const damc_denoiser_t* d) {
  int s = 0;
  for (int j = 0; j < 7; ++j) s += d->blocks[j].dout;
  return s;
}

struct SweepWs {
  float *px, *qt, *t1, *t2, *xs;
  float* outs[7];
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
  SweepWs t;
  t.px = take((long)B * S);
  t.qt = take((long)n * S);
  t.t1 = take((long)n * d->ntemb);
  t.t2 = take((long)n * d->ntemb);
  t.xs = take((long)B * d->nxemb);
  for (int j = 0; j < 7; ++j) t.outs[j] = take((long)B * d->blocks[j].dout);
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
  for (int j = 0; j < 7; ++j) {
    const damc_csq_block_t& b = d->blocks[j];
    if (b.din != din[j] || b.dout != dout[j]) return DAMC_ERR_ARG;
    if (!b.wl || !b.bl || !b.ws || !b.bs || !b.wg || !b.bg || !b.wb) return DAMC_ERR_ARG;
    if (b.din > 1024 || b.dout > 512) return DAMC_ERR_UNSUPPORTED;
  }
  return 0;
}

}  // namespace

extern "C" size_t damc_sweep_workspace_bytes(const damc_denoiser_t* d, int B, int n) {
  if (validate(d) || B <= 0 || n <= 0) return 0;
  return carve(d, B, n, nullptr, nullptr);
}

extern "C" int damc_reverse_sweep(const damc_denoiser_t* d, const float* xemb, float* zt, int B, int n,
                                  const float* temb_in, const float* coef, int with_noise, const float* noise,
                                  uint64_t seed, uint64_t chain_base, float* eps_log, int eps_log_steps,
                                  void* wsp, size_t wsb, void* stream) {
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

  // ---- per-sweep precompute: time-MLP (batch-invariant) and the ctx Linear split
  {
    damc::GemmArgs g;
    g.M = n;
    g.N = nt;
    g.K = nt;
    g.k_per_z = nt;
    g.A = temb_in;
    g.lda = nt;
    g.B = d->tw1;
    g.ldb = nt;
    g.C = w.t1;
    g.ldc = nt;
    g.bias = d->tb1;
    g.bias_mod = nt;
    g.act = DAMC_ACT_SILU;
    if ((rc = damc::launch_gemm(g, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "sweep_pre", 2.0 * n * nt * nt, s)))
      return rc;
    g.A = w.t1;
    g.B = d->tw2;
    g.C = w.t2;
    g.bias = d->tb2;
    g.act = DAMC_ACT_SILU;  // the ctx Linear consumes SiLU(temb)
    if ((rc = damc::launch_gemm(g, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "sweep_pre", 2.0 * n * nt * nt, s)))
      return rc;
    g.A = w.t2;
    g.B = d->wctx_t;
    g.ldb = S;
    g.N = S;
    g.C = w.qt;
    g.ldc = S;
    g.bias = d->bctx;
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
    h.B = d->wctx_x;
    h.ldb = S;
    h.C = w.px;
    h.ldc = S;
    if ((rc = damc::launch_gemm(h, damc::A_DENSE, damc::EPI_STORE, damc::O_DENSE, 1, "sweep_pre", 2.0 * B * nx * S, s)))
      return rc;
  }

  // ---- the sweep: 7 fused block launches per step
  int coloff[7];
  {
    int o = 0;
    for (int j = 0; j < 7; ++j) {
      coloff[j] = o;
      o += d->blocks[j].dout;
    }
  }
  // coef is a HOST table: the per-step scalars travel by value in the kernel arguments
  const float* cf = coef;
  // block inputs: source pointers per block (in0: emb of z)
  float* const* O = w.outs;
  const float* srcA[7] = {nullptr, O[0], O[1], O[2], O[3], O[4], O[5]};
  const float* srcB[7] = {nullptr, nullptr, nullptr, nullptr, O[2], O[1], O[0]};
  const int wa[7] = {0, d->blocks[0].dout, d->blocks[1].dout, d->blocks[2].dout, d->blocks[3].dout,
                     d->blocks[4].dout, d->blocks[5].dout};
  const int wbw[7] = {0, 0, 0, 0, d->blocks[2].dout, d->blocks[1].dout, d->blocks[0].dout};
  double flops_step = 0;
  for (int j = 0; j < 7; ++j) {
    const damc_csq_block_t& b = d->blocks[j];
    flops_step += 2.0 * B * (2.0 * b.din * b.dout + 2.0 * b.dout * b.dout);
  }
  int noisy_k = 0;
  for (int k = 0; k < n; ++k) {
    const float* c = cf + 6 * (size_t)k;
    const bool last = c[5] != 0.f;
    ProfScope ps("denoise_step", flops_step, s);
    for (int j = 0; j < 7; ++j) {
      const damc_csq_block_t& b = d->blocks[j];
      CsqArgs a{};
      a.srcA = srcA[j];
      a.wa = wa[j];
      a.srcB = srcB[j];
      a.wb_ = wbw[j];
      a.emb_mode = j == 0;
      a.z = zt;
      a.bmat = d->bmat;
      a.nz = d->nz;
      a.din = b.din;
      a.dout = b.dout;
      a.B = B;
      a.wl = b.wl;
      a.bl = b.bl;
      a.ws = b.ws;
      a.bs = b.bs;
      a.wg = b.wg;
      a.bg = b.bg;
      a.wb = b.wb;
      a.px = w.px + coloff[j];
      a.ldpx = S;
      a.qt = w.qt + (size_t)k * S + coloff[j];
      a.out = O[j];
      a.final_ = j == 6;
      if (a.final_) {
        a.residual = d->residual;
        a.c0 = c[0];
        a.c1 = c[1];
        a.c2 = c[2];
        a.c3 = c[3];
        a.c4 = c[4];
        a.last = last;
        a.with_noise = with_noise && !last;
        a.noise = (a.with_noise && noise) ? noise + (size_t)noisy_k * B * d->nz : nullptr;
        a.seed = seed;
        a.chain_base = chain_base;
        a.step = (uint64_t)noisy_k;
        a.zt = zt;
        a.eps_log = (eps_log && k < eps_log_steps) ? eps_log + (size_t)k * B * d->nz : nullptr;
      }
      const size_t sm = sizeof(float) * ((size_t)TM * (b.din + 2) + (size_t)TM * (b.dout + 2) + 4 * TM * TN);
      dim3 grid((B + TM - 1) / TM, (b.dout + TN - 1) / TN);
      hipLaunchKernelGGL(csq_block_kernel, grid, dim3(256), sm, s, a);
    }
    if (!last) ++noisy_k;
    DAMC_LAUNCH_CHECK();
  }
  (void)temb_in;
  return 0;
}
