// denoiser_train.hip — the denoiser of the Q update: Diffusion_UnetA forward with
// every intermediate kept, and its backward, for Q.calculate_loss (workspace/src/diffusion_net.py:624-645)
// as trained 6x per iteration (workspace/train_gen_recon.py:211-220).
//
// Per-sample logsnr and xemb make every Linear a real (B x din) GEMM: the fp32 MFMA engine (gemm.hip,
// exact fp32) runs them, with the weights of each ConcatSquash block stacked once per call so a block is
// 2 forward GEMMs ([l | s] = x [Wl; Ws]^T, [bias | gate] = c [Wb; Wg]^T) and 4 backward GEMMs (dx, dctx,
// and the two stacked weight gradients), plus one fused elementwise kernel each way.  The seven ctx
// Linears (SiLU(cat(temb, xemb)) -> dout_b) run as ONE GEMM over their stacked weights.  ~40 launches
// forward + ~70 backward for what PyTorch autograd issues as ~1,200.
#include <algorithm>

#include "gemm.h"
#include "wgrad.h"

namespace damc {
namespace {

constexpr float kTwoPi = 6.283185307179586f;  // 2 * np.pi as the fp32 scalar torch multiplies by
constexpr float kSlope = 0.01f;               // F.leaky_relu(out, negative_slope=0.01) between blocks

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x / (1.f + expf(-x)); }
// d silu: grad * s * (1 + x (1 - s)) (ATen silu_backward)
__device__ __forceinline__ float dsilu(float g, float x) {
  const float s = sigm(x);
  return g * s * (1.f + x * (1.f - s));
}
__device__ __forceinline__ float dlrelu(float g, float pre) { return pre > 0.f ? g : g * kSlope; }

// ------------------------------------------------------------------ weight stacking (one launch per table)
// each descriptor: src (rows x cols, row-major; NULL = zeros) -> dst_t[k * ldt + t_col + o] (transposed)
// and/or dst[(d_row + o) * ldd + k] (copy); 32x32 tiles through LDS
struct PackDesc {
  const float* src;
  float* dst_t;
  float* dst;
  int rows, cols, ldt, t_col, ldd, d_row;
};
constexpr int kPackMax = 40;
struct PackTable {
  int n;
  PackDesc d[kPackMax];
};

__global__ __launch_bounds__(256) void pack_multi_kernel(PackTable tab) {
  const PackDesc D = tab.d[blockIdx.y];
  const int tc_n = (D.cols + 31) / 32, tr_n = (D.rows + 31) / 32;
  if ((int)blockIdx.x >= tr_n * tc_n) return;
  const int tr = blockIdx.x / tc_n, tc = blockIdx.x - tr * tc_n;
  __shared__ float t[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int o = tr * 32 + r, k = tc * 32 + tx;
    float v = 0.f;
    if (o < D.rows && k < D.cols) {
      if (D.src) v = D.src[(long)o * D.cols + k];
      if (D.dst) D.dst[(long)(D.d_row + o) * D.ldd + k] = v;
    }
    t[r][tx] = v;
  }
  __syncthreads();
  if (!D.dst_t) return;
  for (int r = ty; r < 32; r += 8) {
    const int k = tc * 32 + r, o = tr * 32 + tx;
    if (k < D.cols && o < D.rows) D.dst_t[(long)k * D.ldt + D.t_col + o] = t[tx][r];
  }
}

struct Packer {
  PackTable tab{};
  int max_tiles = 0;
  hipStream_t s;
  int rc = 0;
  explicit Packer(hipStream_t st) : s(st) { tab.n = 0; }
  void add(const float* src, int rows, int cols, float* dst_t, int ldt, int t_col, float* dst, int ldd, int d_row) {
    if (tab.n == kPackMax) flush();
    tab.d[tab.n++] = PackDesc{src, dst_t, dst, rows, cols, ldt, t_col, ldd, d_row};
    max_tiles = std::max(max_tiles, ((rows + 31) / 32) * ((cols + 31) / 32));
  }
  void flush() {
    if (tab.n == 0) return;
    hipLaunchKernelGGL(pack_multi_kernel, dim3((unsigned)max_tiles, (unsigned)tab.n), dim3(256), 0, s, tab);
    if (!rc) rc = (int)hipGetLastError();
    tab.n = 0;
    max_tiles = 0;
  }
};

// ------------------------------------------------------------------ gradient scatter (one launch)
struct CopyDesc {
  const float* src;
  float* dst;
  long n;
};
constexpr int kCopyMax = 64;
struct CopyTable {
  int n;
  CopyDesc d[kCopyMax];
};
__global__ __launch_bounds__(256) void copy_multi_kernel(CopyTable tab) {
  const CopyDesc D = tab.d[blockIdx.y];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < D.n; i += (long)gridDim.x * blockDim.x)
    D.dst[i] = D.src[i];
}

// ------------------------------------------------------------------ forward elementwise
__global__ void silu_copy_kernel(const float* __restrict__ x, long n, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = silu_f(x[i]);
}

// emb[:, T:] = xemb (temb already in emb[:, :T]); semb = silu(emb)
__global__ void emb_finish_kernel(float* __restrict__ emb, const float* __restrict__ xemb, int B, int T, int X,
                                  float* __restrict__ semb) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int E = T + X;
  if (i >= (long)B * E) return;
  const int n = (int)(i / E), j = (int)(i - (long)n * E);
  float v;
  if (j < T) {
    v = emb[i];
  } else {
    v = xemb[(long)n * X + j - T];
    emb[i] = v;
  }
  semb[i] = silu_f(v);
}

struct BlockOff {
  int off[8];  // column offset of block b in the stacked ctx output; off[7] = total
};
// c_b[n][j] = silu(u_all[n][off_b + j]); c_b stored contiguously at c + B * off_b
__global__ void ctx_silu_kernel(const float* __restrict__ u, int B, BlockOff bo, float* __restrict__ c) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int D = bo.off[7];
  if (i >= (long)B * D) return;
  const int n = (int)(i / D), col = (int)(i - (long)n * D);
  int b = 0;
  while (col >= bo.off[b + 1]) ++b;
  const int dout = bo.off[b + 1] - bo.off[b];
  c[(long)B * bo.off[b] + (long)n * dout + (col - bo.off[b])] = silu_f(u[i]);
}

// X0 = cat(sin(2 pi v), cos(2 pi v), z) (diffusion_net.py:486-488); zT = z^T (backward operand)
__global__ void input_emb_kernel(const float* __restrict__ v, const float* __restrict__ z, int B, int nz,
                                 float* __restrict__ X0, float* __restrict__ zT) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int h = nz / 2, din = 2 * h + nz;
  if (i >= (long)B * din) return;
  const int n = (int)(i / din), j = (int)(i - (long)n * din);
  float o;
  if (j < h) {
    o = sinf(kTwoPi * v[(long)n * h + j]);
  } else if (j < 2 * h) {
    o = cosf(kTwoPi * v[(long)n * h + j - h]);
  } else {
    o = z[(long)n * nz + j - 2 * h];
    zT[(long)(j - 2 * h) * B + n] = o;
  }
  X0[i] = o;
}

// block output: gate = sigmoid(G), R = (l * gate + bias) + s (diffusion_net.py:438-443); then the next
// block's input lrelu(cat(R, hs)) or, for the last block, eps = z + R (residual) / R
__global__ void csq_combine_kernel(const float* __restrict__ LS, float* __restrict__ BG, int B, int dout,
                                   float* __restrict__ R, float* __restrict__ Xn, int dinn,
                                   const float* __restrict__ hs, const float* __restrict__ z,
                                   float* __restrict__ eps) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * dout) return;
  const int n = (int)(i / dout), j = (int)(i - (long)n * dout);
  const float l = LS[(long)n * 2 * dout + j], s = LS[(long)n * 2 * dout + dout + j];
  const float bb = BG[(long)n * 2 * dout + j];
  const float g = sigm(BG[(long)n * 2 * dout + dout + j]);
  BG[(long)n * 2 * dout + dout + j] = g;
  const float r = (l * g + bb) + s;
  R[i] = r;
  if (eps) {
    eps[i] = z ? z[i] + r : r;
    return;
  }
  Xn[(long)n * dinn + j] = r > 0.f ? r : r * kSlope;
  if (hs) {
    const float hv = hs[i];  // the skip input has the same width as this block's output
    Xn[(long)n * dinn + dout + j] = hv > 0.f ? hv : hv * kSlope;
  }
}

// ------------------------------------------------------------------ backward elementwise
// D = [dl | dR | dgate_pre] (B x 3 dout) and its transpose T (3 dout x B)
__global__ void csq_bwd_kernel(const float* __restrict__ dR, const float* __restrict__ LS,
                               const float* __restrict__ BG, int B, int dout, float* __restrict__ D,
                               float* __restrict__ T) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * dout) return;
  const int n = (int)(i / dout), j = (int)(i - (long)n * dout);
  const float d = dR[i];
  const float l = LS[(long)n * 2 * dout + j], g = BG[(long)n * 2 * dout + dout + j];
  const float dl = d * g;
  const float dgp = (d * l) * (1.f - g) * g;  // sigmoid_backward: grad * (1 - y) * y
  float* Dr = D + (long)n * 3 * dout;
  Dr[j] = dl;
  Dr[dout + j] = d;
  Dr[2 * dout + j] = dgp;
  T[(long)j * B + n] = dl;
  T[(long)(dout + j) * B + n] = d;
  T[(long)(2 * dout + j) * B + n] = dgp;
}

// dX (B x (da + dc)) of a block input lrelu(cat(Ra, Rc)) -> dRa (= or +=) and dRc (= or +=)
__global__ void propagate_kernel(const float* __restrict__ dX, int B, int din, const float* __restrict__ Ra, int da,
                                 float* __restrict__ dRa, int acc_a, const float* __restrict__ Rc,
                                 float* __restrict__ dRc, int acc_c) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * din) return;
  const int n = (int)(i / din), j = (int)(i - (long)n * din);
  const float g = dX[i];
  if (j < da) {
    const long o = (long)n * da + j;
    const float v = dlrelu(g, Ra[o]);
    dRa[o] = acc_a ? dRa[o] + v : v;
  } else {
    const int dc = din - da;
    const long o = (long)n * dc + (j - da);
    const float v = dlrelu(g, Rc[o]);
    dRc[o] = acc_c ? dRc[o] + v : v;
  }
}

// y = g * silu'(x) and its transpose yT (cols x B); ldx = row stride of x and g
__global__ void dsilu_t_kernel(const float* __restrict__ g, const float* __restrict__ x, int B, int cols,
                               float* __restrict__ y, float* __restrict__ yT) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * cols) return;
  const int n = (int)(i / cols), j = (int)(i - (long)n * cols);
  const float v = dsilu(g[i], x[i]);
  y[i] = v;
  if (yT) yT[(long)j * B + n] = v;
}

// demb = dsemb * silu'(emb): dtemb (+ transpose) and dxemb
__global__ void emb_bwd_kernel(const float* __restrict__ dsemb, const float* __restrict__ emb, int B, int T, int X,
                               float* __restrict__ dtemb, float* __restrict__ dtembT, float* __restrict__ dxemb) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int E = T + X;
  if (i >= (long)B * E) return;
  const int n = (int)(i / E), j = (int)(i - (long)n * E);
  const float v = dsilu(dsemb[i], emb[i]);
  if (j < T) {
    dtemb[(long)n * T + j] = v;
    dtembT[(long)j * B + n] = v;
  } else if (dxemb) {
    dxemb[(long)n * X + j - T] = v;
  }
}

// dv = 2 pi (dX0_sin * cos(w) - dX0_cos * sin(w)), w = 2 pi v
__global__ void input_emb_bwd_kernel(const float* __restrict__ dX0, const float* __restrict__ v, int B, int nz,
                                     float* __restrict__ dv) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int h = nz / 2, din = 2 * h + nz;
  if (i >= (long)B * h) return;
  const int n = (int)(i / h), j = (int)(i - (long)n * h);
  const float w = kTwoPi * v[i];
  const float ds = dX0[(long)n * din + j], dc = dX0[(long)n * din + h + j];
  dv[i] = (ds * cosf(w) + dc * -sinf(w)) * kTwoPi;
}

// dz = g (residual) + dX0[:, 2h:] + dzp
__global__ void dz_kernel(const float* __restrict__ g, const float* __restrict__ dX0, const float* __restrict__ dzp,
                          int B, int nz, float* __restrict__ dz) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * nz) return;
  const int n = (int)(i / nz), j = (int)(i - (long)n * nz);
  const int din = 2 * (nz / 2) + nz;
  float v = dX0[(long)n * din + 2 * (nz / 2) + j] + dzp[i];
  if (g) v += g[i];
  dz[i] = v;
}

inline dim3 grid1(long n) { return dim3((unsigned)((n + 255) / 256)); }

// sum of S split-K slabs [S][M][N] (+ bias[n]) into C (row stride ldc), fixed order
__global__ void slab_bias_sum_kernel(const float* __restrict__ slabs, int S, int M, int N,
                                     const float* __restrict__ bias, float* __restrict__ C, long ldc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (long)m * N);
  float acc = 0.f;
  for (int z = 0; z < S; ++z) acc += slabs[(long)z * M * N + i];
  if (bias) acc += bias[n];
  C[(long)m * ldc + n] = acc;
}

// C (M x N, row stride ldc) = A (M x K, lda) . B (K x N row-major, ldb) (+ bias).  A (B x din) activation
// times a weight has M = B <= 256 rows: 1-4 output tiles of the engine, so those GEMMs split K over
// workgroups (>= 2 K tiles each) into slab[S][M][N] and a fixed-order sum adds the slices and the bias.
constexpr int kMaxSplit = 16;
int gemm(const float* A, long lda, const float* Bm, long ldb, const float* bias, float* C, long ldc, int M, int N,
         int K, const char* name, hipStream_t s, float* slab = nullptr) {
  // round 5: every product of this net is small (M = B rows or K = B): one launch of the 16 x 16-per-wave kernel
  // instead of the tiled engine's 1-16 workgroups or its split-K slabs plus a reduce; DAMC_DN_SMALL_GEMM=0 (read per
  // call) keeps the tiled engine
  const char* esg = getenv("DAMC_DN_SMALL_GEMM");
  if (!(esg && esg[0] == '0')) {
    const int rc = launch_small_gemm(A, lda, Bm, ldb, bias, C, ldc, M, N, K, s);
    if (rc != DAMC_ERR_UNSUPPORTED) return rc;
  }
  GemmArgs a;
  a.A = A;
  a.lda = lda;
  a.B = Bm;
  a.ldb = ldb;
  a.M = M;
  a.N = N;
  a.K = K;
  a.act = DAMC_ACT_NONE;
  const long tiles = (long)((M + 127) / 128) * ((N + 127) / 128);
  const int kt = (K + 31) / 32;
  int S = 1;
  if (slab && tiles < 64 && kt >= 4) S = std::min(kMaxSplit, std::max(1, std::min<int>(kt / 2, (int)(128 / tiles))));
  if (S > 1) {
    const int kper = (kt + S - 1) / S * 32;
    S = (K + kper - 1) / kper;
    a.C = slab;
    a.ldc = N;
    a.c_zstride = (long)M * N;
    a.k_per_z = kper;
    int rc = launch_gemm(a, A_DENSE, EPI_STORE, O_DENSE, S, name, 2.0 * M * N * K, s);
    if (rc) return rc;
    hipLaunchKernelGGL(slab_bias_sum_kernel, dim3((unsigned)(((long)M * N + 255) / 256)), dim3(256), 0, s,
                       (const float*)slab, S, M, N, bias, C, ldc);
    return (int)hipGetLastError();
  }
  a.C = C;
  a.ldc = ldc;
  a.k_per_z = K;
  a.bias = bias;
  a.bias_mod = N;
  return launch_gemm(a, A_DENSE, EPI_BIAS_ACT, O_DENSE, 1, name, 2.0 * M * N * K, s);
}

// several independent products of one stage (and the bias gradients as column sums) in ONE launch of the grouped
// small-GEMM kernel (gemm.hip small_gemm_group_kernel; round 5: the Q update issued 53 GEMM launches of 4-20 us, each
// latency-bound on its single-wave K chain).  DAMC_DN_GROUP=0 (read per call), DAMC_DN_SMALL_GEMM=0 or a member the
// kernel does not take: every member on its own (gemm() above, launch_colsum for the column sums)
struct Grp {
  SmallGemm g[SG_GROUP_MAX];
  int n = 0;
  void mm(const float* A, long lda, const float* Bm, long ldb, const float* bias, float* C, long ldc, int M, int N,
          int K) {
    SmallGemm& d = g[n++];
    d.A = A;
    d.lda = lda;
    d.B = Bm;
    d.ldb = ldb;
    d.bias = bias;
    d.C = C;
    d.ldc = ldc;
    d.M = M;
    d.N = N;
    d.K = K;
  }
  // C (N) = column sums of X (R x N, row stride ld)
  void colsum(const float* X, long R, int N, long ld, float* C) {
    SmallGemm& d = g[n++];
    d.a_ones = 1;
    d.B = X;
    d.ldb = ld;
    d.C = C;
    d.ldc = N;
    d.M = 1;
    d.N = N;
    d.K = (int)R;
  }
  int run(float* slab, float* tmp, hipStream_t s) {
    const char* eg = getenv("DAMC_DN_GROUP");
    const char* esg = getenv("DAMC_DN_SMALL_GEMM");
    if (!(eg && eg[0] == '0') && !(esg && esg[0] == '0')) {
      const int rc = launch_small_gemm_group(g, n, s);
      if (rc != DAMC_ERR_UNSUPPORTED) return rc;
    }
    for (int i = 0; i < n; ++i) {
      const SmallGemm& d = g[i];
      const int rc = d.a_ones ? launch_colsum(d.B, d.K, d.N, d.ldb, d.C, tmp, s)
                              : gemm(d.A, d.lda, d.B, d.ldb, d.bias, d.C, d.ldc, d.M, d.N, d.K, "dn_gemm", s,
                                     d.M <= 256 ? slab : nullptr);
      if (rc) return rc;
    }
    return 0;
  }
};

// ------------------------------------------------------------------ workspace
struct DW {
  // packed weights
  float *WLS_T[7], *WLS[7], *WBG_T[7], *WBG[7], *bLS[7], *bBG[7];
  float *WC_T, *WC, *bC, *T1_T, *T2_T, *BmT;
  // forward intermediates
  float *se_in, *a1, *s1, *emb, *semb, *u, *c, *v, *zT, *X[7], *LS[7], *BG[7], *R[7];
  // backward
  float *D, *T, *dX, *dR[7], *dc, *du, *duT, *dsemb, *dtemb, *dtembT, *ds1, *da1, *da1T, *dv, *dzp;
  float *gWLS[7], *gWBG[7], *gbD[7], *gWC, *gbC, *tmp, *slab;
  int off[8];
  int maxd, maxin;
};

int validate(const damc_denoiser_train_t* d) {
  if (!d || d->nz <= 0 || d->nz % 2 || d->ntemb <= 0 || d->nxemb <= 0 || d->ntemb % 2) return DAMC_ERR_ARG;
  if (!d->bmat || !d->tw1 || !d->tb1 || !d->tw2 || !d->tb2) return DAMC_ERR_ARG;
  int o[7], in[7];
  for (int b = 0; b < 7; ++b) {
    const damc_csq_block_t& k = d->blocks[b];
    if (!k.wl || !k.bl || !k.ws || !k.bs || !k.wg || !k.bg || !k.wb || !d->wctx[b] || !d->bctx[b]) return DAMC_ERR_ARG;
    o[b] = k.dout;
    in[b] = k.din;
    if (o[b] <= 0 || in[b] <= 0) return DAMC_ERR_ARG;
  }
  // Diffusion_UnetA wiring (diffusion_net.py:470-533)
  if (in[0] != 2 * (d->nz / 2) + d->nz || in[1] != o[0] || in[2] != o[1] || in[3] != o[2]) return DAMC_ERR_ARG;
  if (in[4] != o[3] + o[2] || in[5] != o[4] + o[1] || in[6] != o[5] + o[0] || o[6] != d->nz) return DAMC_ERR_ARG;
  if (o[3] != o[2] || o[4] != o[1] || o[5] != o[0]) return DAMC_ERR_ARG;  // skip inputs as wide as the output
  return 0;
}

size_t carve(const damc_denoiser_train_t* d, int B, char* base, DW* w) {
  size_t off = 0;
  auto take = [&](long floats) -> float* {
    float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((size_t)std::max(floats, 1L) * sizeof(float) + 255) / 256 * 256;
    return p;
  };
  const int T = d->ntemb, X = d->nxemb, E = T + X, nz = d->nz, h = nz / 2;
  DW t{};
  t.off[0] = 0;
  t.maxd = t.maxin = 0;
  for (int b = 0; b < 7; ++b) {
    t.off[b + 1] = t.off[b] + d->blocks[b].dout;
    t.maxd = std::max(t.maxd, d->blocks[b].dout);
    t.maxin = std::max(t.maxin, d->blocks[b].din);
  }
  const int Dt = t.off[7];
  for (int b = 0; b < 7; ++b) {
    const long di = d->blocks[b].din, dd = d->blocks[b].dout;
    t.WLS_T[b] = take(di * 2 * dd);
    t.WLS[b] = take(2 * dd * di);
    t.WBG_T[b] = take(dd * 2 * dd);
    t.WBG[b] = take(2 * dd * dd);
    t.bLS[b] = take(2 * dd);
    t.bBG[b] = take(2 * dd);
  }
  t.WC_T = take((long)E * Dt);
  t.WC = take((long)Dt * E);
  t.bC = take(Dt);
  t.T1_T = take((long)T * T);
  t.T2_T = take((long)T * T);
  t.BmT = take((long)h * nz);
  t.se_in = take((long)B * T);
  t.a1 = take((long)B * T);
  t.s1 = take((long)B * T);
  t.emb = take((long)B * E);
  t.semb = take((long)B * E);
  t.u = take((long)B * Dt);
  t.c = take((long)B * Dt);
  t.v = take((long)B * h);
  t.zT = take((long)nz * B);
  for (int b = 0; b < 7; ++b) {
    const long di = d->blocks[b].din, dd = d->blocks[b].dout;
    t.X[b] = take(B * di);
    t.LS[b] = take(B * 2 * dd);
    t.BG[b] = take(B * 2 * dd);
    t.R[b] = take(B * dd);
  }
  t.D = take((long)B * 3 * t.maxd);
  t.T = take((long)B * 3 * t.maxd);
  t.dX = take((long)B * t.maxin);
  for (int b = 0; b < 7; ++b) t.dR[b] = take((long)B * d->blocks[b].dout);
  t.dc = take((long)B * Dt);
  t.du = take((long)B * Dt);
  t.duT = take((long)B * Dt);
  t.dsemb = take((long)B * E);
  t.dtemb = take((long)B * T);
  t.dtembT = take((long)B * T);
  t.ds1 = take((long)B * T);
  t.da1 = take((long)B * T);
  t.da1T = take((long)B * T);
  t.dv = take((long)B * h);
  t.dzp = take((long)B * nz);
  for (int b = 0; b < 7; ++b) {
    const long di = d->blocks[b].din, dd = d->blocks[b].dout;
    t.gWLS[b] = take(2 * dd * di);
    t.gWBG[b] = take(2 * dd * dd);
    t.gbD[b] = take(3 * dd);
  }
  t.gWC = take((long)Dt * E);
  t.gbC = take(Dt);
  size_t tmpf = std::max(colsum_tmp_floats(B, 3 * t.maxd), colsum_tmp_floats(B, Dt));
  tmpf = std::max(tmpf, colsum_tmp_floats(B, T));
  t.tmp = take((long)tmpf);
  {  // split-K slabs of the (B x N) GEMMs: N <= max(2 dout, din, sum dout, ntemb + nxemb)
    const long nmax = std::max<long>(std::max(2L * t.maxd, (long)t.maxin), std::max<long>(Dt, E));
    t.slab = take((long)kMaxSplit * B * nmax);
  }
  if (w) *w = t;
  return off;
}

int setup(const damc_denoiser_train_t* d, int B, void* wsp, size_t wsb, DW* w) {
  int rc = validate(d);
  if (rc) return rc;
  if (B <= 0) return DAMC_ERR_ARG;
  const size_t need = carve(d, B, nullptr, nullptr);
  if (!wsp || wsb < need) return DAMC_ERR_WORKSPACE;
  carve(d, B, reinterpret_cast<char*>(wsp), w);
  return 0;
}

#define RC(x)                \
  do {                       \
    const int rc_ = (x);     \
    if (rc_) return rc_;     \
  } while (0)

int forward(const damc_denoiser_train_t* d, const float* zt, const float* se, const float* xemb, int B, float* eps,
            DW& w, hipStream_t s) {
  const int T = d->ntemb, X = d->nxemb, E = T + X, nz = d->nz, h = nz / 2, Dt = w.off[7];
  {  // stack / transpose the live weights (the nets train between calls)
    ProfScope ps("dn_pack", 0.0, s);
    Packer pk(s);
    for (int b = 0; b < 7; ++b) {
      const damc_csq_block_t& k = d->blocks[b];
      const int di = k.din, dd = k.dout;
      pk.add(k.wl, dd, di, w.WLS_T[b], 2 * dd, 0, w.WLS[b], di, 0);
      pk.add(k.ws, dd, di, w.WLS_T[b], 2 * dd, dd, w.WLS[b], di, dd);
      pk.add(k.wb, dd, dd, w.WBG_T[b], 2 * dd, 0, w.WBG[b], dd, 0);
      pk.add(k.wg, dd, dd, w.WBG_T[b], 2 * dd, dd, w.WBG[b], dd, dd);
      pk.add(d->wctx[b], dd, E, w.WC_T, Dt, w.off[b], w.WC, E, w.off[b]);
    }
    pk.add(d->tw1, T, T, w.T1_T, T, 0, nullptr, 0, 0);
    pk.add(d->tw2, T, T, w.T2_T, T, 0, nullptr, 0, 0);
    pk.add(d->bmat, nz, h, w.BmT, nz, 0, nullptr, 0, 0);
    pk.flush();
    for (int b = 0; b < 7; ++b) {  // biases as (dout x 1) columns -> stacked rows
      const damc_csq_block_t& k = d->blocks[b];
      const int dd = k.dout;
      pk.add(k.bl, dd, 1, w.bLS[b], 0, 0, nullptr, 0, 0);
      pk.add(k.bs, dd, 1, w.bLS[b], 0, dd, nullptr, 0, 0);
      pk.add(nullptr, dd, 1, w.bBG[b], 0, 0, nullptr, 0, 0);  // _hyper_bias has no bias
      pk.add(k.bg, dd, 1, w.bBG[b], 0, dd, nullptr, 0, 0);
      pk.add(d->bctx[b], dd, 1, w.bC, 0, w.off[b], nullptr, 0, 0);
    }
    pk.flush();
    RC(pk.rc);
  }
  // time MLP: temb = Lt2(silu(Lt1(se))) written into emb[:, :T] (se kept for dWt1)
  DAMC_CHECK(hipMemcpyAsync(w.se_in, se, sizeof(float) * B * T, hipMemcpyDeviceToDevice, s));
  {  // Lt1 and the input embedding's z B are independent: one launch
    Grp gp;
    gp.mm(w.se_in, T, w.T1_T, T, d->tb1, w.a1, T, B, T, T);
    gp.mm(zt, nz, d->bmat, h, nullptr, w.v, h, B, h, nz);
    RC(gp.run(w.slab, w.tmp, s));
  }
  hipLaunchKernelGGL(silu_copy_kernel, grid1((long)B * T), dim3(256), 0, s, w.a1, (long)B * T, w.s1);
  {
    Grp gp;
    gp.mm(w.s1, T, w.T2_T, T, d->tb2, w.emb, E, B, T, T);
    RC(gp.run(w.slab, w.tmp, s));
  }
  hipLaunchKernelGGL(emb_finish_kernel, grid1((long)B * E), dim3(256), 0, s, w.emb, xemb, B, T, X, w.semb);
  {  // the 7 ctx Linears in one GEMM, then c_b = silu
    Grp gp;
    gp.mm(w.semb, E, w.WC_T, Dt, w.bC, w.u, Dt, B, Dt, E);
    RC(gp.run(w.slab, w.tmp, s));
  }
  BlockOff bo;
  for (int b = 0; b < 8; ++b) bo.off[b] = w.off[b];
  hipLaunchKernelGGL(ctx_silu_kernel, grid1((long)B * Dt), dim3(256), 0, s, w.u, B, bo, w.c);
  // input embedding
  hipLaunchKernelGGL(input_emb_kernel, grid1((long)B * (2 * h + nz)), dim3(256), 0, s, w.v, zt, B, nz, w.X[0], w.zT);
  // blocks; skip inputs: out0 <- in2, out1 <- in1, out2 <- in0
  const int hs_of[7] = {-1, -1, -1, 2, 1, 0, -1};
  for (int b = 0; b < 7; ++b) {
    const int di = d->blocks[b].din, dd = d->blocks[b].dout;
    const float* cb = w.c + (long)B * w.off[b];
    Grp gp;
    gp.mm(w.X[b], di, w.WLS_T[b], 2 * dd, w.bLS[b], w.LS[b], 2 * dd, B, 2 * dd, di);
    gp.mm(cb, dd, w.WBG_T[b], 2 * dd, w.bBG[b], w.BG[b], 2 * dd, B, 2 * dd, dd);
    RC(gp.run(w.slab, w.tmp, s));
    const bool last = b == 6;
    const float* hs = (!last && hs_of[b] >= 0) ? w.R[hs_of[b]] : nullptr;
    hipLaunchKernelGGL(csq_combine_kernel, grid1((long)B * dd), dim3(256), 0, s, w.LS[b], w.BG[b], B, dd, w.R[b],
                       last ? nullptr : w.X[b + 1], last ? 0 : d->blocks[b + 1].din, hs,
                       (last && d->residual) ? zt : nullptr, last ? eps : nullptr);
  }
  return (int)hipGetLastError();
}

int backward(const damc_denoiser_train_t* d, const float* g, int B, const damc_denoiser_grads_t* gr, float* dzt,
             float* dxemb, DW& w, hipStream_t s) {
  const int T = d->ntemb, X = d->nxemb, E = T + X, nz = d->nz, h = nz / 2, Dt = w.off[7];
  // block b's input is lrelu(cat(R[pa], R[pc])) (pc < 0: no skip part); b = 0: the input embedding
  const int pa[7] = {-1, 0, 1, 2, 3, 4, 5}, pc[7] = {-1, -1, -1, -1, 2, 1, 0};
  bool seen[7] = {false, false, false, false, false, false, false};  // dR[b] holds a first contribution
  for (int b = 6; b >= 0; --b) {
    const int di = d->blocks[b].din, dd = d->blocks[b].dout;
    const float* dR = b == 6 ? g : w.dR[b];
    const float* cb = w.c + (long)B * w.off[b];
    hipLaunchKernelGGL(csq_bwd_kernel, grid1((long)B * dd), dim3(256), 0, s, dR, w.LS[b], w.BG[b], B, dd, w.D, w.T);
    {
      Grp gp;
      gp.mm(w.D, 3 * dd, w.WLS[b], di, nullptr, w.dX, di, B, di, 2 * dd);
      gp.mm(w.D + dd, 3 * dd, w.WBG[b], dd, nullptr, w.dc + w.off[b], Dt, B, dd, 2 * dd);
      gp.mm(w.T, B, w.X[b], di, nullptr, w.gWLS[b], di, 2 * dd, di, B);
      gp.mm(w.T + (long)dd * B, B, cb, dd, nullptr, w.gWBG[b], dd, 2 * dd, dd, B);
      gp.colsum(w.D, B, 3 * dd, 3 * dd, w.gbD[b]);
      RC(gp.run(w.slab, w.tmp, s));
    }
    if (b > 0) {
      const int a = pa[b], c = pc[b];
      const int da = d->blocks[a].dout;
      hipLaunchKernelGGL(propagate_kernel, grid1((long)B * di), dim3(256), 0, s, w.dX, B, di, w.R[a], da, w.dR[a],
                         (int)seen[a], c >= 0 ? w.R[c] : nullptr, c >= 0 ? w.dR[c] : nullptr,
                         c >= 0 ? (int)seen[c] : 0);
      seen[a] = true;
      if (c >= 0) seen[c] = true;
    }
  }
  // input embedding (w.dX now holds dX0) -> dBm, dz
  hipLaunchKernelGGL(input_emb_bwd_kernel, grid1((long)B * h), dim3(256), 0, s, w.dX, w.v, B, nz, w.dv);
  {
    Grp gp;
    if (gr->bmat) gp.mm(w.zT, B, w.dv, h, nullptr, gr->bmat, h, nz, h, B);
    if (dzt) gp.mm(w.dv, h, w.BmT, nz, nullptr, w.dzp, nz, B, nz, h);
    if (gp.n) RC(gp.run(w.slab, w.tmp, s));
  }
  if (dzt) {
    hipLaunchKernelGGL(dz_kernel, grid1((long)B * nz), dim3(256), 0, s, d->residual ? g : nullptr, w.dX, w.dzp, B,
                       nz, dzt);
  }
  // ctx: du = dc * silu'(u); dsemb = du Wc; dWc = du^T semb; dbc = colsum(du)
  hipLaunchKernelGGL(dsilu_t_kernel, grid1((long)B * Dt), dim3(256), 0, s, w.dc, w.u, B, Dt, w.du, w.duT);
  {
    Grp gp;
    gp.mm(w.du, Dt, w.WC, E, nullptr, w.dsemb, E, B, E, Dt);
    gp.mm(w.duT, B, w.semb, E, nullptr, w.gWC, E, Dt, E, B);
    gp.colsum(w.du, B, Dt, Dt, w.gbC);
    RC(gp.run(w.slab, w.tmp, s));
  }
  hipLaunchKernelGGL(emb_bwd_kernel, grid1((long)B * E), dim3(256), 0, s, w.dsemb, w.emb, B, T, X, w.dtemb, w.dtembT,
                     dxemb);
  // time MLP
  {
    Grp gp;
    if (gr->tw2) gp.mm(w.dtembT, B, w.s1, T, nullptr, gr->tw2, T, T, T, B);
    if (gr->tb2) gp.colsum(w.dtemb, B, T, T, gr->tb2);
    if (gr->tw1 || gr->tb1) gp.mm(w.dtemb, T, d->tw2, T, nullptr, w.ds1, T, B, T, T);
    if (gp.n) RC(gp.run(w.slab, w.tmp, s));
  }
  if (gr->tw1 || gr->tb1) {
    hipLaunchKernelGGL(dsilu_t_kernel, grid1((long)B * T), dim3(256), 0, s, w.ds1, w.a1, B, T, w.da1, w.da1T);
    // dWt1 = da1^T se (se as kept by the forward)
    Grp gp;
    if (gr->tw1) gp.mm(w.da1T, B, w.se_in, T, nullptr, gr->tw1, T, T, T, B);
    if (gr->tb1) gp.colsum(w.da1, B, T, T, gr->tb1);
    RC(gp.run(w.slab, w.tmp, s));
  }
  // scatter the stacked gradients
  CopyTable ct{};
  long maxn = 0;
  auto add = [&](const float* src, float* dst, long n) {
    if (!dst) return;
    ct.d[ct.n++] = CopyDesc{src, dst, n};
    maxn = std::max(maxn, n);
  };
  auto flush = [&]() -> int {
    if (!ct.n) return 0;
    hipLaunchKernelGGL(copy_multi_kernel, dim3((unsigned)std::min<long>((maxn + 255) / 256, 1024), (unsigned)ct.n),
                       dim3(256), 0, s, ct);
    ct.n = 0;
    maxn = 0;
    return (int)hipGetLastError();
  };
  for (int b = 0; b < 7; ++b) {
    if (ct.n + 9 > kCopyMax) RC(flush());
    const long di = d->blocks[b].din, dd = d->blocks[b].dout;
    add(w.gWLS[b], gr->wl[b], dd * di);
    add(w.gWLS[b] + dd * di, gr->ws[b], dd * di);
    add(w.gWBG[b], gr->wb[b], dd * dd);
    add(w.gWBG[b] + dd * dd, gr->wg[b], dd * dd);
    add(w.gbD[b], gr->bl[b], dd);
    add(w.gbD[b] + dd, gr->bs[b], dd);
    add(w.gbD[b] + 2 * dd, gr->bg[b], dd);
    add(w.gWC + (long)w.off[b] * E, gr->wctx[b], dd * E);
    add(w.gbC + w.off[b], gr->bctx[b], dd);
  }
  RC(flush());
  return 0;
}

}  // namespace
}  // namespace damc

// ------------------------------------------------------------------ Q.calculate_loss glue (round 5)
namespace damc {
namespace {
// The noising around the denoiser in Q.calculate_loss (workspace/src/diffusion_net.py:633-639), the per-sample logsnr
// input of Diffusion_UnetA.forward (:486-491) and its SinusoidalPosEmb (:447-461; the drop-in's fp64 sin / cos of the
// fp32 angle, src/diffusion_net.py), each op rounded as PyTorch's ROCm kernels round it (no contraction; a division by
// a Python scalar is a multiplication by its fp32 reciprocal): one thread per (sample, column) of max(nz, ntemb)
__global__ void q_noise_glue_kernel(const float* __restrict__ u, const float* __restrict__ z,
                                    const float* __restrict__ eps, int B, int nz, float lmin, float lmax,
                                    const float* __restrict__ freqs, int ntemb, float* __restrict__ logsnr,
                                    float* __restrict__ zt, float* __restrict__ temb) {
  const int W = max(nz, ntemb);
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * W) return;
  const int n = (int)(i / W), j = (int)(i - (long)n * W);
  // logsnr_schedule_fn (diffusion_helper_func.py:41-50)
  const float b = atanf(expf(mul_rn(-0.5f, lmax)));
  const float a = sub_rn(atanf(expf(mul_rn(-0.5f, lmin))), b);
  const float l = mul_rn(-2.0f, logf(tanf(add_rn(mul_rn(a, u[n]), b))));
  if (j == 0 && logsnr) logsnr[n] = l;
  if (j < nz) {  // diffusion_forward (:72-78): zt = z sqrt(sigmoid(l)) + sqrt(sigmoid(-l)) eps
    const float sp = 1.0f / add_rn(1.0f, expf(-l)), sm = 1.0f / add_rn(1.0f, expf(l));
    const long o = (long)n * nz + j;
    zt[o] = add_rn(mul_rn(z[o], sqrtf(sp)), mul_rn(sqrtf(sm), eps[o]));
  }
  const int half = ntemb / 2;
  if (j < half) {  // t_in = arctan(exp(-0.5 clamp(l, -20, 20))) / (pi / 2); x *= 1000 / max_time (max_time 1)
    const float c = fminf(fmaxf(l, -20.0f), 20.0f);
    const float t = mul_rn(mul_rn(atanf(expf(mul_rn(-0.5f, c))), 1.0f / 1.5707963267948966f), 1000.0f);
    const float ang = mul_rn(t, freqs[j]);
    temb[(long)n * ntemb + j] = (float)sin((double)ang);
    temb[(long)n * ntemb + half + j] = (float)cos((double)ang);
  }
}

// loss = 0.5 sum_j (eps - pred)^2 per sample (diffusion_net.py:642), and its gradient w.r.t. pred for an incoming
// dL/dloss g: -((0.5 g) (2 (eps - pred))) as autograd's mul / sum / pow / sub backward rounds it
__global__ void q_loss_fwd_kernel(const float* __restrict__ eps, const float* __restrict__ pred, int B, int nz,
                                  float* __restrict__ loss) {
  const int n = blockIdx.x, lane = threadIdx.x;
  float acc = 0.f;
  for (int j = lane; j < nz; j += 64) {
    const float d = sub_rn(eps[(long)n * nz + j], pred[(long)n * nz + j]);
    acc = add_rn(acc, mul_rn(d, d));
  }
  for (int off = 32; off; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) loss[n] = mul_rn(0.5f, acc);
}
__global__ void q_loss_bwd_kernel(const float* __restrict__ eps, const float* __restrict__ pred,
                                  const float* __restrict__ g, long gstride, int B, int nz, float* __restrict__ gpred) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * nz) return;
  const int n = (int)(i / nz);
  const float d = sub_rn(eps[i], pred[i]);
  gpred[i] = -mul_rn(mul_rn(g[n * gstride], 0.5f), mul_rn(2.0f, d));
}
}  // namespace
}  // namespace damc

extern "C" int damc_q_noise_glue(const float* u, const float* z, const float* eps, int batch, int nz,
                                 float logsnr_min, float logsnr_max, const float* freqs, int ntemb, float* logsnr,
                                 float* zt, float* temb_in, void* stream) {
  if (!u || !z || !eps || !freqs || !zt || !temb_in || batch <= 0 || nz <= 0 || ntemb < 2 || ntemb % 2)
    return DAMC_ERR_ARG;
  const long n = (long)batch * std::max(nz, ntemb);
  hipLaunchKernelGGL(damc::q_noise_glue_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), u,
                     z, eps, batch, nz, logsnr_min, logsnr_max, freqs, ntemb, logsnr, zt, temb_in);
  return (int)hipGetLastError();
}

extern "C" int damc_q_loss_forward(const float* eps, const float* eps_pred, int batch, int nz, float* loss,
                                   void* stream) {
  if (!eps || !eps_pred || !loss || batch <= 0 || nz <= 0) return DAMC_ERR_ARG;
  hipLaunchKernelGGL(damc::q_loss_fwd_kernel, dim3((unsigned)batch), dim3(64), 0, as_stream(stream), eps, eps_pred,
                     batch, nz, loss);
  return (int)hipGetLastError();
}

extern "C" int damc_q_loss_backward(const float* eps, const float* eps_pred, const float* grad_loss,
                                    long grad_stride, int batch, int nz, float* grad_eps_pred, void* stream) {
  if (!eps || !eps_pred || !grad_loss || !grad_eps_pred || batch <= 0 || nz <= 0 || grad_stride < 0)
    return DAMC_ERR_ARG;
  const long n = (long)batch * nz;
  hipLaunchKernelGGL(damc::q_loss_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), eps,
                     eps_pred, grad_loss, grad_stride, batch, nz, grad_eps_pred);
  return (int)hipGetLastError();
}

using damc::DW;

extern "C" size_t damc_denoiser_train_workspace_bytes(const damc_denoiser_train_t* d, int B) {
  if (damc::validate(d) || B <= 0) return 0;
  return damc::carve(d, B, nullptr, nullptr);
}

extern "C" int damc_denoiser_train_forward(const damc_denoiser_train_t* d, const float* zt, const float* temb_in,
                                           const float* xemb, int B, float* eps, void* wsp, size_t wsb,
                                           void* stream) {
  DW w;
  int rc = damc::setup(d, B, wsp, wsb, &w);
  if (rc) return rc;
  if (!zt || !temb_in || !xemb || !eps) return DAMC_ERR_ARG;
  return damc::forward(d, zt, temb_in, xemb, B, eps, w, as_stream(stream));
}

extern "C" int damc_denoiser_train_backward(const damc_denoiser_train_t* d, const float* grad_eps, int B,
                                            const damc_denoiser_grads_t* grads, float* grad_zt, float* grad_xemb,
                                            void* wsp, size_t wsb, void* stream) {
  DW w;
  int rc = damc::setup(d, B, wsp, wsb, &w);
  if (rc) return rc;
  if (!grad_eps || !grads) return DAMC_ERR_ARG;
  return damc::backward(d, grad_eps, B, grads, grad_zt, grad_xemb, w, as_stream(stream));
}
