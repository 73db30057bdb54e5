// encoder_train.hip — Conv2d backward for the encoder of the Q update ("encoder bwd,
// reusing the a10 kernels"; Encoder_* workspace/src/diffusion_net.py:227-413, trained by Q.calculate_loss
// :624-645 six times per iteration, train_gen_recon.py:211-220).  Three shapes cover every encoder:
//   (A) k4 s2 p1 with H = 2 Ho: the input gradient is a ConvTranspose2d k4 s2 p1 forward with the conv's own
//       weight read as a transposed-conv weight (in = Cout, out = Cin), so it runs on the generator's
//       phase-split UP2 path (limb engine when the gathered channel count allows); the weight gradient is
//       the generator's O_WGRAD GEMM with the roles swapped (layer "input" = dy on the Ho x Wo grid, layer
//       "output gradient" = x, phase-split) — its reduce writes the (Cout, Cin, 4, 4) layout directly;
//   (B) the first conv, k3 s1 p1 with Cin <= 4: no input gradient (the image); the weight gradient is the
//       output layer's direct kernel (wgrad.hip) with dy in the "activation" role and x in the "delta" role;
//   (C) the last conv, covering its whole input (p0, output 1x1): a dense layer, two fp32 MFMA GEMMs;
//   (A') k4 s2 p1 with H = 2 Ho + 1 (Encoder_mnist's 7 -> 3): x zero-padded by one row and column and dy by one
//       output row and column turn it into (A) exactly — output rows < Ho read input rows < H only, the extra
//       output row reads the zero row and gets dy = 0, so dW and dx[:H, :W] are unchanged — then dx is cropped.
// Biases: fixed-order column sums of dy.
#include <algorithm>

#include "gemm.h"
#include "wgrad.h"

namespace {

using namespace damc;

enum { CASE_NONE = 0, CASE_UP = 1, CASE_FIRST = 2, CASE_DENSE = 3, CASE_UP_ODD = 4, CASE_UP_CPAD = 5 };

int conv_case(int hin, int win, int cin, int cout, int k, int stride, int pad, int* ho_, int* wo_) {
  const int ho = (hin + 2 * pad - k) / stride + 1, wo = (win + 2 * pad - k) / stride + 1;
  *ho_ = ho;
  *wo_ = wo;
  if (ho <= 0 || wo <= 0) return CASE_NONE;
  if (k == 4 && stride == 2 && pad == 1 && hin == 2 * ho && win == 2 * wo && cin % 8 == 0) return CASE_UP;
  if (k == 4 && stride == 2 && pad == 1 && hin == 2 * ho + 1 && win == 2 * wo + 1 && cin % 8 == 0) return CASE_UP_ODD;
  if (k == 3 && stride == 1 && pad == 1 && cin <= 4) return CASE_FIRST;
  // a k4 s2 p1 conv whose input channels are not a multiple of 8 (Encoder_celebaHQ at nif = 4: 4 -> 8): the CASE_UP
  // path on zero channels padded up to the next multiple of 8, then the crop
  if (k == 4 && stride == 2 && pad == 1 && hin == 2 * ho && win == 2 * wo && cin % 8 != 0) return CASE_UP_CPAD;
  if (pad == 0 && ho == 1 && wo == 1 && k == hin && k == win) return CASE_DENSE;
  return CASE_NONE;
}

// the conv read as ConvTranspose2d k4 s2 p1 (input Cout on Ho x Wo -> output Cin on H x W)
damc_layer_t up_view(int hin, int win, int cin, int cout, int ho, int wo) {
  damc_layer_t L{};
  L.kind = DAMC_LAYER_UP2;
  L.cin = cout;
  L.cout = cin;
  L.k = 4;
  L.stride = 2;
  L.pad = 1;
  L.hin = ho;
  L.win = wo;
  L.hout = hin;
  L.wout = win;
  L.act = DAMC_ACT_NONE;
  return L;
}

// limb-engine capability of the transposed view's forward (gemm.hip launch_gemm_x3 constraints)
bool up_x3(int cin, int cout) { return cout % KM_BK == 0 && cin % 8 == 0; }

int up_split(int ho, int wo, int cin, int cout, int Bp, int* S, int* kper) {
  const long M = 4L * cout, N = cin, K = (long)ho * wo * Bp;
  const long base = ((M + 255) / 256) * ((N + 127) / 128) * 4;
  const long nkt = K / 32;
  // >= 512 workgroups, but at most 16 slices: the fixed-order reduce reads every slice once per output
  const long sl = std::max(1L, std::min(std::min((512 + base - 1) / base, 16L), nkt));
  const long kp = (nkt + sl - 1) / sl * 32;
  *kper = (int)kp;
  *S = (int)((K + kp - 1) / kp);
  return 0;
}

// NHWC (B, H, W, C) -> (B, H2, W2, C) with zeros beyond H x W (H2 >= H, W2 >= W), or the crop back (H2 <= H)
__global__ void pad_crop_kernel(const float* __restrict__ x, int B, int H, int W, int C, float* __restrict__ y, int H2,
                                int W2) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * H2 * W2 * C) return;
  long t = i;
  const int c = (int)(t % C);
  t /= C;
  const int xx = (int)(t % W2);
  t /= W2;
  const int yy = (int)(t % H2);
  const int b = (int)(t / H2);
  y[i] = (yy < H && xx < W) ? x[(((long)b * H + yy) * W + xx) * C + c] : 0.f;
}

int pad_crop(const float* x, int B, int H, int W, int C, float* y, int H2, int W2, hipStream_t s) {
  const long n = (long)B * H2 * W2 * C;
  hipLaunchKernelGGL(pad_crop_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, B, H, W, C, y, H2, W2);
  return (int)hipGetLastError();
}

// per sample b: y[b][j][i] = x[b][i][j] for an R x C matrix (the dense last conv's (tap, ci) <-> (ci, tap) orders);
// one thread per output element, outputs contiguous
__global__ void batch_transpose_kernel(const float* __restrict__ x, int nb, int R, int C, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)R * C;
  if (i >= nb * per) return;
  const long b = i / per;
  const int o = (int)(i - b * per), j = o / R, r = o - j * R;
  y[i] = x[b * per + (long)r * C + j];
}

// (n, c) -> (c, n)
__global__ void transpose_kernel(const float* __restrict__ x, int R, int C, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)R * C) return;
  const int r = (int)(i / C), c = (int)(i - (long)r * C);
  y[(long)c * R + r] = x[i];
}

struct Carve {
  char* base;
  size_t off = 0;
  explicit Carve(char* b) : base(b) {}
  template <class T>
  T* take(size_t n) {
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += (n * sizeof(T) + 255) / 256 * 256;
    return p;
  }
};

struct Bufs {
  float *wf = nullptr, *wb = nullptr, *tmp = nullptr, *slab = nullptr, *g = nullptr, *dyT = nullptr, *wk = nullptr;
  unsigned short *dy3 = nullptr, *tin = nullptr, *tdl = nullptr;
  float* part = nullptr;
  float *xp = nullptr, *dyp = nullptr, *dxp = nullptr;  // CASE_UP_ODD: padded x, dy and dx
  float *wc = nullptr, *dwc = nullptr;                   // CASE_UP_CPAD: channel-padded weight and its gradient
};

inline int cpad8(int c) { return (c + 7) / 8 * 8; }

// NHWC channel pad / crop: y (rows, C2) from x (rows, C1), zero past C1
__global__ void chan_pad_kernel(const float* __restrict__ x, long rows, int C1, int C2, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * C2) return;
  const long r = i / C2;
  const int c = (int)(i - r * C2);
  y[i] = c < C1 ? x[r * C1 + c] : 0.f;
}
// conv weight (cout, C1, k, k) <-> (cout, C2, k, k), zero past C1
__global__ void wchan_pad_kernel(const float* __restrict__ w, int cout, int C1, int C2, int kk, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)cout * C2 * kk) return;
  const int t = (int)(i % kk);
  const long r = i / kk;
  const int c = (int)(r % C2), co = (int)(r / C2);
  y[i] = c < C1 ? w[((long)co * C1 + c) * kk + t] : 0.f;
}
int chan_pad(const float* x, long rows, int C1, int C2, float* y, hipStream_t s) {
  const long n = rows * C2;
  hipLaunchKernelGGL(chan_pad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, rows, C1, C2, y);
  return (int)hipGetLastError();
}
int wchan_pad(const float* w, int cout, int C1, int C2, int kk, float* y, hipStream_t s) {
  const long n = (long)cout * C2 * kk;
  hipLaunchKernelGGL(wchan_pad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, cout, C1, C2, kk, y);
  return (int)hipGetLastError();
}

void carve_up(Carve& cv, int B, int ho, int wo, int cin, int cout, Bufs& t) {
  const long M = (long)B * ho * wo;
  const int Bp = (B + 31) / 32 * 32;
  const long P = (long)ho * wo;
  const size_t n = (size_t)cin * cout * 16;
  t.wf = cv.take<float>(n + n * 3 / 2);  // fp32 packing + its x3 copy (damc_pack_generator_layer layout)
  t.wb = cv.take<float>(n + n * 3 / 2);
  t.dy3 = cv.take<unsigned short>((size_t)M * cout * 3);
  t.tin = cv.take<unsigned short>((size_t)cout * P * Bp * 3);
  t.tdl = cv.take<unsigned short>((size_t)4 * cin * P * Bp * 3);
  int S, kp;
  up_split(ho, wo, cin, cout, Bp, &S, &kp);
  t.slab = cv.take<float>((size_t)4 * S * 4 * cout * cin);
}

size_t carve(int B, int hin, int win, int cin, int cout, int k, int stride, int pad, char* base, Bufs* b, int* cs) {
  int ho, wo;
  const int c = conv_case(hin, win, cin, cout, k, stride, pad, &ho, &wo);
  *cs = c;
  Carve cv(base);
  Bufs t;
  const long M = (long)B * ho * wo;
  t.tmp = cv.take<float>(std::max<size_t>(colsum_tmp_floats(M, cout), 1));
  if (c == CASE_UP) {
    carve_up(cv, B, ho, wo, cin, cout, t);
  } else if (c == CASE_UP_ODD) {
    t.xp = cv.take<float>((size_t)B * (hin + 1) * (win + 1) * cin);
    t.dxp = cv.take<float>((size_t)B * (hin + 1) * (win + 1) * cin);
    t.dyp = cv.take<float>((size_t)B * (ho + 1) * (wo + 1) * cout);
    carve_up(cv, B, ho + 1, wo + 1, cin, cout, t);
  } else if (c == CASE_UP_CPAD) {
    const int cp = cpad8(cin);
    t.xp = cv.take<float>((size_t)B * hin * win * cp);
    t.dxp = cv.take<float>((size_t)B * hin * win * cp);
    t.wc = cv.take<float>((size_t)cout * cp * 16);
    t.dwc = cv.take<float>((size_t)cout * cp * 16);
    carve_up(cv, B, ho, wo, cp, cout, t);
  } else if (c == CASE_FIRST) {
    damc_layer_t L = up_view(hin, win, cin, cout, ho, wo);
    L.kind = DAMC_LAYER_SMALLC;
    L.cin = cout;
    L.cout = cin;
    L.k = 3;
    L.stride = 1;
    L.pad = 1;
    t.part = cv.take<float>(smallc_wgrad_part_floats(L, B));
    t.tmp = cv.take<float>(std::max(smallc_wgrad_tmp_floats(L, B), colsum_tmp_floats(M, cout)));
  } else if (c == CASE_DENSE) {
    const long KK = (long)k * k * cin;
    t.dyT = cv.take<float>((size_t)cout * B);
    t.g = cv.take<float>((size_t)B * KK);   // x in (ci, ky, kx) order per sample
    t.wk = cv.take<float>((size_t)B * KK);  // dx in (ci, ky, kx) order per sample
  }
  if (b) *b = t;
  return c == CASE_NONE ? 0 : cv.off;
}

// (A): dW by O_WGRAD with the transposed view's roles, dx by the transposed view's phase-split forward
int backward_up(const float* x, const float* dy, const float* w, int B, int hin, int win, int cin, int cout, int ho,
                int wo, float* dx, float* dw, const Bufs& t, hipStream_t s, void* stream) {
  const long M = (long)B * ho * wo;
  int rc;
  const int Bp = (B + 31) / 32 * 32;
  const long P = (long)ho * wo;
  damc_layer_t L = up_view(hin, win, cin, cout, ho, wo);
  // weight gradient: O_WGRAD with the transposed view's roles (input = dy, output gradient = x)
  if ((rc = launch_transpose_x3(dy, nullptr, B, ho, wo, cout, ho, wo, 1, 1, 0, 0, Bp, t.tin, nullptr, s))) return rc;
  if ((rc = launch_transpose_x3_4ph(x, nullptr, B, hin, win, cin, ho, wo, Bp, t.tdl, (long)cin * P * Bp * 3, nullptr,
                                    0, s)))
    return rc;
  {
    int S, kp;
    up_split(ho, wo, cin, cout, Bp, &S, &kp);
    GemmArgs a;
    a.A3 = t.tin;
    a.B3 = t.tdl;
    a.Cg = cout;
    a.Hin = ho;
    a.Win = wo;
    a.K = (int)(P * Bp);
    a.wg_bp = Bp;
    a.kw = 2;
    a.wg_phases = 4;
    a.M = 4 * cout;
    a.N = cin;
    a.ldc = cin;
    a.c_zstride = (long)a.M * a.N;
    a.b_zstride = (long)cin * a.K;
    a.k_per_z = kp;
    a.C = t.slab;
    if ((rc = launch_wgrad_x3(a, S, "enc_wgrad", 2.0 * M * cout * cin * 16, s))) return rc;
    if ((rc = launch_up2_wgrad_reduce(t.slab, S, cout, cin, dw, s))) return rc;
  }
  if (!dx) return 0;
  // input gradient: the transposed view's forward (phase-split implicit GEMM) over dy
  L.w_fwd = t.wf;
  L.w_bwd = t.wb;
  if ((rc = damc_pack_generator_layer(&L, w, t.wf, t.wb, stream))) return rc;
  const size_t n = (size_t)cin * cout * 16;
  GemmArgs a;
  a.A = dy;
  a.Hin = ho;
  a.Win = wo;
  a.Cg = cout;
  a.Hq = ho;
  a.Wq = wo;
  a.kw = 2;
  a.stride = 1;
  a.B = t.wf;
  a.b_kmajor = conv_kmajor_ok(cout);
  a.ldb = a.b_kmajor ? 4L * cout : cin;
  a.b_zstride = 4L * cout * cin;
  a.C = dx;
  a.ldc = cin;
  a.M = (int)M;
  a.N = cin;
  a.K = 4 * cout;
  a.Hout = hin;
  a.Wout = win;
  a.act = DAMC_ACT_NONE;
  if (up_x3(cin, cout)) {
    // dy staged as fp32 and split into limbs in registers (gemm.hip X3_F32A; bitwise the limb copy, no split launch);
    // DAMC_ENC_BWD_F32A=0 (read per call) gathers the limbs of launch_split_x3
    const char* ef = getenv("DAMC_ENC_BWD_F32A");
    if (!(ef && ef[0] == '0')) {
      a.a_f32 = 1;
    } else {
      if ((rc = launch_split_x3(dy, M * cout, t.dy3, s))) return rc;
      a.A3 = t.dy3;
    }
    a.B3 = reinterpret_cast<const unsigned short*>(t.wf + n);
    a.b_negblk = 1;  // damc_pack_generator_layer's x3 copy (up_view(...)'s forward sign block: generator.hip up2_negk_fwd)
    a.negk = x3_conv_negk((long)ho * wo, cin, 4 * cout, 4);
  }
  return launch_gemm(a, A_CONV, EPI_BIAS_ACT, O_PHASE, 4, "enc_dgrad", 2.0 * M * cout * cin * 16, s);
}

}  // namespace

extern "C" size_t damc_conv2d_backward_workspace_bytes(int B, int hin, int win, int cin, int cout, int k, int stride,
                                                       int pad) {
  if (B <= 0 || hin <= 0 || win <= 0 || cin <= 0 || cout <= 0 || k <= 0 || stride <= 0) return 0;
  int cs;
  return carve(B, hin, win, cin, cout, k, stride, pad, nullptr, nullptr, &cs);
}

// x NHWC (B, hin, win, cin), dy NHWC (B, ho, wo, cout), w PyTorch (cout, cin, k, k) -> dx NHWC (optional),
// dw (cout, cin, k, k), db (cout) (optional)
extern "C" int damc_conv2d_backward_nhwc(const float* x, const float* dy, const float* w, int B, int hin, int win,
                                         int cin, int cout, int k, int stride, int pad, float* dx, float* dw,
                                         float* db, void* wsp, size_t wsb, void* stream) {
  if (!x || !dy || !w || !dw || B <= 0) return DAMC_ERR_ARG;
  int cs;
  const size_t need = carve(B, hin, win, cin, cout, k, stride, pad, nullptr, nullptr, &cs);
  if (cs == CASE_NONE) return DAMC_ERR_UNSUPPORTED;
  if (!wsp || wsb < need) return DAMC_ERR_WORKSPACE;
  Bufs t;
  carve(B, hin, win, cin, cout, k, stride, pad, reinterpret_cast<char*>(wsp), &t, &cs);
  hipStream_t s = as_stream(stream);
  const int ho = (hin + 2 * pad - k) / stride + 1, wo = (win + 2 * pad - k) / stride + 1;
  const long M = (long)B * ho * wo;
  int rc;
  if (db && (rc = launch_colsum(dy, M, cout, cout, db, t.tmp, s))) return rc;
  if (cs == CASE_FIRST) {
    if (dx) return DAMC_ERR_UNSUPPORTED;  // the image needs no gradient
    damc_layer_t L{};
    L.kind = DAMC_LAYER_SMALLC;
    L.cin = cout;  // dy plays the activation (channels across threads) ...
    L.cout = cin;  // ... and x the small-channel "delta" window
    L.k = 3;
    L.stride = 1;
    L.pad = 1;
    L.hin = ho;
    L.win = wo;
    L.hout = hin;
    L.wout = win;
    return launch_smallc_wgrad(L, dy, x, B, t.part, t.tmp, dw, s);
  }
  if (cs == CASE_DENSE) {
    // round 5: both products run in PyTorch's (ci, ky, kx) weight order, so neither the 8.4 M-weight gradient nor the
    // weight itself is permuted (33.5 MB each way for Encoder_cifar10's last conv, 26 + 33 us); the B x k*k*cin
    // input and input gradient are transposed per sample instead (4 MB at B = 128)
    const int KK = k * k * cin, T = k * k;
    const long nx = (long)B * KK;
    // dW (co, (ci,ky,kx)) = dy^T X', X' = the NHWC input per sample in (ci, ky, kx) order
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)(((long)B * cout + 255) / 256)), dim3(256), 0, s, dy, B, cout,
                       t.dyT);
    hipLaunchKernelGGL(batch_transpose_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, s, x, B, T, cin, t.g);
    GemmArgs a;
    a.A = t.dyT;
    a.lda = B;
    a.B = t.g;
    a.ldb = KK;
    a.C = dw;
    a.ldc = KK;
    a.M = cout;
    a.N = KK;
    a.K = B;
    a.k_per_z = B;
    // the small-GEMM kernel (one 16 x 16 tile per wave: 32K waves here instead of the tiled engine's 512 workgroups
    // with K = B = 128 each), the tiled engine where it does not apply
    rc = launch_small_gemm(a.A, a.lda, a.B, a.ldb, nullptr, a.C, a.ldc, a.M, a.N, a.K, s);
    if (rc == DAMC_ERR_UNSUPPORTED) rc = launch_gemm(a, A_DENSE, EPI_STORE, O_DENSE, 1, "enc_wgrad", 2.0 * cout * KK * B, s);
    if (rc) return rc;
    if (dx) {  // dX' = dy W with W (co, (ci,ky,kx)) as stored, then back to NHWC per sample
      GemmArgs d;
      d.A = dy;
      d.lda = cout;
      d.B = w;
      d.ldb = KK;
      d.C = t.wk;
      d.ldc = KK;
      d.M = B;
      d.N = KK;
      d.K = cout;
      d.k_per_z = cout;
      rc = launch_small_gemm(d.A, d.lda, d.B, d.ldb, nullptr, d.C, d.ldc, d.M, d.N, d.K, s);
      if (rc == DAMC_ERR_UNSUPPORTED) rc = launch_gemm(d, A_DENSE, EPI_STORE, O_DENSE, 1, "enc_dgrad", 2.0 * B * KK * cout, s);
      if (rc) return rc;
      hipLaunchKernelGGL(batch_transpose_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, s,
                         (const float*)t.wk, B, cin, T, dx);
    }
    return (int)hipGetLastError();
  }
  if (cs == CASE_UP) return backward_up(x, dy, w, B, hin, win, cin, cout, ho, wo, dx, dw, t, s, stream);
  if (cs == CASE_UP_CPAD) {  // CASE_UP on channels padded with zeros to a multiple of 8, then the crops
    const int cp = cpad8(cin);
    const long rows = (long)B * hin * win;
    if ((rc = chan_pad(x, rows, cin, cp, t.xp, s))) return rc;
    if ((rc = wchan_pad(w, cout, cin, cp, 16, t.wc, s))) return rc;
    if ((rc = backward_up(t.xp, dy, t.wc, B, hin, win, cp, cout, ho, wo, dx ? t.dxp : nullptr, t.dwc, t, s, stream)))
      return rc;
    if ((rc = wchan_pad(t.dwc, cout, cp, cin, 16, dw, s))) return rc;  // (cout, cp, 4, 4) -> (cout, cin, 4, 4)
    return dx ? chan_pad(t.dxp, rows, cp, cin, dx, s) : 0;
  }
  // CASE_UP_ODD: (A) on the padded tensors, then the crop
  if ((rc = pad_crop(x, B, hin, win, cin, t.xp, hin + 1, win + 1, s))) return rc;
  if ((rc = pad_crop(dy, B, ho, wo, cout, t.dyp, ho + 1, wo + 1, s))) return rc;
  if ((rc = backward_up(t.xp, t.dyp, w, B, hin + 1, win + 1, cin, cout, ho + 1, wo + 1, dx ? t.dxp : nullptr, dw, t, s,
                        stream)))
    return rc;
  return dx ? pad_crop(t.dxp, B, hin + 1, win + 1, cin, dx, hin, win, s) : 0;
}

// ---------------------------------------------------------------------------------------------------------------
// The whole encoder of the Q update in two calls (round 5): damc_encoder_train_forward runs every stage the way
// damc.training's per-stage loop did (conv on the limb engine or the fp32 engine, InstanceNorm + LeakyReLU keeping
// the conv output and the statistics), damc_encoder_train_backward every stage's InstanceNorm and Conv2d backward;
// the host issues one call each way instead of ~4 per stage (the Q update is host-bound).
namespace {
struct EncTrainPlan {
  int n, H[DAMC_MAX_ENC_LAYERS + 1], W[DAMC_MAX_ENC_LAYERS + 1];
  bool limb[DAMC_MAX_ENC_LAYERS], head[DAMC_MAX_ENC_LAYERS];
  size_t nbx[DAMC_MAX_ENC_LAYERS], wbytes[DAMC_MAX_ENC_LAYERS], convws[DAMC_MAX_ENC_LAYERS];
  size_t inws[DAMC_MAX_ENC_LAYERS], inbws[DAMC_MAX_ENC_LAYERS], cbws[DAMC_MAX_ENC_LAYERS];
  long x_off, y_off[DAMC_MAX_ENC_LAYERS], st_off[DAMC_MAX_ENC_LAYERS], out_off[DAMC_MAX_ENC_LAYERS];
  size_t saved_floats;
  // workspace regions (bytes)
  size_t w_at, conv_at, in_at, inb_at, cb_at, bufa_at, bufb_at, ws_bytes;
};

inline size_t up256(size_t b) { return (b + 255) / 256 * 256; }

// 0 = supported (p filled), else a DAMC error code
int enc_train_plan(const damc_encoder_t* e, int B, EncTrainPlan* p) {
  if (!e || B <= 0 || e->n_layers < 1 || e->n_layers > DAMC_MAX_ENC_LAYERS || e->nc <= 0 || e->h <= 0 || e->w <= 0)
    return DAMC_ERR_ARG;
  p->n = e->n_layers;
  p->H[0] = e->h;
  p->W[0] = e->w;
  long off = 0;
  auto take = [&](long floats) {
    const long o = off;
    off += (floats + 63) / 64 * 64;  // 256-B aligned views
    return o;
  };
  p->x_off = take((long)B * e->h * e->w * e->nc);
  size_t wmax = 0, cmax = 0, imax = 0, ibmax = 0, cbmax = 0, amax = 0;
  int cin_expect = e->nc;
  for (int i = 0; i < p->n; ++i) {
    const damc_enc_layer_t& L = e->layers[i];
    if (L.cin != cin_expect || L.cout <= 0 || L.k <= 0 || L.stride <= 0 || !L.w_src) return DAMC_ERR_ARG;
    const bool norm = L.in_gamma != nullptr;
    if (norm != (i + 1 < p->n) || (norm && !L.in_beta) || !L.bias) return DAMC_ERR_UNSUPPORTED;
    const int hin = p->H[i], win = p->W[i];
    const int ho = (hin + 2 * L.pad - L.k) / L.stride + 1, wo = (win + 2 * L.pad - L.k) / L.stride + 1;
    if (ho <= 0 || wo <= 0) return DAMC_ERR_ARG;
    p->H[i + 1] = ho;
    p->W[i + 1] = wo;
    p->nbx[i] = e->engine == DAMC_ENGINE_LIMB
                    ? damc_conv2d_x3_workspace_bytes(B, hin, win, L.cin, L.cout, L.k, L.stride, L.pad)
                    : 0;
    p->limb[i] = p->nbx[i] > 0;
    if (p->limb[i]) {
      p->wbytes[i] = damc_conv2d_x3_bytes(L.cout, L.cin, L.k);
      p->convws[i] = p->nbx[i];
    } else {
      p->wbytes[i] = (size_t)L.cout * L.cin * L.k * L.k * sizeof(float);
      p->convws[i] = damc_conv2d_workspace_floats(B, hin, win, L.cin, L.cout, L.k, L.stride, L.pad) * sizeof(float);
    }
    // the dense head (launch_dense_head_x3) for a last conv covering its input; its slabs in the conv workspace
    const long KH = (long)L.cin * L.k * L.k;
    p->head[i] = p->limb[i] && !norm && L.pad == 0 && ho == 1 && wo == 1 && L.k == hin && L.k == win &&
                 L.cout % 64 == 0 && KH % 512 == 0 && (uintptr_t)L.w_src % 16 == 0;
    if (p->head[i]) p->convws[i] = std::max(p->convws[i], (size_t)(KH / 512) * B * L.cout * sizeof(float));
    p->cbws[i] = damc_conv2d_backward_workspace_bytes(B, hin, win, L.cin, L.cout, L.k, L.stride, L.pad);
    if (p->cbws[i] == 0) return DAMC_ERR_UNSUPPORTED;
    const long act = (long)B * ho * wo * L.cout;
    if (norm) {
      p->inws[i] = damc_instnorm_workspace_floats(B, ho * wo, L.cout) * sizeof(float);
      p->inbws[i] = damc_instnorm_bwd_workspace_floats(B, ho * wo, L.cout) * sizeof(float);
      p->y_off[i] = take(act);
      p->st_off[i] = take(2L * B * L.cout);
      p->out_off[i] = take(act);
    } else {
      p->inws[i] = p->inbws[i] = 0;
      p->y_off[i] = p->st_off[i] = p->out_off[i] = -1;
      if (ho != 1 || wo != 1) return DAMC_ERR_UNSUPPORTED;  // xemb = the last conv's (B, cout) output
    }
    wmax = std::max(wmax, p->wbytes[i]);
    cmax = std::max(cmax, p->convws[i]);
    imax = std::max(imax, p->inws[i]);
    ibmax = std::max(ibmax, p->inbws[i]);
    cbmax = std::max(cbmax, p->cbws[i]);
    amax = std::max(amax, (size_t)act);
    amax = std::max(amax, (size_t)B * hin * win * L.cin);
    cin_expect = L.cout;
  }
  p->saved_floats = (size_t)off;
  size_t w = 0;
  p->w_at = w;
  w += up256(wmax);
  p->conv_at = w;
  w += up256(cmax);
  p->in_at = w;
  w += up256(imax);
  p->inb_at = w;
  w += up256(ibmax);
  p->cb_at = w;
  w += up256(cbmax);
  p->bufa_at = w;
  w += up256(amax * sizeof(float));
  p->bufb_at = w;
  w += up256(amax * sizeof(float));
  p->ws_bytes = std::max<size_t>(w, 256);
  return 0;
}
}  // namespace

extern "C" size_t damc_encoder_train_saved_floats(const damc_encoder_t* e, int B) {
  EncTrainPlan p;
  return enc_train_plan(e, B, &p) ? 0 : p.saved_floats;
}

extern "C" size_t damc_encoder_train_workspace_bytes(const damc_encoder_t* e, int B) {
  EncTrainPlan p;
  return enc_train_plan(e, B, &p) ? 0 : p.ws_bytes;
}

extern "C" int damc_encoder_train_forward(const damc_encoder_t* e, const float* x, int B, float* saved, float* xemb,
                                          void* workspace, size_t workspace_bytes, void* stream) {
  EncTrainPlan p;
  int rc = enc_train_plan(e, B, &p);
  if (rc) return rc;
  if (!x || !saved || !xemb) return DAMC_ERR_ARG;
  if (!workspace || workspace_bytes < p.ws_bytes) return DAMC_ERR_WORKSPACE;
  char* ws = static_cast<char*>(workspace);
  float* h = saved + p.x_off;
  const char* hde = getenv("DAMC_ENC_HEAD");  // (read per call) 0: the last conv on the limb GEMM, as in the stage calls
  const bool head_on = !(hde && hde[0] == '0');
  if ((rc = damc_nchw_to_nhwc(x, B, e->nc, e->h * e->w, h, stream))) return rc;
  for (int i = 0; i < p.n; ++i) {
    const damc_enc_layer_t& L = e->layers[i];
    const int hin = p.H[i], win = p.W[i], ho = p.H[i + 1], wo = p.W[i + 1];
    const bool norm = L.in_gamma != nullptr;
    float* y = norm ? saved + p.y_off[i] : xemb;
    if (p.head[i] && head_on && (uintptr_t)xemb % 16 == 0) {
      // the last conv as the inference encoder's dense head (no limb copy of the weight): the NHWC input (kept for the
      // backward) per sample to (ci, ky, kx) order in bufa, then the head's two launches
      const int T = L.k * L.k, K = T * L.cin;
      float* a = reinterpret_cast<float*>(ws + p.bufa_at);
      const long nx = (long)B * K;
      hipLaunchKernelGGL(batch_transpose_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, as_stream(stream), h,
                         B, T, L.cin, a);
      rc = launch_dense_head_x3(a, L.w_src, L.bias, B, L.cout, K, reinterpret_cast<float*>(ws + p.conv_at),
                                p.convws[i] / sizeof(float), xemb, as_stream(stream));
    } else if (p.limb[i]) {
      if ((rc = damc_pack_conv2d_x3(L.w_src, L.cout, L.cin, L.k, ws + p.w_at, stream))) return rc;
      rc = damc_conv2d_x3_nhwc(h, B, hin, win, L.cin, ws + p.w_at, L.bias, L.cout, L.k, L.stride, L.pad, y,
                               ws + p.conv_at, p.convws[i], stream);
    } else {
      float* wp = reinterpret_cast<float*>(ws + p.w_at);
      if ((rc = damc_pack_conv2d(L.w_src, L.cout, L.cin, L.k, wp, stream))) return rc;
      rc = damc_conv2d_nhwc(h, B, hin, win, L.cin, wp, L.bias, L.cout, L.k, L.stride, L.pad, y,
                            reinterpret_cast<float*>(ws + p.conv_at), p.convws[i] / sizeof(float), stream);
    }
    if (rc) return rc;
    if (!norm) break;
    float* out = saved + p.out_off[i];
    if ((rc = damc_instnorm_lrelu_train_nhwc(y, B, ho * wo, L.cout, L.in_gamma, L.in_beta, L.in_eps, L.slope, out,
                                             saved + p.st_off[i], reinterpret_cast<float*>(ws + p.in_at), stream)))
      return rc;
    h = out;
  }
  return 0;
}

extern "C" int damc_encoder_train_backward(const damc_encoder_t* e, const float* saved, const float* grad_xemb, int B,
                                           const damc_encoder_grads_t* g, void* workspace, size_t workspace_bytes,
                                           void* stream) {
  EncTrainPlan p;
  int rc = enc_train_plan(e, B, &p);
  if (rc) return rc;
  if (!saved || !grad_xemb || !g) return DAMC_ERR_ARG;
  if (!workspace || workspace_bytes < p.ws_bytes) return DAMC_ERR_WORKSPACE;
  char* ws = static_cast<char*>(workspace);
  float* bufa = reinterpret_cast<float*>(ws + p.bufa_at);
  float* bufb = reinterpret_cast<float*>(ws + p.bufb_at);
  const float* dh = grad_xemb;
  for (int i = p.n - 1; i >= 0; --i) {
    const damc_enc_layer_t& L = e->layers[i];
    const int hin = p.H[i], win = p.W[i], ho = p.H[i + 1], wo = p.W[i + 1];
    const float* dy = dh;
    if (L.in_gamma) {
      if ((rc = damc_instnorm_lrelu_backward_nhwc(saved + p.y_off[i], saved + p.st_off[i], dh, B, ho * wo, L.cout,
                                                  L.in_gamma, L.in_beta, L.slope, bufa, g->gamma[i], g->beta[i],
                                                  reinterpret_cast<float*>(ws + p.inb_at), stream)))
        return rc;
      dy = bufa;
    }
    const float* hin_p = i == 0 ? saved + p.x_off : saved + p.out_off[i - 1];
    float* dw = g->w[i] ? g->w[i] : reinterpret_cast<float*>(ws + p.w_at);  // dw is required by the conv backward
    if (!g->w[i] && p.wbytes[i] < (size_t)L.cout * L.cin * L.k * L.k * sizeof(float)) return DAMC_ERR_WORKSPACE;
    if ((rc = damc_conv2d_backward_nhwc(hin_p, dy, L.w_src, B, hin, win, L.cin, L.cout, L.k, L.stride, L.pad,
                                        i > 0 ? bufb : nullptr, dw, g->b[i], ws + p.cb_at, p.cbws[i], stream)))
      return rc;
    dh = bufb;
  }
  return 0;
}
