// gemm.h — host interface of the fp32 MFMA implicit-GEMM engine (gemm.hip).
#pragma once
#include <cstdlib>
#include "common.h"

namespace damc {

enum AMode { A_DENSE = 0, A_CONV = 1, A_CONV_SCALAR = 2 };
enum Epi { EPI_STORE = 0, EPI_BIAS_ACT = 1, EPI_MASK = 2, EPI_RESID = 3, EPI_GATE = 4 };
enum OMode { O_DENSE = 0, O_PHASE = 1, O_WGRAD = 2 };

// C[M,N] (+)= A[M,K] · B[K,N], K reduced in fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 fmaf chains).
//   A_DENSE       : A[m*lda + k]
//   A_CONV(_SCALAR): A = NHWC tensor X[B][Hin][Win][Cg]; m -> (b, qy, qx) on an Hq x Wq grid,
//                   k -> (ky, kx, ci) with ci fastest; value X[b][qy*stride-pad_y+ky][qx*stride-pad_x+kx][ci]
//   O_PHASE       : blockIdx.z = output phase (py,px) of a k4 s2 p1 transposed conv; the GEMM is the
//                   2x2 conv with pad (1-py, 1-px) and row m = (b,qy,qx) is stored at output pixel
//                   (b, 2qy+py, 2qx+px) of a Hout x Wout NHWC map; B advanced by z*b_zstride
//   O_DENSE       : blockIdx.z = split-K slice: k in [z*k_per_z, (z+1)*k_per_z), C advanced by z*c_zstride
//   O_WGRAD       : (limb engine only) weight gradient of a generator layer over pixel-major transposed
//                   operands (wgrad.hip): A = x3 [Cg][K] input channels, K = (qy, qx, n) with n fastest over
//                   wg_bp (a multiple of 32) samples; GEMM row m = (tap, ci) with tap = (ty, tx) on a kw x kw
//                   grid reads A row ci shifted by (ty - pad_y, tx - pad_x) pixels (zero outside the
//                   Hin x Win grid); B = x3 [N][K] (per phase: + ph * b_zstride).  blockIdx.z = phase *
//                   slices + split-K slice; wg_phases = 4 (k4 s2 p1 ConvT, pad = 1 - phase) or 1 (no
//                   shift); C advanced by z * c_zstride (EPI_STORE only)
//   b_kmajor      : B is stored transposed, Bt[n*ldb + k] (k contiguous).  Only the K-major convolution
//                   engine reads this layout: A_CONV with conv_kmajor_ok(Cg), no split-K.
// default k per sign block of the limb engine (GemmArgs::negk; the encoder, the weight gradients and every layer
// whose generator.hip up2_negk rule does not pick 1024)
#ifndef DAMC_X3_NEGK
#define DAMC_X3_NEGK 512
#endif
constexpr int X3_NEGK = DAMC_X3_NEGK;

struct GemmArgs {
  const float* A = nullptr;
  long lda = 0;
  int Hin = 1, Win = 1, Cg = 1, Hq = 1, Wq = 1, kw = 1, stride = 1, pad_y = 0, pad_x = 0;
  const float* B = nullptr;
  long ldb = 0;
  long b_zstride = 0;
  float* C = nullptr;
  long ldc = 0;
  long c_zstride = 0;
  int M = 0, N = 0, K = 0, k_per_z = 0;
  const float* bias = nullptr;
  int bias_mod = 1;
  int act = DAMC_ACT_NONE;
  float slope = 0.f;
  const float* mask = nullptr;  // EPI_MASK: post-activation at the same output index
  int mask_act = DAMC_ACT_LRELU;
  float mask_slope = 0.2f;
  const float* xres = nullptr;  // EPI_RESID: target (row-major like C)
  float inv_s2 = 1.f;
  float* xhat = nullptr;
  float* sqerr = nullptr;       // EPI_RESID: accumulates |t - x|^2 * inv_s2 / 2 (diagnostics)
  int Hout = 1, Wout = 1;
  int b_kmajor = 0;
  // limb engine (gemm_x3_kernel): A and B as x3 bf16 limb tensors (see gemm.hip); when A3 is set the
  // fp32 A / B pointers are not read
  const unsigned short* A3 = nullptr;
  const unsigned short* B3 = nullptr;
  // limb engine output: an x3 copy of the epilogue result (C may then be null: fp32 not stored)
  unsigned short* C3 = nullptr;
  // limb engine: sign bits of the epilogue result (bit e of byte idx/8 = out[idx + e] > 0), and for
  // EPI_MASK the LReLU' mask read from such bits instead of from the fp32 `mask`
  unsigned char* sgn = nullptr;
  const unsigned char* mask_sgn = nullptr;
  // O_WGRAD geometry (see above)
  int wg_phases = 1, wg_bp = 0;
  // EPI_GATE: v + bias[n], then sigmoid on the columns n < gate_cols (a ConcatSquash block's hyper gate and
  // hyper bias computed by one GEMM, diffusion_net.py:441-443)
  int gate_cols = 0;
  // limb engine: B3 holds -B on the odd blocks of negk consecutive k of every row (launch_split_x3_negblk),
  // and the kernel subtracts those blocks' sums (the MFMA's truncation bias then alternates sign; gemm.hip)
  int b_negblk = 0;
  // limb engine: k per sign block = per MFMA accumulation block = per split-K slab (a power of two >= 32); the
  // packer of B3 and every launch reading it use the same value (generator.hip up2_negk: 512 or 1024 per layer)
  int negk = X3_NEGK;
  // x3_skinny_kernel: the B operand as fp32 rows [N][K] (k contiguous), split into the B3 limbs in registers (the RNE
  // split of the packer: bitwise the B3 operand, 2/3 of its bytes); null: B3 is read
  const float* b32k = nullptr;
  // limb engine: the A operand is the fp32 tensor A (NHWC), staged as fp32 and split into limbs in registers
  // (gemm_x3_kernel variant X3_F32A: 4 B per gathered element instead of 6 B of limbs); A3 unused
  int a_f32 = 0;
  // host pointer (EPI_BIAS_ACT, O_DENSE, no C3 / sgn): when set and the launch splits K into register-layout slabs
  // (kslab_reg), the reduce is skipped and the slab count is written here for a consumer that sums the slabs itself
  // (the encoder's InstanceNorm; slab layout: gemm.hip x3_ksplit_reduce_tile_kernel); 0 = the launcher reduced or did
  // not split, C holds the result
  int* ksplit_deferred = nullptr;
  // clock probe (damc_clock_probe; diagnostics, off in timed work): thread 0 of each workgroup stores {s_memtime,
  // s_memrealtime} before its K loop and after it, at clk[4 * (workgroup % clk_n)]
  unsigned long long* clk = nullptr;
  int clk_n = 0;
  // fused output-layer projection (O_PHASE, EPI_BIAS_ACT, N <= 256): after the epilogue, every output pixel's
  // activated row h (N channels) is projected on the next layer's packed weights, proj_out[pixel][n] =
  // sum_c h[c] proj_w[n][c] for n < proj_np (launch_proj_rows has the same arithmetic); proj_nostore: h itself
  // (C) is not written (set by the launcher only where the projection ran in this kernel)
  const float* proj_w = nullptr;
  float* proj_out = nullptr;
  int proj_np = 0, proj_ldw = 0, proj_nostore = 0;
  // one chain per 128-channel chunk (gemm.hip PROJ_CHUNK), chunk j into proj_out + j * proj_pstride (floats; the whole
  // batch's npix * proj_np); the gather adds the partials in order
  long proj_pstride = 0;
  // limb engine, O_PHASE / O_DENSE: split-K over ksplit slices of k_per_z (a multiple of X3_NEGK) when the grid
  // would under-fill the chip; the slices' fp32 tiles go to kslab [zdim * ksplit][M][N] and a fixed-order reduce
  // applies the epilogue.  kslab = scratch the caller owns (kslab_floats of it); null: never split
  int ksplit = 1;
  float* kslab = nullptr;
  long kslab_floats = 0;
  // split-K: sign blocks per workgroup (each block's sum still goes to its own slab; ksplit / kbpw workgroups along
  // K), so a small batch fills the chip without paying a prologue and epilogue per 256 k
  int kbpw = 1;
  // split-K slab layout: 0 row-major [M][N] per block; 1 the 256 x 128 kernel's register layout, per block
  // [tile][wave][4 x 4 tiles][64 lanes] f32x4 (16-B stores straight from the accumulators; the reduce maps back)
  int kslab_reg = 0;
  // split-K in-GEMM ordered fix-up (gemm.hip X3_FIXUP; register-layout slabs on the F32A path, grids of <= 256
  // workgroups): 2 X3_KTICKETS words -- an arrival counter per (phase, output tile), then a claim word per (phase, tile,
  // slice) -- zero when the call began; each launch tags the words it touches with its epoch (kepoch = ++*kepoch_ctr, a
  // host counter of the call, < 2^16), so one zeroing per call serves all of its launches; null: the separate reduce
  // launch.  Callers set them only where they zeroed the words (the posterior call, once per call)
  unsigned* kticket = nullptr;
  unsigned* kepoch_ctr = nullptr;
  unsigned kepoch = 0;
  unsigned* fixup_probe = nullptr;  // damc_x3_fixup_probe's counters (diagnostics; null: off)
  // limb engine, A_CONV (not O_WGRAD): 1 = the K walk of a 4 x 4 conv is channel-slice-major with parity-grouped taps
  // (x3_walk_tap): K tile kt = 32 channels 32 (kt / 16) .. of tap x3_walk_tap(kt % 16), and the weight operand is
  // packed in that order (x3_conv_walk); 0 = tap-major
  int kwalk = 0;
  // InstanceNorm statistics of the epilogue result (round 6; limb engine, O_DENSE, EPI_BIAS_ACT, unsplit 256 x 128
  // tiles: the encoder's norms): per (sample, 256-row strip, channel) {n, mean, m2} at
  // in_part[((b * N + n) * in_S + strip) * 3] (in_stats_kernel's layout, in_merge_kernel reads it), computed by
  // strip256_stats from the stored values; in_hw = output rows per sample (a multiple of 256), in_S = in_hw / 256.
  // in_done (host): the caller sets it to 1; a launcher that cannot write the statistics (a split-K or narrow launch)
  // clears it, and the caller then runs encoder.hip's in_strip_stats_kernel (the same arithmetic) over C
  float* in_part = nullptr;
  int in_hw = 0, in_S = 0;
  int* in_done = nullptr;
};

// InstanceNorm statistics of one 256-row strip (256 consecutive output pixels of one sample) for 128 channels, by 512
// threads: thread t takes channel t & 127 over rows 64 (t >> 7) .. + 63 in two passes (the sum, mean = sum / 64, then
// the centred squares), and threads t < 128 merge the four quarters in order (Chan's pairwise update, in_stats_kernel's
// wmerge at equal counts).  Fixed partition and order, every operation non-contractable, so the same values give the
// same statistics in the conv's epilogue (gemm_x3_kernel, LDS tile) and in the stand-alone kernel (encoder.hip
// in_strip_stats_kernel, global rows): the statistics, and so the normalised activation, do not depend on whether the
// conv ran split, nor on the batch.  y: row r, channel c at y[r * ld + c] (LDS or global); live: c < the channel count;
// red: 1024 floats of LDS; {n, mean, m2} returned in threads t < 128 (after the one barrier inside)
__device__ __forceinline__ void strip256_stats(const float* y, long ld, int tid, bool live, float* red, float (&st)[3]) {
  const int c = tid & 127, q = tid >> 7;
  const float* col = y + (long)q * 64 * ld + c;
  float s = 0.f, m2 = 0.f;
  if (live) {
#pragma unroll 16
    for (int r = 0; r < 64; ++r) s = add_rn(s, col[r * ld]);
    const float mean = mul_rn(s, 0.015625f);
#pragma unroll 16
    for (int r = 0; r < 64; ++r) {
      const float d = sub_rn(col[r * ld], mean);
      m2 = __builtin_fmaf(d, d, m2);
    }
    s = mean;
  }
  red[q * 256 + c] = s;
  red[q * 256 + 128 + c] = m2;
  __syncthreads();
  if (tid < 128) {
    float n = 64.f, mu = red[c], M2 = red[128 + c];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float mb = red[k * 256 + c], m2b = red[k * 256 + 128 + c];
      const float fb = k == 1 ? 0.5f : k == 2 ? (1.f / 3.f) : 0.25f;  // 64 / (n + 64)
      const float d = sub_rn(mb, mu);
      mu = add_rn(mu, mul_rn(d, fb));
      M2 = add_rn(add_rn(M2, m2b), mul_rn(mul_rn(mul_rn(d, d), n), fb));
      n = add_rn(n, 64.f);
    }
    st[0] = n;
    st[1] = mu;
    st[2] = M2;
  }
}
// opt-in (round 6): the encoder's 4 x 4 convs walk K slice-major with their taps grouped by (ky, kx) parity: a stride-2
// tap reads one parity class of the input pixels, the four taps of a class read the same pixels shifted, and a
// 32-channel slice keeps a workgroup's reuse distance within the XCD's L2.  At CelebA-HQ B=64 it cuts FETCH per conv
// 2.4x (2862 / 2043 / 1142 / 349 MB -> 1183 / 739 / 370 / 168 MB) at the same time (1422 vs 1437 us for the first
// k4 s2 conv; the convs run at 200-230 TFLOP/s, compute-bound like the generator's), and measured 2-4 % slower on the
// CIFAR / CelebA-64 encoders (profiles/r06/enc_walk_ab.txt), so tap-major stays the default.  position pos -> tap
__host__ __device__ inline int x3_walk_tap(int pos) {
  const int c = pos >> 2, j = pos & 3;
  return ((c >> 1) + 2 * (j >> 1)) * 4 + (c & 1) + 2 * (j & 1);
}
__host__ __device__ inline int x3_walk_pos(int tap) {
  const int ky = tap >> 2, kx = tap & 3;
  return (((ky & 1) << 1) | (kx & 1)) * 4 + ((ky >> 1) << 1) + (kx >> 1);
}
// whether a k x k conv on cin channels takes the walk (packers and GEMM launches of one call read it alike);
// DAMC_ENC_WALK=1 (read per call) enables it
inline int x3_conv_walk(int k, int cin) {
  const char* e = getenv("DAMC_ENC_WALK");
  return (k == 4 && cin % 32 == 0 && e && e[0] == '1') ? 1 : 0;
}
// words per half of GemmArgs::kticket (counters, claims): a split grid has < 256 unsplit tiles x phases, the fix-up grid
// <= 256 workgroups
constexpr int X3_KTICKETS = 1024;
// k per sign block of a limb-engine conv weight (GemmArgs::negk), from the conv's shape alone (never the batch, so a
// batch split over ranks runs the blocks, slabs and sums of the whole batch).  W16 = (256 x 128 output tiles of the
// GEMM at 16 samples) x K measures how finely a 16-sample batch must split K to fill the chip:
//   W16 >= 2^18: 1024 (512-k blocks would already leave two per workgroup, so the 1024-k block halves the slabs and
//                still fills the chip: every UP2 GEMM of CIFAR-10 ngf=128 and CelebA-HQ);
//   W16 >= 2^16: 512 (CelebA-64 ngf=128);
//   below:       256 (SVHN ngf=64: its per-config batch of 64 fills the chip only with 256-k slices).
// Measured (profiles/r05/negk_ab.txt, posterior step ms, 1024 / 512 / 256 where run): CIFAR B=16 0.452 / 0.487 /
// 0.539, CelebA-HQ B=8 1.229 / 1.244 / 1.39, CelebA-64 B=32 0.525 / 0.421 / 0.476, B=256 - / 2.06 / 2.19, SVHN B=64
// 0.374 / 0.279 / 0.248.  Every length keeps the limb engine's error at or below the fp32-MFMA engine's (DESIGN.md
// section 4).  DAMC_X3_NEGK_RULE=256 / 512 / 1024 (read per call; the packing and the launches of one call read it
// alike) pins it for A/B.
inline int x3_conv_negk(long m_per_sample, int N, int K, int zdim) {
  const char* e = getenv("DAMC_X3_NEGK_RULE");
  int nk;
  if (e && e[0] == '2') {
    nk = 256;
  } else if (e && e[0] == '5') {
    nk = 512;
  } else if (e && e[0] == '1') {
    nk = 1024;
  } else {
    const long w16 = ((16 * m_per_sample + 255) / 256) * ((N + 127) / 128) * zdim * (long)K;
    nk = w16 >= (1L << 18) ? 1024 : w16 >= (1L << 16) ? 512 : 256;
  }
  while (nk > 256 && K % nk != 0) nk >>= 1;
  return nk;
}
// the fused output-layer projection as a kernel of its own: P[pix][n] = sum_c h[pix][c] w[n][c] (c < C <= 256,
// C % 16 == 0; n < np, np = 32 or 64; w rows ldw floats), bitwise the fused form (same MFMA sequence per row); for
// C > 128 the two 128-channel chunks' sums go to P and P + pstride
constexpr int PROJ_CHUNK = 128;  // channels per output-layer projection chain (one F32A N tile)
int launch_proj_rows(const float* h, long npix, int C, const float* w, int ldw, int np, float* P, long pstride,
                     hipStream_t s);
// slab floats a limb-engine conv of this shape uses when split (0: it runs unsplit); workspace sizing
long x3_ksplit_floats(int M, int N, int K, int zdim, int negk = X3_NEGK);

// The K-major convolution engine (a K tile never straddles a filter tap) applies when the gathered
// channel count is a multiple of its K tile; weight packers pick the B layout with this predicate.
constexpr int KM_BK = 32;
inline bool conv_kmajor_ok(int Cg) { return Cg > 0 && Cg % KM_BK == 0; }

// fp32 [n/C rows][C] -> x3 limb layout [rows][C/8][3][8] bf16 (n % 8 == 0, 16-B aligned)
int launch_split_x3(const float* x, long n, unsigned short* y, hipStream_t s);
// the same for a weight operand whose rows are K long, with the values of the odd X3_NEGK-blocks of each row
// negated (exact); the GEMM launches that read it set GemmArgs::b_negblk
int launch_split_x3_negblk(const float* x, long n, int K, unsigned short* y, hipStream_t s, int negk = X3_NEGK);
// the same reordered for the channel-major K walk: a row's K = taps * Cg values [tap][c] are stored
// [c / sw][tap][c % sw] (sw channels per slice), sign blocks counted in that order
int launch_split_x3_cmaj(const float* x, long n, int K, int Cg, int sw, unsigned short* y, hipStream_t s,
                         int negk = X3_NEGK);
// the x3 copy of a conv weight (rows of K = taps * Cg) in the order the library's limb-engine kernels walk K:
// slice-major with sign-alternating blocks when the default variant walks channel-major (DAMC_X3_VARIANT & 8),
// else tap-major (launch_split_x3_negblk)
int launch_split_x3_conv(const float* x, long n, int K, int Cg, unsigned short* y, hipStream_t s, int negk = X3_NEGK);
// the same for a 4 x 4 conv's K-major rows (K = 16 Cg, Cg % 32 == 0) in the x3_conv_walk order
int launch_split_x3_walk(const float* x, long n, int K, int Cg, unsigned short* y, hipStream_t s, int negk = X3_NEGK);
// generator-layer packing through LDS tiles (fp32 + x3 in one pass; damc_pack_generator_layer); 1 = layout not
// covered (the caller falls back to the element-wise packing + launch_split_x3_conv)
int launch_pack_up2_tiled(const float* w, int cin, int cout, float* wf, unsigned short* wf3, float* wb,
                          unsigned short* wb3, hipStream_t s, int negk_f = X3_NEGK, int negk_b = X3_NEGK);
int launch_pack_proj_tiled(const float* w, int cin, int cout, int kk, float* wf, float* wb, unsigned short* wb3,
                           hipStream_t s);

// a PyTorch Conv2d weight (cout, cin, k, k), cin % 8 == 0, straight to the limb B operand of the conv (the order
// launch_split_x3_conv gives damc_pack_conv2d's K-major packing)
int launch_pack_conv_x3(const float* w, int cout, int cin, int k, unsigned short* y, hipStream_t s);
// several Conv2d weights (PyTorch layout) to their limb B operands in one launch (the LDS-transposing kernel):
// n <= 8 layers, each cin % 128 == 0 or cin == 64, k * k <= 32, w 16-B aligned; returns 1 (nothing launched) otherwise
struct PackConvList {
  int n;
  int walk[8];  // layer i's limbs in the x3_conv_walk order (pack_conv_x3_many_prep fills it)
  const float* w[8];
  unsigned short* y[8];
  int cin[8], taps[8], cc[8], blk0[9];
  int ready;   // set by pack_conv_x3_many_prep (blk0 then holds workgroup offsets, not couts)
  int lds;     // dynamic LDS bytes per workgroup (prep)
  int cout[8];  // (prep) each layer's output channels: the device-side bound of a workgroup's weight rows
  int* err;     // optional device status word: a workgroup outside the list ORs 1 into it and writes nothing
};
bool pack_conv_x3_many_ok(const float* w, int cin, int k);
// fills in cc and lds and turns blk0[i + 1] (layer i's cout on entry) into running workgroup offsets, once (ready);
// nonzero when a layer is not covered or l was already prepared
int pack_conv_x3_many_prep(PackConvList& l);
// launches a list (prepared here unless ready)
int launch_pack_conv_x3_many(PackConvList l, hipStream_t s);

// the limb form of 8 consecutive fp32 values (the engine's RNE split: v = hi + mid + lo to 24 significand bits),
// stored as one x3 octet [3][8] bf16 at dst (16-B aligned)
__device__ __forceinline__ void store_x3_octet(const float (&v)[8], unsigned short* dst) {
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  bf16x8_t h, m, l;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 b0 = (__bf16)v[e];
    const float r1 = sub_rn(v[e], (float)b0);
    const __bf16 b1 = (__bf16)r1;
    h[e] = b0;
    m[e] = b1;
    l[e] = (__bf16)(sub_rn(r1, (float)b1));
  }
  bf16x8_t* o = reinterpret_cast<bf16x8_t*>(dst);
  o[0] = h;
  o[1] = m;
  o[2] = l;
}

// one workgroup (nthr threads, pk_t = CC * (taps + 1) floats of LDS) of the LDS-transposing conv weight packing
// (gemm.hip pack_conv_x3_lds_kernel; also run by the encoder's first-layer kernel as extra workgroups): workgroup blk
// of a prepared list = (layer, co, chunk of CC input channels).  The chunk's CC * k * k floats are one contiguous run
// of the PyTorch layout (read as f32x4), transposed in LDS to (tap, channel); each tap's CC / 8 limb octets are
// CC * 6 contiguous bytes of the K-major output, odd sign blocks negated
__device__ __forceinline__ void pack_conv_x3_block(const PackConvList& l, int blk, int tid, int nthr, float* pk_t) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  // bound (workgroup-uniform, before any access): the workgroup must name a weight row of the prepared list; one that
  // does not (a grid larger than the list) writes nothing and flags the status word
  const bool in_list = l.ready && l.n >= 1 && l.n <= 8 && blk >= 0 && blk < l.blk0[l.n];
  int li = 0;
  while (in_list && li + 1 < l.n && blk >= l.blk0[li + 1]) ++li;
  blk -= l.blk0[li];
  const int CC = l.cc[li], cin = l.cin[li], taps = l.taps[li], nch = CC > 0 ? cin / CC : 0;
  const int co = nch > 0 ? blk / nch : 0, cc0 = (blk - co * nch) * CC, tp1 = taps + 1, n4 = CC * taps / 4;
  if (!in_list || nch <= 0 || co >= l.cout[li] || cc0 + CC > cin) {
    if (tid == 0 && l.err) atomicOr(l.err, 1);
    return;
  }
  const f32x4_t* src = reinterpret_cast<const f32x4_t*>(l.w[li] + ((long)co * cin + cc0) * taps);
  for (int q = tid; q < n4; q += nthr) {
    const f32x4_t v = src[q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int f = 4 * q + e, ci = f / taps;
      pk_t[ci * tp1 + (f - ci * taps)] = v[e];
    }
  }
  __syncthreads();
  const int oc = CC / 8, cin8 = cin / 8, walk = l.walk[li];
  unsigned short* o = l.y[li] + 24L * (long)co * taps * cin8;
  for (int q = tid; q < taps * oc; q += nthr) {
    const int tap = q / oc, c8 = q - tap * oc, c = cc0 + c8 * 8;
    // the octet's K index in the walk the GEMM runs: tap-major (tap cin + c), or slice-major with the taps in
    // x3_walk_pos order; the sign block follows it
    const int kk = walk ? (c >> 5) * taps * 32 + x3_walk_pos(tap) * 32 + (c & 31) : tap * cin + c;
    const float sg = ((kk / X3_NEGK) & 1) ? -1.f : 1.f;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = sg * pk_t[(c8 * 8 + e) * tp1 + tap];
    store_x3_octet(v, o + 24L * (kk >> 3));
  }
}

// the encoder's dense head (encoder.hip enc_head_x3_kernel): out[M][N] = A . W^T + bias on the limb product, A [M][K]
// and W [N][K] fp32 (a PyTorch Conv2d weight covering its whole input, with A the samples' CHW rows); N % 64 == 0,
// K % 512 == 0, 16-B aligned A / W / slab / out; slab: K / 512 * M * N floats of scratch
int launch_dense_head_x3(const float* a, const float* w, const float* bias, int M, int N, int K, float* slab,
                         size_t slab_floats, float* out, hipStream_t s);

// O_WGRAD on the limb engine: zdim = wg_phases * split-K slices
int launch_wgrad_x3(const GemmArgs& a, int slices, const char* prof_name, double flops, hipStream_t s);

// small fp32 GEMMs in one launch (gemm.hip small_gemm_kernel): C = act(A . B + bias[n % bias_mod]) (bias_mod 0: n),
// A (M x K, K % 4 == 0, lda % 4 == 0, 16-B aligned), B (K x N row-major); one 16 x 16 output tile per wave, exact
// fp32 products, fp32 accumulation
int launch_small_gemm(const float* A, long lda, const float* B, long ldb, const float* bias, float* C, long ldc, int M,
                      int N, int K, hipStream_t s, int bias_mod = 0, int act = DAMC_ACT_NONE, float slope = 0.f);
// up to SG_GROUP_MAX independent small GEMMs in one launch (gemm.hip small_gemm_group_kernel): one 16 x 16 tile per
// 4-wave workgroup, K split over the waves, partials summed in a fixed order; a_ones (M = 1): A is a row of ones (C =
// column sums of B)
struct SmallGemm {
  const float* A = nullptr;
  const float* B = nullptr;
  const float* bias = nullptr;
  float* C = nullptr;
  long lda = 0, ldb = 0, ldc = 0;
  int M = 0, N = 0, K = 0, bias_mod = 0, act = DAMC_ACT_NONE;
  float slope = 0.f;
  int a_ones = 0;
  int b_t = 0;  // B given transposed: N rows of K (row stride ldb >= K, 16-B aligned), e.g. a PyTorch Linear weight
};
constexpr int SG_GROUP_MAX = 8;
struct SmallGemmGroup {
  int n;
  int tile_end[SG_GROUP_MAX];
  SmallGemm d[SG_GROUP_MAX];
};
int launch_small_gemm_group(const SmallGemm* g, int n, hipStream_t s);
int launch_gemm(const GemmArgs& a, AMode am, Epi epi, OMode om, int zdim, const char* prof_name, double flops,
                hipStream_t s);

// up to GEMM_GROUP_MAX independent A_DENSE / O_DENSE GEMMs (no split-K, float4-aligned rows) in one launch of the
// generic engine; each result is bitwise the one launch_gemm gives it
constexpr int GEMM_GROUP_MAX = 8;
struct GemmGroup {
  GemmArgs a[GEMM_GROUP_MAX];
  int start[GEMM_GROUP_MAX + 1];
  int n;
};
int launch_gemm_group(const GemmArgs* a, int n, Epi epi, const char* prof_name, double flops, hipStream_t s);

}  // namespace damc
