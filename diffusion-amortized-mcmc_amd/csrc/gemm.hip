// gemm.hip — fp32 MFMA implicit-GEMM engine for the generator / encoder convolutions.
//
// Block tile (64*MT) x 128 x BK, 256 threads = 4 waves in a 2x2 grid; a wave owns (32*MT) x 64 =
// MT x 2 tiles of v_mfma_f32_32x32x2_f32 (exact fp32: a k-ordered fmaf chain per output; gfx950
// has no xf32).  Operands are staged global -> registers -> LDS (k-major images: every MFMA operand
// read is one conflict-free ds_read_b32 of 32 consecutive floats per half-wave), double-buffered
// with one barrier per K-tile.  Schedule per tile: all fragments of the tile -> registers, store the
// next tile into the other LDS buffer, issue the global loads of the tile after that, then the
// tile's MFMAs back to back (the loads land under them).  Gather addresses are 32-bit element
// offsets off the tensor base (every tensor here has < 2^31 elements).  Blocks are remapped so each
// XCD owns a contiguous run of tiles (shared A rows stay in its L2).
//
// Config (BK, OCC, MT): K-tile depth, workgroups per CU for the launch bounds, MFMA tiles per wave
// along M.  tools/gemm_bench.hip A/B-tests them on the generator's convolutions.
#include "gemm.h"

namespace damc {

constexpr int BN = 128;

template <int BK, int MT>
struct TileCfg {
  static constexpr int BM = 64 * MT;
  // A is written transposed with ds_write_b32: lanes (a_kq, m) of a half-wave must hit 32 banks
  static constexpr int LDA = (BK == 16) ? BM + 2 : BM + 1;
  static constexpr int LDB = BN;
  static constexpr int AQ = BK / 4;              // float4 slots per A row
  static constexpr int AROWS_V = BM * BK / 1024; // A float4 loads per thread (vector path)
  static constexpr int AROWS_S = BM * BK / 256;  // A scalar loads per thread
  static constexpr int BROWS_V = BK / 8;         // B float4 loads per thread
  static constexpr int BROWS_S = BK / 2;         // B scalar loads per thread
};

template <int AM, int EPI, int OM, bool BVEC, int BK, int OCC, int MT>
__global__ __launch_bounds__(256, OCC) void gemm_f32_kernel(GemmArgs p) {
  typedef TileCfg<BK, MT> C;
  constexpr int BM = C::BM;
  __shared__ float As[2][BK * C::LDA];
  __shared__ float Bs[2][BK * C::LDB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- XCD-aware tile remap (bijective for any grid size)
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ntn = (p.N + BN - 1) / BN;
  const int tm = wgid / ntn, tn = wgid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.z;

  int pad_y = p.pad_y, pad_x = p.pad_x;
  const float* Bg = p.B;
  int kbeg = 0, kend = p.K;
  int py = 0, px = 0;
  if (OM == O_PHASE) {
    py = z >> 1;
    px = z & 1;
    pad_y = 1 - py;
    pad_x = 1 - px;
    Bg += (long)z * p.b_zstride;
  } else {
    kbeg = z * p.k_per_z;
    kend = min(p.K, kbeg + p.k_per_z);
  }
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // ---- per-thread A rows
  const int a_kq = tid % C::AQ;  // float4 slot within the k tile (vector paths)
  const int a_ml = tid / C::AQ;  // rows a_ml + AVSTEP*j
  constexpr int AVSTEP = 256 / C::AQ;
  const int s_kk = tid % BK;     // scalar path k
  const int s_ml = tid / BK;     // rows s_ml + ASSTEP*j
  constexpr int ASSTEP = 256 / BK;
  constexpr int AROWS = (AM == A_CONV_SCALAR) ? C::AROWS_S : C::AROWS_V;
  int a_pix[AROWS], a_iy[AROWS], a_ix[AROWS];  // first pixel of the sample / top-left input tap
  const int hwq = p.Hq * p.Wq;
  const int hwin = p.Hin * p.Win;
#pragma unroll
  for (int j = 0; j < AROWS; ++j) {
    const int m = m0 + ((AM == A_CONV_SCALAR) ? (s_ml + ASSTEP * j) : (a_ml + AVSTEP * j));
    const bool ok = m < p.M;
    if (AM == A_DENSE) {
      a_pix[j] = m * (int)p.lda;
      a_iy[j] = ok ? 0 : -0x40000000;  // poisons the row bound check
      a_ix[j] = 0;
    } else {
      const int mm = ok ? m : 0;
      const int b = mm / hwq;
      const int r = mm - b * hwq;
      const int qy = r / p.Wq, qx = r - qy * p.Wq;
      a_pix[j] = b * hwin;
      a_iy[j] = ok ? qy * p.stride - pad_y : -0x40000000;
      a_ix[j] = qx * p.stride - pad_x;
    }
  }
  // when Cg is a multiple of BK a whole K-tile sits inside one filter tap: the tap decomposition
  // is then tile-uniform (scalar) instead of a per-lane division
  const bool tap_uniform = (AM == A_CONV) && (p.Cg % BK == 0);
  const unsigned Hin = (unsigned)p.Hin, Win = (unsigned)p.Win;

  f32x4 ra[C::AROWS_V];
  float rs[C::AROWS_S];
  f32x4 rb[C::BROWS_V];
  float rbs[C::BROWS_S];

  auto load_a = [&](int k0) {
    if (AM == A_CONV_SCALAR) {
      const int k = k0 + s_kk;
      int ky = 0, kx = 0, ci = 0;
      const bool kin = k < kend;
      if (kin) {
        const int tap = k / p.Cg;
        ci = k - tap * p.Cg;
        ky = tap / p.kw;
        kx = tap - ky * p.kw;
      }
#pragma unroll
      for (int j = 0; j < C::AROWS_S; ++j) {
        const int iy = a_iy[j] + ky, ix = a_ix[j] + kx;
        const bool ok = kin && (unsigned)iy < Hin && (unsigned)ix < Win;
        rs[j] = ok ? p.A[(a_pix[j] + iy * p.Win + ix) * p.Cg + ci] : 0.f;
      }
    } else {
      const int k = k0 + 4 * a_kq;
      const bool kin = k < kend;
      if (AM == A_DENSE) {
#pragma unroll
        for (int j = 0; j < C::AROWS_V; ++j) {
          ra[j] = (kin && a_iy[j] == 0) ? *reinterpret_cast<const f32x4*>(p.A + (a_pix[j] + k))
                                        : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      } else {
        int ky = 0, kx = 0, ci = 0;
        if (tap_uniform) {
          const int tap = k0 / p.Cg;
          ci = k0 - tap * p.Cg + 4 * a_kq;
          ky = tap / p.kw;
          kx = tap - ky * p.kw;
        } else if (kin) {
          const int tap = k / p.Cg;
          ci = k - tap * p.Cg;
          ky = tap / p.kw;
          kx = tap - ky * p.kw;
        }
#pragma unroll
        for (int j = 0; j < C::AROWS_V; ++j) {
          const int iy = a_iy[j] + ky, ix = a_ix[j] + kx;
          const bool ok = kin && (unsigned)iy < Hin && (unsigned)ix < Win;
          ra[j] = ok ? *reinterpret_cast<const f32x4*>(p.A + ((a_pix[j] + iy * p.Win + ix) * p.Cg + ci))
                     : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  };
  auto store_a = [&](int buf) {
    float* as = As[buf];
    if (AM == A_CONV_SCALAR) {
#pragma unroll
      for (int j = 0; j < C::AROWS_S; ++j) as[s_kk * C::LDA + s_ml + ASSTEP * j] = rs[j];
    } else {
#pragma unroll
      for (int j = 0; j < C::AROWS_V; ++j) {
        const int ml = a_ml + AVSTEP * j;
        as[(4 * a_kq + 0) * C::LDA + ml] = ra[j].x;
        as[(4 * a_kq + 1) * C::LDA + ml] = ra[j].y;
        as[(4 * a_kq + 2) * C::LDA + ml] = ra[j].z;
        as[(4 * a_kq + 3) * C::LDA + ml] = ra[j].w;
      }
    }
  };
  // B tile: BK k-rows x 128 n
  const int b_row = tid >> 5, b_c4 = tid & 31;    // vector path: 8 rows per pass
  const int bs_n = tid & 127, bs_row = tid >> 7;  // scalar path: 2 rows per pass
  const int ldb = (int)p.ldb;
  auto load_b = [&](int k0) {
    if (BVEC) {
      const int n = n0 + 4 * b_c4;
#pragma unroll
      for (int j = 0; j < C::BROWS_V; ++j) {
        const int k = k0 + b_row + 8 * j;
        rb[j] = (k < kend && n < p.N) ? *reinterpret_cast<const f32x4*>(Bg + (k * ldb + n))
                                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      const int n = n0 + bs_n;
#pragma unroll
      for (int j = 0; j < C::BROWS_S; ++j) {
        const int k = k0 + bs_row + 2 * j;
        rbs[j] = (k < kend && n < p.N) ? Bg[k * ldb + n] : 0.f;
      }
    }
  };
  auto store_b = [&](int buf) {
    float* bs = Bs[buf];
    if (BVEC) {
#pragma unroll
      for (int j = 0; j < C::BROWS_V; ++j)
        *reinterpret_cast<f32x4*>(bs + (b_row + 8 * j) * C::LDB + 4 * b_c4) = rb[j];
    } else {
#pragma unroll
      for (int j = 0; j < C::BROWS_S; ++j) bs[(bs_row + 2 * j) * C::LDB + bs_n] = rbs[j];
    }
  };

  f32x16 acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    load_a(kbeg);
    load_b(kbeg);
    store_a(0);
    store_b(0);
    if (nk > 1) {
      load_a(kbeg + BK);
      load_b(kbeg + BK);
    }
  }
  __syncthreads();

  const int lrow = lane & 31, lk = lane >> 5;
  const int am0 = wm * (32 * MT) + lrow, bn0 = wn * 64 + lrow;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const float* as = As[cur];
    const float* bs = Bs[cur];
    float fa[BK / 2][MT], fb[BK / 2][2];
#pragma unroll
    for (int s2 = 0; s2 < BK / 2; ++s2) {
      const int kk = 2 * s2 + lk;
#pragma unroll
      for (int i = 0; i < MT; ++i) fa[s2][i] = as[kk * C::LDA + am0 + 32 * i];
      fb[s2][0] = bs[kk * C::LDB + bn0];
      fb[s2][1] = bs[kk * C::LDB + bn0 + 32];
    }
    if (kt + 1 < nk) {
      store_a(cur ^ 1);
      store_b(cur ^ 1);
      if (kt + 2 < nk) {
        load_a(kbeg + (kt + 2) * BK);
        load_b(kbeg + (kt + 2) * BK);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < BK / 2; ++s2)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s2][i], fb[s2][0], acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s2][i], fb[s2][1], acc[i][1], 0, 0, 0);
      }
    __syncthreads();
  }

  // ---- epilogue: lane holds col = lane&31, rows (r&3) + 8(r>>2) + 4(lane>>5) of each 32x32 tile
  float* Cz = p.C;
  if (OM == O_DENSE) Cz += (long)z * p.c_zstride;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * (32 * MT) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m >= p.M) continue;
      long rowoff;
      if (OM == O_PHASE) {
        const int b = m / hwq;
        const int rr = m - b * hwq;
        const int qy = rr / p.Wq, qx = rr - qy * p.Wq;
        rowoff = (((long)b * p.Hout + 2 * qy + py) * p.Wout + 2 * qx + px) * p.ldc;
      } else {
        rowoff = (long)m * p.ldc;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + j * 32 + lrow;
        if (n >= p.N) continue;
        float v = acc[i][j][r];
        const long idx = rowoff + n;
        if (EPI == EPI_BIAS_ACT) {
          if (p.bias) v += p.bias[n % p.bias_mod];
          v = act_apply(v, p.act, p.slope);
        } else if (EPI == EPI_MASK) {
          v *= act_grad_from_out(p.mask[idx], p.mask_act, p.mask_slope);
        } else if (EPI == EPI_RESID) {
          if (p.bias) v += p.bias[n % p.bias_mod];
          const float t = act_apply(v, p.act, p.slope);
          if (p.xhat) p.xhat[idx] = t;
          const float res = t - p.xres[idx];
          if (p.sqerr) atomicAdd(p.sqerr, 0.5f * p.inv_s2 * res * res);
          v = res * p.inv_s2 * act_grad_from_out(t, p.act, p.slope);
        }
        Cz[idx] = v;
      }
    }
  }
}

template <int AM, int EPI, int OM, bool BV, int BK, int OCC, int MT>
static void launch_t(const GemmArgs& a, int zdim, hipStream_t s) {
  const int bm = 64 * MT;
  const int ntm = (a.M + bm - 1) / bm, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn, 1, zdim);
  hipLaunchKernelGGL((gemm_f32_kernel<AM, EPI, OM, BV, BK, OCC, MT>), grid, dim3(256), 0, s, a);
}

// tile configuration used by the library (tools/gemm_bench.hip A/B-tests alternatives)
#ifndef DAMC_GEMM_BK
#define DAMC_GEMM_BK 32  // measured best on the B=128 generator convs (profiles/r01/gemm_bench.txt)
#endif
#ifndef DAMC_GEMM_OCC
#define DAMC_GEMM_OCC 2
#endif
#ifndef DAMC_GEMM_MT
#define DAMC_GEMM_MT 2
#endif

int launch_gemm(const GemmArgs& a, AMode am, Epi epi, OMode om, int zdim, const char* prof_name, double flops,
                hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return DAMC_ERR_ARG;
  // 32-bit element offsets inside the kernel
  const double a_elems = (am == A_DENSE) ? (double)a.M * a.lda : (double)a.Hin * a.Win * a.Cg * ((double)a.M / ((double)a.Hq * a.Wq) + 1);
  if (a_elems >= 2147483647.0 || (double)a.K * a.ldb >= 2147483647.0) return DAMC_ERR_UNSUPPORTED;
  const bool bvec = (a.ldb % 4 == 0) && (a.N % 4 == 0) && ((uintptr_t)a.B % 16 == 0);
  if (am == A_DENSE && (a.lda % 4 != 0 || a.K % 4 != 0 || (uintptr_t)a.A % 16 != 0)) am = A_CONV_SCALAR;
  if (am == A_CONV && (a.Cg % 4 != 0 || (uintptr_t)a.A % 16 != 0)) am = A_CONV_SCALAR;
  GemmArgs b = a;
  if (am == A_CONV_SCALAR && a.Hq == 1 && a.Wq == 1 && a.Hin == 1 && a.Win == 1 && a.kw == 1) {
    // dense-as-scalar: treat A (M,K) as an NHWC map with one pixel of Cg = lda channels
    b.Cg = (int)a.lda;
  }
  ProfScope ps(prof_name, flops, s);
  constexpr int BKc = DAMC_GEMM_BK, OCCc = DAMC_GEMM_OCC, MTc = DAMC_GEMM_MT;
#define DAMC_G(AM_, EPI_, OM_)                                                          \
  if (am == AM_ && epi == EPI_ && om == OM_) {                                          \
    if (bvec) launch_t<AM_, EPI_, OM_, true, BKc, OCCc, MTc>(b, zdim, s);               \
    else launch_t<AM_, EPI_, OM_, false, BKc, OCCc, MTc>(b, zdim, s);                   \
    return (int)hipGetLastError();                                                      \
  }
  DAMC_G(A_DENSE, EPI_STORE, O_DENSE)
  DAMC_G(A_DENSE, EPI_BIAS_ACT, O_DENSE)
  DAMC_G(A_DENSE, EPI_MASK, O_DENSE)
  DAMC_G(A_DENSE, EPI_RESID, O_DENSE)
  DAMC_G(A_CONV, EPI_BIAS_ACT, O_PHASE)
  DAMC_G(A_CONV, EPI_MASK, O_DENSE)
  DAMC_G(A_CONV, EPI_BIAS_ACT, O_DENSE)
  DAMC_G(A_CONV, EPI_STORE, O_DENSE)
  DAMC_G(A_CONV_SCALAR, EPI_STORE, O_DENSE)
  DAMC_G(A_CONV_SCALAR, EPI_BIAS_ACT, O_DENSE)
  DAMC_G(A_CONV_SCALAR, EPI_MASK, O_DENSE)
  DAMC_G(A_CONV_SCALAR, EPI_RESID, O_DENSE)
  DAMC_G(A_CONV_SCALAR, EPI_BIAS_ACT, O_PHASE)
  DAMC_G(A_CONV_SCALAR, EPI_MASK, O_PHASE)
#undef DAMC_G
  return DAMC_ERR_UNSUPPORTED;
}

}  // namespace damc

#ifndef DAMC_GEMM_NO_C_API
extern "C" int damc_gemm(const float* a, int lda, const float* b, int ldb, const float* bias, float* c, int ldc,
                         int m, int n, int k, int act, float slope, void* stream) {
  damc::GemmArgs g;
  g.A = a;
  g.lda = lda;
  g.B = b;
  g.ldb = ldb;
  g.C = c;
  g.ldc = ldc;
  g.M = m;
  g.N = n;
  g.K = k;
  g.k_per_z = k;
  g.bias = bias;
  g.bias_mod = n;
  g.act = act;
  g.slope = slope;
  return damc::launch_gemm(g, damc::A_DENSE, damc::EPI_BIAS_ACT, damc::O_DENSE, 1, "gemm", 2.0 * m * n * k,
                           as_stream(stream));
}
#endif
