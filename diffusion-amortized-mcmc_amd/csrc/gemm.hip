// gemm.hip — fp32 MFMA implicit-GEMM engine for the generator / encoder convolutions.
//
// Tile 128x128x16, 256 threads = 4 waves in a 2x2 grid, each wave 64x64 = 2x2 tiles of
// v_mfma_f32_32x32x2_f32 (exact fp32: a k-ordered fmaf chain per output, no xf32 on gfx950).
// Operands are staged global -> registers -> LDS (k-major images so every MFMA operand read is
// one conflict-free ds_read_b32 of 32 consecutive floats per half-wave), double-buffered with one
// barrier per K-tile: the next tile's global loads are issued before the current tile's MFMAs.
// Blocks are remapped so each XCD owns a contiguous run of tiles (shared A rows stay in its L2).
#include "gemm.h"

namespace damc {

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int LDA_S = BM + 2;  // 4*LDA_S == 8 (mod 32): the transposing ds_write_b32 of A is conflict-free
constexpr int LDB_S = BN;

template <int AM, int EPI, int OM, bool BVEC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs p) {
  __shared__ float As[2][BK * LDA_S];
  __shared__ float Bs[2][BK * LDB_S];

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

  // ---- per-thread A rows (vector paths: 2 rows x one float4 of k; scalar path: 8 rows x 1 k)
  const int a_kq = tid & 3;       // float4 slot within the 16-wide k tile
  const int a_ml = tid >> 2;      // 0..63 (+64)
  const int s_kk = tid & 15;      // scalar path k
  const int s_ml = tid >> 4;      // 0..15 (+16*j)
  constexpr int AROWS = (AM == A_CONV_SCALAR) ? 8 : 2;
  int a_b[AROWS], a_iy[AROWS], a_ix[AROWS];
  bool a_ok[AROWS];
  const long hwq = (long)p.Hq * p.Wq;
#pragma unroll
  for (int j = 0; j < AROWS; ++j) {
    const int m = m0 + ((AM == A_CONV_SCALAR) ? (s_ml + 16 * j) : (a_ml + 64 * j));
    a_ok[j] = m < p.M;
    if (AM == A_DENSE) {
      a_b[j] = m;
      a_iy[j] = 0;
      a_ix[j] = 0;
    } else {
      const int mm = a_ok[j] ? m : 0;
      const int b = (int)(mm / hwq);
      const int r = (int)(mm - b * hwq);
      const int qy = r / p.Wq, qx = r - qy * p.Wq;
      a_b[j] = b;
      a_iy[j] = qy * p.stride - pad_y;
      a_ix[j] = qx * p.stride - pad_x;
    }
  }

  f32x4 ra[2];
  float rs[8];
  f32x4 rb[2];
  float rbs[8];

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
      for (int j = 0; j < 8; ++j) {
        const int iy = a_iy[j] + ky, ix = a_ix[j] + kx;
        const bool ok = kin && a_ok[j] && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
        rs[j] = ok ? p.A[(((long)a_b[j] * p.Hin + iy) * p.Win + ix) * p.Cg + ci] : 0.f;
      }
    } else {
      const int k = k0 + 4 * a_kq;
      const bool kin = k < kend;
      if (AM == A_DENSE) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          ra[j] = (kin && a_ok[j]) ? *reinterpret_cast<const f32x4*>(p.A + (long)a_b[j] * p.lda + k)
                                   : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      } else {
        int ky = 0, kx = 0, ci = 0;
        if (kin) {
          const int tap = k / p.Cg;
          ci = k - tap * p.Cg;
          ky = tap / p.kw;
          kx = tap - ky * p.kw;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int iy = a_iy[j] + ky, ix = a_ix[j] + kx;
          const bool ok = kin && a_ok[j] && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
          ra[j] = ok ? *reinterpret_cast<const f32x4*>(p.A + (((long)a_b[j] * p.Hin + iy) * p.Win + ix) * p.Cg + ci)
                     : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  };
  auto store_a = [&](int buf) {
    float* as = As[buf];
    if (AM == A_CONV_SCALAR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) as[s_kk * LDA_S + s_ml + 16 * j] = rs[j];
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ml = a_ml + 64 * j;
        as[(4 * a_kq + 0) * LDA_S + ml] = ra[j].x;
        as[(4 * a_kq + 1) * LDA_S + ml] = ra[j].y;
        as[(4 * a_kq + 2) * LDA_S + ml] = ra[j].z;
        as[(4 * a_kq + 3) * LDA_S + ml] = ra[j].w;
      }
    }
  };
  // B tile: 16 k-rows x 128 n
  const int b_row = tid >> 5, b_c4 = tid & 31;   // vector path
  const int bs_n = tid & 127, bs_row = tid >> 7; // scalar path
  auto load_b = [&](int k0) {
    if (BVEC) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = k0 + b_row + 8 * j;
        const int n = n0 + 4 * b_c4;
        rb[j] = (k < kend && n < p.N) ? *reinterpret_cast<const f32x4*>(Bg + (long)k * p.ldb + n)
                                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = k0 + bs_row + 2 * j;
        const int n = n0 + bs_n;
        rbs[j] = (k < kend && n < p.N) ? Bg[(long)k * p.ldb + n] : 0.f;
      }
    }
  };
  auto store_b = [&](int buf) {
    float* bs = Bs[buf];
    if (BVEC) {
#pragma unroll
      for (int j = 0; j < 2; ++j) *reinterpret_cast<f32x4*>(bs + (b_row + 8 * j) * LDB_S + 4 * b_c4) = rb[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) bs[(bs_row + 2 * j) * LDB_S + bs_n] = rbs[j];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    load_a(kbeg);
    load_b(kbeg);
    store_a(0);
    store_b(0);
  }
  __syncthreads();

  const int lrow = lane & 31, lk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_a(kbeg + (kt + 1) * BK);
      load_b(kbeg + (kt + 1) * BK);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a0 = as[(kk + lk) * LDA_S + wm * 64 + lrow];
      const float a1 = as[(kk + lk) * LDA_S + wm * 64 + 32 + lrow];
      const float b0 = bs[(kk + lk) * LDB_S + wn * 64 + lrow];
      const float b1 = bs[(kk + lk) * LDB_S + wn * 64 + 32 + lrow];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) {
      store_a(cur ^ 1);
      store_b(cur ^ 1);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds col = lane&31, rows (r&3) + 8(r>>2) + 4(lane>>5) of each 32x32 tile
  float* Cz = p.C;
  if (OM == O_DENSE) Cz += (long)z * p.c_zstride;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m >= p.M) continue;
      long rowoff;
      if (OM == O_PHASE) {
        const int b = (int)(m / hwq);
        const int rr = (int)(m - b * hwq);
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

template <int AM, int EPI, int OM, bool BV>
static void launch_t(const GemmArgs& a, int zdim, hipStream_t s) {
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn, 1, zdim);
  hipLaunchKernelGGL((gemm_f32_kernel<AM, EPI, OM, BV>), grid, dim3(256), 0, s, a);
}

int launch_gemm(const GemmArgs& a, AMode am, Epi epi, OMode om, int zdim, const char* prof_name, double flops,
                hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return DAMC_ERR_ARG;
  const bool bvec = (a.ldb % 4 == 0) && (a.N % 4 == 0) && ((uintptr_t)a.B % 16 == 0);
  if (am == A_DENSE && (a.lda % 4 != 0 || a.K % 4 != 0 || (uintptr_t)a.A % 16 != 0)) am = A_CONV_SCALAR;
  if (am == A_CONV && (a.Cg % 4 != 0 || (uintptr_t)a.A % 16 != 0)) am = A_CONV_SCALAR;
  GemmArgs b = a;
  if (am == A_CONV_SCALAR && a.Hq == 1 && a.Wq == 1 && a.Hin == 1 && a.Win == 1 && a.kw == 1) {
    // dense-as-scalar: treat A (M,K) as an NHWC map with one pixel of Cg = lda channels
    b.Cg = (int)a.lda;
  }
  ProfScope ps(prof_name, flops, s);
#define DAMC_G(AM_, EPI_, OM_)                                                          \
  if (am == AM_ && epi == EPI_ && om == OM_) {                                          \
    if (bvec) launch_t<AM_, EPI_, OM_, true>(b, zdim, s);                               \
    else launch_t<AM_, EPI_, OM_, false>(b, zdim, s);                                   \
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
