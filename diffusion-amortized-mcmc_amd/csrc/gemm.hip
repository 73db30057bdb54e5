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
#include <algorithm>
#include <cstdlib>
#include <type_traits>

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

// ---- epilogue: lane holds col = lane&31, rows (r&3) + 8(r>>2) + 4(lane>>5) of each 32x32 tile
// output row offset of GEMM row m (O_PHASE: pixel (b, 2qy+py, 2qx+px) of the Hout x Wout map)
template <int OM>
__device__ __forceinline__ long gemm_row_offset(const GemmArgs& p, int m, int py, int px) {
  if (OM == O_PHASE) {
    const int hwq = p.Hq * p.Wq;
    const int b = m / hwq;
    const int rr = m - b * hwq;
    const int qy = rr / p.Wq, qx = rr - qy * p.Wq;
    return (((long)b * p.Hout + 2 * qy + py) * p.Wout + 2 * qx + px) * p.ldc;
  }
  return (long)m * p.ldc;
}

// one output element: epilogue arithmetic + store (idx = row offset + n)
template <int EPI>
__device__ __forceinline__ void epi_element(const GemmArgs& p, float* Cz, long idx, int n, bool bias_wrap, float v) {
  if (EPI == EPI_BIAS_ACT) {
    if (p.bias) v += p.bias[bias_wrap ? n % p.bias_mod : n];
    v = act_apply(v, p.act, p.slope);
  } else if (EPI == EPI_MASK) {
    v *= act_grad_from_out(p.mask[idx], p.mask_act, p.mask_slope);
  } else if (EPI == EPI_GATE) {
    if (p.bias) v += p.bias[n];
    if (n < p.gate_cols) v = 1.f / (1.f + expf(-v));
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

// rowtab: optional per-block table of gemm_row_offset for rows m0 .. m0 + 32*MT*2 - 1
template <int EPI, int OM, int MT>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& p, f32x16 (&acc)[MT][2], int m0, int n0, int wm,
                                              int wn, int lane, int z, int py, int px,
                                              const long* rowtab = nullptr) {
  const int lrow = lane & 31;
  float* Cz = p.C;
  if (OM == O_DENSE) Cz += (long)z * p.c_zstride;
  const bool bias_wrap = p.bias_mod < p.N;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ml = wm * (32 * MT) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int m = m0 + ml;
      if (m >= p.M) continue;
      const long rowoff = rowtab ? rowtab[ml] : gemm_row_offset<OM>(p, m, py, px);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + j * 32 + lrow;
        if (n >= p.N) continue;
        epi_element<EPI>(p, Cz, rowoff + n, n, bias_wrap, acc[i][j][r]);
      }
    }
  }
}

// the same for a wave's 4 x 4 grid of 16x16 accumulators (col = lane&15, row = 4(lane>>4) + r)
template <int EPI, int OM>
__device__ __forceinline__ void gemm_epilogue16(const GemmArgs& p, f32x4 (&acc)[4][4], int m0, int n0, int wm, int wn,
                                                int lane, int z, int py, int px, const long* rowtab) {
  float* Cz = p.C;
  if (OM == O_DENSE) Cz += (long)z * p.c_zstride;
  const bool bias_wrap = p.bias_mod < p.N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ml = wm * 64 + i * 16 + 4 * (lane >> 4) + r;
      const int m = m0 + ml;
      if (m >= p.M) continue;
      const long rowoff = rowtab ? rowtab[ml] : gemm_row_offset<OM>(p, m, py, px);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + (lane & 15);
        if (n >= p.N) continue;
        epi_element<EPI>(p, Cz, rowoff + n, n, bias_wrap, acc[i][j][r]);
      }
    }
  }
}

// XCD-aware bijective remap: consecutive work-group ids land on one XCD (dispatch is round-robin over 8)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// supertile raster: linear id l in [0, T * P) -> (M tile tm, pair p), blocks of SM x SP ids (SP = min(4, P) pairs
// fastest, then SM = 32 / SP M tiles), blocks ordered M-major; edge blocks are smaller.  Bijective.
__device__ __forceinline__ void supertile(int l, int T, int P, int& tm, int& p) {
  const int SP = P < 4 ? P : 4;
  const int SMf = 32 / SP;
  const int SM = T < SMf ? T : SMf;
  const int rowsz = SM * P;              // ids of one full block row (SM M tiles, all pairs)
  const int tmb = l / rowsz;
  const int sm = min(SM, T - tmb * SM);  // M tiles in this block row (smaller on the last)
  int rem = l - tmb * rowsz;
  const int pb = rem / (sm * SP);        // full pair blocks come first; the last may be narrower
  const int sp = min(SP, P - pb * SP);
  rem -= pb * sm * SP;
  tm = tmb * SM + rem / sp;
  p = pb * SP + rem % sp;
}

// one block tile of the generic engine: tile wgid (already XCD-remapped) of the (M, N) grid, z = blockIdx.z
template <int AM, int EPI, int OM, bool BVEC, int BK, int MT, int SCHED>
__device__ __forceinline__ void gemm_f32_tile(const GemmArgs& p, const int wgid, const int z) {
  typedef TileCfg<BK, MT> C;
  constexpr int BM = C::BM;
  __shared__ float As[2][BK * C::LDA];
  __shared__ float Bs[2][BK * C::LDB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int ntn = (p.N + BN - 1) / BN;
  const int tm = wgid / ntn, tn = wgid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;

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
    auto mfma_steps = [&](int s_lo, int s_hi) {
#pragma unroll
      for (int s2 = 0; s2 < BK / 2; ++s2) {
        if (s2 < s_lo || s2 >= s_hi) continue;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s2][i], fb[s2][0], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s2][i], fb[s2][1], acc[i][1], 0, 0, 0);
        }
      }
    };
    auto stage_next = [&]() {
      if (kt + 1 < nk) {
        store_a(cur ^ 1);
        store_b(cur ^ 1);
        if (kt + 2 < nk) {
          load_a(kbeg + (kt + 2) * BK);
          load_b(kbeg + (kt + 2) * BK);
        }
      }
    };
    if (SCHED == 0) {
      stage_next();
      mfma_steps(0, BK / 2);
    } else if (SCHED == 1) {
      // keep the MFMA block before the barrier (hipcc otherwise hoists the barrier and its
      // lgkmcnt(0) above the MFMAs, serialising the LDS writes in front of them)
      stage_next();
      mfma_steps(0, BK / 2);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      // first half of the MFMAs, then the LDS writes + next global loads, then the second half
      mfma_steps(0, BK / 4);
      __builtin_amdgcn_sched_barrier(0);
      stage_next();
      __builtin_amdgcn_sched_barrier(0);
      mfma_steps(BK / 4, BK / 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }

  gemm_epilogue<EPI, OM, MT>(p, acc, m0, n0, wm, wn, lane, z, py, px);
}

template <int AM, int EPI, int OM, bool BVEC, int BK, int OCC, int MT, int SCHED>
__global__ __launch_bounds__(256, OCC) void gemm_f32_kernel(GemmArgs p) {
  // XCD-aware tile remap (bijective for any grid size)
  gemm_f32_tile<AM, EPI, OM, BVEC, BK, MT, SCHED>(p, xcd_remap(blockIdx.x, gridDim.x), blockIdx.z);
}

// independent GEMMs of one shape class in one launch: group g owns the remapped tile ids [start[g], start[g+1]), so
// the tiles of all of them share the chip instead of each launch's last partial round idling half of it
template <int AM, int EPI, int OM, bool BVEC, int BK, int OCC, int MT, int SCHED>
__global__ __launch_bounds__(256, OCC) void gemm_f32_group_kernel(GemmGroup g) {
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  int j = 0;
#pragma unroll
  for (int t = 1; t < GEMM_GROUP_MAX; ++t) j += (t < g.n && wgid >= g.start[t]) ? 1 : 0;
  gemm_f32_tile<AM, EPI, OM, BVEC, BK, MT, SCHED>(g.a[j], wgid - g.start[j], 0);
}

// ================================================================================================
// Small fp32 GEMMs (the Q update's denoiser: B = 128-row activations times weights, and the weight gradients with
// K = B): C (M x N, ldc) = A (M x K row-major, lda) . B (K x N row-major, ldb) (+ bias[n]), exact fp32 products on
// v_mfma_f32_16x16x4f32 with fp32 accumulation.  One 16 x 16 output tile per wave, the whole K in one chain, operands
// straight from memory into registers (KU 16-k steps of loads in flight), so a 128 x 512 product is 256 waves in ONE
// launch -- the tiled engine gave it 4 workgroups, or split K into slabs plus a reduce launch.  Lane (m, q) supplies
// A[row m][k0 + 4 q + e] and B[k0 + 4 q + e][col m] to MFMA step e (proj16's k bijection).
template <int KU>
__global__ __launch_bounds__(256) void small_gemm_kernel(const float* __restrict__ A, long lda, const float* __restrict__ B,
                                                         long ldb, const float* __restrict__ bias, float* __restrict__ C,
                                                         long ldc, int M, int N, int K, int bias_mod, int act,
                                                         float slope) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntn = (N + 15) >> 4;
  const long tile = (long)blockIdx.x * 4 + wave;
  const int tm = (int)(tile / ntn), tn = (int)(tile - (long)tm * ntn);
  if (tm * 16 >= M) return;  // wave-uniform
  const int m = lane & 15, q = lane >> 4;
  const int row = tm * 16 + m, col = tn * 16 + m;
  const bool rok = row < M, cok = col < N;
  const float* Ar = A + (long)(rok ? row : 0) * lda;
  const float* Bc = B + (cok ? col : 0);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 16 * KU) {
    f32x4 a[KU], b[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {  // K % 4 == 0: a lane's 4 k are all in range or all out; loads from clamped
      const int k = k0 + 16 * u + 4 * q;  // (valid) addresses, then zeroed, so no load sits in a branch
      const bool kin = k < K;
      const int kk = kin ? k : 0;
      a[u] = *reinterpret_cast<const f32x4*>(Ar + kk);
#pragma unroll
      for (int e = 0; e < 4; ++e) b[u][e] = Bc[(long)(kk + e) * ldb];
      if (!(rok && kin)) a[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!(cok && kin)) b[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_sched_barrier(0);  // the KU steps' loads all in flight before the first MFMA waits
#pragma unroll
    for (int u = 0; u < KU; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][e], b[u][e], acc, 0, 0, 0);
  }
  if (!cok) return;
  const float bv = bias ? bias[bias_mod > 0 ? col % bias_mod : col] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = tm * 16 + 4 * q + r;
    if (rr < M) C[(long)rr * ldc + col] = act_apply(acc[r] + bv, act, slope);
  }
}

int launch_small_gemm(const float* A, long lda, const float* B, long ldb, const float* bias, float* C, long ldc, int M,
                      int N, int K, hipStream_t s, int bias_mod, int act, float slope) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < N || ldc < N) return DAMC_ERR_ARG;
  if (K % 4 != 0 || lda % 4 != 0 || (reinterpret_cast<uintptr_t>(A) & 15) != 0) return DAMC_ERR_UNSUPPORTED;  // f32x4 A
  ProfScope ps("small_gemm", 2.0 * M * N * K, s);
  const long tiles = (long)((M + 15) / 16) * ((N + 15) / 16);
  hipLaunchKernelGGL(small_gemm_kernel<4>, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, A, lda, B, ldb, bias, C,
                     ldc, M, N, K, bias_mod, act, slope);
  return (int)hipGetLastError();
}

// Up to SG_GROUP_MAX independent small GEMMs (SmallGemm, gemm.h) in ONE launch, one 16 x 16 output tile per 4-wave
// workgroup with K split over the waves in four contiguous runs of 16-k steps (a quarter of the single-wave kernel's
// dependent load rounds), the wave partials summed in LDS in a fixed order ((w0 + w1) + w2) + w3.  a_ones: A is a row of
// ones (M = 1): C = the column sums of B, the bias gradients of the denoiser's Linears as one more member of the group.
template <int KU>
__global__ __launch_bounds__(256) void small_gemm_group_kernel(SmallGemmGroup g) {
  __shared__ f32x4 red[3][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int blk = blockIdx.x;
  int gi = 0;
  while (gi + 1 < g.n && blk >= g.tile_end[gi]) ++gi;  // workgroup-uniform
  const SmallGemm& D = g.d[gi];
  const int tile = blk - (gi ? g.tile_end[gi - 1] : 0);
  const int M = D.M, N = D.N, K = D.K;
  const int ntn = (N + 15) >> 4;
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int m = lane & 15, q = lane >> 4;
  const int row = tm * 16 + m, col = tn * 16 + m;
  const bool rok = row < M, cok = col < N;
  const float* Ar = D.A + (long)(rok && !D.a_ones ? row : 0) * D.lda;
  const long ldb = D.ldb;
  const float* Bc = D.b_t ? D.B + (long)(cok ? col : 0) * ldb : D.B + (cok ? col : 0);
  const int k16 = (K + 15) >> 4, per = (k16 + 3) >> 2;
  const int kb = wave * per * 16, ke = min(K, kb + per * 16);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += 16 * KU) {
    f32x4 a[KU], b[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {  // K % 4 == 0: a lane's 4 k are all in range or all out
      const int k = k0 + 16 * u + 4 * q;
      const bool kin = k < ke;
      const int kk = kin ? k : 0;
      a[u] = D.a_ones ? f32x4{1.f, 1.f, 1.f, 1.f} : *reinterpret_cast<const f32x4*>(Ar + kk);
      if (D.b_t) {
        b[u] = *reinterpret_cast<const f32x4*>(Bc + kk);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) b[u][e] = Bc[(long)(kk + e) * ldb];
      }
      if (!(rok && kin)) a[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!(cok && kin)) b[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < KU; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][e], b[u][e], acc, 0, 0, 0);
  }
  if (wave) red[wave - 1][lane] = acc;
  __syncthreads();
  if (wave || !cok) return;
  acc = ((acc + red[0][lane]) + red[1][lane]) + red[2][lane];
  const float bv = D.bias ? D.bias[D.bias_mod > 0 ? col % D.bias_mod : col] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = tm * 16 + 4 * q + r;
    if (rr < M) D.C[(long)rr * D.ldc + col] = act_apply(acc[r] + bv, D.act, D.slope);
  }
}

int launch_small_gemm_group(const SmallGemm* g, int n, hipStream_t s) {
  if (n < 1 || n > SG_GROUP_MAX) return DAMC_ERR_ARG;
  SmallGemmGroup grp{};
  long tot = 0;
  double flops = 0.0;
  for (int i = 0; i < n; ++i) {
    const SmallGemm& d = g[i];
    if ((!d.A && !d.a_ones) || !d.B || !d.C || d.M <= 0 || d.N <= 0 || d.K <= 0 || d.ldb < (d.b_t ? d.K : d.N) ||
        d.ldc < d.N || (d.a_ones && d.M != 1) || (!d.a_ones && d.lda < d.K))
      return DAMC_ERR_ARG;
    if (d.K % 4 != 0 || (!d.a_ones && (d.lda % 4 != 0 || (reinterpret_cast<uintptr_t>(d.A) & 15) != 0)))
      return DAMC_ERR_UNSUPPORTED;  // f32x4 A
    if (d.b_t && (d.ldb % 4 != 0 || (reinterpret_cast<uintptr_t>(d.B) & 15) != 0)) return DAMC_ERR_UNSUPPORTED;
    grp.d[i] = d;
    tot += (long)((d.M + 15) / 16) * ((d.N + 15) / 16);
    if (tot >= (1L << 31)) return DAMC_ERR_UNSUPPORTED;
    grp.tile_end[i] = (int)tot;
    flops += 2.0 * d.M * d.N * d.K;
  }
  grp.n = n;
  ProfScope ps("small_gemm_group", flops, s);
  hipLaunchKernelGGL(small_gemm_group_kernel<4>, dim3((unsigned)tot), dim3(256), 0, s, grp);
  return (int)hipGetLastError();
}

// ================================================================================================
// K-major convolution engine (A_CONV with Cg % 32 == 0, B packed [n][k]).
//
// Both operands are staged k-contiguous: a global float4 (4 consecutive channels of one pixel, or 4
// consecutive k of one weight row) -> one ds_write_b128 -> the MFMA fragments come back as
// ds_read_b128 through a k-permutation (MFMA step s of k-quad q uses k = 8q + 4(lane>>5) + s, the same
// bijection on A and B, so every lane's 4 consecutive steps are one 16-B read).  Rows are padded to
// 36 floats: any 16 consecutive rows then cover all 64 banks, which makes both the b128 reads (16-lane
// groups of rows) and the b128 writes (8-lane groups along one row) conflict-free.
// Since a 32-wide K tile never straddles a filter tap, the tap walk is a scalar counter; each A row
// carries a bitmask of the taps that land inside the image (computed once), and every load is a
// buffer load whose offset is pushed out of the descriptor's range when the tap is padding, so the
// hardware returns zeros -- no per-load bounds arithmetic or exec-mask branches in the K loop.
constexpr int KM_BM = 128;
constexpr int KM_RS = KM_BK + 4;
constexpr unsigned KM_OOB = 0xF0000000u;  // any offset >= the descriptor size reads as zero

// PIPE 0: per tile {fragments of tile kt -> regs, stage tile kt+1, load tile kt+2, MFMAs, barrier}.
// PIPE 1: fragments register-prefetched one tile ahead; per tile {barrier, fragments of kt+1 -> regs,
//         stage tile kt+2, load tile kt+3, MFMAs of kt} so the MFMA operands are resident when the
//         barrier releases and the LDS traffic runs under the MFMAs.
#ifndef DAMC_KM_PIPE
#define DAMC_KM_PIPE 3
#endif
// DBG (timing experiments only, wrong results): 1 = every row loads the same cache lines,
// 2 = no global loads in the K loop
template <int EPI, int OM, int PIPE = DAMC_KM_PIPE, int DBG = 0>
__global__ __launch_bounds__(256, 2) void gemm_km_kernel(GemmArgs p) {
  constexpr int BK = KM_BK, RS = KM_RS, BM = KM_BM, MT = 2;
  __shared__ __attribute__((aligned(16))) float As[2][BM * RS];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * RS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntn = (p.N + BN - 1) / BN;
  const int tm = wgid / ntn, tn = wgid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.z;

  int pad_y = p.pad_y, pad_x = p.pad_x, py = 0, px = 0;
  const float* Bg = p.B;
  if (OM == O_PHASE) {
    py = z >> 1;
    px = z & 1;
    pad_y = 1 - py;
    pad_x = 1 - px;
    Bg += (long)z * p.b_zstride;
  }
  const int Cg = p.Cg, kw = p.kw, Win = p.Win;
  const int kh = p.K / Cg / kw;
  // O_DENSE: blockIdx.z is a split-K slice [kbeg, kend) (k_per_z a multiple of BK)
  const int kbeg = (OM == O_DENSE) ? z * p.k_per_z : 0;
  const int kend = (OM == O_DENSE) ? min(p.K, kbeg + p.k_per_z) : p.K;
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  const int hwq = p.Hq * p.Wq;
  const int nimg = (p.M + hwq - 1) / hwq;
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, nimg * p.Hin * Win * Cg * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)Bg, (short)0, p.N * (int)p.ldb * 4, 0x00020000);

  // ---- per-thread rows: A rows / B rows (tid>>3) + 32j, float4 slot tid&7 of the K tile
  const int q4 = tid & 7, r0 = tid >> 3;
  int abase[4];
  unsigned amask[4], boff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + r0 + 32 * j;
    unsigned msk = 0;
    int base = 0;
    if (m < p.M) {
      const int b = m / hwq;
      const int r = m - b * hwq;
      const int qy = r / p.Wq, qx = r - qy * p.Wq;
      const int iy0 = qy * p.stride - pad_y, ix0 = qx * p.stride - pad_x;
      base = ((b * p.Hin + iy0) * Win + ix0) * Cg;
      for (int ky = 0; ky < kh; ++ky)
        for (int kx = 0; kx < kw; ++kx)
          if ((unsigned)(iy0 + ky) < (unsigned)p.Hin && (unsigned)(ix0 + kx) < (unsigned)Win)
            msk |= 1u << (ky * kw + kx);
    }
    abase[j] = base * 4 + q4 * 16;
    amask[j] = msk;
    boff[j] = (unsigned)((n0 + r0 + 32 * j) * (int)p.ldb * 4 + q4 * 16);  // rows >= N fall out of range
    if (DBG == 1) {
      abase[j] = q4 * 16;
      amask[j] = 0xFFFFFFFFu;
      boff[j] = q4 * 16;
    }
  }

  // ---- scalar tap walk over the K tiles still to be loaded
  int tap = kbeg / Cg, ci0 = kbeg - (kbeg / Cg) * Cg;
  int tky = tap / kw, tkx = tap - (tap / kw) * kw;
  unsigned aoff[4];
  auto set_tap = [&]() {
    const int toff = DBG == 1 ? 0 : (tky * Win + tkx) * Cg * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) aoff[j] = ((amask[j] >> (tap & 31)) & 1u) ? (unsigned)(abase[j] + toff) : KM_OOB;
  };
  set_tap();
  f32x4 ra[4], rb[4];
  auto load_ab = [&](int k0) {
    if (DBG == 2) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      ra[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, (int)aoff[j], DBG == 1 ? 0 : ci0 * 4, 0));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      rb[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsB, (int)boff[j], DBG == 1 ? 0 : k0 * 4, 0));
    ci0 += BK;
    if (ci0 == Cg) {
      ci0 = 0;
      ++tap;
      if (++tkx == kw) {
        tkx = 0;
        ++tky;
      }
      set_tap();
    }
  };
  // branch-free form for the interleaved pipelines (one basic block per K step): a tile past the end
  // of K loads nothing (every offset out of range) and the tap walk advances with selects
  auto load_ab_nb = [&](int k0) {
    const bool live = k0 < kend;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      ra[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, (int)(live ? aoff[j] : KM_OOB), ci0 * 4, 0));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      rb[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsB, (int)(live ? boff[j] : KM_OOB), k0 * 4, 0));
    ci0 += BK;
    const int wrap = ci0 == Cg;
    ci0 = wrap ? 0 : ci0;
    tap = min(tap + wrap, 31);
    tkx += wrap;
    const int wx = tkx == kw;
    tkx = wx ? 0 : tkx;
    tky += wx;
    set_tap();
  };
  auto store_ab = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *reinterpret_cast<f32x4*>(&As[buf][(r0 + 32 * j) * RS + 4 * q4]) = ra[j];
      *reinterpret_cast<f32x4*>(&Bs[buf][(r0 + 32 * j) * RS + 4 * q4]) = rb[j];
    }
  };

  f32x16 acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lrow = lane & 31, lk = lane >> 5;
  const int afr = (wm * 64 + lrow) * RS + 4 * lk, bfr = (wn * 64 + lrow) * RS + 4 * lk;
  auto read_frags = [&](int buf, f32x4 (&fa)[4][MT], f32x4 (&fb)[4][2]) {
    const float* as = As[buf];
    const float* bs = Bs[buf];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int i = 0; i < MT; ++i) fa[q][i] = *reinterpret_cast<const f32x4*>(as + afr + 32 * i * RS + 8 * q);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[q][j] = *reinterpret_cast<const f32x4*>(bs + bfr + 32 * j * RS + 8 * q);
    }
  };
  auto mfma_tile = [&](const f32x4 (&fa)[4][MT], const f32x4 (&fb)[4][2]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q][i][s2], fb[q][0][s2], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q][i][s2], fb[q][1][s2], acc[i][1], 0, 0, 0);
        }
  };

  constexpr int SG_MFMA = 0x8, SG_VMEM_RD = 0x20, SG_DS_RD = 0x100, SG_DS_WR = 0x200;
  if (PIPE == 0 || PIPE == 2) {  // PIPE >= 3: the prefetch structure below
    if (nk > 0) {
      load_ab(kbeg);
      store_ab(0);
      if (nk > 1) load_ab(kbeg + BK);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      f32x4 fa[4][MT], fb[4][2];
      if (PIPE == 0) {
        read_frags(cur, fa, fb);
        if (kt + 1 < nk) {
          store_ab(cur ^ 1);
          if (kt + 2 < nk) load_ab(kbeg + (kt + 2) * BK);
        }
        mfma_tile(fa, fb);
      } else {
        // stores past the last tile land in the buffer nobody reads again; loads past K are empty
        read_frags(cur, fa, fb);
        store_ab(cur ^ 1);
        load_ab_nb(kbeg + (kt + 2) * BK);
        mfma_tile(fa, fb);
        // the first k-quad's 4 fragments, then the remaining reads, stores and loads one per MFMA
        __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 4, 0);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 1, 0);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_WR, 1, 0);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
          __builtin_amdgcn_sched_group_barrier(SG_VMEM_RD, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 36, 0);
      }
      __syncthreads();
    }
  } else {
    // prologue: tiles 0 and 1 staged, tile 2 in flight, fragments of tile 0 resident
    if (nk > 0) {
      load_ab(kbeg);
      store_ab(0);
      if (nk > 1) {
        load_ab(kbeg + BK);
        store_ab(1);
        if (nk > 2) load_ab(kbeg + 2 * BK);
      }
    }
    __syncthreads();
    f32x4 f0a[4][MT], f0b[4][2], f1a[4][MT], f1b[4][2];
    if (nk > 0) read_frags(0, f0a, f0b);
    auto step = [&](int kt, const f32x4 (&fca)[4][MT], const f32x4 (&fcb)[4][2], f32x4 (&fna)[4][MT],
                    f32x4 (&fnb)[4][2]) {
      __syncthreads();
      if (PIPE == 1) {
        if (kt + 1 < nk) read_frags((kt + 1) & 1, fna, fnb);
        if (kt + 2 < nk) {
          store_ab(kt & 1);
          if (kt + 3 < nk) load_ab(kbeg + (kt + 3) * BK);
        }
        mfma_tile(fca, fcb);
      } else {
        read_frags((kt + 1) & 1, fna, fnb);
        store_ab(kt & 1);
        load_ab_nb(kbeg + (kt + 3) * BK);
        mfma_tile(fca, fcb);
        // one LDS read / LDS write / global load per MFMA gap, so every wave always has MFMAs ready
        if (PIPE == 3) {  // 16 reads, 8 writes, 8 loads on the first 32 MFMAs
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 1, 0);
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_DS_WR, 1, 0);
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_VMEM_RD, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 32, 0);
        } else if (PIPE == 4) {  // the same order spread over all 64 MFMAs
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_DS_WR, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_VMEM_RD, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
          }
        } else {  // PIPE 5: global loads first (they have the longest latency), then reads, then writes
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_DS_WR, 1, 0);
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_VMEM_RD, 1, 0);
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
            __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 32, 0);
        }
      }
    };
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, f0a, f0b, f1a, f1b);
      if (kt + 1 < nk) step(kt + 1, f1a, f1b, f0a, f0b);
    }
  }
  if (OM == O_PHASE) {
    // one row-offset division per row instead of one per (row, lane): table in the (drained) A buffer
    long* rowtab = reinterpret_cast<long*>(&As[0][0]);
    __syncthreads();
    if (tid < BM) rowtab[tid] = gemm_row_offset<OM>(p, m0 + tid, py, px);
    __syncthreads();
    gemm_epilogue<EPI, OM, MT>(p, acc, m0, n0, wm, wn, lane, z, py, px, rowtab);
  } else {
    gemm_epilogue<EPI, OM, MT>(p, acc, m0, n0, wm, wn, lane, z, py, px);
  }
}

// The first layer's input gradient at per-rank batches (dz_slabs: M = B <= 32 dense rows as a 1 x 1 "convolution",
// split-K slices of k_per_z, EPI_STORE into per-slice slabs): one workgroup per (slice, 128 columns), 4 waves of 32
// columns, every fragment straight from memory into registers with 4 K tiles' loads in flight (the 128 x 128 kernel
// walks a slice's 8 K tiles through a 2-3 deep LDS pipeline, latency-bound at this size).  The same 32x32x2 MFMA
// sequence per output (k-quad q, then step s; lane half lk takes k = 8 q + 4 lk + s of each 32-deep tile) from zero
// per slice, so every slab value is bitwise gemm_km_kernel's.
// MT = 2 (round 5, DAMC_KM_SKINNY_MT=2 since round 6): M <= 64 as two 32-row tiles per wave (SVHN's per-config batch of 64 at nz = 100 left the tiled
// kernel 22 us for a 52 MFLOP product), two K tiles' loads in flight so the fragments stay within the VGPRs
template <int MT>
__global__ __launch_bounds__(256) void km_skinny_kernel(GemmArgs p) {
  constexpr int KU = 4 / MT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lrow = lane & 31, lk = lane >> 5;
  // blockIdx.z: 32 MT-row block of the rows (round 5: M up to 128 as two 64-row blocks)
  const int z = blockIdx.x, n0 = blockIdx.y * 128 + wave * 32, rb0 = blockIdx.z * 32 * MT;
  const int kbeg = z * p.k_per_z, kend = min(p.K, kbeg + p.k_per_z);
  const int nk = kend > kbeg ? (kend - kbeg) / KM_BK : 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.Cg * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.N * (int)p.ldb * 4, 0x00020000);
  constexpr int OOB = 0x7FFFFFF0;
  int aoff[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
    aoff[t] = rb0 + 32 * t + lrow < p.M ? ((rb0 + 32 * t + lrow) * p.Cg + 4 * lk) * 4 : OOB;
  const int boff = n0 + lrow < p.N ? ((n0 + lrow) * (int)p.ldb + 4 * lk) * 4 : OOB;
  f32x16 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  for (int kt = 0; kt < nk; kt += KU) {
    f32x4 fa[MT][KU][4], fb[KU][4];
#pragma unroll
    for (int u = 0; u < KU; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool live = kt + u < nk;
        const int k0 = (kbeg + (kt + u) * KM_BK + 8 * q) * 4;
#pragma unroll
        for (int t = 0; t < MT; ++t)
          fa[t][u][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      ra, live ? aoff[t] : OOB, live ? k0 : 0, 0));
        fb[u][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rb, live ? boff : OOB, live ? k0 : 0, 0));
      }
    __builtin_amdgcn_sched_barrier(0);  // every load of the batch issued before the first MFMA waits on one
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (kt + u >= nk) break;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int t = 0; t < MT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[t][u][q][s2], fb[u][q][s2], acc[t], 0, 0, 0);
    }
  }
  float* Cz = p.C + (long)z * p.c_zstride;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = rb0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * lk, n = n0 + lrow;
      if (m < p.M && n < p.N) Cz[(long)m * p.ldc + n] = acc[t][r];
    }
}

template <int EPI, int OM, int PIPE = DAMC_KM_PIPE, int DBG = 0>
static void launch_km_t(const GemmArgs& a, int zdim, hipStream_t s) {
  const int ntm = (a.M + KM_BM - 1) / KM_BM, ntn = (a.N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_km_kernel<EPI, OM, PIPE, DBG>), dim3(ntm * ntn, 1, zdim), dim3(256), 0, s, a);
}

// K-major dispatch; splits the batch so every launch's gathered tensor stays below 2^31 bytes
static int launch_gemm_km(const GemmArgs& a, Epi epi, OMode om, int zdim, hipStream_t s) {
  const int taps = a.Cg > 0 ? a.K / a.Cg : 0;
  if (!conv_kmajor_ok(a.Cg) || taps * a.Cg != a.K || a.kw <= 0 || taps % a.kw != 0 || taps > 32) return DAMC_ERR_ARG;
  if (om == O_PHASE && zdim != 4) return DAMC_ERR_ARG;
  if (om == O_DENSE && (a.k_per_z <= 0 || a.k_per_z % KM_BK != 0 ||
                        (long)zdim * a.k_per_z < a.K || (long)(zdim - 1) * a.k_per_z >= a.K))
    return DAMC_ERR_ARG;
  if (a.ldb < a.K || ((uintptr_t)a.A | (uintptr_t)a.B) % 16 != 0 || (a.ldb % 4) != 0) return DAMC_ERR_ARG;
  if ((double)a.N * a.ldb * 4 >= 2147483647.0) return DAMC_ERR_UNSUPPORTED;
  const long hwq = (long)a.Hq * a.Wq;
  if (a.M % hwq != 0) return DAMC_ERR_ARG;
  const long img = (long)a.Hin * a.Win * a.Cg;  // floats per gathered image
  const long nimg = a.M / hwq;
  // DAMC_KM_CHUNK_BYTES lowers the per-launch limit (tests exercise the chunked path on small inputs)
  static const long lim = [] {
    const char* e = getenv("DAMC_KM_CHUNK_BYTES");
    const long v = e ? atol(e) : 0;
    return (v > 0 && v < 2147483647L) ? v : 2147483647L;
  }();
  const long per = (lim / 4 - 1) / img;
  if (per < 1) return DAMC_ERR_UNSUPPORTED;
  const long cimg = (om == O_PHASE) ? (long)a.Hout * a.Wout * a.ldc : hwq * a.ldc;  // output floats per image
  for (long b0 = 0; b0 < nimg; b0 += per) {
    const long nb = std::min(per, nimg - b0);
    GemmArgs c = a;
    c.A = a.A + b0 * img;
    c.C = a.C + b0 * cimg;
    if (a.mask) c.mask = a.mask + b0 * cimg;
    c.M = (int)(nb * hwq);
    // dz_slabs at per-rank batches: km_skinny_kernel (bitwise gemm_km_kernel); DAMC_KM_SKINNY=0 (read per call) keeps
    // the tiled kernel
    const char* esk = getenv("DAMC_KM_SKINNY");
    // rows: up to 64 (two 32-row tiles per wave); DAMC_KM_SKINNY_ROWS (read per call) moves the limit for A/B (128, as
    // two 64-row blocks: 38.3 us against the tiled kernel's 28.6 at the headline's B = 128, profiles/r05/skinny128_ab.txt)
    const char* ekr = getenv("DAMC_KM_SKINNY_ROWS");
    const int km_rows = ekr ? atoi(ekr) : 64;
    if (epi == EPI_STORE && om == O_DENSE && c.M <= km_rows && c.Hin == 1 && c.Win == 1 && c.Hq == 1 && c.Wq == 1 &&
        c.kw == 1 && c.Cg == c.K && !(esk && esk[0] == '0')) {
      // rows in 32-row workgroups of km_skinny_kernel<1> (round 6: SVHN B=64's two workgroups per slice took 11.4 us
      // against 17.2 for one 64-row workgroup of <2>, half the MFMA chain per wave, profiles/r06/km_skinny_mt.txt);
      // DAMC_KM_SKINNY_MT=2 (read per call) keeps <2> for 33-64 rows
      const char* emt = getenv("DAMC_KM_SKINNY_MT");
      const bool mt1 = c.M <= 32 || !(emt && emt[0] == '2');
      const dim3 g((unsigned)zdim, (unsigned)((c.N + 127) / 128), (unsigned)((c.M + (mt1 ? 31 : 63)) / (mt1 ? 32 : 64)));
      if (mt1)
        hipLaunchKernelGGL(km_skinny_kernel<1>, g, dim3(256), 0, s, c);
      else
        hipLaunchKernelGGL(km_skinny_kernel<2>, g, dim3(256), 0, s, c);
      continue;
    }
#define DAMC_KM(E_, O_)                \
  if (epi == E_ && om == O_) {         \
    launch_km_t<E_, O_>(c, zdim, s);   \
    continue;                          \
  }
    DAMC_KM(EPI_BIAS_ACT, O_PHASE)
    DAMC_KM(EPI_MASK, O_DENSE)
    DAMC_KM(EPI_BIAS_ACT, O_DENSE)
    DAMC_KM(EPI_STORE, O_DENSE)
#undef DAMC_KM
    return DAMC_ERR_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

// ================================================================================================
// Limb engine: fp32-accurate convolution GEMM on bf16 MFMA.
//
// Every fp32 operand value a is carried as three bf16 limbs a = a0 + a1 + a2 (RNE splits: a0 = bf16(a),
// a1 = bf16(a - a0), a2 = bf16(a - a0 - a1); both subtractions are exact, so the limbs hold all 24
// significand bits).  A product a*b is the sum of the six limb products with i + j <= 2; the dropped
// three are below 2^-23 |ab|.  Each limb product is exact in the MFMA (8 x 8 significand bits) and the
// sum is accumulated in fp32 by v_mfma_f32_32x32x16_bf16, smallest terms first.  Error against fp64 is
// the fp32 GEMM's (tools/gemm_bench.hip prints both), at 16/6 of the fp32-MFMA rate per clock.
//
// "x3" tensor layout: a row of C channels is C/8 octets, each octet stored as [limb][8] bf16 (48 B), so
// a 32-channel K tile of one row is 192 contiguous bytes.  The A operand is an NHWC x3 map gathered by
// the same tap walk as the K-major engine (a K tile never straddles a tap, padding taps read zero
// through an out-of-range buffer offset); B is x3 over K, [n][K/8][3][8].
//
// Block 256 x 128, 8 waves (4 along M x 2 along N), each wave 64 x 64 of accumulators.
// LDS rows are the 192 B of a K tile, unpadded, with the four 48-B octets of row r stored at octet
// position q ^ ((r >> 1) & 3): the ds_read_b128 lane groups of a 16x16x32 fragment read ({0-3,12-15,
// 20-27}, ...) then hit 16 distinct 4-bank groups, and the staging writes are lane-linear (each thread
// stores the PHYSICAL chunk id % 12 of row id / 12 and gathers the matching logical chunk), so 8-lane
// write groups are contiguous.  Double-buffered: 2 x 384 rows x 192 B = 147,456 B, one workgroup per CU.
constexpr int X3_BM = 256, X3_BN = 128, X3_BK = 32, X3_ROWB = 192;
__device__ __forceinline__ int x3_swz(int row) { return (row >> 1) & 3; }
// F32A (variant bit 2097152): the A operand staged as fp32, one 128-B row of 8 16-B chunks per K tile, physical chunk
// = logical chunk ^ f32a_swz(row & 15).  A lane of a 16x16x32 fragment read (row lane & 15, octet q = lane >> 4)
// takes logical chunks 2q and 2q + 1 in two ds_read_b128; with u = (r >> 1) & 7 and the bit-1 flip on rows 4-11
// (the rows the b128 lane groups pair with the other octet) every 16-lane group hits 16 distinct 4-bank groups.
constexpr int X3_F32A = 2097152, X3A_ROWB = 128;
// X3_NARROW (variant bit 4194304): a 64 x 128 block tile, 8 waves 2 (M) x 4 (N) of 32 x 32 (2 x 2 MFMA tiles each),
// 74 KB of LDS so two workgroups share a CU: a small-batch conv fills the chip without split-K slabs (every output
// takes the default tile's MFMA sequence, so it is bitwise the default and the split forms)
constexpr int X3_NARROW = 4194304;
// split-K with the in-GEMM ordered fix-up (GemmArgs::kticket; the F32A register-slab path): the last workgroup of a
// tile to arrive sums the tile's slabs in slab order and runs the unsplit epilogue, so no reduce launch follows
constexpr int X3_FIXUP = 8388608;
constexpr int X3_FIXUP_WAIT = 3000;  // the fix-up's bounded wait for the other slices: 30 us of s_memrealtime (100 MHz)
static unsigned* g_fixup_probe = nullptr;  // damc_x3_fixup_probe (diagnostics)
__device__ __forceinline__ int f32a_swz(int r) { return ((r >> 1) & 7) ^ ((((r >> 2) ^ (r >> 3)) & 1) << 1); }
static_assert(X3_NEGK % 32 == 0 && (X3_NEGK & (X3_NEGK - 1)) == 0, "sign blocks are whole K tiles, a power of two");
constexpr int X3_CHUNKS = 12;  // 16-B chunks per row and K tile (4 octets x 3 limbs)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// V: variant bits (tools/gemm_bench.hip A/B): 256 = fragment reads in MFMA order (below), 1 = v_mfma_f32_16x16x32_bf16 on a 4x4 grid of 16x16 tiles per
// wave, 2 = s_setprio(1) around the MFMA cluster, 4 = LDS-DMA staging (buffer_load ... lds straight into
// the lane-linear LDS image, issued one K tile ahead; no staging registers or ds_write), 16 = supertile
// raster (32 = one MFMA accumulation chain over all of K: no blocking, no sign alternation; A/B only) (a 1-D grid; each XCD's 32 concurrent workgroups form a block of <= 8 M tiles x 4 (N tile, phase) pairs
// with the 4 phases of an N tile adjacent, so the phases' overlapping input windows and the weight panels are
// shared in L2 instead of every XCD streaming all phases' panels; DMA and non-WGRAD only)
#ifndef DAMC_X3_VARIANT
#define DAMC_X3_VARIANT 261  // measured best (profiles/r02/gemm_bench_rdorder.txt; round 1: 5)
#endif
// RNE limb split of 8 consecutive values: v = h + m + l (to 24 significand bits)
__device__ __forceinline__ void split3_octet(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 b0 = (__bf16)v[e];
    const float r1 = sub_rn(v[e], (float)b0);
    const __bf16 b1 = (__bf16)r1;
    const float r2 = sub_rn(r1, (float)b1);
    h[e] = b0;
    m[e] = b1;
    l[e] = (__bf16)r2;
  }
}

// Output-layer projection of 16 rows of an LDS tile (row stride ts floats, C channels, C % 16 == 0) on
// v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation): lane (row m = lane & 15, quarter q = lane >> 4) reads
// the f32x4 run c = 16 g + 4 q .. + 3 of its row and of weight row n = 16 t + m, element e feeding MFMA step e (one k
// bijection for both operands).  acc[t][r] = P[row r0 + 4 q + r][16 t + m].  gemm_x3_kernel's fused epilogue and
// proj_rows_kernel share it, so the two forms are bitwise equal.
template <int NT>
__device__ __forceinline__ void proj16(const float* tile, int ts, int r0, int C, const float* w, int ldw,
                                       f32x4 (&acc)[NT]) {
  const int lane = threadIdx.x & 63, m = lane & 15, q = lane >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int g = 0; g < C / 16; ++g) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(tile + (r0 + m) * ts + 16 * g + 4 * q);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(w + (long)(16 * t + m) * ldw + 16 * g + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[e], acc[t], 0, 0, 0);
    }
  }
}

// proj16 with the b operands preloaded into registers (w[g][t] = weight row 16 t + m, k = 16 g + 4 q .. + 3, as
// x3_ksplit_reduce_proj_kernel holds them): the same MFMA sequence per output, so bitwise proj16
template <int NT>
__device__ __forceinline__ void proj16_pre(const float* tile, int ts, int r0, int C, const f32x4 (&w)[PROJ_CHUNK / 16][4],
                                           f32x4 (&acc)[NT]) {
  const int lane = threadIdx.x & 63, m = lane & 15, q = lane >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < PROJ_CHUNK / 16; ++g) {
    if (16 * g >= C) break;
    const f32x4 a = *reinterpret_cast<const f32x4*>(tile + (r0 + m) * ts + 16 * g + 4 * q);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], w[g][t][e], acc[t], 0, 0, 0);
  }
}

// the projection alone: 128 pixels per workgroup (8 waves x 16 rows) staged in LDS with gemm_x3_kernel's WIDE tile
// stride, then proj16 (NT = np / 16) per 128-channel chunk (PROJ_CHUNK): chunk j's chain goes to partial buffer j
// (P + j npix np), and the gather adds the partials in order -- the chunking of the F32A tile's fused projection, whose
// workgroups each hold one 128-channel N tile
template <int NT>
__global__ __launch_bounds__(512) void proj_rows_kernel(const float* __restrict__ h, long npix, int C,
                                                        const float* __restrict__ w, int ldw, float* __restrict__ P,
                                                        long pstride) {
  constexpr int TS = 256 + 4;
  __shared__ __attribute__((aligned(16))) float tile[128 * TS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long p0 = (long)blockIdx.x * 128;
  const int c4 = C / 4;
  for (int i = tid; i < 128 * c4; i += 512) {
    const int r = i / c4, c = (i - r * c4) * 4;
    const long pix = p0 + r;
    *reinterpret_cast<f32x4*>(tile + r * TS + c) =
        pix < npix ? *reinterpret_cast<const f32x4*>(h + pix * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  const int m = lane & 15, q = lane >> 4;
  for (int c0 = 0; c0 < C; c0 += PROJ_CHUNK) {  // one chain per 128-channel chunk, into its own partial buffer
    f32x4 acc[NT];
    proj16<NT>(tile + c0, TS, wave * 16, min(PROJ_CHUNK, C - c0), w + c0, ldw, acc);
    float* Pc = P + (c0 / PROJ_CHUNK) * pstride;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long pix = p0 + wave * 16 + 4 * q + r;
        if (pix < npix) Pc[pix * (16 * NT) + 16 * t + m] = acc[t][r];
      }
  }
}

int launch_proj_rows(const float* h, long npix, int C, const float* w, int ldw, int np, float* P, long pstride,
                     hipStream_t s) {
  if (C <= 0 || C > 256 || C % 16 || (np != 32 && np != 64) || npix <= 0) return DAMC_ERR_ARG;
  if (C > PROJ_CHUNK && pstride < npix * np) return DAMC_ERR_ARG;
  const dim3 grid((unsigned)((npix + 127) / 128));
  if (np == 32)
    hipLaunchKernelGGL(proj_rows_kernel<2>, grid, dim3(512), 0, s, h, npix, C, w, ldw, P, pstride);
  else
    hipLaunchKernelGGL(proj_rows_kernel<4>, grid, dim3(512), 0, s, h, npix, C, w, ldw, P, pstride);
  return (int)hipGetLastError();
}

template <int EPI, int OM, int V = DAMC_X3_VARIANT>
__global__ __launch_bounds__(512, (V & X3_NARROW) ? 2 : 1) void gemm_x3_kernel(GemmArgs p) {
  constexpr bool M16 = (V & 1) != 0;
  // 262144: 16-deep K stages in a 4-slot LDS ring (three stages in flight across raw barriers, counted vmcnt), each
  // MFMA taking two limb products over 16 k (P16 main loop below)
  constexpr bool P16 = (V & 262144) != 0;
  constexpr bool DMA_OK_P16 = (V & 4) != 0;
  // 524288: a 128 x 256 block tile (waves 2 along M x 4 along N, each still 64 x 64) instead of 256 x 128: no
  // half-empty tile at M = 128 (the first layer, M = B) and half the A gather per K tile
  constexpr bool WIDE = (V & 524288) != 0;
  static_assert(!(WIDE && P16), "one layout variant at a time");
  constexpr bool NARROW = (V & X3_NARROW) != 0;
  static_assert(!NARROW || (!WIDE && !P16 && M16 && (V & 4) && !(V & (8 | 16 | 32 | 64 | 2048 | 1048576 | 2097152))),
                "NARROW: the default LDS-DMA tap-major path, unsplit");
  constexpr int BM = WIDE ? 128 : NARROW ? 64 : X3_BM, BN = WIDE ? 256 : X3_BN;
  // X3_F32A: A staged as fp32 (4 B per element instead of 6 B of limbs) and split into its RNE limbs in registers after
  // the fragment read, the same split as the producing epilogue's, so the MFMA operands and results are bitwise the
  // limb path's; waves 8 along M x 1 along N (each 32 x 128), so every A element is split by one wave only
  constexpr bool F32A = (V & X3_F32A) != 0;
  static_assert(!F32A || (OM != O_WGRAD && M16 && (V & 4) && (V & 256) && !WIDE && !P16 &&
                          !(V & (32 | 64 | 512 | 1024 | 2048 | 4096 | 8192 | 16384 | 32768 | 65536 | 131072))),
                "F32A: the default 16x16-tile LDS-DMA path (A/B builds: + the channel-major walk 8, the raster 16)");
  constexpr int AROWB = F32A ? X3A_ROWB : X3_ROWB, ESZ = F32A ? 4 : 6;
  constexpr int AJ = (BM * (F32A ? 8 : X3_CHUNKS) + 511) / 512, BJ = BN * X3_CHUNKS / 512;  // NARROW: 1.5 -> 2
  constexpr int BUFB = BM * AROWB + BN * X3_ROWB;  // one LDS buffer (A image, then B image)
  // K tiles per MFMA accumulation block = the GEMM's sign block (GemmArgs::negk, a power of two >= 32); 64: A/B of
  // the block length (no b_negblk)
  const int FLOG = __builtin_ctz((unsigned)p.negk >> 5) + ((V & 64) ? 2 : 0), FLUSH = 1 << FLOG;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * (BM + BN) * X3_ROWB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = (WIDE || NARROW) ? wave >> 2 : wave >> 1, wn = (WIDE || NARROW) ? wave & 3 : wave & 1;
  unsigned long long clk_t0 = 0, clk_r0 = 0;
  if (p.clk && tid == 0) {
    clk_t0 = __builtin_amdgcn_s_memtime();
    clk_r0 = __builtin_amdgcn_s_memrealtime();
  }
  constexpr bool RASTER = (V & 16) != 0 && OM != O_WGRAD;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntn = (p.N + BN - 1) / BN;
  int tm, tn, z;
  if constexpr (RASTER) {
    const int nph = OM == O_PHASE ? 4 : 1;
    const int ntm = (p.M + BM - 1) / BM;
    int pr;
    supertile(wgid, ntm, ntn * nph, tm, pr);
    tn = pr / nph;
    z = pr - tn * nph;
  } else {
    tm = wgid / ntn;
    tn = wgid - tm * ntn;
    z = blockIdx.z;
  }
  const int m0 = tm * BM, n0 = tn * BN;

  int pad_y = p.pad_y, pad_x = p.pad_x, py = 0, px = 0;
  const unsigned short* Bg = p.B3;
  // split-K (O_PHASE / O_DENSE): z = phase * (ksplit / kbpw) + workgroup slice of kbpw sign blocks
  const bool KSPLIT = OM != O_WGRAD && p.ksplit > 1;
  // split-K into register-layout slabs (GemmArgs::kslab_reg; launched only split, 256 x 128 16x16-tile path): a
  // compile-time variant, so the block-total registers of the unsplit kernel drop out
  constexpr bool KREG = (V & 1048576) != 0;
  static_assert(!KREG || (M16 && !(V & (32 | 2048 | 65536 | 131072 | 262144 | 524288))), "KREG: default tiles only");
  // in-GEMM ordered fix-up of the split-K slabs (round 6; the protocol is described where the epilogue runs it)
  constexpr bool FIXUP = (V & X3_FIXUP) != 0;
  static_assert(!FIXUP || (KREG && F32A), "FIXUP: the F32A register-slab split-K path");
  const int nslz = KSPLIT ? p.ksplit / p.kbpw : 1;
  const int zph = KSPLIT ? z / nslz : z, zsl = KSPLIT ? z - zph * nslz : 0;
  if (OM == O_PHASE) {
    py = zph >> 1;
    px = zph & 1;
    pad_y = 1 - py;
    pad_x = 1 - px;
    Bg += (long)zph * p.b_zstride * 3;
  }
  int kbeg = 0, kend = p.K;
  if (KSPLIT) {
    kbeg = zsl * p.k_per_z;
    kend = min(p.K, kbeg + p.k_per_z);
  }
  if constexpr (OM == O_WGRAD) {  // z = phase * slices + split-K slice
    const int nsl = gridDim.z / p.wg_phases;
    const int ph = z / nsl, sl = z - ph * nsl;
    if (p.wg_phases == 4) {
      py = ph >> 1;
      px = ph & 1;
      pad_y = 1 - py;
      pad_x = 1 - px;
    } else {
      pad_y = pad_x = 0;
    }
    Bg += (long)ph * p.b_zstride * 3;
    kbeg = sl * p.k_per_z;
    kend = min(p.K, kbeg + p.k_per_z);
  }
  const int Cg = p.Cg, kw = p.kw, Win = p.Win;
  const int kh = p.K / Cg / kw;
  const int nk = (OM == O_WGRAD || KSPLIT) ? max(kend - kbeg, 0) / X3_BK : p.K / X3_BK;
  const int kt0 = kbeg / X3_BK;  // global index of the first K tile (sign blocks follow the global index)
  const int hwq = p.Hq * p.Wq;
  const int nimg = (p.M + hwq - 1) / hwq;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      F32A ? (void*)p.A : (void*)p.A3, (short)0, (OM == O_WGRAD) ? Cg * p.K * 6 : nimg * p.Hin * Win * Cg * ESZ,
      0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)Bg, (short)0, p.N * p.K * 6, 0x00020000);

  // ---- per-thread chunks: chunk id = tid + 512 j -> (row id / 12, 16-B chunk id % 12)
  int abase[AJ];
  unsigned amask[AJ], boff[BJ];
  int alds[AJ], blds[BJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    // P16: 16-deep K stages, rows of 6 chunks in global order (the first X3P_AJ entries are used)
    const int nch = F32A ? 8 : P16 ? 6 : X3_CHUNKS;
    const int id = tid + 512 * j, row = id / nch, ch = id - row * nch;
    const int m = m0 + row;
    unsigned msk = 0;
    int base = 0;
    if constexpr (OM == O_WGRAD) {
      // row m = (tap, ci): A row ci shifted by (dy, dx) pixels = (dy * Win + dx) * wg_bp elements; the shift
      // is packed into the mask word ((dy+1) | (dx+1) << 2), all-ones for rows beyond M
      msk = 0xFFFFFFFFu;
      if (m < p.M) {
        const int t = m / Cg, ci = m - t * Cg;
        const int ty = t / kw, tx = t - ty * kw;
        const int dy = ty - pad_y, dx = tx - pad_x;
        base = ci * p.K + (dy * Win + dx) * p.wg_bp;
        msk = (unsigned)(dy + 1) | ((unsigned)(dx + 1) << 2);
      }
    } else if (m < p.M) {
      const int b = m / hwq;
      const int r = m - b * hwq;
      const int qy = r / p.Wq, qx = r - qy * p.Wq;
      const int iy0 = qy * p.stride - pad_y, ix0 = qx * p.stride - pad_x;
      base = ((b * p.Hin + iy0) * Win + ix0) * Cg;
      for (int ky = 0; ky < kh; ++ky)
        for (int kx = 0; kx < kw; ++kx)
          if ((unsigned)(iy0 + ky) < (unsigned)p.Hin && (unsigned)(ix0 + kx) < (unsigned)Win)
            msk |= 1u << (ky * kw + kx);
    }
    const int q = (ch / 3) ^ x3_swz(row), limb = ch - (ch / 3) * 3;  // logical octet of physical chunk ch
    abase[j] = F32A ? base * 4 + ((id & 7) ^ f32a_swz(row & 15)) * 16
                    : P16 ? base * 6 + ch * 16 : base * 6 + q * 48 + limb * 16;
    amask[j] = msk;
    alds[j] = row * X3_ROWB + ch * 16;
  }
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    const int nch = P16 ? 6 : X3_CHUNKS;
    const int id = tid + 512 * j, row = id / nch, ch = id - row * nch;
    const int q = (ch / 3) ^ x3_swz(row), limb = ch - (ch / 3) * 3;
    boff[j] = (unsigned)((n0 + row) * p.K * 6 + (P16 ? ch * 16 : q * 48 + limb * 16));  // rows >= N fall out of range
    blds[j] = (BM + row) * X3_ROWB + ch * 16;
  }

  int tap = 0, ci0 = 0, tky = 0, tkx = 0;
  // GemmArgs::kwalk (a 4 x 4 conv, the default / F32A LDS-DMA paths): K tile kt = channels 32 (kt / 16) .. of tap
  // x3_walk_tap(kt % 16); wpos = kt % 16
  const bool walk = OM == O_DENSE && p.kwalk != 0;  // (the encoder's convs; compile-time off for the ConvT phases)
  int wpos = 0;
  if (OM != O_WGRAD && kbeg > 0) {  // a split slice starts mid-walk
    if (walk) {
      const int kt = kbeg / X3_BK;
      wpos = kt & 15;
      ci0 = (kt >> 4) * X3_BK;
      tap = x3_walk_tap(wpos);
    } else {  // tap-major: K tile = (tap, 32 channels)
      tap = kbeg / Cg;
      ci0 = kbeg - tap * Cg;
    }
    tky = tap / kw;
    tkx = tap - tky * kw;
  }
  unsigned aoff[AJ];
  auto set_tap = [&]() {
    const int toff = (tky * Win + tkx) * Cg * ESZ;
#pragma unroll
    for (int j = 0; j < AJ; ++j) aoff[j] = ((amask[j] >> (tap & 31)) & 1u) ? (unsigned)(abase[j] + toff) : KM_OOB;
  };
  set_tap();
  // the next K tile's (channels, tap): tap-major, or the 4 x 4 conv walk
  auto next_ktile = [&]() {
    if (walk) {
      if (++wpos == 16) {
        wpos = 0;
        ci0 += X3_BK;
      }
      tap = x3_walk_tap(wpos);
      tky = tap >> 2;
      tkx = tap & 3;
      set_tap();
      return;
    }
    ci0 += X3_BK;
    if (ci0 == Cg) {
      ci0 = 0;
      ++tap;
      if (++tkx == kw) {
        tkx = 0;
        ++tky;
      }
      set_tap();
    }
  };
  u32x4 ra[AJ], rb[BJ];
  auto load_ab = [&](int k0) {
#pragma unroll
    for (int j = 0; j < AJ; ++j)
      ra[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, (int)aoff[j], ci0 * 6, 0));
#pragma unroll
    for (int j = 0; j < BJ; ++j)
      rb[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsB, (int)boff[j], k0 * 6, 0));
    next_ktile();
  };
  auto store_ab = [&](int buf) {
    unsigned char* base = smem + buf * (BM + BN) * X3_ROWB;
#pragma unroll
    for (int j = 0; j < AJ; ++j) *reinterpret_cast<u32x4*>(base + alds[j]) = ra[j];
#pragma unroll
    for (int j = 0; j < BJ; ++j) *reinterpret_cast<u32x4*>(base + blds[j]) = rb[j];
  };
  // channel-major walk: the next tile's (slice, tap), advanced after the tile's barrier (its VALU work then
  // overlaps the trailing MFMAs; before the DMA issue it delayed the next tile, before the barrier it kept the
  // barrier from being hoisted)
  constexpr bool CMAJ = (V & 8) != 0 && OM != O_WGRAD;
  constexpr int CMAJ_SW = X3_BK;  // channels per slice of the channel-major walk (64 measured the same)
  int cmaj_h = 0;  // K tile within the current slice (slices of CMAJ_SW channels)
  auto advance_cmaj = [&]() {
    if (++cmaj_h < CMAJ_SW / X3_BK) {
      ci0 += X3_BK;
      return;
    }
    cmaj_h = 0;
    ci0 -= CMAJ_SW - X3_BK;
    ++tap;
    if (++tkx == kw) {
      tkx = 0;
      if (++tky == kh) {
        tky = 0;
        tap = 0;
        ci0 += CMAJ_SW;
      }
    }
    set_tap();
  };
  // LDS-DMA form: chunk id -> LDS byte 16 id, so each wave-instruction fills 1 KiB at a wave-uniform base
  typedef __attribute__((address_space(3))) void* lds_t;
  const int wbase = (tid & ~63) * 16;
  auto dma_ab = [&](int k0, int buf) {
    unsigned char* base = smem + buf * BUFB + wbase;
    if constexpr (OM == O_WGRAD) {
      // the K tile is 32 samples of ONE pixel (wg_bp % 32 == 0): a chunk is live when its shifted pixel
      // lies inside the grid
      const int pix = k0 / p.wg_bp;
      const int qy = pix / Win, qx = pix - qy * Win;
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int dy = (int)(amask[j] & 3u) - 1, dx = (int)((amask[j] >> 2) & 3u) - 1;
        const bool live = amask[j] != 0xFFFFFFFFu && (unsigned)(qy + dy) < (unsigned)p.Hin &&
                          (unsigned)(qx + dx) < (unsigned)Win;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16,
                                                 live ? (int)(abase[j] + k0 * 6) : (int)KM_OOB, 0, 0, 0);
      }
    } else if constexpr (CMAJ) {
      // K tile kt = (channel slice kt / taps, tap kt % taps), walked incrementally; the weights are stored in
      // the same slice-major order (launch_split_x3_cmaj), so B stays the sequential column k0
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (int)aoff[j], ci0 * ESZ, 0, 0);
    } else if constexpr ((V & 16384) != 0) {
      // timing probe (wrong results): no A DMA after the first tile
      if (k0 == kbeg) {
#pragma unroll
        for (int j = 0; j < AJ; ++j)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (int)aoff[j], ci0 * 6, 0, 0);
      }
    } else if constexpr ((V & 4096) != 0) {
      // timing probe (tools/gemm_bench.hip only, wrong results): every workgroup loads the same 64 KB, so the DMA
      // is served by a hot L2 (issue cost and L2 latency only)
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (tid * 16 + 8192 * j) & 0xFFFF,
                                                 0, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (int)aoff[j], ci0 * ESZ, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j)
      if (!(V & 32768) || k0 == kbeg)  // 32768: timing probe (wrong results), no B DMA after the first tile
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t)(base + BM * AROWB + 512 * 16 * j), 16,
                                               (V & 4096) ? ((tid * 16 + 8192 * j) & 0xFFFF) : (int)boff[j],
                                               (V & 4096) ? 0 : k0 * 6, 0, 0);
    if constexpr (OM != O_WGRAD && !CMAJ) next_ktile();
  };

  // 65536 / 131072 (A/B): the default path's DMA in two parts, B and half of A at the tile start, the other half of A
  // after a quarter / half of the tile's MFMAs
  auto dma_part = [&](int k0, int buf, int part) {
    unsigned char* base = smem + buf * (BM + BN) * X3_ROWB + wbase;
    if (part == 0) {
#pragma unroll
      for (int j = 0; j < BJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t)(base + BM * X3_ROWB + 512 * 16 * j), 16, (int)boff[j],
                                                 k0 * 6, 0, 0);
#pragma unroll
      for (int j = 0; j < AJ / 2; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (int)aoff[j], ci0 * 6, 0, 0);
    } else {
#pragma unroll
      for (int j = AJ / 2; j < AJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (int)aoff[j], ci0 * 6, 0, 0);
      ci0 += X3_BK;
      if (ci0 == Cg) {
        ci0 = 0;
        ++tap;
        if (++tkx == kw) {
          tkx = 0;
          ++tky;
        }
        set_tap();
      }
    }
  };

  // Blocked accumulation: the MFMA chain runs over FLUSH K tiles, then adds into tot (a second fp32 sum
  // over the blocks, round-to-nearest VALU adds) and restarts from zero.  Rounding error of one output then
  // grows with sqrt(K/32 * FLUSH) + K/32/sqrt(FLUSH) instead of K/32: ~3x less at K = 16384
  // (tools/diag_hq.py), for 64 VGPRs and 64 v_add_f32 per FLUSH tiles.
  // Sign alternation (b_negblk): v_mfma_f32_16x16x32_bf16 aligns its 32 products and the accumulator before
  // one rounding and drops the low bits toward -inf, a bias of -0.19 x 2^-24 max|term| per instruction on
  // random operands that flips sign when the operands are negated (tools/mfma_bias.hip).  A bias that keeps
  // its sign survives every later layer and the first layer's 32768-term sum where rounding noise cancels
  // (tools/diag_chain.py: 3x the CPU's error on CelebA-HQ's z gradient); with -B stored on odd blocks and
  // those blocks subtracted, consecutive blocks' biases cancel.
  f32x16 acc[2][2], tot[2][2];
  f32x4 acc16[4][4], tot16[4][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = tot[i][j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc16[i][j] = tot16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 32x32x16: fragment of k16 step s, lane half h = octet 2s + h of the row, limb l at +16 l
  // 16x16x32: lane quarter q = octet q of the row (the whole 32-deep K tile in one MFMA)
  // (tile bases are multiples of 16 rows, so the row swizzle is a function of lrow alone)
  const int lrow = M16 ? (lane & 15) : (lane & 31), loct = M16 ? (lane >> 4) : (lane >> 5);
  const int sw = x3_swz(lrow);
  const int afr = (wm * 64 + lrow) * X3_ROWB, bfr = (BM + wn * 64 + lrow) * X3_ROWB;
  const int oct16 = (loct ^ sw) * 48;                                         // 16x16x32
  const int oct32[2] = {((loct) ^ sw) * 48, ((2 + loct) ^ sw) * 48};          // 32x32x16, k16 step s

  // 128: static priority for the younger half of the workgroup (waves 4-7 lose VALU / LDS issue arbitration to
  // their older SIMD partners at every tile start; MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if constexpr ((V & 128) != 0) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  auto flush16 = [&](int ktd) {  // block flush after the MFMAs of K tile ktd
    const float sg = (p.b_negblk && (((ktd + kt0) >> FLOG) & 1)) ? -1.f : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) tot16[i][j][r] = __builtin_fmaf(sg, acc16[i][j][r], tot16[i][j][r]);
        acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
  };
  if constexpr (NARROW) {
    // ---- 64 x 128 tile: A chunks 512 .. 767 are issued by waves 0-3 only (wave-uniform guard); per K tile each wave
    // reads 2 A + 2 B tiles (12 ds_read_b128) and runs 24 MFMAs, smallest limb products first
    auto dma_n = [&](int k0, int buf) {
      unsigned char* base = smem + buf * BUFB + wbase;
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        if (512 * j + (tid & ~63) < BM * X3_CHUNKS)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (int)aoff[j], ci0 * 6, 0, 0);
#pragma unroll
      for (int j = 0; j < BJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t)(base + BM * X3_ROWB + 512 * 16 * j), 16, (int)boff[j],
                                                 k0 * 6, 0, 0);
      ci0 += X3_BK;
      if (ci0 == Cg) {
        ci0 = 0;
        ++tap;
        if (++tkx == kw) {
          tkx = 0;
          ++tky;
        }
        set_tap();
      }
    };
    if (nk > 0) dma_n(kbeg, 0);
    __syncthreads();
    const int afn = (wm * 32 + lrow) * X3_ROWB, bfn = (BM + wn * 32 + lrow) * X3_ROWB;
    for (int kt = 0; kt < nk; ++kt) {
      const unsigned char* base = smem + (kt & 1) * BUFB;
      if (kt + 1 < nk) dma_n(kbeg + (kt + 1) * X3_BK, (kt + 1) & 1);
      bf16x8 fa[2][3], fb[2][3];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int l = 0; l < 3; ++l) {
          fa[t][l] = *reinterpret_cast<const bf16x8*>(base + afn + t * 16 * X3_ROWB + oct16 + l * 16);
          fb[t][l] = *reinterpret_cast<const bf16x8*>(base + bfn + t * 16 * X3_ROWB + oct16 + l * 16);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 c = acc16[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
          acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
        }
      __syncthreads();
      if (((kt + 1) & (FLUSH - 1)) == 0) {
        const float sg = (p.b_negblk && (((kt + kt0) >> FLOG) & 1)) ? -1.f : 1.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) tot16[i][j][r] = __builtin_fmaf(sg, acc16[i][j][r], tot16[i][j][r]);
            acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
    }
  } else if constexpr (F32A) {
    // ---- fp32 A image (X3A_ROWB rows, f32a_swz), limb B image; wave w owns rows 32 w .. 32 w + 31 and all 128 columns:
    // acc16[2 a + (t >> 2)][t & 3] is A tile a (16 rows) x B tile t (16 columns).  A runs one tile ahead of B: during
    // tile kt's MFMAs (limb fragments of A(kt) in registers, B(kt) read from LDS one 16-column tile ahead) each wave
    // reads its fp32 rows of A(kt + 1) (4 ds_read_b128) and splits them into the next tile's limbs (split3_octet, the
    // producing epilogue's RNE split), so the split's VALU runs in the MFMA gaps.  LDS-DMA: B(kt + 1) and A(kt + 2)
    // are issued at the start of tile kt into the buffers tile kt - 1 finished with; the end-of-tile barrier lands
    // them.  Double-buffered: 2 x (256 x 128 + 128 x 192) B.
    auto dma_a = [&](int buf) {
      unsigned char* dst = smem + buf * BUFB + wbase;
#pragma unroll
      for (int j = 0; j < AJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(dst + 512 * 16 * j), 16, (int)aoff[j], ci0 * ESZ, 0, 0);
      next_ktile();
    };
    auto dma_b = [&](int k0, int buf) {
      unsigned char* dst = smem + buf * BUFB + BM * X3A_ROWB + wbase;
#pragma unroll
      for (int j = 0; j < BJ; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t)(dst + 512 * 16 * j), 16, (int)boff[j], k0 * 6, 0, 0);
    };
    const int fs = f32a_swz(lrow);
    const int ca0 = ((2 * loct) ^ fs) * 16, ca1 = ((2 * loct + 1) ^ fs) * 16;
    const int arow = (wave * 32 + lrow) * X3A_ROWB, brow = BM * X3A_ROWB + lrow * X3_ROWB + oct16;
    auto rd_a = [&](const unsigned char* buf, f32x4 (&av)[2][2]) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        av[a][0] = *reinterpret_cast<const f32x4*>(buf + arow + a * 16 * X3A_ROWB + ca0);
        av[a][1] = *reinterpret_cast<const f32x4*>(buf + arow + a * 16 * X3A_ROWB + ca1);
      }
    };
    // RNE limb split of elements e, e + 1 of A tile a (split3_octet's arithmetic, element by element)
    auto split2 = [&](const f32x4 (&av)[2][2], bf16x8 (&f)[2][3], int a, int e) {
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const float v = av[a][(e + d) >> 2][(e + d) & 3];
        const __bf16 b0 = (__bf16)v;
        const float r1 = sub_rn(v, (float)b0);
        const __bf16 b1 = (__bf16)r1;
        const float r2 = sub_rn(r1, (float)b1);
        f[a][0][e + d] = b0;
        f[a][1][e + d] = b1;
        f[a][2][e + d] = (__bf16)r2;
      }
    };
    auto rd_split = [&](const unsigned char* buf, bf16x8 (&f)[2][3]) {
      f32x4 av[2][2];
      rd_a(buf, av);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int e = 0; e < 8; e += 2) split2(av, f, a, e);
    };
    bf16x8 fx[2][3], fy[2][3], fb[2][3];
    if (nk > 0) {
      dma_a(0);
      dma_b(kbeg, 0);
    }
    if (nk > 1) dma_a(1);
    __syncthreads();
    rd_split(smem, fx);
    constexpr int SG_MFMA = 0x8, SG_VALU = 0x2, SG_DS_RD = 0x100;
    auto tile = [&](int kt, bf16x8 (&fc)[2][3], bf16x8 (&fn)[2][3]) {
      const unsigned char* base = smem + (kt & 1) * BUFB;
      if (kt + 1 < nk) dma_b(kbeg + (kt + 1) * X3_BK, (kt + 1) & 1);
      if (kt + 2 < nk) dma_a(kt & 1);
      // A(kt + 1): read and split unconditionally (past the last tile it is stale, in-bounds LDS, never used); two
      // elements per B tile, in that tile's MFMA gaps
      f32x4 av[2][2];
      rd_a(smem + ((kt + 1) & 1) * BUFB, av);
      auto rd_b = [&](int t, int slot) {
#pragma unroll
        for (int l = 0; l < 3; ++l) fb[slot][l] = *reinterpret_cast<const bf16x8*>(base + brow + t * 16 * X3_ROWB + l * 16);
      };
      rd_b(0, 0);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (t + 1 < 8) rd_b(t + 1, (t + 1) & 1);
        const int sl = t & 1;
        split2(av, fn, t >> 2, (t & 3) * 2);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          f32x4 c = acc16[2 * a + (t >> 2)][t & 3];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[a][2], fb[sl][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[a][1], fb[sl][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[a][0], fb[sl][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[a][1], fb[sl][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[a][0], fb[sl][1], c, 0, 0, 0);
          acc16[2 * a + (t >> 2)][t & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fc[a][0], fb[sl][0], c, 0, 0, 0);
        }
      }
      // schedule: the 4 A reads and B tiles 0 and 1 (6 reads) first, then per B tile t its 12 MFMAs with the split's
      // VALU in their gaps, then B tile t + 2's reads (into the slot tile t's MFMAs just released)
      __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 10, 0);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
#pragma unroll
        for (int m = 0; m < 12; ++m) {
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
          __builtin_amdgcn_sched_group_barrier(SG_VALU, 1, 0);
        }
        if (t + 2 < 8) __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
      }
      // the next tile's limbs are complete before the barrier: otherwise the compiler sinks the split into the next
      // tile, where it runs ahead of the first MFMAs instead of in this tile's gaps
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int l = 0; l < 3; ++l) asm volatile("" : "+v"(fn[a][l]));
      __syncthreads();
      if (((kt + 1) & (FLUSH - 1)) != 0) return;
      if constexpr (KREG) {
        // the register slab layout of the 4 x 2 wave grid (x3_ksplit_reduce_tile_kernel): A tile a of this wave is
        // row tile (w & 1) * 2 + a of wave row w >> 1, B tile t is column tile t & 3 of wave column t >> 2
        const float sg = (p.b_negblk && (((kt + kt0) >> FLOG) & 1)) ? -1.f : 1.f;
        const int ntile = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
        const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.kslab + ((long)zph * p.ksplit + zsl * p.kbpw) * ntile * (BM * BN)), (short)0,
            p.kbpw * ntile * (BM * BN) * 4, 0x00020000);
        const int soff = ((kt >> FLOG) * ntile + tm * ntn + tn) * (BM * BN * 4);
        const int voff = ((wave >> 1) * 2 * 1024 + ((wave & 1) * 2) * 4 * 64 + lane) * 16;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int a = i >> 1, wnp = i & 1;
            acc16[i][j] *= sg;
            if (m0 + wave * 32 + a * 16 < p.M) {
              // the whole offset in the VGPR, soffset the inline constant 0 (round 6; was SGPR soffset + an `s_nop 4`):
              // the VMEM-store-data hazard -- a > 64-bit store's data VGPRs rewritten by the next VALU before the store
              // has read them -- needs a wait state that LLVM's GCNHazardRecognizer (createsVALUHazard) inserts only
              // for MUBUF stores whose soffset is not an SGPR; with an SGPR soffset it assumed the exemption, the
              // register allocator reused the data VGPRs for the next tile's scaled copy at once, and 3 of every 16
              // slab tiles held the next tile's values on gfx950 (gemm_bench eq, profiles/r04/f32a_kreg_hazard.txt).
              // With soffset = 0 the recognizer pads the hazard itself (profiles/r06/kreg_store_isa.txt);
              // test_f32a_posterior_is_bitwise (B=16, register slabs) stays the gate
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc16[i][j]), rsl,
                                                     voff + soff + (wnp * 1024 + (a * 4 + j) * 64) * 16, 0,
                                                     FIXUP ? 16 : 0);
            }
            acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      } else {
        flush16(kt);
      }
    };
    for (int kt = 0; kt < nk; kt += 2) {  // two tiles per trip: the limb sets trade roles without register moves
      tile(kt, fx, fy);
      if (kt + 1 < nk) tile(kt + 1, fy, fx);
    }
  } else if constexpr (P16) {
    // ---- 16-deep K stages: stage s (16 k) of the A and B tiles is 384 rows x 96 B (three limbs of two octets, global
    // order, conflict-free for every fragment pattern below without a swizzle), slot s & 3 of a 4-slot ring; the DMA
    // of stage s + 3 is issued at the start of stage s, so three stages are in flight across each raw barrier and a
    // wave waits (counted vmcnt) only for the stage the next one reads.  Per (A tile, B tile) three MFMAs, each over 16
    // k of two limb products: [h|l].[l|h] (hl + lh), [h|m].[m|h] (hm + mh), [h|m].[h|m] (hh + mm).
    static_assert(DMA_OK_P16 && !CMAJ && M16, "P16: LDS-DMA, tap-major walk, 16x16 tiles");
    constexpr int PROWB = 96, PSLOT = (BM + BN) * PROWB;
    static_assert(4 * PSLOT <= 2 * (BM + BN) * X3_ROWB, "P16 ring exceeds the LDS");
    const int nks = 2 * nk;
    const bool lo4 = __builtin_amdgcn_readfirstlane(tid) < 256;  // waves 0-3 also issue the second B piece
    auto pdma = [&](int s) {
      const int k0 = kbeg + s * 16;
      unsigned char* base = smem + (s & 3) * PSLOT + wbase;
      if constexpr (OM == O_WGRAD) {
        const int pix = k0 / p.wg_bp;
        const int qy = pix / Win, qx = pix - qy * Win;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int dy = (int)(amask[j] & 3u) - 1, dx = (int)((amask[j] >> 2) & 3u) - 1;
          const bool live = amask[j] != 0xFFFFFFFFu && (unsigned)(qy + dy) < (unsigned)p.Hin &&
                            (unsigned)(qx + dx) < (unsigned)Win;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16,
                                                   live ? (int)(abase[j] + k0 * 6) : (int)KM_OOB, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_t)(base + 512 * 16 * j), 16, (int)aoff[j], ci0 * 6, 0, 0);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t)(base + BM * PROWB), 16, (int)boff[0], k0 * 6, 0, 0);
      if (lo4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_t)(base + BM * PROWB + 512 * 16), 16, (int)boff[1], k0 * 6,
                                                 0, 0);
      if constexpr (OM != O_WGRAD) {
        ci0 += 16;
        if (ci0 == Cg) {
          ci0 = 0;
          ++tap;
          if (++tkx == kw) {
            tkx = 0;
            ++tky;
          }
          set_tap();
        }
      }
    };
    // wait until at most `younger` stage groups issued after the one needed are still in flight (5 pieces per stage
    // on waves 0-3, 4 on waves 4-7)
    auto vwait = [&](int younger) {
      if (lo4) {
        if (younger >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    };
    for (int s = 0; s < 3; ++s)
      if (s < nks) pdma(s);
    vwait((1 < nks) + (2 < nks));
    __builtin_amdgcn_s_barrier();
    // fragment byte offsets of this lane: row m = lane & 15, k-group q = lane >> 4 reads octet q & 1 of limb h (q < 2)
    // or the pattern's second limb
    const int lrow16 = lane & 15, q4 = lane >> 4, o3 = (q4 & 1) * 3;
    const int cA1 = (o3 + (q4 < 2 ? 0 : 1)) * 16, cA2 = (o3 + (q4 < 2 ? 0 : 2)) * 16;
    const int cB2 = (o3 + (q4 < 2 ? 1 : 0)) * 16, cB3 = (o3 + (q4 < 2 ? 2 : 0)) * 16;
    const int arow = (wm * 64 + lrow16) * PROWB, brow = (BM + wn * 64 + lrow16) * PROWB;
    bf16x8 fa1[4], fa2[4], fb1[4], fb2[4], fb3[4];
    constexpr int SG_MFMA = 0x8, SG_DS_RD = 0x100;
    for (int s = 0; s < nks; ++s) {
      if (s + 3 < nks) pdma(s + 3);
      const unsigned char* sb = smem + (s & 3) * PSLOT;
      auto rd_a = [&](int t) {
        fa1[t] = *reinterpret_cast<const bf16x8*>(sb + arow + t * 16 * PROWB + cA1);
        fa2[t] = *reinterpret_cast<const bf16x8*>(sb + arow + t * 16 * PROWB + cA2);
      };
      auto rd_b = [&](int t) {
        fb1[t] = *reinterpret_cast<const bf16x8*>(sb + brow + t * 16 * PROWB + cA1);
        fb2[t] = *reinterpret_cast<const bf16x8*>(sb + brow + t * 16 * PROWB + cB2);
        fb3[t] = *reinterpret_cast<const bf16x8*>(sb + brow + t * 16 * PROWB + cB3);
      };
      auto mf = [&](int i, int j) {
        f32x4 c = acc16[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa2[i], fb3[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[i], fb2[j], c, 0, 0, 0);
        acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[i], fb1[j], c, 0, 0, 0);
      };
      rd_a(0);
      rd_b(0);
      rd_b(1);
      mf(0, 0);
      rd_b(2);
      mf(0, 1);
      rd_b(3);
      mf(0, 2);
      rd_a(1);
      mf(0, 3);
      rd_a(2);
#pragma unroll
      for (int j = 0; j < 4; ++j) mf(1, j);
      rd_a(3);
#pragma unroll
      for (int i = 2; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mf(i, j);
      __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 8, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 2, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 2, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 12, 0);
      __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 2, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 24, 0);
      // the next stage's DMA has landed (this wave's pieces; the barrier covers the other waves'), and this stage's
      // reads are retired before any wave re-fills its slot
      vwait((s + 2 < nks) + (s + 3 < nks));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (!(V & 32) && ((s + 1) & (2 * FLUSH - 1)) == 0) flush16(s >> 1);
    }
  } else {
  constexpr bool DMA = (V & 4) != 0;
  static_assert(OM != O_WGRAD || DMA, "O_WGRAD runs on the LDS-DMA staging path only");
  static_assert(!CMAJ || DMA, "the channel-major walk runs on the LDS-DMA staging path only");
  if (DMA) {
    if (nk > 0) dma_ab(kbeg, 0);
    if constexpr (CMAJ) advance_cmaj();
  } else if (nk > 0) {
    load_ab(0);
    store_ab(0);
    if (nk > 1) load_ab(X3_BK);
  }
  __syncthreads();
  bf16x8 pfa[4][3], pfb[4][3];  // the read-order path's fragments
  // 2048: waves 4-7 run half a tile behind (the stagger of MI355X_MICROARCH.md, two waves per SIMD, item 9); every
  // accumulator still takes its tiles' MFMAs in the same order and is flushed at the same block ends: bitwise the
  // unstaggered kernel
  const bool stag = M16 && (V & 256) && (V & 2048) && DMA && __builtin_amdgcn_readfirstlane(tid) >= 256;

  auto mfp = [&](int i, int j) {  // the six limb products of A tile i x B tile j, smallest first
    f32x4 c = acc16[i][j];
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pfa[i][2], pfb[j][0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pfa[i][1], pfb[j][1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pfa[i][0], pfb[j][2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pfa[i][1], pfb[j][0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pfa[i][0], pfb[j][1], c, 0, 0, 0);
    acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pfa[i][0], pfb[j][0], c, 0, 0, 0);
  };
  // one loop per wave role (a runtime branch inside a shared loop made the compiler keep both roles' fragment sets
  // live: 316 VGPRs spilled)
  auto kloop = [&](auto S_) {
    constexpr bool S = decltype(S_)::value;
    for (int kt = 0; kt < nk; ++kt) {
      const unsigned char* base = smem + (kt & 1) * (BM + BN) * X3_ROWB;
      // DMA: the next tile goes into the other buffer (read before the previous barrier) now; the
      // barrier at the end of this tile (its vmcnt(0)) lands it
      // (issuing it later — after the fragment reads, or mid-MFMA — measured 10-15 % slower)
      // timing probes (tools/gemm_bench.hip only, wrong results): 512 no DMA after the first tile, 1024 fragment reads
      // of the first tile only
      // 8192 (with the stagger): the staggered waves issue their share of the DMA after their trailing half tile, so
      // the two waves of a SIMD never issue DMA at the same time (each covers the other's DMA issue with MFMAs)
      constexpr bool LATE = S && (V & 8192) != 0;
      constexpr int SPLIT = (V & 65536) ? 1 : (V & 131072) ? 2 : 0;
      static_assert(SPLIT == 0 || (OM != O_WGRAD && !CMAJ && !(V & (512 | 2048 | 4096 | 16384 | 32768))), "probe mix");
      const bool dnext = DMA && kt + 1 < nk && !(V & 512);
      if (SPLIT && dnext) dma_part(kbeg + (kt + 1) * X3_BK, (kt + 1) & 1, 0);
      else if (dnext && !(LATE && kt > 0)) dma_ab(kbeg + (kt + 1) * X3_BK, (kt + 1) & 1);
      if (M16 && (V & 256)) {
        // 256: fragment reads one group ahead of the MFMAs that consume them, in the order those MFMAs run (A tile 0
        // against B tiles 0..3, then A tiles 1..3), pinned by sched_group_barrier: the first MFMAs wait for 6 reads
        // instead of the ~15 the default schedule puts in front of its first lgkmcnt(0).  2.5-3.9 % less time on
        // the four CIFAR shapes, bit-identical results (profiles/r02/gemm_bench_rdorder.txt).  Measured and dropped:
        // reading the next tile's first fragments after the barrier into the registers the trailing MFMAs free
        // (cross-tile pipeline, 1-2 % slower than this), all reads issued by the end of A row 0 so the barrier moves
        // up (5-8 % slower), A tile 3 read later so it moves down (0-2 % slower).
        bf16x8 (&fa)[4][3] = pfa, (&fb)[4][3] = pfb;  // [tile][limb]
        const bool rd = !(V & 1024) || kt == 0;
        auto rd_a = [&](int t) {
          if (!rd) return;
#pragma unroll
          for (int l = 0; l < 3; ++l) fa[t][l] = *reinterpret_cast<const bf16x8*>(base + afr + t * 16 * X3_ROWB + oct16 + l * 16);
        };
        auto rd_b = [&](int t) {
          if (!rd) return;
#pragma unroll
          for (int l = 0; l < 3; ++l) fb[t][l] = *reinterpret_cast<const bf16x8*>(base + bfr + t * 16 * X3_ROWB + oct16 + l * 16);
        };
        auto mf = [&](int i, int j) {
          f32x4 c = acc16[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
          acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
        };
        constexpr int SG_MFMA = 0x8, SG_DS_RD = 0x100;
        if constexpr (S) {
          // 2048, waves 4-7: the second half (A tiles 2, 3) of the previous tile's MFMAs from the registers its
          // fragments still hold, that tile's block flush, then this tile's reads and its first half, so that on every
          // SIMD one wave is at MFMAs while its partner waits for its fragment reads after the barrier
          if (kt > 0) {
#pragma unroll
            for (int i = 2; i < 4; ++i)
#pragma unroll
              for (int j = 0; j < 4; ++j) mf(i, j);
            __builtin_amdgcn_sched_barrier(0);
            if (!(V & 32) && (kt & (FLUSH - 1)) == 0) flush16(kt - 1);
            if (LATE && kt + 1 < nk && !(V & 512)) dma_ab(kbeg + (kt + 1) * X3_BK, (kt + 1) & 1);
          }
          rd_a(0);
          rd_b(0);
          rd_b(1);
          mf(0, 0);
          rd_b(2);
          mf(0, 1);
          rd_b(3);
          mf(0, 2);
          rd_a(1);
          mf(0, 3);
          rd_a(2);
#pragma unroll
          for (int j = 0; j < 4; ++j) mf(1, j);
          rd_a(3);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 9, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 24, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __syncthreads();
          if constexpr (CMAJ) advance_cmaj();
          continue;
        }
        if constexpr (SPLIT != 0) {
          rd_a(0);
          rd_b(0);
          rd_b(1);
          mf(0, 0);
          rd_b(2);
          mf(0, 1);
          rd_b(3);
          mf(0, 2);
          rd_a(1);
          mf(0, 3);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 9, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (SPLIT == 1 && dnext) dma_part(kbeg + (kt + 1) * X3_BK, (kt + 1) & 1, 1);
          __builtin_amdgcn_sched_barrier(0);
          rd_a(2);
#pragma unroll
          for (int j = 0; j < 4; ++j) mf(1, j);
          rd_a(3);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_group_barrier(SG_MFMA, 24, 0);
          __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (SPLIT == 2 && dnext) dma_part(kbeg + (kt + 1) * X3_BK, (kt + 1) & 1, 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 2; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) mf(i, j);
          __syncthreads();
          if (!(V & 32) && ((kt + 1) & (FLUSH - 1)) == 0) flush16(kt);
          continue;
        }
        rd_a(0);
        rd_b(0);
        rd_b(1);
        mf(0, 0);
        rd_b(2);
        mf(0, 1);
        rd_b(3);
        mf(0, 2);
        rd_a(1);
        mf(0, 3);
        rd_a(2);
#pragma unroll
        for (int j = 0; j < 4; ++j) mf(1, j);
        rd_a(3);
#pragma unroll
        for (int i = 2; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) mf(i, j);
        __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 9, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 6, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 24, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DS_RD, 3, 0);
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 48, 0);
      } else if (M16) {
        bf16x8 fa[4][3], fb[4][3];  // [tile][limb]
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int l = 0; l < 3; ++l) {
            fa[t][l] = *reinterpret_cast<const bf16x8*>(base + afr + t * 16 * X3_ROWB + oct16 + l * 16);
            fb[t][l] = *reinterpret_cast<const bf16x8*>(base + bfr + t * 16 * X3_ROWB + oct16 + l * 16);
          }
        if (!DMA && kt + 1 < nk) {
          store_ab((kt + 1) & 1);
          if (kt + 2 < nk) load_ab((kt + 2) * X3_BK);
        }
        if (V & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f32x4 c = acc16[i][j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
            acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
          }
        if (V & 2) __builtin_amdgcn_s_setprio(0);
      } else {
        bf16x8 fa[2][2][3], fb[2][2][3];  // [s][tile][limb]
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int l = 0; l < 3; ++l) {
              fa[s][t][l] = *reinterpret_cast<const bf16x8*>(base + afr + t * 32 * X3_ROWB + oct32[s] + l * 16);
              fb[s][t][l] = *reinterpret_cast<const bf16x8*>(base + bfr + t * 32 * X3_ROWB + oct32[s] + l * 16);
            }
        if (!DMA && kt + 1 < nk) {
          store_ab((kt + 1) & 1);
          if (kt + 2 < nk) load_ab((kt + 2) * X3_BK);
        }
        if (V & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              f32x16 c = acc[i][j];
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i][2], fb[s][j][0], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i][1], fb[s][j][1], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i][0], fb[s][j][2], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i][1], fb[s][j][0], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i][0], fb[s][j][1], c, 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][i][0], fb[s][j][0], c, 0, 0, 0);
            }
        if (V & 2) __builtin_amdgcn_s_setprio(0);
      }
      __syncthreads();
      if constexpr (CMAJ) advance_cmaj();
      // block flush after the barrier: the compiler keeps hoisting the barrier above the tile's trailing MFMAs
      // (a flush between them and the barrier measured 6-8 % slower)
      if (KREG) {
        if (((kt + 1) & (FLUSH - 1)) != 0) continue;
        // split-K: every sign block's signed sum straight from the accumulators into its own slab, in the register
        // layout (one 16-B store per lane and tile: 1 KB per wave-instruction); x3_ksplit_reduce_kernel maps back
        // buffer stores: one VGPR of offset (wave, lane), the rest scalar, so the 256 accumulator VGPRs do not spill
        const float sg = (p.b_negblk && (((kt + kt0) >> FLOG) & 1)) ? -1.f : 1.f;
        const int ntile = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
        const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.kslab + ((long)zph * p.ksplit + zsl * p.kbpw) * ntile * (BM * BN)), (short)0,
            p.kbpw * ntile * (BM * BN) * 4, 0x00020000);
        const int soff = ((kt >> FLOG) * ntile + tm * ntn + tn) * (BM * BN * 4);
        const int voff = (wave * 1024 + lane) * 16;
        const bool live = m0 + wm * 64 < p.M;  // a wave whose 64 rows are all past M stores nothing (the reduce skips them)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc16[i][j] *= sg;
            if (live)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc16[i][j]), rsl, voff,
                                                     soff + (i * 4 + j) * 1024, 0);
            acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      } else if (!(V & 32) && ((kt + 1) & (FLUSH - 1)) == 0) {
        const float sg = (p.b_negblk && (((kt + kt0) >> FLOG) & 1)) ? -1.f : 1.f;
        if (M16) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma unroll
              for (int r = 0; r < 4; ++r) tot16[i][j][r] = __builtin_fmaf(sg, acc16[i][j][r], tot16[i][j][r]);
              acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        } else {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                tot[i][j][r] = __builtin_fmaf(sg, acc[i][j][r], tot[i][j][r]);
                acc[i][j][r] = 0.f;
              }
        }
      }
    }
    if (S && nk > 0) {  // the staggered waves' trailing half tile
#pragma unroll
      for (int i = 2; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mfp(i, j);
      if (!(V & 32) && (nk & (FLUSH - 1)) == 0) flush16(nk - 1);
    }
  };
  if (stag)
    kloop(std::true_type{});
  else
    kloop(std::false_type{});

  }
  if (p.clk && tid == 0) {  // the K loop's shader clocks over its 100 MHz ticks (damc_clock_probe)
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* c = p.clk + 4 * ((blockIdx.z * gridDim.x + blockIdx.x) % (unsigned)p.clk_n);
    c[0] = clk_t0;
    c[1] = clk_r0;
    c[2] = t1;
    c[3] = r1;
  }
  if (KREG && !FIXUP) return;  // every block already in its slab
  if constexpr (!FIXUP) {  // the last partial block
    const float sg = (p.b_negblk && nk > 0 && (((nk - 1 + kt0) >> FLOG) & 1)) ? -1.f : 1.f;
    if (M16) {
      constexpr int MI = NARROW ? 2 : 4;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc16[i][j][r] = __builtin_fmaf(sg, acc16[i][j][r], tot16[i][j][r]);
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_fmaf(sg, acc[i][j][r], tot[i][j][r]);
    }
  }
  // ---- epilogue through LDS: the block's 256 x 128 fp32 tile, then one thread per (row, channel octet):
  // 2 x 16-B fp32 stores and (C3) 3 x 16-B limb stores per octet, each row's 128 channels contiguous
  constexpr int TS = BN + 4;  // tile row stride (floats): 4-row groups of a 16x16 store land 16 banks apart
  static_assert(BM * TS * 4 + BM * 8 <= 2 * (BM + BN) * X3_ROWB, "epilogue tile exceeds the LDS");
  static_assert(!FIXUP || BM * TS * 4 + BM * 8 <= 2 * (BM + BN) * X3_ROWB - 16, "the fix-up's last word overlaps the tile");
  float* tile = reinterpret_cast<float*>(smem);
  long* rowtab = reinterpret_cast<long*>(smem + BM * TS * 4);
  float* Cz = p.C;
  if ((OM == O_DENSE || OM == O_WGRAD) && Cz) Cz += (long)(KSPLIT ? zph : z) * p.c_zstride;
  // one (row, channel octet) of the tile through the epilogue (bias + act / LReLU' mask, sign bits, fp32, limbs)
  auto octet = [&](int row, int oct) {
    const int n = n0 + oct * 8;
    const long rowoff = rowtab[row];
    if (rowoff < 0 || n >= p.N) return;
    const long idx = rowoff + n;
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(tile + row * TS + oct * 8);
    const f32x4 t1 = *reinterpret_cast<const f32x4*>(tile + row * TS + oct * 8 + 4);
    float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    if (EPI == EPI_BIAS_ACT) {
      if (p.bias) {
        const int nb = p.bias_mod < p.N ? n % p.bias_mod : n;
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + nb);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + nb + 4);
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bb[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = act_apply(v[e], p.act, p.slope);
    } else if (EPI == EPI_MASK) {
      if (p.mask_sgn) {  // LReLU' from the sign bits of the activation: 1 where it was > 0, else slope
        const unsigned bits = p.mask_sgn[idx >> 3];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= ((bits >> e) & 1u) ? 1.f : p.mask_slope;
      } else {
        const f32x4 k0 = *reinterpret_cast<const f32x4*>(p.mask + idx);
        const f32x4 k1 = *reinterpret_cast<const f32x4*>(p.mask + idx + 4);
        const float kk[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= act_grad_from_out(kk[e], p.mask_act, p.mask_slope);
      }
    }
    if (p.sgn) {
      unsigned bits = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) bits |= (v[e] > 0.f ? 1u : 0u) << e;
      p.sgn[idx >> 3] = (unsigned char)bits;
    }
    if (Cz && !p.proj_nostore) {
      *reinterpret_cast<f32x4*>(Cz + idx) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(Cz + idx + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
    if (p.C3) {
      bf16x8 h, m, l;
      split3_octet(v, h, m, l);
      bf16x8* o = reinterpret_cast<bf16x8*>(p.C3 + 3 * idx);
      o[0] = h;
      o[1] = m;
      o[2] = l;
    }
    if ((OM == O_PHASE && EPI == EPI_BIAS_ACT && (WIDE || F32A) && p.proj_out) ||
        (OM == O_DENSE && EPI == EPI_BIAS_ACT && !WIDE && !NARROW && p.in_part)) {  // the stored row back into the tile
      *reinterpret_cast<f32x4*>(tile + row * TS + oct * 8) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(tile + row * TS + oct * 8 + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  };
  // FIXUP: the output-layer projection's weights (proj16's b operands of this N tile's chunk), preloaded into registers
  // while the slices wait, so a band's projection does not chain on their loads (proj16_pre)
  f32x4 pw[PROJ_CHUNK / 16][4];
  // the epilogue of tile rows [r_lo, r_hi) (the whole tile except in the fix-up's bands; rowtab is -1 outside)
  auto epilogue = [&](int r_lo, int r_hi) {
    if constexpr (FIXUP) {
      for (int id = tid; id < (r_hi - r_lo) * (BN / 8); id += 512) octet(r_lo + id / (BN / 8), id % (BN / 8));
    } else {
#pragma unroll 2
      for (int it = 0; it < BM * BN / 8 / 512; ++it) {
        const int id = tid + 512 * it;
        octet(id / (BN / 8), id % (BN / 8));
      }
    }
    if constexpr (OM == O_PHASE && EPI == EPI_BIAS_ACT && (WIDE || F32A)) {
      // fused output-layer projection (GemmArgs::proj_out), proj16 as proj_rows_kernel, P indexed by the output pixel,
      // one chain per 128-channel chunk into partial buffer chunk (proj_rows_kernel's chunking).  WIDE: the tile holds
      // every channel (n0 == 0, N <= 256), 8 waves x 16 rows, all chunks.  F32A: the tile holds channels n0 .. n0 + 127
      // = chunk n0 / 128, 8 waves x 32 rows (two 16-row groups each)
      if (p.proj_out) {
        __syncthreads();
        const int m = lane & 15, q = lane >> 4;
        auto store = [&](auto NT_) {
          constexpr int NT = decltype(NT_)::value;
          constexpr int RG = F32A ? 2 : 1;
#pragma unroll
          for (int g = 0; g < RG; ++g) {
            const int r0 = F32A ? wave * 32 + g * 16 : wave * 16;
            if (r0 + 16 <= r_lo || r0 >= r_hi) continue;  // FIXUP: a 16-row group outside the band (wave-uniform)
            for (int c0 = 0; c0 < (F32A ? BN : p.N); c0 += PROJ_CHUNK) {
              const int cc = F32A ? n0 : c0;  // global channel of the chunk's first column
              if (cc >= p.N) break;
              f32x4 acc[NT];
              if constexpr (FIXUP)
                proj16_pre<NT>(tile + c0, TS, r0, min(PROJ_CHUNK, p.N - cc), pw, acc);
              else
                proj16<NT>(tile + c0, TS, r0, min(PROJ_CHUNK, p.N - cc), p.proj_w + cc, p.proj_ldw, acc);
              float* Pc = p.proj_out + (cc / PROJ_CHUNK) * p.proj_pstride;
#pragma unroll
              for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const long ro = rowtab[r0 + 4 * q + r];
                  if (ro >= 0) Pc[(ro / p.ldc) * (16 * NT) + 16 * t + m] = acc[t][r];
                }
            }
          }
        };
        if (p.proj_np == 32)
          store(std::integral_constant<int, 2>{});
        else
          store(std::integral_constant<int, 4>{});
      }
    }
  };
  if constexpr (FIXUP) {
    // ---- split-K in-GEMM ordered fix-up, spread over the tile's slices (MI355X_MICROARCH.md, inter-workgroup visibility,
    // first row of the sc1 hand-off table).  Every slice stored its slabs sc1 (write-through); each wave drains them,
    // then behind a barrier lane 0 counts the slice in (one agent-scope CAS on the tile's epoch-tagged counter) and waits,
    // bounded, until every slice of the tile has arrived (the launch has <= 256 workgroups at one per CU, so they are
    // co-resident on an otherwise idle chip).  Slice j then claims band j of the tile's 16-row tiles (a CAS on the band's
    // claim word, exactly once per launch) and sums the band's slabs 0 .. ksplit - 1 in order with sc1 loads into the LDS
    // tile -- x3_ksplit_reduce_tile_kernel's order and roundings -- and runs the unsplit epilogue on those rows.  The last
    // slice to arrive never waits: after its own band it claims every band still unclaimed (a slice whose wait ran out
    // leaves its band), so each band is combined exactly once whatever the residency.  Words are tagged with the launch's
    // epoch (GemmArgs::kepoch), so the counters need zeroing once per call, not per launch.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long t_drained = __builtin_amdgcn_s_memrealtime();
    // LDS words past the epilogue's tile and row table, in the one LDS array: [0] own band claimed, [1] last, [2] bands
    unsigned* sw = reinterpret_cast<unsigned*>(smem + sizeof(smem) - 16);
    const int ntile = ((p.M + BM - 1) / BM) * ntn;
    const int tix = zph * ntile + tm * ntn + tn;
    const int nband = min(nslz, 16);
    const unsigned ep = p.kepoch;
    unsigned* cnt = p.kticket + tix;
    unsigned* claim = p.kticket + X3_KTICKETS + (long)tix * nslz;
    auto try_claim = [&](int b) -> bool {
      unsigned w = __hip_atomic_load(claim + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while ((w >> 16) != ep)
        if (__hip_atomic_compare_exchange_strong(claim + b, &w, (ep << 16) | 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          return true;
      return false;
    };
    if constexpr (OM == O_PHASE && EPI == EPI_BIAS_ACT) {
      if (p.proj_out) {  // F32A: this N tile is the chunk n0 / PROJ_CHUNK
        const int cw = min(PROJ_CHUNK, p.N - n0), nt = p.proj_np / 16, mm = lane & 15, qq = lane >> 4;
        // buffer loads, zeros past the chunk's columns or rows through an out-of-range offset (no branch per load)
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            (void*)p.proj_w, (short)0, p.proj_np * p.proj_ldw * 4, 0x00020000);
#pragma unroll
        for (int g = 0; g < PROJ_CHUNK / 16; ++g)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            pw[g][t] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                           rw, (16 * g < cw && t < nt) ? (n0 + (16 * t + mm) * p.proj_ldw + 16 * g + 4 * qq) * 4
                                                       : (int)KM_OOB, 0, 0));
      }
    }
    if (tid == 0) {
      unsigned w = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), mine;
      for (;;) {
        mine = ((w >> 16) == ep ? (w & 0xFFFFu) : 0u) + 1u;
        if (__hip_atomic_compare_exchange_strong(cnt, &w, (ep << 16) | mine, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          break;
      }
      const bool last = mine == (unsigned)nslz;
      bool ok = last;
      if (!last) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned long long dt = 0;
        for (;;) {
          const unsigned v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dt = __builtin_amdgcn_s_memrealtime() - t0;
          if ((v >> 16) == ep && (v & 0xFFFFu) >= (unsigned)nslz) {
            ok = true;
            break;
          }
          if (dt > (unsigned long long)X3_FIXUP_WAIT) break;
          __builtin_amdgcn_s_sleep(2);
        }
        if (p.fixup_probe) {
          atomicMax(p.fixup_probe + 3, (unsigned)dt);
          atomicAdd(p.fixup_probe + 4, (unsigned)dt);
        }
      }
      sw[0] = (ok && zsl < nband && try_claim(zsl)) ? 1u : 0u;
      sw[1] = last ? 1u : 0u;
      if (p.fixup_probe) {
        atomicAdd(p.fixup_probe, 1u);
        if (!ok) atomicAdd(p.fixup_probe + 1, 1u);
        if (last) atomicAdd(p.fixup_probe + 5, 1u);
      }
    }
    __syncthreads();
    // damc_clock_probe on a fix-up launch (diagnostics): realtime stamps {K-loop end, slabs drained, wait over, bands
    // done} instead of the clock pairs
    unsigned long long* ck = (p.clk && tid == 0)
                                 ? p.clk + 4 * ((blockIdx.z * gridDim.x + blockIdx.x) % (unsigned)p.clk_n) : nullptr;
    if (ck) {
      ck[0] = ck[3];  // K-loop end
      ck[1] = t_drained;
      ck[2] = __builtin_amdgcn_s_memrealtime();  // wait over
    }
    const bool own_ok = sw[0] != 0, last = sw[1] != 0;
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.kslab + (long)zph * p.ksplit * ntile * (BM * BN)), (short)0, p.ksplit * ntile * (BM * BN) * 4,
        0x00020000);
    // band b = 16-row tiles [16 b / nband, 16 (b + 1) / nband): thread (wn = tid >> 8, column tile ci, lane l) owns one
    // f32x4 of the register slab layout per row tile (rows 4 (l >> 4) .. + 3, column wn 64 + ci 16 + (l & 15)); the
    // (row tile, slab) pairs go 16 loads at a time, each added into the LDS tile in slab order (0 + slab 0 + slab 1 ..)
    auto band = [&](int b) {
      const int rt0 = b * 16 / nband, rt1 = (b + 1) * 16 / nband, np = (rt1 - rt0) * p.ksplit;
      const int wnb = tid >> 8, ci = (tid >> 6) & 3;
      __syncthreads();  // the previous band's epilogue is done with the tile
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};  // the running sum of the current row tile's slabs
      for (int q0 = 0; q0 < np; q0 += 16) {
        f32x4 t[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int q = q0 + k, rt = rt0 + q / p.ksplit, sl = q - (q / p.ksplit) * p.ksplit;
          const int off = ((((rt >> 2) * 2 + wnb) * 16 + (rt & 3) * 4 + ci) * 64 + lane) * 16;
          // no branch around the load (a "load or zero" select made each load wait for the last one): an invalid
          // pair's offset falls outside the buffer, which returns zeros
          t[k] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsl, (q < np && m0 + rt * 16 < p.M) ? off : (int)KM_OOB,
                                                           (sl * ntile + tm * ntn + tn) * (BM * BN * 4), 16));
        }
        __builtin_amdgcn_sched_barrier(0);  // all 16 loads issued before the first add waits on one
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int q = q0 + k, rt = rt0 + q / p.ksplit, sl = q - (q / p.ksplit) * p.ksplit;
          // 0 + slab 0 + slab 1 + ..., as the reduce; pairs past the band leave acc alone (a select, no branch)
          const f32x4 nx = (sl == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc) + t[k];
          acc = q < np ? nx : acc;
          if (q < np && sl == p.ksplit - 1) {
            float* d = tile + (rt * 16 + 4 * (lane >> 4)) * TS + wnb * 64 + ci * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) d[r * TS] = acc[r];
          }
        }
      }
      if (tid < BM)
        rowtab[tid] = (tid >= rt0 * 16 && tid < rt1 * 16 && m0 + tid < p.M) ? gemm_row_offset<OM>(p, m0 + tid, py, px)
                                                                           : -1L;
      __syncthreads();
      epilogue(rt0 * 16, rt1 * 16);
    };
    if (own_ok) band(zsl);
    if (last) {
      if (wave == 0) {  // the bands nobody claimed, one CAS per band in parallel lanes
        const bool got = lane < nband && lane != zsl && try_claim(lane);
        const unsigned long long m = __builtin_amdgcn_ballot_w64(got);
        if (lane == 0) {
          sw[2] = (unsigned)m;
          if (p.fixup_probe && m) atomicAdd(p.fixup_probe + 2, (unsigned)__builtin_popcountll(m));
        }
      }
      __syncthreads();
      unsigned m = sw[2];
      while (m) {
        const int b = __builtin_ctz(m);
        m &= m - 1;
        band(b);
      }
    }
    if (ck) ck[3] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  if (tid < BM) rowtab[tid] = (m0 + tid < p.M) ? gemm_row_offset<OM>(p, m0 + tid, py, px) : -1L;
  if (F32A) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tile[(wave * 32 + (i >> 1) * 16 + 4 * (lane >> 4) + r) * TS + ((i & 1) * 4 + j) * 16 + (lane & 15)] =
              acc16[i][j][r];
  } else if (NARROW) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tile[(wm * 32 + i * 16 + 4 * (lane >> 4) + r) * TS + wn * 32 + j * 16 + (lane & 15)] = acc16[i][j][r];
  } else if (M16) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tile[(wm * 64 + i * 16 + 4 * (lane >> 4) + r) * TS + wn * 64 + j * 16 + (lane & 15)] = acc16[i][j][r];
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          tile[(wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * TS + wn * 64 + j * 32 + (lane & 31)] =
              acc[i][j][r];
  }
  __syncthreads();
  if (KSPLIT && !FIXUP) {  // row-major slabs (one block per workgroup): the fp32 tile into its slab; the reduce applies the epilogue
    float* sl = p.kslab + ((long)zph * p.ksplit + zsl) * p.M * p.N;
#pragma unroll 2
    for (int it = 0; it < BM * BN / 8 / 512; ++it) {
      const int id = tid + 512 * it, row = id / (BN / 8), oct = id % (BN / 8);
      const int m = m0 + row, n = n0 + oct * 8;
      if (m >= p.M || n >= p.N) continue;
      float* d = sl + (long)m * p.N + n;
      *reinterpret_cast<f32x4*>(d) = *reinterpret_cast<const f32x4*>(tile + row * TS + oct * 8);
      *reinterpret_cast<f32x4*>(d + 4) = *reinterpret_cast<const f32x4*>(tile + row * TS + oct * 8 + 4);
    }
    return;
  }
  epilogue(0, BM);
  if constexpr (OM == O_DENSE && EPI == EPI_BIAS_ACT && !WIDE && !NARROW && !FIXUP && BM == 256 && BN == 128) {
    // the encoder norm's statistics of this tile (GemmArgs::in_part): its 256 rows are one strip of one sample
    static_assert(BM * TS * 4 + BM * 8 + 1024 * 4 <= 2 * (BM + BN) * X3_ROWB, "statistics scratch exceeds the LDS");
    if (p.in_part && !KSPLIT) {  // workgroup-uniform
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem + BM * TS * 4 + BM * 8);
      float st[3];
      strip256_stats(tile, TS, tid, n0 + (tid & 127) < p.N, red, st);
      if (tid < 128 && n0 + tid < p.N) {
        const int b = m0 / p.in_hw, sp = (m0 - b * p.in_hw) >> 8;
        float* o = p.in_part + (((long)b * p.N + n0 + tid) * p.in_S + sp) * 3;
        o[0] = st[0];
        o[1] = st[1];
        o[2] = st[2];
      }
    }
  }
}

// the split-K reduce: one thread per (phase, row, channel octet); the slices in fixed order, then the limb GEMM's
// epilogue (bias + act or the LReLU' mask, sign bits, fp32 and limb outputs) on the sum
// the epilogue of one output octet (8 consecutive channels n .. n + 7 of GEMM row m) from its fp32 sums
template <int EPI, int OM>
__device__ __forceinline__ void x3_octet_epilogue(const GemmArgs& p, int m, int n, int py, int px, float (&v)[8]);
template <int EPI>
__device__ __forceinline__ void x3_octet_epilogue_at(const GemmArgs& p, long idx, int n, float (&v)[8]);

// register slab layout, one wave per 16x16 MFMA tile: lane l sums its f32x4 (rows 4 (l >> 4) .. + 3, column l & 15)
// over the blocks in order (1 KB per wave-load; a thread per 4 rows x 8 channels measured 5-10 % slower per step at B=8-32), then the tile goes through
// LDS and 32 lanes apply the octet epilogue
template <int EPI, int OM>
__global__ __launch_bounds__(256) void x3_ksplit_reduce_tile_kernel(GemmArgs p, int zdim) {
  __shared__ float red[4][16][17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long blk = (long)blockIdx.x * 4 + w;  // ((phase * ntile + tile) * 8 + wave) * 16 + tile16
  const int ntm = (p.M + X3_BM - 1) / X3_BM, ntn = (p.N + X3_BN - 1) / X3_BN;
  const long ntile = (long)ntm * ntn;
  const int ij = (int)(blk & 15), wave = (int)((blk >> 4) & 7);
  const long tl = blk >> 7;
  const int tile = (int)(tl % ntile), ph = (int)(tl / ntile);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int m0 = tm * X3_BM + (wave >> 1) * 64 + (ij >> 2) * 16, n0 = tn * X3_BN + (wave & 1) * 64 + (ij & 3) * 16;
  const bool live = ph < zdim && m0 < p.M && n0 < p.N;  // wave-uniform
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (live) {
    const long sstride = ntile * (X3_BM * X3_BN / 4);
    const f32x4* src = reinterpret_cast<const f32x4*>(p.kslab) + (long)ph * p.ksplit * sstride +
                       (((long)tile * 8 + wave) * 16 + ij) * 64 + lane;
    // the blocks in order, the sign already applied; four slabs' loads in flight before their adds (one load per
    // trip left each lane waiting a memory round trip per slab: 11.5 us for 8 MB at CIFAR B=16)
    int sl = 0;
    for (; sl + 4 <= p.ksplit; sl += 4) {
      const f32x4 t0 = src[(long)sl * sstride], t1 = src[(long)(sl + 1) * sstride];
      const f32x4 t2 = src[(long)(sl + 2) * sstride], t3 = src[(long)(sl + 3) * sstride];
      v += t0;
      v += t1;
      v += t2;
      v += t3;
    }
    for (; sl < p.ksplit; ++sl) v += src[(long)sl * sstride];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][4 * (lane >> 4) + r][lane & 15] = v[r];
  __syncthreads();
  if (!live || lane >= 32) return;
  const int row = lane >> 1, oc = (lane & 1) * 8, m = m0 + row, n = n0 + oc;
  if (m >= p.M || n >= p.N) return;
  float o[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = red[w][row][oc + c];
  const int py = OM == O_PHASE ? ph >> 1 : 0, px = OM == O_PHASE ? ph & 1 : 0;
  x3_octet_epilogue<EPI, OM>(p, m, n, py, px, o);
}

// the split-K reduce of a ConvT forward whose epilogue also runs the output layer's projection (GemmArgs::proj_out,
// register slab layout): one workgroup of 4 waves per (phase, 256 x 128 tile, 64-row quarter).  Wave w sums the 8
// 16x16 tiles of rows 16 w .. + 15 of the quarter (x3_ksplit_reduce_tile_kernel's per-lane order) into an LDS tile,
// the octet epilogue writes the sign bits (and C unless proj_nostore) and leaves the activated rows in the tile, and
// wave w projects its 16 rows with proj16 into the chunk's partial buffer -- the F32A tile's fused epilogue on the
// same sums, so the result is bitwise the unsplit kernel's, without the fp32 activation's write and re-read by
// proj_rows_kernel
template <int NT>
__global__ __launch_bounds__(256) void x3_ksplit_reduce_proj_kernel(GemmArgs p, int zdim) {
  constexpr int TS = X3_BN + 4, RW = 64;
  __shared__ __attribute__((aligned(16))) float tile[RW * TS];
  __shared__ long rowtab[RW];
  __shared__ int rowpix[RW];  // rowtab / ldc: the projection's output row
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntm = (p.M + X3_BM - 1) / X3_BM, ntn = (p.N + X3_BN - 1) / X3_BN;
  const long ntile = (long)ntm * ntn;
  const int qtr = blockIdx.x & 3;
  const long tl = blockIdx.x >> 2;
  const int tile_i = (int)(tl % ntile), ph = (int)(tl / ntile);
  if (ph >= zdim) return;  // workgroup-uniform
  const int tm = tile_i / ntn, tn = tile_i - tm * ntn;
  const int py = ph >> 1, px = ph & 1;
  const int r16 = qtr * RW + 16 * w;  // this wave's 16 rows within the 256-row tile
  const int wm = r16 >> 6, ti = (r16 & 63) >> 4;
  const long sstride = ntile * (X3_BM * X3_BN / 4);
  const f32x4* src = reinterpret_cast<const f32x4*>(p.kslab) + (long)ph * p.ksplit * sstride + (long)tile_i * 8 * 16 * 64;
  f32x4 v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the chunk's projection weights (proj16's b operands: row 16 t + m, k = 16 g + 4 q .. + 3) into registers first,
  // so their loads overlap the slab loads instead of chaining through proj16's k loop
  const int cc = tn * X3_BN, cw = min(PROJ_CHUNK, p.N - cc);
  const int mm = lane & 15, qq = lane >> 4;
  f32x4 wb[PROJ_CHUNK / 16][NT];
#pragma unroll
  for (int g = 0; g < PROJ_CHUNK / 16; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t)
      wb[g][t] = 16 * g < cw ? *reinterpret_cast<const f32x4*>(p.proj_w + cc + (long)(16 * t + mm) * p.proj_ldw + 16 * g + 4 * qq)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
  if (tm * X3_BM + r16 < p.M) {  // wave-uniform
    // two slabs' 16 loads in flight before their adds (in slab order per output)
    int sl = 0;
    for (; sl + 2 <= p.ksplit; sl += 2) {
      f32x4 t[2][8];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < 8; ++u) {  // u = (wave_n, j): columns 64 (u >> 2) + 16 (u & 3)
          const int wv = wm * 2 + (u >> 2), ij = ti * 4 + (u & 3);
          t[h][u] = src[(long)(sl + h) * sstride + ((long)wv * 16 + ij) * 64 + lane];
        }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] += t[h][u];
    }
    for (; sl < p.ksplit; ++sl) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int wv = wm * 2 + (u >> 2), ij = ti * 4 + (u & 3);
        v[u] += src[(long)sl * sstride + ((long)wv * 16 + ij) * 64 + lane];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) tile[(16 * w + 4 * (lane >> 4) + r) * TS + 16 * u + (lane & 15)] = v[u][r];
  if (tid < RW) {
    const int m = tm * X3_BM + qtr * RW + tid;
    const long ro = m < p.M ? gemm_row_offset<O_PHASE>(p, m, py, px) : -1;
    rowtab[tid] = ro;
    rowpix[tid] = ro >= 0 ? (int)(ro / p.ldc) : -1;
  }
  __syncthreads();
  GemmArgs q = p;
  if (p.proj_nostore) q.C = nullptr;
  for (int o = tid; o < RW * 16; o += 256) {
    const int row = o >> 4, oc = (o & 15) * 8;
    const int m = tm * X3_BM + qtr * RW + row, n = tn * X3_BN + oc;
    if (m >= p.M || n >= p.N) continue;
    float e8[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) e8[c] = tile[row * TS + oc + c];
    x3_octet_epilogue_at<EPI_BIAS_ACT>(q, rowtab[row] + n, n, e8);
    *reinterpret_cast<f32x4*>(tile + row * TS + oc) = f32x4{e8[0], e8[1], e8[2], e8[3]};
    *reinterpret_cast<f32x4*>(tile + row * TS + oc + 4) = f32x4{e8[4], e8[5], e8[6], e8[7]};
  }
  __syncthreads();
  // proj16's arithmetic (same MFMA sequence per output) with the preloaded weights
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < PROJ_CHUNK / 16; ++g) {
    if (16 * g >= cw) break;
    const f32x4 a = *reinterpret_cast<const f32x4*>(tile + (16 * w + mm) * TS + 16 * g + 4 * qq);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], wb[g][t][e], acc[t], 0, 0, 0);
  }
  float* Pc = p.proj_out + (cc / PROJ_CHUNK) * p.proj_pstride;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pix = rowpix[16 * w + 4 * qq + r];
      if (pix >= 0) Pc[(long)pix * (16 * NT) + 16 * t + mm] = acc[t][r];
    }
}

template <int EPI, int OM>
__global__ void x3_ksplit_reduce_kernel(GemmArgs p, int zdim) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int noct = p.N / 8;
  if (i >= (long)zdim * p.M * noct) return;
  const int oct = (int)(i % noct);
  const long r = i / noct;
  const int m = (int)(r % p.M), ph = (int)(r / p.M);
  const int py = OM == O_PHASE ? ph >> 1 : 0, px = OM == O_PHASE ? ph & 1 : 0;
  const int n = oct * 8;
  // the blocks in order from 0: each add the kernel's fmaf(sign, block, tot) with the sign already applied
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int sl = 0; sl < p.ksplit; ++sl) {
    const float* src = p.kslab + ((long)(ph * p.ksplit + sl) * p.M + m) * p.N + n;
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(src);
    const f32x4 t1 = *reinterpret_cast<const f32x4*>(src + 4);
    v[0] += t0.x; v[1] += t0.y; v[2] += t0.z; v[3] += t0.w;
    v[4] += t1.x; v[5] += t1.y; v[6] += t1.z; v[7] += t1.w;
  }
  x3_octet_epilogue<EPI, OM>(p, m, n, py, px, v);
}

// the octet epilogue at output offset idx (row offset + n)
template <int EPI>
__device__ __forceinline__ void x3_octet_epilogue_at(const GemmArgs& p, long idx, int n, float (&v)[8]) {
  if (EPI == EPI_BIAS_ACT) {
    if (p.bias) {
      const int nb = p.bias_mod < p.N ? n % p.bias_mod : n;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += p.bias[nb + e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = act_apply(v[e], p.act, p.slope);
  } else if (EPI == EPI_MASK) {
    if (p.mask_sgn) {
      const unsigned bits = p.mask_sgn[idx >> 3];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= ((bits >> e) & 1u) ? 1.f : p.mask_slope;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= act_grad_from_out(p.mask[idx + e], p.mask_act, p.mask_slope);
    }
  }
  if (p.sgn) {
    unsigned bits = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) bits |= (v[e] > 0.f ? 1u : 0u) << e;
    p.sgn[idx >> 3] = (unsigned char)bits;
  }
  if (p.C) {
    *reinterpret_cast<f32x4*>(p.C + idx) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(p.C + idx + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
  if (p.C3) {
    bf16x8 h, mm, l;
    split3_octet(v, h, mm, l);
    bf16x8* o = reinterpret_cast<bf16x8*>(p.C3 + 3 * idx);
    o[0] = h;
    o[1] = mm;
    o[2] = l;
  }
}
template <int EPI, int OM>
__device__ __forceinline__ void x3_octet_epilogue(const GemmArgs& p, int m, int n, int py, int px, float (&v)[8]) {
  x3_octet_epilogue_at<EPI>(p, gemm_row_offset<OM>(p, m, py, px) + n, n, v);
}

// Skinny limb GEMM for the first layer at per-rank batches (z . W, M = B <= 32 rows, K <= negk: one sign block,
// a 1 x 1 "convolution" of dense rows): 4 waves per workgroup, each 16 rows x 64 columns; the K tiles go from memory
// straight into registers (two tiles' 30 loads of 16 B per lane in flight, no LDS staging, no barrier) -- the
// 128 x 256 kernel streams its 50 MB of weight limbs through a two-deep LDS pipeline that left each workgroup
// latency-bound at 4 K tiles.  Same fragments (octet q of the tile per lane quarter), the same six-product MFMA
// sequence and the same block fold (fmaf(+1, acc, 0)), then gemm_x3_kernel's octet epilogue (x3_octet_epilogue):
// every output is bitwise the 128 x 256 kernel's (tests/test_gpu_langevin.py).
// Round 5: each wave takes 16 rows x 16 NTW columns (NTW = 2 by default: twice the waves of the 64-column form, which
// serialised its loads at 86 VGPRs, and half those of NTW = 1, whose 1024 workgroups measured 5-17 us slower per CIFAR
// B=16 step), and
// F32B reads the weights as fp32 rows split in registers with the packer's RNE split (2/3 of the limb bytes).  The
// MFMA sequence per output is unchanged, so every output is still bitwise the 128 x 256 kernel's.
template <bool F32B, int NTW>
__global__ __launch_bounds__(256) void x3_skinny_kernel(GemmArgs p) {
  constexpr int WC = 16 * NTW, KU = 4;  // columns per wave, K tiles per batch of loads
  __shared__ __attribute__((aligned(16))) float st[4][16][WC + 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, q = lane >> 4;
  const int n0 = (blockIdx.x * 4 + wave) * WC, r0 = blockIdx.y * 16;
  if (n0 >= p.N) return;  // wave-uniform; the waves share no barrier
  const int K8 = p.K >> 3, nk = p.K >> 5;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A3, (short)0, p.M * p.K * 6, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = F32B ? __builtin_amdgcn_make_buffer_rsrc((void*)p.b32k, (short)0, p.N * p.K * 4, 0x00020000)
                                        : __builtin_amdgcn_make_buffer_rsrc((void*)p.B3, (short)0, p.N * p.K * 6, 0x00020000);
  constexpr int OOB = 0x7FFFFFF0;
  const int aoff = (r0 + m < p.M) ? ((r0 + m) * K8 + q) * 48 : OOB;
  int boff[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
    boff[t] = (n0 + 16 * t + m < p.N) ? (F32B ? ((n0 + 16 * t + m) * p.K + 8 * q) * 4 : ((n0 + 16 * t + m) * K8 + q) * 48)
                                      : OOB;
  f32x4 acc[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto ld = [&](const __amdgpu_buffer_rsrc_t& r, int off, int kt, int l) {
    // the sgpr offset must be wave-uniform (a per-lane soffset made the compiler wrap every load in a waterfall loop);
    // an out-of-range lane's voffset (OOB) alone takes the load out of range
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, kt * 192 + l * 16, 0));
  };
  for (int kt = 0; kt < nk; kt += KU) {
    bf16x8 fa[KU][3], fb[KU][NTW][3];
    if constexpr (F32B) {
      // 8 fp32 of row n per lane and K tile (two 16-B loads), split as the packer splits (K <= negk: sign block 0)
      f32x4 fv[KU][NTW][2];
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const bool live = kt + u < nk;
#pragma unroll
        for (int l = 0; l < 3; ++l) fa[u][l] = ld(ra, live ? aoff : OOB, kt + u, l);
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            fv[u][t][h] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, live ? boff[t] : OOB, (kt + u) * 128 + h * 16, 0));
      }
      __builtin_amdgcn_sched_barrier(0);  // every load of the batch issued before the split waits on one
#pragma unroll
      for (int u = 0; u < KU; ++u)
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          const float v[8] = {fv[u][t][0][0], fv[u][t][0][1], fv[u][t][0][2], fv[u][t][0][3],
                              fv[u][t][1][0], fv[u][t][1][1], fv[u][t][1][2], fv[u][t][1][3]};
          split3_octet(v, fb[u][t][0], fb[u][t][1], fb[u][t][2]);
        }
    } else {
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const bool live = kt + u < nk;
#pragma unroll
        for (int l = 0; l < 3; ++l) {
          fa[u][l] = ld(ra, live ? aoff : OOB, kt + u, l);
#pragma unroll
          for (int t = 0; t < NTW; ++t) fb[u][t][l] = ld(rb, live ? boff[t] : OOB, kt + u, l);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // every load of the batch issued before the first MFMA waits on one
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (kt + u >= nk) break;
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        f32x4 c = acc[t];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][2], fb[u][t][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][1], fb[u][t][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][0], fb[u][t][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][1], fb[u][t][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][0], fb[u][t][1], c, 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][0], fb[u][t][0], c, 0, 0, 0);
      }
    }
  }
  // the block fold of gemm_x3_kernel's last partial block (tot = 0, sign block 0 positive), then the epilogue
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) st[wave][4 * q + r][16 * t + m] = __builtin_fmaf(1.f, acc[t][r], 0.f);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  constexpr int NOCT = 16 * WC / 8;  // (row, octet) items of the wave's tile
#pragma unroll
  for (int j = 0; j < (NOCT + 63) / 64; ++j) {
    const int id = lane + 64 * j, row = id / (WC / 8), oct = id % (WC / 8);
    const int mg = r0 + row, n = n0 + 8 * oct;
    if (id >= NOCT || mg >= p.M || n >= p.N) continue;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = st[wave][row][8 * oct + e];
    x3_octet_epilogue<EPI_BIAS_ACT, O_DENSE>(p, mg, n, 0, 0, v);
  }
}

// split-K plan of a limb-engine conv: an under-filled grid (see below; DAMC_X3_KSPLIT_WGS pins the bound) splits K
// into its negk sign blocks (GemmArgs::negk), one per slice.  A slice's tile is then exactly the unsplit kernel's block sum (sign applied), and the reduce adds
// the blocks in the kernel's order with the kernel's single rounding per block: the split result is bitwise the
// unsplit one, so a batch split over ranks (or calls) still reproduces the one-call chains bit for bit
int x3_ksplit(int M, int N, int K, int zdim, int bm, int bn, int negk = X3_NEGK) {
  // DAMC_X3_KSPLIT=0 disables; DAMC_X3_KSPLIT_WGS: the grid size below which a conv splits (A/B)
  const char* ev = getenv("DAMC_X3_KSPLIT");  // per call: tests compare both paths in one process
  const bool on = !(ev && ev[0] == '0');
  static const long below = [] {
    const char* e = getenv("DAMC_X3_KSPLIT_WGS");
    return e ? atol(e) : -1L;
  }();
  const long wgs = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * zdim;
  if (!on || K % negk != 0 || K / negk < 2) return 1;
  const int ks = K / negk;
  // default: below 128 workgroups always; below 256 (half the chip idle) when K has at most 16 sign blocks, since
  // the slab bytes grow with K (CIFAR B=16/32 per-rank steps -2.6 / -1.5 %, B=64's K=8192 dgrad stays unsplit)
  const bool split = below >= 0 ? wgs < below : (wgs < 128 || (wgs < 256 && ks <= 16));
  return split ? ks : 1;
}

long x3_ksplit_floats(int M, int N, int K, int zdim, int negk) {  // either block layout (gemm_x3_kernel, V & 524288)
  const int ks = std::max(x3_ksplit(M, N, K, zdim, X3_BM, X3_BN, negk), x3_ksplit(M, N, K, zdim, 128, 256, negk));
  // the register slab layout covers whole 256 x 128 tiles
  const long padded = (long)((M + X3_BM - 1) / X3_BM) * X3_BM * ((N + X3_BN - 1) / X3_BN) * X3_BN;
  return ks > 1 ? (long)zdim * ks * std::max((long)M * N, padded) : 0;
}

template <int EPI, int OM, int V = DAMC_X3_VARIANT>
static int launch_x3_t(const GemmArgs& a0, int zdim, hipStream_t s) {
  GemmArgs a = a0;
  constexpr int BM = (V & 524288) ? 128 : X3_BM, BN = (V & 524288) ? 256 : X3_BN;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  // the norm statistics in the epilogue (GemmArgs::in_part): the unsplit 256 x 128 dense tile only; every other launch
  // clears in_done and leaves them to the caller's kernel
  auto no_stats = [&]() {
    if (a.in_part && a.in_done) *a.in_done = 0;
    a.in_part = nullptr;
  };
  if (a.in_part && !(OM == O_DENSE && EPI == EPI_BIAS_ACT && BM == 256 && BN == 128 && zdim == 1 && a.in_hw > 0 &&
                     a.in_hw % 256 == 0 && a.M % a.in_hw == 0 && a.in_S == a.in_hw / 256))
    no_stats();
  if constexpr (V == DAMC_X3_VARIANT && OM != O_WGRAD) {
    // opt-in (DAMC_X3_NARROW=1, read per call): an under-filled grid that the 64 x 128 tile fills (>= 256 workgroups)
    // runs unsplit on it instead of split-K.  Measured slower at the CIFAR B=16 per-rank step: 158.7 / 152.2 us for the
    // L2 forward / L3 dgrad against 121 / 122 us for split-K + reduce (profiles/r04/b16_narrow_kernel_stats.csv): the
    // 32 x 32 wave tile reads 2x the LDS fragments per MFMA and stages 1.5x the bytes per flop
    const char* en = getenv("DAMC_X3_NARROW");
    const long nnm = (a.M + 63) / 64;
    if (a.kslab && !a.proj_out && !a.kwalk && en && en[0] == '1' && (long)ntm * ntn * zdim < 256 &&
        nnm * ntn * zdim >= 256) {
      no_stats();
      a.ksplit = 1;
      a.kbpw = 1;
      a.kslab_reg = 0;
      hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, (V & ~(8 | 16)) | X3_NARROW>), dim3((unsigned)(nnm * ntn), 1, zdim), dim3(512), 0, s,
                         a);
      return 0;
    }
  }
  if (OM != O_WGRAD && a.kslab && !(V & 16)) {
    const int ks = x3_ksplit(a.M, a.N, a.K, zdim, BM, BN, a.negk);
    if (ks > 1 && (long)zdim * ks * a.M * a.N <= a.kslab_floats && a.N % 8 == 0) {
      no_stats();
      a.ksplit = ks;
      const int nostore0 = a.proj_nostore;  // the caller's: honoured where the reduce runs the projection itself
      a.proj_nostore = 0;  // the reduce writes C; the projection then runs as proj_rows_kernel over it
      auto proj_after = [&]() {
        if (OM == O_PHASE && a.proj_out)
          return launch_proj_rows(a.C, (long)(a.M / (a.Hq * a.Wq)) * a.Hout * a.Wout, a.N, a.proj_w, a.proj_ldw,
                                  a.proj_np, a.proj_out, a.proj_pstride, s);
        return 0;
      };
      // sign blocks per workgroup: the most (a power of two dividing ks) that still leaves >= 256 workgroups, so one
      // round covers the chip (the default 16x16-tile path only); DAMC_X3_KSPLIT_BPW (read per call) pins it
      int bpw = 1;
      if ((V & ~X3_F32A) == DAMC_X3_VARIANT && (V & 1) && !(V & (2048 | 65536 | 131072 | 262144))) {
        const char* eb = getenv("DAMC_X3_KSPLIT_BPW");
        if (eb) {
          bpw = std::max(1, atoi(eb));
          while (bpw > 1 && ks % bpw) bpw >>= 1;
        } else {
          while (ks % (2 * bpw) == 0 && (long)ntm * ntn * zdim * ks / (2 * bpw) >= 256) bpw *= 2;
        }
      }
      // the register slab layout on the default 16x16-tile path (256 x 128 tiles), row-major slabs (one block per
      // workgroup) otherwise; DAMC_X3_KSLAB_REG=0, read per call, forces row-major
      const char* er = getenv("DAMC_X3_KSLAB_REG");
      a.kslab_reg = (!(er && er[0] == '0') && BM == X3_BM && BN == X3_BN && (V & 1) && (V & 4) &&
                     !(V & (32 | 2048 | 65536 | 131072 | 262144)) && (long)zdim * ks * ntm * ntn * BM * BN <= a.kslab_floats &&
                     (long)bpw * ntm * ntn * BM * BN * 4 < (1L << 31))
                        ? 1 : 0;
      if (!a.kslab_reg) bpw = 1;
      a.kbpw = bpw;
      a.k_per_z = a.K / ks * bpw;
      if constexpr ((V & ~X3_F32A) == DAMC_X3_VARIANT && OM != O_WGRAD && (V & 1) && (V & 4) &&
                    !(V & (32 | 2048 | 65536 | 131072 | 262144 | 524288))) {
        if constexpr ((V & X3_F32A) != 0 && ((EPI == EPI_BIAS_ACT && OM == O_PHASE) || (EPI == EPI_MASK && OM == O_DENSE))) {
          // round 6, opt-in (DAMC_X3_FIXUP=1, read per call): the in-GEMM ordered fix-up instead of the reduce launch
          // (bitwise; gemm_x3_kernel X3_FIXUP) where the caller provides zeroed counters.  Measured slower at every
          // per-rank batch (CIFAR B=16 0.474-0.485 against 0.410 ms per step, SVHN B=64 0.386-0.391 against
          // 0.216-0.226; profiles/r06/fixup_ab.txt): the slabs' write-through, the wait for the tile's slowest slice
          // and the bands' reads of 32 MB of slabs put 15-20 us on every launch's tail (profiles/r06/fixup_timeline.txt),
          // more than the 9-17 us reduce launch they replace
          const char* ef = getenv("DAMC_X3_FIXUP");
          const long grid = (long)ntm * ntn * zdim * (ks / bpw);
          if (a.kslab_reg && a.kticket && a.kepoch_ctr && *a.kepoch_ctr < 65535u && ef && ef[0] == '1' &&
              grid <= 256 && grid <= X3_KTICKETS && (long)ks * ntm * ntn * BM * BN * 4 < (1L << 31)) {
            a.kepoch = ++*a.kepoch_ctr;  // this launch's tag on the counters and claims (16 bits; zeroed per call)
            a.fixup_probe = g_fixup_probe;
            a.proj_nostore = nostore0;  // the epilogue runs the fused projection itself, as the unsplit kernel does
            hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, V | 1048576 | X3_FIXUP>), dim3(ntm * ntn, 1, zdim * ks / bpw),
                               dim3(512), 0, s, a);
            return 0;
          }
        }
        if (a.kslab_reg)
          hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, V | 1048576>), dim3(ntm * ntn, 1, zdim * ks / bpw), dim3(512), 0,
                             s, a);
        else
          hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, V>), dim3(ntm * ntn, 1, zdim * ks / bpw), dim3(512), 0, s, a);
      } else {
        a.kslab_reg = 0;
        hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, V>), dim3(ntm * ntn, 1, zdim * ks / bpw), dim3(512), 0, s, a);
      }
      if (a.kslab_reg) {  // one wave per 16x16 tile, four per workgroup
        if (EPI == EPI_BIAS_ACT && OM == O_DENSE && a.ksplit_deferred && !a.C3 && !a.sgn) {
          *a.ksplit_deferred = ks;  // the consumer sums the slabs (GemmArgs::ksplit_deferred)
          return 0;
        }
        // a ConvT forward with the fused output-layer projection: the reduce runs the projection too (bitwise the
        // reduce + proj_rows_kernel); DAMC_REDUCE_PROJ=0 (read per call) keeps the two kernels
        const char* erp = getenv("DAMC_REDUCE_PROJ");
        if (OM == O_PHASE && EPI == EPI_BIAS_ACT && a.proj_out && a.N % 16 == 0 && a.N <= 256 &&
            (a.N <= PROJ_CHUNK || a.N % PROJ_CHUNK == 0) && (a.proj_np == 32 || a.proj_np == 64) &&
            !(erp && erp[0] == '0')) {
          a.proj_nostore = nostore0;
          const unsigned nwg = (unsigned)(zdim * ntm * ntn * 4);
          if (a.proj_np == 32)
            hipLaunchKernelGGL((x3_ksplit_reduce_proj_kernel<2>), dim3(nwg), dim3(256), 0, s, a, zdim);
          else
            hipLaunchKernelGGL((x3_ksplit_reduce_proj_kernel<4>), dim3(nwg), dim3(256), 0, s, a, zdim);
          return (int)hipGetLastError();
        }
        const long waves = (long)zdim * ntm * ntn * 128;
        hipLaunchKernelGGL((x3_ksplit_reduce_tile_kernel<EPI, OM>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s,
                           a, zdim);
        return proj_after();
      }
      const long tot = (long)zdim * a.M * (a.N / 8);
      hipLaunchKernelGGL((x3_ksplit_reduce_kernel<EPI, OM>), dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, a,
                         zdim);
      return proj_after();
    }
  }
  a.ksplit = 1;
  a.kbpw = 1;
  a.kslab_reg = 0;
  if constexpr ((V & X3_F32A) != 0 && OM == O_PHASE && !(V & 16)) {
    // round 5: the unsplit F32A ConvT forward on the supertile raster (bit 16: each XCD's concurrent workgroups cover
    // <= 8 M tiles x the 4 phases of an N tile, so the phases' overlapping input windows and weight panels are shared
    // in its L2).  Bitwise the default raster; CIFAR B=128 upconv_fwd FETCH 1059 -> 705 MB per launch at the same
    // time (548 vs 551 us; profiles/r05/walk_ab.txt).  DAMC_X3_RASTER=0 (read per call) keeps the default raster
    const char* er = getenv("DAMC_X3_RASTER");
    if (!(er && er[0] == '0')) {
      hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, V | 16>), dim3(ntm * ntn * zdim, 1, 1), dim3(512), 0, s, a);
      return 0;
    }
  }
  if ((V & 16) && OM != O_WGRAD)  // supertile raster: phases folded into a 1-D grid
    hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, V>), dim3(ntm * ntn * zdim, 1, 1), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_x3_kernel<EPI, OM, V>), dim3(ntm * ntn, 1, zdim), dim3(512), 0, s, a);
  return 0;
}

// fp32 [rows][C] -> x3 [rows][C/8][3][8]; one thread per channel octet
__global__ void split_x3_kernel(const float* __restrict__ x, long n8, unsigned short* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const f32x4 v0 = reinterpret_cast<const f32x4*>(x)[2 * i];
  const f32x4 v1 = reinterpret_cast<const f32x4*>(x)[2 * i + 1];
  const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  bf16x8 h, m, l;
  split3_octet(v, h, m, l);
  bf16x8* o = reinterpret_cast<bf16x8*>(y) + 3 * i;
  o[0] = h;
  o[1] = m;
  o[2] = l;
}

// rows of K values; octets in odd negk-blocks of a row negated
__global__ void split_x3_negblk_kernel(const float* __restrict__ x, long n8, int K8, unsigned short* __restrict__ y,
                                       int negk) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const long k8 = i % K8;
  const float sg = ((k8 * 8 / negk) & 1) ? -1.f : 1.f;
  const f32x4 v0 = reinterpret_cast<const f32x4*>(x)[2 * i];
  const f32x4 v1 = reinterpret_cast<const f32x4*>(x)[2 * i + 1];
  const float v[8] = {sg * v0.x, sg * v0.y, sg * v0.z, sg * v0.w, sg * v1.x, sg * v1.y, sg * v1.z, sg * v1.w};
  bf16x8 h, m, l;
  split3_octet(v, h, m, l);
  bf16x8* o = reinterpret_cast<bf16x8*>(y) + 3 * i;
  o[0] = h;
  o[1] = m;
  o[2] = l;
}

int launch_split_x3_negblk(const float* x, long n, int K, unsigned short* y, hipStream_t s, int negk) {
  if (K <= 0 || K % 8 != 0 || n % K != 0 || ((uintptr_t)x | (uintptr_t)y) % 16 != 0) return DAMC_ERR_ARG;
  const long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(split_x3_negblk_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, x, n8, K / 8, y, negk);
  return (int)hipGetLastError();
}

// weight rows of K = taps * Cg values in tap-major order [tap][c] -> x3 in slice-major order
// [c / 32][tap][c % 32] (the channel-major K walk, V & 8), odd negk-blocks of the new order negated
__global__ void split_x3_cmaj_kernel(const float* __restrict__ x, long n8, int K8, int Cg8, int taps, int sw8,
                                     unsigned short* __restrict__ y, int negk) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // source octet
  if (i >= n8) return;
  const long row = i / K8;
  const int k8 = (int)(i - row * K8);
  const int tp = k8 / Cg8, c8 = k8 - tp * Cg8;  // octet c8 of tap tp
  const int d8 = (c8 / sw8) * taps * sw8 + tp * sw8 + c8 % sw8;  // destination octet within the row
  const float sg = ((d8 * 8 / negk) & 1) ? -1.f : 1.f;
  const f32x4 v0 = reinterpret_cast<const f32x4*>(x)[2 * i];
  const f32x4 v1 = reinterpret_cast<const f32x4*>(x)[2 * i + 1];
  const float v[8] = {sg * v0.x, sg * v0.y, sg * v0.z, sg * v0.w, sg * v1.x, sg * v1.y, sg * v1.z, sg * v1.w};
  bf16x8 h, m, l;
  split3_octet(v, h, m, l);
  bf16x8* o = reinterpret_cast<bf16x8*>(y) + 3 * (row * K8 + d8);
  o[0] = h;
  o[1] = m;
  o[2] = l;
}

int launch_split_x3_cmaj(const float* x, long n, int K, int Cg, int sw, unsigned short* y, hipStream_t s, int negk) {
  if (K <= 0 || Cg <= 0 || sw <= 0 || sw % 8 != 0 || Cg % sw != 0 || K % Cg != 0 || n % K != 0 ||
      ((uintptr_t)x | (uintptr_t)y) % 16 != 0)
    return DAMC_ERR_ARG;
  const long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(split_x3_cmaj_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, x, n8, K / 8, Cg / 8,
                     K / Cg, sw / 8, y, negk);
  return (int)hipGetLastError();
}

// rows of K = 16 Cg values in tap-major order [tap][c] -> x3 in the 4 x 4 conv walk (x3_conv_walk: [c / 32][x3_walk_pos
// (tap)][c % 32]), sign blocks counted in the walk order
__global__ void split_x3_walk_kernel(const float* __restrict__ x, long n8, int K8, int Cg8,
                                     unsigned short* __restrict__ y, int negk) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // source octet
  if (i >= n8) return;
  const long row = i / K8;
  const int k8 = (int)(i - row * K8);
  const int tp = k8 / Cg8, c = (k8 - tp * Cg8) * 8;
  const int kk = (c >> 5) * 16 * 32 + x3_walk_pos(tp) * 32 + (c & 31);
  const float sg = ((kk / negk) & 1) ? -1.f : 1.f;
  const f32x4 v0 = reinterpret_cast<const f32x4*>(x)[2 * i];
  const f32x4 v1 = reinterpret_cast<const f32x4*>(x)[2 * i + 1];
  const float v[8] = {sg * v0.x, sg * v0.y, sg * v0.z, sg * v0.w, sg * v1.x, sg * v1.y, sg * v1.z, sg * v1.w};
  bf16x8 h, m, l;
  split3_octet(v, h, m, l);
  bf16x8* o = reinterpret_cast<bf16x8*>(y) + 3 * (row * K8 + (kk >> 3));
  o[0] = h;
  o[1] = m;
  o[2] = l;
}

int launch_split_x3_walk(const float* x, long n, int K, int Cg, unsigned short* y, hipStream_t s, int negk) {
  if (Cg <= 0 || Cg % 32 != 0 || K != 16 * Cg || n % K != 0 || ((uintptr_t)x | (uintptr_t)y) % 16 != 0)
    return DAMC_ERR_ARG;
  const long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(split_x3_walk_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, x, n8, K / 8, Cg / 8,
                     y, negk);
  return (int)hipGetLastError();
}

int launch_split_x3_conv(const float* x, long n, int K, int Cg, unsigned short* y, hipStream_t s, int negk) {
  if ((DAMC_X3_VARIANT & 8) != 0 && Cg % 32 == 0) return launch_split_x3_cmaj(x, n, K, Cg, 32, y, s, negk);
  return launch_split_x3_negblk(x, n, K, y, s, negk);
}

// ---- generator-layer weight packing through LDS tiles (damc_pack_generator_layer's hot layouts): a ConvTranspose2d
// weight W[ci][co][tap] (kk <= 16 taps) read in contiguous rows, written as whole octets of the packed matrix, with
// its x3 copy (sign-alternating negk blocks, split_x3_negblk_kernel's values) in the same pass -- the per-call
// packing was scattered 4-byte stores plus a second read for the limb split.
__device__ __forceinline__ void pack_store_octet(const float (&v)[8], long flat, int k, float* __restrict__ out,
                                                 unsigned short* __restrict__ x3, int negk) {
  f32x4* o = reinterpret_cast<f32x4*>(out + flat);
  o[0] = f32x4{v[0], v[1], v[2], v[3]};
  o[1] = f32x4{v[4], v[5], v[6], v[7]};
  if (x3) {
    const float sg = ((k / negk) & 1) ? -1.f : 1.f;
    const float u[8] = {sg * v[0], sg * v[1], sg * v[2], sg * v[3], sg * v[4], sg * v[5], sg * v[6], sg * v[7]};
    bf16x8 h, m, l;
    split3_octet(u, h, m, l);
    bf16x8* y = reinterpret_cast<bf16x8*>(x3) + 3 * (flat / 8);
    y[0] = h;
    y[1] = m;
    y[2] = l;
  }
}

// out[ci][tap][co] = W[ci][co][tap]; x3 rows ci of K = kk * cout. Block: one ci, 128 output channels (kk <= 64).
constexpr int PK_ROW_CO = 128;
__global__ void __launch_bounds__(256) pack_rowT_kernel(const float* __restrict__ w, int cout, int kk,
                                                        float* __restrict__ out, unsigned short* __restrict__ x3,
                                                        int negk) {
  __shared__ float t[PK_ROW_CO * 65];
  const int ci = blockIdx.y, co0 = blockIdx.x * PK_ROW_CO;
  const int nco = min(PK_ROW_CO, cout - co0), nco8 = nco / 8, ld = kk + 1;
  const float* src = w + ((long)ci * cout + co0) * kk;
  for (int e = threadIdx.x; e < nco * kk; e += 256) t[(e / kk) * ld + e % kk] = src[e];
  __syncthreads();
  for (int o = threadIdx.x; o < kk * nco8; o += 256) {
    const int tap = o / nco8, c8 = o - tap * nco8;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[(c8 * 8 + j) * ld + tap];
    const int k = tap * cout + co0 + c8 * 8;
    pack_store_octet(v, (long)ci * kk * cout + k, k, out, x3, negk);
  }
}

// out[seg][ci] with seg(co, tap) = the ConvT forward row order: UP2 ((phase * cout + co) * 4 + ty * 2 + tx, x3 rows
// of 4 Cin per (phase, co)), PROJ (tap * cout + co, x3 rows of Cin). Block: 32 input x 128 / kk output channels (each
// input channel's run of 128 contiguous weights).
__global__ void __launch_bounds__(256) pack_colT_kernel(const float* __restrict__ w, int cin, int cout, int kk, int up2,
                                                        float* __restrict__ out, unsigned short* __restrict__ x3,
                                                        int negk) {
  __shared__ float t[32 * 129];
  const int cot = 128 / kk, ci0 = blockIdx.x * 32, co0 = blockIdx.y * cot, rl = 128, ld = rl + 1;
  for (int e = threadIdx.x; e < 32 * rl; e += 256) {
    const int cl = e / rl, r = e - cl * rl;
    t[cl * ld + r] = w[((long)(ci0 + cl) * cout + co0) * kk + r];
  }
  __syncthreads();
  for (int o = threadIdx.x; o < rl * 4; o += 256) {
    const int c8 = o & 3, r = o >> 2, col = r / kk, tap = r - col * kk, co = co0 + col;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[(c8 * 8 + j) * ld + r];
    long seg;
    int k = ci0 + c8 * 8;
    if (up2) {  // ky = 3 - py - 2 ty (the stride-2 phase decomposition, generator.hip pack_up2_kernel)
      const int ky = tap >> 2, kx = tap & 3, py = (3 - ky) & 1, px = (3 - kx) & 1;
      const int tt = ((3 - ky - py) >> 1) * 2 + ((3 - kx - px) >> 1);
      seg = ((long)(py * 2 + px) * cout + co) * 4 + tt;
      k += tt * cin;
    } else {
      seg = (long)tap * cout + co;
    }
    pack_store_octet(v, seg * cin + ci0 + c8 * 8, k, out, x3, negk);
  }
}

static bool pack_tiled_ok(const void* a, const void* b, const void* c, const void* d) {
  return (DAMC_X3_VARIANT & 8) == 0 &&  // the negblk limb order (launch_split_x3_conv)
         (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)d) % 16) == 0;
}

// 1 = layout not covered (the caller packs element-wise)
int launch_pack_up2_tiled(const float* w, int cin, int cout, float* wf, unsigned short* wf3, float* wb,
                          unsigned short* wb3, hipStream_t s, int negk_f, int negk_b) {
  if (cin % KM_BK != 0 || cout % KM_BK != 0 || !pack_tiled_ok(wf, wf3, wb, wb3)) return 1;
  hipLaunchKernelGGL(pack_colT_kernel, dim3(cin / 32, cout / 8), dim3(256), 0, s, w, cin, cout, 16, 1, wf, wf3, negk_f);
  hipLaunchKernelGGL(pack_rowT_kernel, dim3((cout + PK_ROW_CO - 1) / PK_ROW_CO, cin), dim3(256), 0, s, w, cout, 16,
                     wb, wb3, negk_b);
  return (int)hipGetLastError();
}

int launch_pack_proj_tiled(const float* w, int cin, int cout, int kk, float* wf, float* wb, unsigned short* wb3,
                           hipStream_t s) {
  if (kk > 64 || 128 % kk != 0 || cin % 32 != 0 || cout % 8 != 0 || cout % (128 / kk) != 0 ||
      !pack_tiled_ok(wf, wb, wb3, nullptr))
    return 1;
  hipLaunchKernelGGL(pack_rowT_kernel, dim3((cout + PK_ROW_CO - 1) / PK_ROW_CO, cin), dim3(256), 0, s, w, cout, kk,
                     wf, (unsigned short*)nullptr, X3_NEGK);
  hipLaunchKernelGGL(pack_colT_kernel, dim3(cin / 32, cout / (128 / kk)), dim3(256), 0, s, w, cin, cout, kk, 0, wb, wb3,
                     X3_NEGK);
  return (int)hipGetLastError();
}

// a PyTorch Conv2d weight (cout, cin, k, k) straight to the limb engine's B operand of the conv, [co][(ky, kx, ci)]
// with sign-alternating blocks (launch_split_x3_negblk of damc_pack_conv2d's K-major packing, in one pass)
__global__ void pack_conv_x3_kernel(const float* __restrict__ w, int cout, int cin, int k, unsigned short* __restrict__ y) {
  const int K = k * k * cin, K8 = K / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)cout * K8) return;
  const int co = (int)(i / K8), k8 = (int)(i - (long)co * K8);
  const int kk = k8 * 8, tap = kk / cin, ci0 = kk - tap * cin;  // cin % 8 == 0: an octet never straddles a tap
  const float sg = ((kk / X3_NEGK) & 1) ? -1.f : 1.f;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = sg * w[((long)co * cin + ci0 + e) * k * k + tap];
  bf16x8 h, m, l;
  split3_octet(v, h, m, l);
  bf16x8* o = reinterpret_cast<bf16x8*>(y) + 3 * i;
  o[0] = h;
  o[1] = m;
  o[2] = l;
}

// the same packing, one thread per (co, input-channel octet): its 8 channels' k*k taps are 8 * k * k contiguous
// floats of the PyTorch layout, read 4 taps at a time as f32x4 (k * k % 4 == 0); adjacent threads write adjacent
// 48-B limb octets of each tap (the thread-per-output-octet kernel above reads 4 B at a 64-B stride, every line 16x)
__global__ void pack_conv_x3_taps_kernel(const float* __restrict__ w, int cout, int cin, int k,
                                         unsigned short* __restrict__ y, int walk) {
  // one thread per (co, 4-tap group, channel octet), octets fastest: 4x the threads of one per (co, octet) walking
  // all its taps (CIFAR encoder: 4 launches 69 -> ~25 us per Q(x) call), same values and stores
  const int cin8 = cin / 8, taps = k * k, K8 = taps * cin8, tq = taps / 4;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)cout * tq * cin8) return;
  const int c8 = (int)(i % cin8);
  const long r = i / cin8;
  const int t0 = 4 * (int)(r % tq), co = (int)(r / tq);
  const f32x4* src = reinterpret_cast<const f32x4*>(w + ((long)co * cin + c8 * 8) * taps);
  bf16x8* o = reinterpret_cast<bf16x8*>(y) + 3L * co * K8;
  f32x4 q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] = src[(e * taps + t0) / 4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int c = c8 * 8;  // the octet's K index in the GEMM's walk (x3_conv_walk), which also sets its sign block
    const int kk = walk ? (c >> 5) * taps * 32 + x3_walk_pos(t0 + t) * 32 + (c & 31) : (t0 + t) * cin + c;
    const float sg = ((kk / X3_NEGK) & 1) ? -1.f : 1.f;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = sg * q[e][t];
    bf16x8 h, m, l;
    split3_octet(v, h, m, l);
    bf16x8* d = o + 3L * (kk >> 3);
    d[0] = h;
    d[1] = m;
    d[2] = l;
  }
}

// the same packing through LDS, one workgroup per (layer, co, chunk of CC input channels) (pack_conv_x3_block, gemm.h):
// every byte is read and written once, in full lines (the tap-group kernel below reads each 64-B line from 4 waves
// far apart).  Several layers share one launch (the encoder's per-call packing: one dispatch instead of one per layer)
__global__ __launch_bounds__(256) void pack_conv_x3_lds_kernel(PackConvList l) {
  extern __shared__ float pk_t[];  // [CC][taps + 1]
  pack_conv_x3_block(l, blockIdx.x, threadIdx.x, 256, pk_t);
}

bool pack_conv_x3_many_ok(const float* w, int cin, int k) {
  return (DAMC_X3_VARIANT & 8) == 0 && k > 0 && k * k <= 32 && (uintptr_t)w % 16 == 0 && (cin % 128 == 0 || cin == 64);
}

int pack_conv_x3_many_prep(PackConvList& l) {
  if (l.ready || l.n < 1 || l.n > 8) return 1;
  size_t sm = 0;
  l.blk0[0] = 0;
  for (int i = 0; i < l.n; ++i) {
    if (l.taps[i] <= 0 || l.taps[i] > 32 || (uintptr_t)l.w[i] % 16 || (uintptr_t)l.y[i] % 16 ||
        !(l.cin[i] % 128 == 0 || l.cin[i] == 64) || l.blk0[i + 1] <= 0)
      return 1;
    l.cc[i] = l.cin[i] % 128 == 0 ? 128 : 64;
    l.walk[i] = l.taps[i] == 16 ? x3_conv_walk(4, l.cin[i]) : 0;
    sm = std::max(sm, (size_t)l.cc[i] * (l.taps[i] + 1) * sizeof(float));
  }
  for (int i = 0; i < l.n; ++i) {
    l.cout[i] = l.blk0[i + 1];
    l.blk0[i + 1] = l.blk0[i] + l.blk0[i + 1] * (l.cin[i] / l.cc[i]);
  }
  // the grid is exactly the work list: one workgroup per (layer, co, channel chunk), nothing more
  long total = 0;
  for (int i = 0; i < l.n; ++i) total += (long)l.cout[i] * (l.cin[i] / l.cc[i]);
  if (total != l.blk0[l.n]) return 1;
  l.lds = (int)sm;
  l.ready = 1;
  return 0;
}

int launch_pack_conv_x3_many(PackConvList l, hipStream_t s) {
  if (!l.ready && pack_conv_x3_many_prep(l)) return 1;
  hipLaunchKernelGGL(pack_conv_x3_lds_kernel, dim3((unsigned)l.blk0[l.n]), dim3(256), (size_t)l.lds, s, l);
  return (int)hipGetLastError();
}

int launch_pack_conv_x3(const float* w, int cout, int cin, int k, unsigned short* y, hipStream_t s) {
  if ((DAMC_X3_VARIANT & 8) != 0) return DAMC_ERR_UNSUPPORTED;  // the channel-major walk needs the slice-major order
  if (cout <= 0 || cin % 8 != 0 || k <= 0 || (uintptr_t)y % 16 != 0) return DAMC_ERR_ARG;
  static const bool lds = [] {  // DAMC_PACK_CONV_LDS=0: the tap-group kernel below (A/B)
    const char* e = getenv("DAMC_PACK_CONV_LDS");
    return !(e && e[0] == '0');
  }();
  const int taps = k * k;
  if (lds && pack_conv_x3_many_ok(w, cin, k)) {
    PackConvList l{};
    l.n = 1;
    l.w[0] = w;
    l.y[0] = y;
    l.cin[0] = cin;
    l.taps[0] = taps;
    l.blk0[1] = cout;
    return launch_pack_conv_x3_many(l, s);
  }
  if ((k * k) % 4 == 0 && (uintptr_t)w % 16 == 0) {
    const long nt = (long)cout * (k * k / 4) * (cin / 8);
    hipLaunchKernelGGL(pack_conv_x3_taps_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, w, cout, cin, k,
                       y, x3_conv_walk(k, cin));
    return (int)hipGetLastError();
  }
  if (x3_conv_walk(k, cin)) return DAMC_ERR_UNSUPPORTED;  // (k = 4: the taps kernel above always takes it)
  const long n = (long)cout * k * k * cin / 8;
  hipLaunchKernelGGL(pack_conv_x3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, cout, cin, k, y);
  return (int)hipGetLastError();
}

int launch_split_x3(const float* x, long n, unsigned short* y, hipStream_t s) {
  if (n % 8 != 0 || ((uintptr_t)x | (uintptr_t)y) % 16 != 0) return DAMC_ERR_ARG;
  const long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(split_x3_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, x, n8, y);
  return (int)hipGetLastError();
}

// limb-engine dispatch (A3 / B3 set, A_CONV geometry as the K-major engine); splits the batch so every
// launch's gathered x3 tensor stays below 2^31 bytes
// damc_clock_probe: the buffer O_PHASE limb-engine launches stamp (null: off)
static unsigned long long* g_clk = nullptr;
static int g_clk_n = 0;
static unsigned g_clk_launch = 0;  // DAMC_CLOCK_REGIONS=R (tools): every limb-engine launch stamps region launch % R

// an at-most-128-row GEMM whose K holds >= 8 sign blocks (the encoder's last conv: M = B, N = nemb, K = 16 Cin): the
// 64 x 128 tile split into its sign blocks (row-major slabs, x3_ksplit_reduce_kernel), 4x the workgroups of the
// 128 x 256 layout's split (CIFAR B=128: 16 x 16 = 256 instead of 64); bitwise the same (one slab per sign block)
template <int EPI>
static void launch_x3_narrow_split(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int ks = a.K / a.negk;
  a.ksplit = ks;
  a.kbpw = 1;
  a.kslab_reg = 0;
  a.k_per_z = a.negk;
  a.proj_nostore = 0;
  const int ntm = (a.M + 63) / 64, ntn = (a.N + X3_BN - 1) / X3_BN;
  hipLaunchKernelGGL((gemm_x3_kernel<EPI, O_DENSE, (DAMC_X3_VARIANT & ~(8 | 16)) | X3_NARROW>), dim3(ntm * ntn, 1, ks), dim3(512), 0, s,
                     a);
  const long tot = (long)a.M * (a.N / 8);
  hipLaunchKernelGGL((x3_ksplit_reduce_kernel<EPI, O_DENSE>), dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, a,
                     1);
}

// the skinny first-layer kernel's row limit: 32.  DAMC_X3_SKINNY_ROWS (read per call) moves it for A/B; at the
// headline's B = 128 the skinny form (8 x N / 64 workgroups, bitwise the same) took 81.8 us against 30.4 us for the
// 128 x 256 layout (profiles/r05/skinny128_ab.txt)
static int x3_skinny_max_rows() {
  const char* e = getenv("DAMC_X3_SKINNY_ROWS");
  return e ? atoi(e) : 32;
}

static int launch_gemm_x3(const GemmArgs& a, Epi epi, OMode om, int zdim, hipStream_t s) {
  const int taps = a.Cg > 0 ? a.K / a.Cg : 0;
  if (!(a.a_f32 ? a.A != nullptr : a.A3 != nullptr) || !a.B3 || a.Cg % X3_BK != 0 || taps * a.Cg != a.K || a.kw <= 0 ||
      taps % a.kw != 0 || taps > 32)
    return DAMC_ERR_ARG;
  if ((om == O_PHASE) != (zdim == 4) || (om == O_DENSE && zdim != 1)) return DAMC_ERR_ARG;
  // the 4 x 4 conv walk (GemmArgs::kwalk): O_DENSE, 16 taps of whole 32-channel slices, the default / F32A tiles only
  if (a.kwalk && (om != O_DENSE || taps != 16 || a.kw != 4 || a.Cg % 32 != 0 || (DAMC_X3_VARIANT & ~0x105) != 0))
    return DAMC_ERR_ARG;
  if (((uintptr_t)a.A3 | (uintptr_t)a.A | (uintptr_t)a.B3 | (uintptr_t)a.C | (uintptr_t)a.C3 | (uintptr_t)a.mask) % 16 !=
      0)
    return DAMC_ERR_ARG;
  if (!a.C && !a.C3) return DAMC_ERR_ARG;
  if (epi == EPI_MASK && !a.mask && !a.mask_sgn) return DAMC_ERR_ARG;
  if (a.mask_sgn && a.mask_act != DAMC_ACT_LRELU) return DAMC_ERR_ARG;
  // octet epilogue: 8 consecutive channels per thread, 16-B aligned rows and bias
  if (a.N % 8 != 0 || a.ldc % 8 != 0 || (a.bias && ((uintptr_t)a.bias % 16 != 0 || a.bias_mod % 8 != 0)))
    return DAMC_ERR_UNSUPPORTED;
  if ((double)a.N * a.K * 6 >= 2147483647.0) return DAMC_ERR_UNSUPPORTED;
  const long hwq = (long)a.Hq * a.Wq;
  if (a.M % hwq != 0) return DAMC_ERR_ARG;
  const long img = (long)a.Hin * a.Win * a.Cg;  // elements per gathered image
  const long nimg = a.M / hwq;
  static const long lim = [] {
    const char* e = getenv("DAMC_KM_CHUNK_BYTES");
    const long v = e ? atol(e) : 0;
    return (v > 0 && v < 2147483647L) ? v : 2147483647L;
  }();
  const long per = (lim / 6 - 1) / img;
  if (per < 1) return DAMC_ERR_UNSUPPORTED;
  const long cimg = (om == O_PHASE) ? (long)a.Hout * a.Wout * a.ldc : hwq * a.ldc;
  if (a.ksplit_deferred) *a.ksplit_deferred = 0;
  for (long b0 = 0; b0 < nimg; b0 += per) {
    const long nb = std::min(per, nimg - b0);
    GemmArgs c = a;
    if (nimg > per) c.ksplit_deferred = nullptr;  // one launch's slabs only
    static const int regions = [] {
      const char* e = getenv("DAMC_CLOCK_REGIONS");
      return e ? std::max(1, atoi(e)) : 1;
    }();
    if (g_clk && (om == O_PHASE || regions > 1)) {
      const int per_region = g_clk_n / regions;
      c.clk = g_clk + 4L * per_region * (g_clk_launch++ % regions);
      c.clk_n = per_region;
    }
    if (a.A3) c.A3 = a.A3 + b0 * img * 3;
    if (a.a_f32) c.A = a.A + b0 * img;
    if (a.in_part) c.in_part = a.in_part + b0 * hwq / (a.in_hw > 0 ? a.in_hw : 1) * (long)a.N * a.in_S * 3;
    if (a.C) c.C = a.C + b0 * cimg;
    if (a.C3) c.C3 = a.C3 + b0 * cimg * 3;
    if (a.sgn) c.sgn = a.sgn + b0 * cimg / 8;
    if (a.mask_sgn) c.mask_sgn = a.mask_sgn + b0 * cimg / 8;
    if (a.mask) c.mask = a.mask + b0 * cimg;
    c.M = (int)(nb * hwq);
    if (a.proj_out) {  // the fused output-layer projection (GemmArgs::proj_out, 128-channel chunks)
      if (om != O_PHASE || epi != EPI_BIAS_ACT || a.N > 256 || a.N % 16 || !a.C || !a.proj_w ||
          (a.proj_np != 32 && a.proj_np != 64) || (a.N > PROJ_CHUNK && a.proj_pstride <= 0))
        return DAMC_ERR_ARG;
      c.proj_out = a.proj_out + b0 * (long)a.Hout * a.Wout * a.proj_np;
      if (c.a_f32) {  // the F32A tile: each 128-channel N tile projects its chunk
        if (a.N > PROJ_CHUNK && a.N % PROJ_CHUNK) return DAMC_ERR_UNSUPPORTED;
        if (const int rc_ = launch_x3_t<EPI_BIAS_ACT, O_PHASE, DAMC_X3_VARIANT | X3_F32A>(c, zdim, s)) return rc_;
      } else {  // the 128 x 256 layout: one N tile holding every channel
        if (const int rc_ = launch_x3_t<EPI_BIAS_ACT, O_PHASE, DAMC_X3_VARIANT | 524288>(c, zdim, s)) return rc_;
      }
      continue;
    }
    // at most 128 rows (the first layer, M = B <= 128): the 128 x 256 block layout, no half-empty 256-row tile
    // (bitwise the default layout: every output takes the same MFMA sequence; 46.6 -> 35.7 us for CIFAR's B = 128
    // first layer, tools/gemm_bench.hip).  DAMC_X3_WIDE=0 (read per call) keeps the default layout
    const char* ew = getenv("DAMC_X3_WIDE");
    // the first layer at per-rank batches: the skinny kernel (bitwise the 128 x 256 layout); DAMC_X3_SKINNY=0 (read
    // per call) keeps the tiled kernel
    const char* esk = getenv("DAMC_X3_SKINNY");
    if (epi == EPI_BIAS_ACT && om == O_DENSE && !c.kwalk && c.M <= x3_skinny_max_rows() && c.K <= c.negk && c.Hin == 1 &&
        c.Win == 1 &&
        c.kw == 1 && c.Cg == c.K && c.A3 && !c.a_f32 && !c.proj_out && !(esk && esk[0] == '0')) {
      // fp32 weights split in registers where the caller passes them (2/3 of the limb bytes; bitwise the same
      // operands); DAMC_X3_SKINNY_F32B=0 (read per call) reads the limbs
      const char* efb = getenv("DAMC_X3_SKINNY_F32B");
      if (c.in_part && c.in_done) *c.in_done = 0;  // no norm statistics from this kernel
      const dim3 gsk((unsigned)((c.N + 63) / 64), (unsigned)((c.M + 15) / 16));
      // 32 columns per wave by default (NTW = 2: CIFAR B=16 step -5 to -17 us, B=32 -4 us against 16 columns, same-box
      // pairs in profiles/r05/skinny_ntw_ab.txt); DAMC_X3_SKINNY_NTW=1 (read per call) keeps 16
      const char* ent = getenv("DAMC_X3_SKINNY_NTW");
      if (!(ent && ent[0] == '1') && c.b32k && (c.K % 32) == 0 && (uintptr_t)c.b32k % 16 == 0 && !(efb && efb[0] == '0'))
        hipLaunchKernelGGL((x3_skinny_kernel<true, 2>), dim3((unsigned)((c.N + 127) / 128), gsk.y), dim3(256), 0, s, c);
      else if (c.b32k && (c.K % 32) == 0 && (uintptr_t)c.b32k % 16 == 0 && !(efb && efb[0] == '0'))
        hipLaunchKernelGGL((x3_skinny_kernel<true, 1>), gsk, dim3(256), 0, s, c);
      else
        hipLaunchKernelGGL((x3_skinny_kernel<false, 1>), gsk, dim3(256), 0, s, c);
      continue;
    }
    const char* ens = getenv("DAMC_X3_NARROW_SPLIT");  // (read per call) 0: the 128 x 256 layout below
    if (epi == EPI_BIAS_ACT && om == O_DENSE && c.M <= 128 && !c.a_f32 && !c.proj_out && c.kslab && !c.kwalk &&
        c.K % c.negk == 0 && c.K / c.negk >= 8 && c.N % 8 == 0 && (long)(c.K / c.negk) * c.M * c.N <= c.kslab_floats &&
        !(ens && ens[0] == '0')) {
      if (c.in_part && c.in_done) *c.in_done = 0;  // no norm statistics from this kernel
      launch_x3_narrow_split<EPI_BIAS_ACT>(c, s);
      continue;
    }
    if (epi == EPI_BIAS_ACT && om == O_DENSE && c.M <= 128 && !c.a_f32) {
      if (!(ew && ew[0] == '0')) {
        if (const int rc_ = launch_x3_t<EPI_BIAS_ACT, O_DENSE, DAMC_X3_VARIANT | 524288>(c, zdim, s)) return rc_;
        continue;
      }
    }
    if (ew && ew[0] == '2' && !c.a_f32) {  // A/B only: every limb GEMM on the 128 x 256 layout (bitwise the default)
      if (epi == EPI_BIAS_ACT && om == O_PHASE) {
        if (const int rc_ = launch_x3_t<EPI_BIAS_ACT, O_PHASE, DAMC_X3_VARIANT | 524288>(c, zdim, s)) return rc_;
        continue;
      }
      if (epi == EPI_MASK && om == O_DENSE) {
        if (const int rc_ = launch_x3_t<EPI_MASK, O_DENSE, DAMC_X3_VARIANT | 524288>(c, zdim, s)) return rc_;
        continue;
      }
    }
#define DAMC_X3(E_, O_)                                                      \
  if (epi == E_ && om == O_) {                                               \
    const int rc_ = c.a_f32 ? launch_x3_t<E_, O_, DAMC_X3_VARIANT | X3_F32A>(c, zdim, s) \
                            : launch_x3_t<E_, O_>(c, zdim, s);               \
    if (rc_) return rc_;                                                     \
    continue;                                                                \
  }
    DAMC_X3(EPI_BIAS_ACT, O_PHASE)
    DAMC_X3(EPI_MASK, O_DENSE)
    DAMC_X3(EPI_BIAS_ACT, O_DENSE)
    DAMC_X3(EPI_STORE, O_DENSE)
#undef DAMC_X3
    return DAMC_ERR_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

// O_WGRAD: A3 [Cg][K] and B3 [wg_phases][N][K] pixel-major x3 operands, C = fp32 slabs
// [wg_phases * slices][M][ldc] (EPI_STORE); slice length k_per_z (a multiple of 32)
int launch_wgrad_x3(const GemmArgs& a, int slices, const char* prof_name, double flops, hipStream_t s) {
  if (!a.A3 || !a.B3 || !a.C || a.C3 || a.sgn || a.M <= 0 || a.N <= 0 || a.K <= 0 || slices < 1) return DAMC_ERR_ARG;
  if (a.wg_phases != 1 && a.wg_phases != 4) return DAMC_ERR_ARG;
  if (a.wg_bp <= 0 || a.wg_bp % X3_BK != 0 || a.K % a.wg_bp != 0 || a.K / a.wg_bp != a.Hin * a.Win)
    return DAMC_ERR_ARG;
  if (a.k_per_z <= 0 || a.k_per_z % X3_BK != 0 || (long)a.k_per_z * slices < a.K) return DAMC_ERR_ARG;
  if (a.kw < 1 || a.kw > 2 || a.M != a.kw * a.kw * a.Cg || (a.wg_phases == 1 && a.kw != 1)) return DAMC_ERR_ARG;
  if (a.N % 8 != 0 || a.ldc % 8 != 0 || a.ldc < a.N || a.c_zstride < (long)a.M * a.ldc) return DAMC_ERR_ARG;
  if (((uintptr_t)a.A3 | (uintptr_t)a.B3 | (uintptr_t)a.C) % 16 != 0) return DAMC_ERR_ARG;
  if ((double)a.Cg * a.K * 6 >= 2147483647.0 || (double)a.N * a.K * 6 >= 2147483647.0) return DAMC_ERR_UNSUPPORTED;
  constexpr int BM = (DAMC_X3_VARIANT & 524288) ? 128 : X3_BM, BN = (DAMC_X3_VARIANT & 524288) ? 256 : X3_BN;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  ProfScope ps(prof_name, flops, s);
  hipLaunchKernelGGL((gemm_x3_kernel<EPI_STORE, O_WGRAD>), dim3(ntm * ntn, 1, a.wg_phases * slices), dim3(512), 0, s,
                     a);
  return (int)hipGetLastError();
}

#ifndef DAMC_GEMM_SCHED
#define DAMC_GEMM_SCHED 0  // hipcc's own placement measured best (profiles/r01/gemm_bench.txt)
#endif
template <int AM, int EPI, int OM, bool BV, int BK, int OCC, int MT, int SCHED = DAMC_GEMM_SCHED>
static void launch_t(const GemmArgs& a, int zdim, hipStream_t s) {
  const int bm = 64 * MT;
  const int ntm = (a.M + bm - 1) / bm, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn, 1, zdim);
  hipLaunchKernelGGL((gemm_f32_kernel<AM, EPI, OM, BV, BK, OCC, MT, SCHED>), grid, dim3(256), 0, s, a);
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

int launch_gemm_group(const GemmArgs* a, int n, Epi epi, const char* prof_name, double flops, hipStream_t s) {
  if (n < 1 || n > GEMM_GROUP_MAX) return DAMC_ERR_ARG;
  if (epi != EPI_GATE && epi != EPI_STORE) return DAMC_ERR_UNSUPPORTED;
  GemmGroup g;
  const int bm = 64 * DAMC_GEMM_MT;
  int tot = 0;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& x = a[i];
    if (x.M <= 0 || x.N <= 0 || x.K <= 0 || x.A3 || x.b_kmajor || x.k_per_z < x.K) return DAMC_ERR_ARG;
    // the dense vector path only: float4 rows of A and B
    if (x.lda % 4 || x.K % 4 || x.ldb % 4 || x.N % 4 || ((uintptr_t)x.A | (uintptr_t)x.B) % 16) return DAMC_ERR_UNSUPPORTED;
    if ((double)x.M * x.lda >= 2147483647.0 || (double)x.K * x.ldb >= 2147483647.0) return DAMC_ERR_UNSUPPORTED;
    g.a[i] = x;
    g.start[i] = tot;
    tot += ((x.M + bm - 1) / bm) * ((x.N + BN - 1) / BN);
  }
  for (int i = n; i <= GEMM_GROUP_MAX; ++i) g.start[i] = tot;
  g.n = n;
  ProfScope ps(prof_name, flops, s);
  constexpr int BKc = DAMC_GEMM_BK, OCCc = DAMC_GEMM_OCC, MTc = DAMC_GEMM_MT;
  if (epi == EPI_GATE)
    hipLaunchKernelGGL((gemm_f32_group_kernel<A_DENSE, EPI_GATE, O_DENSE, true, BKc, OCCc, MTc, DAMC_GEMM_SCHED>),
                       dim3(tot), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_f32_group_kernel<A_DENSE, EPI_STORE, O_DENSE, true, BKc, OCCc, MTc, DAMC_GEMM_SCHED>),
                       dim3(tot), dim3(256), 0, s, g);
  return (int)hipGetLastError();
}

int launch_gemm(const GemmArgs& a, AMode am, Epi epi, OMode om, int zdim, const char* prof_name, double flops,
                hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return DAMC_ERR_ARG;
  if (a.A3 || (a.a_f32 && a.B3)) {
    if (am != A_CONV) return DAMC_ERR_ARG;
    ProfScope ps(prof_name, flops, s);
    return launch_gemm_x3(a, epi, om, zdim, s);
  }
  if (a.b_kmajor) {
    if (am != A_CONV) return DAMC_ERR_ARG;
    ProfScope ps(prof_name, flops, s);
    return launch_gemm_km(a, epi, om, zdim, s);
  }
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
  DAMC_G(A_DENSE, EPI_GATE, O_DENSE)
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

void set_fixup_probe(unsigned* buf) { g_fixup_probe = buf; }

void set_clock_probe(unsigned long long* buf, int n) {
  g_clk = (buf && n > 0) ? buf : nullptr;
  g_clk_n = g_clk ? n : 0;
  g_clk_launch = 0;
}

}  // namespace damc

#ifndef DAMC_GEMM_NO_C_API
extern "C" int damc_clock_probe(unsigned long long* buf, int n_slots) {
  damc::set_clock_probe(buf, n_slots);
  return 0;
}

extern "C" int damc_x3_fixup_probe(unsigned* buf) {
  damc::set_fixup_probe(buf);
  return 0;
}

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
