// ebm.hip — latent EBM energy/gradient, the fused Langevin z-update with in-kernel Philox noise,
// and the persistent prior chain (all n steps of sample_langevin_prior_z in one launch).
//
// _netE (workspace/src/diffusion_net.py:207-223): E(z) = w3 . lrelu(W2 lrelu(W1 z + b1) + b2) + b3
//   grad_z E = W1^T [ lrelu'(a1) * W2^T ( lrelu'(a2) * w3 ) ]
// A workgroup owns R chains (rows).  Rows are independent, so the chains never communicate:
// the prior kernel runs every step with z resident in LDS.  At R <= 8 rows per workgroup the
// FC layers are tiny-M GEMMs bound by latency, not FLOPs: each layer splits its K axis over the
// 1024-thread workgroup (float4 weight columns x strided k-groups, all loads of a thread in flight
// at once) and adds the k-group partials in a fixed order in LDS.
#include <cstdlib>

#include "common.h"
#include "gemm.h"

namespace {

constexpr int EBM_THREADS = 1024;  // 16 waves: the K axis of every layer is split over the workgroup

struct EbmSmem {
  float* zs;   // [R][nz]
  float* h1;   // [R][nh]  lrelu(a1)
  float* h2;   // [R][nh]  lrelu(a2)
  float* g2;   // [R][nh]
  float* g1;   // [R][nh]
  float* gz;   // [R][nz]
  float* red;  // [32]
  float* part; // [G][R][N] k-group partial sums, G*N <= 4*EBM_THREADS (+ scalar-path slack)
};

__host__ __device__ inline size_t ebm_part_floats(int R) { return (size_t)R * (4 * EBM_THREADS + 4 * 256); }

__host__ __device__ inline size_t ebm_smem_floats(int R, int nz, int nh) {
  return (size_t)R * nz * 2 + (size_t)R * nh * 4 + 32 + ebm_part_floats(R);
}

__device__ inline EbmSmem ebm_carve(float* base, int R, int nz, int nh) {
  EbmSmem s;
  s.zs = base;
  s.h1 = s.zs + R * nz;
  s.h2 = s.h1 + R * nh;
  s.g2 = s.h2 + R * nh;
  s.g1 = s.g2 + R * nh;
  s.gz = s.g1 + R * nh;
  s.red = s.gz + R * nz;
  s.part = s.red + 32;
  return s;
}

// One fully connected layer for R rows: y[r][n] = sum_k W[k*N + n] x[r][k]  (W k-major, n contiguous).
// Thread t owns the float4 column group nq = t % NQ and the k-group kg = t / NQ (k = kg, kg+G, ...), so
// each thread's ~K/G weight loads are independent and all in flight at once; the G partial sums are
// then added in k-group order by fin(r, n, sum) (a fixed order: deterministic, batch-independent).
// Ends with a barrier.
template <int R, typename Fin>
__device__ __forceinline__ void fc_rows(const float* __restrict__ W, int K, int N, const float* x, float* part,
                                        Fin fin) {
  const int tid = threadIdx.x;
  const bool v4 = (N & 3) == 0;
  const int NQ = v4 ? (N >> 2) : N;  // column groups (float4, or scalar when N % 4 != 0)
  const int G = EBM_THREADS / NQ;
  const int nq = tid % NQ, kg = tid / NQ;
  if (kg < G) {
    if (v4) {
      f32x4 acc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int k = kg; k < K; k += G) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(W + (long)k * N + 4 * nq);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float xv = x[r * K + k];
          acc[r].x = fmaf(w.x, xv, acc[r].x);
          acc[r].y = fmaf(w.y, xv, acc[r].y);
          acc[r].z = fmaf(w.z, xv, acc[r].z);
          acc[r].w = fmaf(w.w, xv, acc[r].w);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) *reinterpret_cast<f32x4*>(part + ((long)kg * R + r) * N + 4 * nq) = acc[r];
    } else {
      float acc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.f;
      for (int k = kg; k < K; k += G) {
        const float w = W[(long)k * N + nq];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fmaf(w, x[r * K + k], acc[r]);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) part[((long)kg * R + r) * N + nq] = acc[r];
    }
  }
  __syncthreads();
  for (int i = tid; i < R * N; i += EBM_THREADS) {
    float sum = part[i];
    for (int g = 1; g < G; ++g) sum += part[(long)g * R * N + i];
    fin(i / N, i - (i / N) * N, sum);
  }
  __syncthreads();
}

// Computes gz = grad_z sum_r E(z_r) for the R rows in s.zs; if energy != nullptr also writes
// per-row energies (valid rows only).  All EBM_THREADS threads participate; ends with a barrier.
template <int R>
__device__ void ebm_rows(const damc_ebm_t& e, EbmSmem& s, int nvalid, float* energy_rows) {
  const int nz = e.nz, nh = e.nh;
  const float sl = e.slope;
  const float* b1 = e.b1;
  const float* b2 = e.b2;
  const float* w3 = e.w3;
  float* h1 = s.h1;
  float* h2 = s.h2;
  float* g2 = s.g2;
  float* g1 = s.g1;
  float* gz = s.gz;
  // layer 1: a1 = W1 z + b1 ; h1 = lrelu(a1)      (w1t is (nz, nh))
  fc_rows<R>(e.w1t, nz, nh, s.zs, s.part, [&](int r, int j, float v) {
    v += b1[j];
    h1[r * nh + j] = v > 0.f ? v : v * sl;
  });
  // layer 2: a2 = W2 h1 + b2 ; h2 = lrelu(a2) ; g2 = w3 * lrelu'(a2)     (w2t is (nh, nh))
  fc_rows<R>(e.w2t, nh, nh, h1, s.part, [&](int r, int j, float v) {
    v += b2[j];
    const bool pos = v > 0.f;
    h2[r * nh + j] = pos ? v : v * sl;
    g2[r * nh + j] = pos ? w3[j] : w3[j] * sl;
  });
  // energies (optional): e_r = w3 . h2_r + b3, one wave per row
  if (energy_rows) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int r = wave; r < R; r += EBM_THREADS / 64) {
      float v = 0.f;
      for (int j = lane; j < nh; j += 64) v = fmaf(w3[j], h2[r * nh + j], v);
      v = wave_sum(v);
      if (lane == 0 && r < nvalid) energy_rows[r] = v + e.b3[0];
    }
  }
  // layer 2 backward: g1 = (W2^T g2) * lrelu'(a1)      (w2 is (nh, nh) = [j][k])
  fc_rows<R>(e.w2, nh, nh, g2, s.part, [&](int r, int k, float v) {
    g1[r * nh + k] = h1[r * nh + k] > 0.f ? v : v * sl;
  });
  // layer 1 backward: gz = W1^T g1                     (w1 is (nh, nz) = [j][c])
  fc_rows<R>(e.w1, nh, nz, g1, s.part, [&](int r, int c, float v) { gz[r * nz + c] = v; });
}

__device__ __forceinline__ float noise_at(const float* noise, long noise_idx, int with_noise, uint64_t seed,
                                          uint64_t chain, uint64_t step, int c, uint32_t stream_id) {
  if (!with_noise) return 0.f;
  if (noise) return noise[noise_idx];
  float n4[4];
  philox_normal4(seed, chain, step, (uint32_t)(c >> 2), stream_id, n4);
  return pick4(n4, c);
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  __syncthreads();
  return t;  // valid in thread 0
}

// ---- posterior update: g = sum_s lik_slab[s] + grad E + z ; z <- (z - c1 g) + step xi
template <int R>
__global__ __launch_bounds__(EBM_THREADS) void posterior_update_kernel(damc_ebm_t e, int use_ebm, float* z, const float* slabs,
                                                                int nslab, long slab_stride, int B, int nz, float c1,
                                                                float step, int with_noise, const float* noise,
                                                                uint64_t seed, uint64_t step_idx, uint64_t chain_base,
                                                                float* diag) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nh = use_ebm ? e.nh : 0;
  EbmSmem s = ebm_carve(smem, R, nz, nh);
  const int row0 = blockIdx.x * R;
  const int nvalid = min(R, B - row0);
  for (int i = threadIdx.x; i < R * nz; i += blockDim.x) {
    const int r = i / nz;
    s.zs[i] = r < nvalid ? z[(long)(row0 + r) * nz + (i - r * nz)] : 0.f;
  }
  __syncthreads();
  float erow[R];
  float* eptr = nullptr;
  __shared__ float en_rows[R];
  if (use_ebm) {
    eptr = diag ? en_rows : nullptr;
    ebm_rows<R>(e, s, nvalid, eptr);
  }
  (void)erow;
  float zsq = 0.f, gsum = 0.f;
  for (int i = threadIdx.x; i < nvalid * nz; i += blockDim.x) {
    const int r = i / nz, c = i - r * nz;
    const long gi = (long)(row0 + r) * nz + c;
    float g = 0.f;
    for (int k = 0; k < nslab; ++k) g += slabs[(long)k * slab_stride + gi];
    if (use_ebm) g += s.gz[i];
    const float zv = s.zs[i];
    g += zv;
    zsq += zv * zv;
    gsum += g;
    float zn = sub_rn(zv, mul_rn(c1, g));
    if (with_noise) {
      const float xi = noise_at(noise, gi, 1, seed, chain_base + row0 + r, step_idx, c, DAMC_STREAM_POSTERIOR);
      zn = add_rn(zn, mul_rn(step, xi));
    }
    z[gi] = zn;
  }
  if (diag) {
    float et = 0.f;
    if (use_ebm && threadIdx.x == 0)
      for (int r = 0; r < nvalid; ++r) et += en_rows[r];
    const float zs_t = block_sum(zsq, s.red);
    const float gs_t = block_sum(gsum, s.red);
    if (threadIdx.x == 0) {
      atomicAdd(&diag[0], et);
      atomicAdd(&diag[2], 0.5f * zs_t);
      atomicAdd(&diag[3], gs_t / (float)((long)B * nz));
    }
  }
}

// ---- prior chain: every step in one launch, z resident in LDS
template <int R>
__global__ __launch_bounds__(EBM_THREADS) void prior_chain_kernel(damc_ebm_t e, float* z, int B, int n_steps, float c1, float step,
                                                           int with_noise, const float* noise, uint64_t seed,
                                                           uint64_t step_offset, uint64_t chain_base, float* diag) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nz = e.nz;
  EbmSmem s = ebm_carve(smem, R, nz, e.nh);
  __shared__ float en_rows[R];
  const int row0 = blockIdx.x * R;
  const int nvalid = min(R, B - row0);
  for (int i = threadIdx.x; i < R * nz; i += blockDim.x) {
    const int r = i / nz;
    s.zs[i] = r < nvalid ? z[(long)(row0 + r) * nz + (i - r * nz)] : 0.f;
  }
  __syncthreads();
  for (int it = 0; it < n_steps; ++it) {
    ebm_rows<R>(e, s, nvalid, diag ? en_rows : nullptr);
    float zsq = 0.f;
    for (int i = threadIdx.x; i < nvalid * nz; i += blockDim.x) {
      const int r = i / nz, c = i - r * nz;
      const float zv = s.zs[i];
      zsq += zv * zv;
      const float g = s.gz[i] + zv;
      float zn = sub_rn(zv, mul_rn(c1, g));
      if (with_noise) {
        const long ni = ((long)it * B + row0 + r) * nz + c;
        const float xi =
            noise_at(noise, ni, 1, seed, chain_base + row0 + r, step_offset + it, c, DAMC_STREAM_PRIOR);
        zn = add_rn(zn, mul_rn(step, xi));
      }
      s.zs[i] = zn;
    }
    if (diag) {
      const float zs_t = block_sum(zsq, s.red);
      if (threadIdx.x == 0) {
        float et = 0.f;
        for (int r = 0; r < nvalid; ++r) et += en_rows[r];
        atomicAdd(&diag[2 * it + 0], et);
        atomicAdd(&diag[2 * it + 1], 0.5f * zs_t);
      }
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < nvalid * nz; i += blockDim.x) {
    const int r = i / nz;
    z[(long)(row0 + r) * nz + (i - r * nz)] = s.zs[i];
  }
}

template <int R>
__global__ __launch_bounds__(EBM_THREADS) void ebm_energy_grad_kernel(damc_ebm_t e, const float* z, int B, float* energy,
                                                               float* grad) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nz = e.nz;
  EbmSmem s = ebm_carve(smem, R, nz, e.nh);
  const int row0 = blockIdx.x * R;
  const int nvalid = min(R, B - row0);
  for (int i = threadIdx.x; i < R * nz; i += blockDim.x) {
    const int r = i / nz;
    s.zs[i] = r < nvalid ? z[(long)(row0 + r) * nz + (i - r * nz)] : 0.f;
  }
  __syncthreads();
  ebm_rows<R>(e, s, nvalid, energy ? energy + row0 : nullptr);
  for (int i = threadIdx.x; i < nvalid * nz; i += blockDim.x) grad[(long)row0 * nz + i] = s.gz[i];
}

__global__ void z_update_kernel(float* z, const float* g, long n, int nz, float c1, float step, int with_noise,
                                const float* noise, uint64_t seed, uint64_t step_idx, uint64_t chain_base) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long r = i / nz;
  const int c = (int)(i - r * nz);
  const float zv = z[i];
  float zn = sub_rn(zv, mul_rn(c1, g[i] + zv));
  if (with_noise) {
    const float xi = noise_at(noise, i, 1, seed, chain_base + r, step_idx, c, DAMC_STREAM_POSTERIOR);
    zn = add_rn(zn, mul_rn(step, xi));
  }
  z[i] = zn;
}

__global__ void philox_normal_kernel(float* out, int n_steps, int B, int nz, uint64_t seed, uint64_t step_offset,
                                     uint64_t chain_base, uint32_t stream_id) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)n_steps * B * nz;
  if (i >= n) return;
  const long st = i / ((long)B * nz);
  const long rem = i - st * B * nz;
  const long r = rem / nz;
  const int c = (int)(rem - r * nz);
  float n4[4];
  philox_normal4(seed, chain_base + r, step_offset + st, (uint32_t)(c >> 2), stream_id, n4);
  out[i] = pick4(n4, c);
}

// ================================================================================================
// Register-resident EBM (the default for nh <= 208, nz <= 128: _netE at every BASELINE config).
//
// The prior chain (and one posterior update) of ONE chain per 1024-thread workgroup, with both weight matrices
// held in VGPRs for the whole launch: W1 (nh x nz) and W2 (nh x nh) are read from HBM/L2 once per launch instead
// of once per step (the streaming version re-read ~0.5 MB per workgroup per step, ~3.5 us at one CU's L2
// bandwidth).  Wave w owns rows j = 13 w + r (r < 13) of both matrices; lane l owns the columns k = l + 64 i:
//   w2[r][i] = W2[13 w + r][l + 64 i] (i < 4),  w1[r][i] = W1[13 w + r][l + 64 i] (i < 2)   -> 78 VGPRs.
// Forward products (W z, W2 h1) are per-lane partial sums over the lane's columns for the wave's 13 rows, summed
// over the 64 lanes by a halving exchange (17 shuffles for 16 rows instead of 13 x 6); the lane ends up holding
// row (lane >> 2) & 15.  Backward products (W2^T g2, W1^T g1) are per-lane partial sums over the wave's rows for
// the lane's columns (the row factors g2 / g1 broadcast by readlane), summed over the 16 waves through LDS.
// At one chain per workgroup the FC layers are matrix-vector products: MFMA would run them at 1/16 of its
// width (16x16x4: 16 columns of which one is live), the same f32 rate as the VALU FMAs used here
// (MI355X_MICROARCH.md: f32 MFMA = the f32 vector rate), so the VALU is the right unit.
constexpr int EB_THREADS = 1024, EB_WAVES = 16, EB_RW = 13, EB_K2 = 4, EB_K1 = 2;
bool ebm_reg_ok(int nz, int nh) { return nz > 0 && nz <= 64 * EB_K1 && nh > 0 && nh <= EB_WAVES * EB_RW; }

// cross-lane moves without the LDS crossbar: DPP within 16-lane rows, v_permlane16/32_swap across them
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_QUAD_XOR1 = 0xB1, DPP_QUAD_XOR2 = 0x4E, DPP_ROW_SHL4 = 0x104, DPP_ROW_SHR4 = 0x114,
              DPP_ROW_ROR8 = 0x128;

// the pair sum across lanes l and l ^ 32 (a in the lower half, b in the upper): one v_permlane32_swap moves the
// upper lanes' a down and the lower lanes' b up, so own + partner is the sum of the two outputs in every lane
__device__ __forceinline__ float pair_sum32(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// the same across l and l ^ 16 (v_permlane16_swap: odd 16-lane rows of the first operand <-> even rows of the
// second)
__device__ __forceinline__ float pair_sum16(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// v[16]: per-lane partial sums of 16 rows -> the sum over the 64 lanes of row (lane >> 2) & 15, in every lane
// (a halving exchange: at each level a lane keeps half of its rows and adds its partner's copy of them; the
// same additions in the same order as with __shfl_xor, without ds_bpermute's LDS round trips)
__device__ __forceinline__ float reduce16_rows(float (&v)[16], int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = pair_sum32(v[i], v[i + 8]);  // lane half 32: rows i (low) / i + 8 (high)
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pair_sum16(v[i], v[i + 4]);
  {
    const bool up = lane & 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float keep = up ? v[i + 2] : v[i], send = up ? v[i] : v[i + 2];
      v[i] = keep + dpp<DPP_ROW_ROR8>(send);  // row_ror:8 = lane ^ 8 within the 16-lane row
    }
  }
  {
    const bool up = lane & 4;
    const float keep = up ? v[1] : v[0], send = up ? v[0] : v[1];
    const float from_hi = dpp<DPP_ROW_SHL4>(send), from_lo = dpp<DPP_ROW_SHR4>(send);
    v[0] = keep + (up ? from_lo : from_hi);
  }
  float t = v[0];
  t += dpp<DPP_QUAD_XOR2>(t);
  t += dpp<DPP_QUAD_XOR1>(t);
  return t;
}

enum { EB_PRIOR = 0, EB_POSTERIOR = 1, EB_GRAD = 2 };

struct EbArgs {
  damc_ebm_t e;
  float* z;            // (B, nz): updated in place (PRIOR, POSTERIOR); read (GRAD)
  const float* glik;   // POSTERIOR: likelihood gradient (B, nz)
  float* energy;       // GRAD: (B) or null
  float* grad;         // GRAD: (B, nz)
  int B, n_steps;
  float c1, step;
  int with_noise;
  const float* noise;  // injected: PRIOR (n_steps, B, nz), POSTERIOR (B, nz)
  uint64_t seed, step_offset, chain_base;
  float* diag;         // PRIOR: (n_steps, 2) {sum E, |z|^2/2};  POSTERIOR: (4) {sum E, -, |z|^2/2, mean grad}
  // POSTERIOR with nslab > 1: glik is the sum of nslab split-K slabs (slab k at slabs + k * slab_stride), added in
  // slab_sum4_kernel's fixed order (16 groups of every 16th slab, then the groups in order), so the fused sum is
  // bitwise the separate kernel's
  const float* slabs;
  int nslab;
  long slab_stride;
  unsigned short* z3;  // POSTERIOR: the new z also as x3 limbs [B][nz/8][3][8] (the limb-engine first layer's A), or null
};

__device__ __forceinline__ float block_sum1024(float v, float* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int w = 0; w < EB_WAVES; ++w) t += red[w];
  return t;  // valid in thread 0
}

template <int MODE>
__global__ __launch_bounds__(EB_THREADS) void ebm_reg_kernel(EbArgs a) {
  const damc_ebm_t& e = a.e;
  const int nz = e.nz, nh = e.nh;
  const float sl = e.slope;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chain = blockIdx.x;
  __shared__ float zs[64 * EB_K1];
  __shared__ float xs[64 * EB_K1];  // this step's noise
  __shared__ float h1s[EB_WAVES * EB_RW];
  __shared__ float part2[EB_WAVES][64 * EB_K2];
  __shared__ float part1[EB_WAVES][64 * EB_K1];
  __shared__ float red[EB_WAVES];
  __shared__ float gpart[16][64 * EB_K1];  // POSTERIOR: the 16 slab-group sums of glik

  // ---- POSTERIOR: the likelihood gradient's split-K slabs, summed as slab_sum4_kernel does (its loads are in flight
  // while the weights load; the barrier below publishes the group sums)
  if (MODE == EB_POSTERIOR && a.nslab > 1) {
    const int c = tid & (64 * EB_K1 - 1), gp = tid / (64 * EB_K1);
#pragma unroll
    for (int h = 0; h < 16 / (EB_THREADS / (64 * EB_K1)); ++h) {
      const int g = gp + (EB_THREADS / (64 * EB_K1)) * h;
      float acc = 0.f;
      if (c < nz) {
        const float* src = a.slabs + (long)chain * nz + c;
#pragma unroll 16
        for (int k = g; k < a.nslab; k += 16) acc += src[(long)k * a.slab_stride];
      }
      gpart[g][c] = acc;
    }
  }

  // ---- weights -> registers (once per launch); column-coalesced rows
  float w2[EB_RW][EB_K2], w1[EB_RW][EB_K1];
#pragma unroll
  for (int r = 0; r < EB_RW; ++r) {
    const int j = EB_RW * wave + r;
#pragma unroll
    for (int i = 0; i < EB_K2; ++i) {
      const int k = lane + 64 * i;
      w2[r][i] = (j < nh && k < nh) ? e.w2[(long)j * nh + k] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < EB_K1; ++i) {
      const int c = lane + 64 * i;
      w1[r][i] = (j < nh && c < nz) ? e.w1[(long)j * nz + c] : 0.f;
    }
  }
  // this lane's reduced row and its per-row constants
  const int rr = (lane >> 2) & 15;
  const int jr = EB_RW * wave + rr;
  const bool rok = rr < EB_RW && jr < nh;
  const float b1r = rok ? e.b1[jr] : 0.f, b2r = rok ? e.b2[jr] : 0.f, w3r = rok ? e.w3[jr] : 0.f;
  // z of this chain -> LDS
  if (tid < 64 * EB_K1) zs[tid] = tid < nz ? a.z[(long)chain * nz + tid] : 0.f;
  __syncthreads();

  const int nsteps = MODE == EB_PRIOR ? a.n_steps : 1;
  for (int it = 0; it < nsteps; ++it) {
    // ---- this step's noise, off the update's critical path: drawn by the last two waves (wave 15 owns 5 live
    // rows of 13 at nh = 200) into LDS before the FC work; the barriers below publish it to the update
    const bool draw = MODE != EB_GRAD && a.with_noise && wave >= EB_WAVES - 2;
    if (draw) {
      const int c = tid - (EB_WAVES - 2) * 64;
      if (c < nz) {
        xs[c] = MODE == EB_PRIOR
                    ? noise_at(a.noise, ((long)it * a.B + chain) * nz + c, 1, a.seed, a.chain_base + chain,
                               a.step_offset + it, c, DAMC_STREAM_PRIOR)
                    : noise_at(a.noise, (long)chain * nz + c, 1, a.seed, a.chain_base + chain, a.step_offset, c,
                               DAMC_STREAM_POSTERIOR);
      }
    }
    // ---- layer 1 forward: a1 = W1 z + b1, h1 = lrelu(a1)
    float zl[EB_K1];
#pragma unroll
    for (int i = 0; i < EB_K1; ++i) zl[i] = zs[lane + 64 * i];
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = 0.f;
      if (r < EB_RW) {
#pragma unroll
        for (int i = 0; i < EB_K1; ++i) p = fmaf(w1[r][i], zl[i], p);
      }
      v[r] = p;
    }
    const float a1 = reduce16_rows(v, lane) + b1r;
    const float m1 = a1 > 0.f ? 1.f : sl;  // lrelu'(a1) of row jr
    if (rok && (lane & 3) == 0) h1s[jr] = a1 > 0.f ? a1 : a1 * sl;
    __syncthreads();
    // ---- layer 2 forward: a2 = W2 h1 + b2; g2 = w3 lrelu'(a2)
    float hl[EB_K2];
#pragma unroll
    for (int i = 0; i < EB_K2; ++i) {
      const int k = lane + 64 * i;
      hl[i] = k < nh ? h1s[k] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = 0.f;
      if (r < EB_RW) {
#pragma unroll
        for (int i = 0; i < EB_K2; ++i) p = fmaf(w2[r][i], hl[i], p);
      }
      v[r] = p;
    }
    const float a2 = reduce16_rows(v, lane) + b2r;
    const float g2 = rok ? (a2 > 0.f ? w3r : w3r * sl) : 0.f;
    const bool want_e = (MODE == EB_PRIOR || MODE == EB_POSTERIOR) ? a.diag != nullptr : a.energy != nullptr;
    float en = 0.f;
    if (want_e && rok && (lane & 3) == 0) en = w3r * (a2 > 0.f ? a2 : a2 * sl);
    // ---- layer 2 backward: partial (W2^T g2)[k] over this wave's rows
    float q2[EB_K2] = {};
#pragma unroll
    for (int r = 0; r < EB_RW; ++r) {
      const float gr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g2), 4 * r));
#pragma unroll
      for (int i = 0; i < EB_K2; ++i) q2[i] = fmaf(w2[r][i], gr, q2[i]);
    }
#pragma unroll
    for (int i = 0; i < EB_K2; ++i) part2[wave][lane + 64 * i] = q2[i];
    __syncthreads();
    // ---- g1 = (W2^T g2) * lrelu'(a1) for this wave's rows: lane (row l >> 2, quarter l & 3) sums 4 waves
    float g1 = 0.f;
    if (lane < 4 * EB_RW) {
      const int j = EB_RW * wave + (lane >> 2), w0 = 4 * (lane & 3);
      if (j < nh) g1 = part2[w0][j] + part2[w0 + 1][j] + part2[w0 + 2][j] + part2[w0 + 3][j];
    }
    g1 += dpp<DPP_QUAD_XOR1>(g1);
    g1 += dpp<DPP_QUAD_XOR2>(g1);
    g1 *= m1;  // lane l < 52 holds row l >> 2 = rr: its own a1
    // ---- layer 1 backward: partial (W1^T g1)[c] over this wave's rows
    float q1[EB_K1] = {};
#pragma unroll
    for (int r = 0; r < EB_RW; ++r) {
      const float gr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g1), 4 * r));
#pragma unroll
      for (int i = 0; i < EB_K1; ++i) q1[i] = fmaf(w1[r][i], gr, q1[i]);
    }
#pragma unroll
    for (int i = 0; i < EB_K1; ++i) part1[wave][lane + 64 * i] = q1[i];
    __syncthreads();
    // ---- gz = sum over waves; the update (fixed summation orders: deterministic, batch-independent)
    float zsq = 0.f, gsum = 0.f;
    if (tid < nz) {
      float gz = 0.f;
#pragma unroll
      for (int w = 0; w < EB_WAVES; ++w) gz += part1[w][tid];
      const long gi = (long)chain * nz + tid;
      const float zv = zs[tid];
      if (MODE == EB_GRAD) {
        a.grad[gi] = gz;
      } else {
        float gl = 0.f;
        if (MODE == EB_POSTERIOR) {
          if (a.nslab > 1) {
            gl = gpart[0][tid];
#pragma unroll
            for (int j = 1; j < 16; ++j) gl += gpart[j][tid];
          } else {
            gl = a.glik[gi];
          }
        }
        float g = (MODE == EB_POSTERIOR) ? gl + gz : gz;
        g += zv;
        zsq = zv * zv;
        gsum = g;
        float zn = sub_rn(zv, mul_rn(a.c1, g));
        if (a.with_noise) zn = add_rn(zn, mul_rn(a.step, xs[tid]));
        zs[tid] = zn;
        if (MODE == EB_POSTERIOR && a.z3) {  // RNE limbs (gemm.hip split3_octet's arithmetic), x3 octet layout
          const __bf16 b0 = (__bf16)zn;
          const float r1 = sub_rn(zn, (float)b0);
          const __bf16 b1 = (__bf16)r1;
          const __bf16 b2 = (__bf16)(sub_rn(r1, (float)b1));
          __bf16* o = reinterpret_cast<__bf16*>(a.z3) + ((long)chain * (nz >> 3) + (tid >> 3)) * 24 + (tid & 7);
          o[0] = b0;
          o[8] = b1;
          o[16] = b2;
        }
      }
    }
    if (want_e) {  // uniform branch
      const float et = block_sum1024(en, red);
      if (MODE == EB_GRAD) {
        if (tid == 0) a.energy[chain] = et + e.b3[0];
      } else {
        const float zt = block_sum1024(zsq, red);
        if (MODE == EB_PRIOR) {
          if (tid == 0) {
            atomicAdd(&a.diag[2 * it + 0], et + e.b3[0]);
            atomicAdd(&a.diag[2 * it + 1], 0.5f * zt);
          }
        } else {
          const float gt = block_sum1024(gsum, red);
          if (tid == 0) {
            atomicAdd(&a.diag[0], et + e.b3[0]);
            atomicAdd(&a.diag[2], 0.5f * zt);
            atomicAdd(&a.diag[3], gt / (float)((long)a.B * nz));
          }
        }
      }
    }
    __syncthreads();
  }
  if (MODE != EB_GRAD && tid < nz) a.z[(long)chain * nz + tid] = zs[tid];
}

// ------------------------------------------------------------------ MFMA prior chain for large batches
// 16 chains per workgroup as one 16-row tile: every FC layer of _netE (and of its backward) is a real GEMM
// [16 x K] . [K x N] on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation).  The activations live in
// LDS; the weights stream from L2 in PyTorch / packed-transpose layouts, each lane reading f32x4 runs through the
// k-permutation of the MFMA steps (step s of k-group g reads k = 16 g + 4 (lane >> 4) + s on both operands).
// Output tiles of 16 columns go round-robin to the 8 waves.  Per step: a1 = z W1^T, a2 = h1 W2^T, g1 = (g2 W2) *
// lrelu'(a1), gz = g1 W1 (2,116 MFMAs per 16 chains at nz = 128, nh = 200).  The fp32 MFMA issues at the fp32 VALU
// rate (MI355X_MICROARCH.md), so this pays only by batching: at B chains it runs ceil(B / 16) workgroups where the
// register-resident VALU kernel runs B (one per CU at a time); damc_prior_langevin takes it from
// DAMC_EBM_MFMA_MIN_B chains up (bench: tools/ebm_profile.py).
constexpr int EM_THREADS = 512, EM_WAVES = 8, EM_ROWS = 16;
constexpr int EM_MAXW = 256;         // nz, nh <= 256
constexpr int EM_LD = EM_MAXW + 4;   // LDS row stride (floats)
bool ebm_mfma_ok(int nz, int nh) { return nz > 0 && nh > 0 && nz <= EM_MAXW && nh <= EM_MAXW && (nz & 15) == 0; }

// acc[r] (row 4 (lane >> 4) + r, column n0 + (lane & 15)) of x[16][K] . W^T, W row n at w + n * ldw (k contiguous,
// rows >= N and k >= K read as zero); x rows in LDS with stride EM_LD, zero-padded to a multiple of 16
__device__ __forceinline__ f32x4 em_tile(const float* xs, const float* __restrict__ w, long ldw, int n0, int N, int K) {
  const int lane = threadIdx.x & 63, m = lane & 15, q = lane >> 4;
  const int n = n0 + m;
  const float* wr = w + (long)n * ldw;
  const int ng = (K + 15) >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int g0 = 0; g0 < ng; g0 += 8) {
    f32x4 wv[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int k = 16 * (g0 + c) + 4 * q;
      wv[c] = (g0 + c < ng && n < N && k < K) ? *reinterpret_cast<const f32x4*>(wr + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (g0 + c < ng) {
        const f32x4 xv = *reinterpret_cast<const f32x4*>(xs + m * EM_LD + 16 * (g0 + c) + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[e], wv[c][e], acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

__global__ __launch_bounds__(EM_THREADS) void prior_chain_mfma_kernel(EbArgs a) {
  const damc_ebm_t& e = a.e;
  const int nz = e.nz, nh = e.nh;
  const float sl = e.slope;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, q = lane >> 4;
  const int r0 = blockIdx.x * EM_ROWS;
  __shared__ __attribute__((aligned(16))) float zs[EM_ROWS * EM_LD];
  __shared__ __attribute__((aligned(16))) float h1[EM_ROWS * EM_LD];  // lrelu(a1), then g1
  __shared__ __attribute__((aligned(16))) float a1s[EM_ROWS * EM_LD];
  __shared__ __attribute__((aligned(16))) float g2[EM_ROWS * EM_LD];
  __shared__ float red[2][EM_WAVES];
  const int kz = (nz + 15) & ~15, kh = (nh + 15) & ~15;
  // z of the 16 chains -> LDS, zero padding of the K tails (never written again)
  for (int i = tid; i < EM_ROWS * EM_LD; i += EM_THREADS) {
    const int r = i / EM_LD, c = i - r * EM_LD;
    zs[i] = (r0 + r < a.B && c < nz) ? a.z[(long)(r0 + r) * nz + c] : 0.f;
    h1[i] = 0.f;
    g2[i] = 0.f;
  }
  __syncthreads();
  const bool want_e = a.diag != nullptr;
  for (int it = 0; it < a.n_steps; ++it) {
    // ---- a1 = z W1^T + b1 -> h1 = lrelu(a1) (and a1 for the backward mask)
    for (int t = wave; 16 * t < kh; t += EM_WAVES) {
      const f32x4 acc = em_tile(zs, e.w1, nz, 16 * t, nh, nz);
      const int n = 16 * t + m;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = n < nh ? acc[r] + e.b1[n] : 0.f;
        a1s[(4 * q + r) * EM_LD + n] = v;
        h1[(4 * q + r) * EM_LD + n] = v > 0.f ? v : v * sl;
      }
    }
    __syncthreads();
    // ---- a2 = h1 W2^T + b2 -> g2 = w3 lrelu'(a2); energy terms w3 lrelu(a2)
    float en = 0.f;
    for (int t = wave; 16 * t < kh; t += EM_WAVES) {
      const f32x4 acc = em_tile(h1, e.w2, nh, 16 * t, nh, nh);
      const int n = 16 * t + m;
      const float w3 = n < nh ? e.w3[n] : 0.f;
      const float b2 = n < nh ? e.b2[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[r] + b2;
        g2[(4 * q + r) * EM_LD + n] = n < nh ? (v > 0.f ? w3 : w3 * sl) : 0.f;
        if (want_e && n < nh && r0 + 4 * q + r < a.B) en += w3 * (v > 0.f ? v : v * sl);
      }
    }
    __syncthreads();
    // ---- g1 = (g2 W2) * lrelu'(a1): reduction over layer-2 rows, B operand w2t[k][n] = W2[n][k]
    for (int t = wave; 16 * t < kh; t += EM_WAVES) {
      const f32x4 acc = em_tile(g2, e.w2t, nh, 16 * t, nh, nh);
      const int k = 16 * t + m;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a1 = a1s[(4 * q + r) * EM_LD + k];
        h1[(4 * q + r) * EM_LD + k] = k < nh ? acc[r] * (a1 > 0.f ? 1.f : sl) : 0.f;
      }
    }
    __syncthreads();
    // ---- gz = g1 W1 (B operand w1t[c][n] = W1[n][c]); g = gz + z; z <- z - c1 g (+ step xi)
    float zsq = 0.f;
    for (int t = wave; 16 * t < kz; t += EM_WAVES) {
      const f32x4 acc = em_tile(h1, e.w1t, nh, 16 * t, nz, nh);
      const int c = 16 * t + m;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 4 * q + r;
        if (row < a.B && c < nz) {
          const float zv = zs[(4 * q + r) * EM_LD + c];
          const float g = acc[r] + zv;
          zsq += zv * zv;
          float zn = sub_rn(zv, mul_rn(a.c1, g));
          if (a.with_noise) {
            const float xi = noise_at(a.noise, ((long)it * a.B + row) * nz + c, 1, a.seed, a.chain_base + row,
                                      a.step_offset + it, c, DAMC_STREAM_PRIOR);
            zn = add_rn(zn, mul_rn(a.step, xi));
          }
          zs[(4 * q + r) * EM_LD + c] = zn;
        }
      }
    }
    if (want_e) {  // uniform branch: per-workgroup sums of E and |z|^2 / 2, added to the step's diagnostics
      en = wave_sum(en);
      zsq = wave_sum(zsq);
      if (lane == 0) {
        red[0][wave] = en;
        red[1][wave] = zsq;
      }
    }
    __syncthreads();
    if (want_e && tid == 0) {
      float et = 0.f, zt = 0.f;
      for (int w = 0; w < EM_WAVES; ++w) {
        et += red[0][w];
        zt += red[1][w];
      }
      const int rows = min(EM_ROWS, a.B - r0);
      atomicAdd(&a.diag[2 * it + 0], et + rows * e.b3[0]);
      atomicAdd(&a.diag[2 * it + 1], 0.5f * zt);
    }
  }
  for (int i = tid; i < EM_ROWS * nz; i += EM_THREADS) {
    const int r = i / nz, c = i - r * nz;
    if (r0 + r < a.B) a.z[(long)(r0 + r) * nz + c] = zs[r * EM_LD + c];
  }
}

// rows per workgroup: per step a workgroup streams all four weight panels (~0.5 MB, L2-resident) once,
// so few rows per workgroup = more workgroups in flight = lower latency for these tiny batches
constexpr int RP = 2;  // prior chain
constexpr int RU = 2;  // posterior update

// fc_rows needs every layer width <= EBM_THREADS (one column group per thread at least) and the
// carved LDS within the default 64 KB dynamic allocation
bool ebm_shape_ok(int R, int nz, int nh) {
  return nz > 0 && nz <= EBM_THREADS && nh >= 0 && nh <= EBM_THREADS &&
         ebm_smem_floats(R, nz, nh) * sizeof(float) <= 65536;
}

}  // namespace

// host helpers used by generator.hip
// the register-resident update kernel runs (and can sum split-K slabs and write z's limbs itself) for this EBM
bool damc_posterior_update_fusable(const damc_ebm_t* e, int nz) { return e && e->nz == nz && ebm_reg_ok(nz, e->nh); }

int damc_launch_posterior_update(const damc_ebm_t* e, float* z, const float* slabs, int nslab, long slab_stride, int B,
                                 int nz, double step, int with_noise, const float* noise, uint64_t seed,
                                 uint64_t step_idx, uint64_t chain_base, float* diag, hipStream_t s,
                                 unsigned short* z3, bool* wrote_z3) {
  if (wrote_z3) *wrote_z3 = false;
  damc_ebm_t ev{};
  int use_ebm = 0;
  if (e) {
    ev = *e;
    use_ebm = 1;
    if (ev.nz != nz) return DAMC_ERR_ARG;
  }
  const float c1 = (float)(0.5 * step * step);  // float32(0.5 * s * s), the reference's scalar
  if (use_ebm && ebm_reg_ok(nz, ev.nh)) {
    EbArgs a{};
    a.e = ev;
    a.z = z;
    a.glik = slabs;
    a.slabs = slabs;
    a.nslab = nslab;
    a.slab_stride = slab_stride;
    a.z3 = (z3 && nz % 8 == 0) ? z3 : nullptr;
    if (wrote_z3) *wrote_z3 = a.z3 != nullptr;
    a.B = B;
    a.c1 = c1;
    a.step = (float)step;
    a.with_noise = with_noise;
    a.noise = noise;
    a.seed = seed;
    a.step_offset = step_idx;
    a.chain_base = chain_base;
    a.diag = diag;
    ProfScope ps("posterior_update", 4.0 * B * ((double)nz * ev.nh + (double)ev.nh * ev.nh), s);
    hipLaunchKernelGGL(ebm_reg_kernel<EB_POSTERIOR>, dim3(B), dim3(EB_THREADS), 0, s, a);
    return (int)hipGetLastError();
  }
  if (!ebm_shape_ok(RU, nz, use_ebm ? ev.nh : 0)) return DAMC_ERR_UNSUPPORTED;
  const size_t sm = ebm_smem_floats(RU, nz, use_ebm ? ev.nh : 0) * sizeof(float);
  ProfScope ps("posterior_update", 0.0, s);
  hipLaunchKernelGGL((posterior_update_kernel<RU>), dim3((B + RU - 1) / RU), dim3(EBM_THREADS), sm, s, ev, use_ebm, z, slabs,
                     nslab, slab_stride, B, nz, c1, (float)step, with_noise, noise, seed, step_idx, chain_base, diag);
  return (int)hipGetLastError();
}

extern "C" int damc_pack_ebm(const damc_ebm_t* e, float* w1t, float* w2t, void* stream);

// the chain count from which engine 0 picks the MFMA engine: DAMC_EBM_MFMA_MIN_B read once per process (default
// 2048); damc.langevin reads it through this entry point, so Python and the library never disagree
extern "C" int damc_ebm_mfma_min_chains(void) {
  static const int v = [] {
    const char* e = getenv("DAMC_EBM_MFMA_MIN_B");
    return e ? atoi(e) : 2048;
  }();
  return v;
}

// engine: 0 = by batch size (MFMA from DAMC_EBM_MFMA_MIN_B chains up), 1 = register-resident VALU, 2 = MFMA
static int prior_langevin_impl(const damc_ebm_t* e, float* z, int B, int n_steps, double step, int with_noise,
                               const float* noise, uint64_t seed, uint64_t step_offset, uint64_t chain_base,
                               float* diag, void* stream, int engine) {
  if (!e || !z || B <= 0 || n_steps < 0) return DAMC_ERR_ARG;
  if (!e->w1t || !e->w2t) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  if (diag) DAMC_CHECK(hipMemsetAsync(diag, 0, sizeof(float) * 2 * (size_t)n_steps, s));
  if (n_steps == 0) return 0;
  const float c1 = (float)(0.5 * step * step);  // float32(0.5 * s * s), the reference's scalar
  const int mfma_min_b = damc_ebm_mfma_min_chains();
  if (engine == 2 && !ebm_mfma_ok(e->nz, e->nh)) return DAMC_ERR_UNSUPPORTED;
  if (ebm_mfma_ok(e->nz, e->nh) && (engine == 2 || (engine == 0 && B >= mfma_min_b))) {
    EbArgs a{};
    a.e = *e;
    a.z = z;
    a.B = B;
    a.n_steps = n_steps;
    a.c1 = c1;
    a.step = (float)step;
    a.with_noise = with_noise;
    a.noise = noise;
    a.seed = seed;
    a.step_offset = step_offset;
    a.chain_base = chain_base;
    a.diag = diag;
    ProfScope ps("prior_chain_mfma", 4.0 * (double)B * n_steps * ((double)e->nz * e->nh + (double)e->nh * e->nh), s);
    hipLaunchKernelGGL(prior_chain_mfma_kernel, dim3((B + EM_ROWS - 1) / EM_ROWS), dim3(EM_THREADS), 0, s, a);
    return (int)hipGetLastError();
  }
  if (ebm_reg_ok(e->nz, e->nh)) {
    EbArgs a{};
    a.e = *e;
    a.z = z;
    a.B = B;
    a.n_steps = n_steps;
    a.c1 = c1;
    a.step = (float)step;
    a.with_noise = with_noise;
    a.noise = noise;
    a.seed = seed;
    a.step_offset = step_offset;
    a.chain_base = chain_base;
    a.diag = diag;
    ProfScope ps("prior_chain", 4.0 * (double)B * n_steps * ((double)e->nz * e->nh + (double)e->nh * e->nh), s);
    hipLaunchKernelGGL(ebm_reg_kernel<EB_PRIOR>, dim3(B), dim3(EB_THREADS), 0, s, a);
    return (int)hipGetLastError();
  }
  if (!ebm_shape_ok(RP, e->nz, e->nh)) return DAMC_ERR_UNSUPPORTED;
  const size_t sm = ebm_smem_floats(RP, e->nz, e->nh) * sizeof(float);
  ProfScope ps("prior_chain", 4.0 * (double)B * n_steps * ((double)e->nz * e->nh + (double)e->nh * e->nh), s);
  hipLaunchKernelGGL((prior_chain_kernel<RP>), dim3((B + RP - 1) / RP), dim3(EBM_THREADS), sm, s, *e, z, B, n_steps, c1, (float)step,
                     with_noise, noise, seed, step_offset, chain_base, diag);
  return (int)hipGetLastError();
}

extern "C" int damc_prior_langevin(const damc_ebm_t* e, float* z, int B, int n_steps, double step, int with_noise,
                                   const float* noise, uint64_t seed, uint64_t step_offset, uint64_t chain_base,
                                   float* diag, void* stream) {
  return prior_langevin_impl(e, z, B, n_steps, step, with_noise, noise, seed, step_offset, chain_base, diag, stream, 0);
}

extern "C" int damc_prior_langevin_engine(const damc_ebm_t* e, float* z, int B, int n_steps, double step,
                                          int with_noise, const float* noise, uint64_t seed, uint64_t step_offset,
                                          uint64_t chain_base, float* diag, int engine, void* stream) {
  if (engine < 0 || engine > 2) return DAMC_ERR_ARG;
  return prior_langevin_impl(e, z, B, n_steps, step, with_noise, noise, seed, step_offset, chain_base, diag, stream,
                             engine);
}

extern "C" int damc_ebm_energy_grad(const damc_ebm_t* e, const float* z, int B, float* energy, float* grad,
                                    void* stream) {
  if (!e || !z || !grad || B <= 0) return DAMC_ERR_ARG;
  if (ebm_reg_ok(e->nz, e->nh)) {
    EbArgs a{};
    a.e = *e;
    a.z = const_cast<float*>(z);
    a.energy = energy;
    a.grad = grad;
    a.B = B;
    hipLaunchKernelGGL(ebm_reg_kernel<EB_GRAD>, dim3(B), dim3(EB_THREADS), 0, as_stream(stream), a);
    return (int)hipGetLastError();
  }
  if (!ebm_shape_ok(RP, e->nz, e->nh)) return DAMC_ERR_UNSUPPORTED;
  const size_t sm = ebm_smem_floats(RP, e->nz, e->nh) * sizeof(float);
  hipLaunchKernelGGL((ebm_energy_grad_kernel<RP>), dim3((B + RP - 1) / RP), dim3(EBM_THREADS), sm, as_stream(stream), *e, z, B,
                     energy, grad);
  return (int)hipGetLastError();
}

extern "C" int damc_z_update(float* z, const float* g, int B, int nz, double step, int with_noise, const float* noise,
                             uint64_t seed, uint64_t step_index, uint64_t chain_base, void* stream) {
  if (!z || !g || B <= 0 || nz <= 0) return DAMC_ERR_ARG;
  const long n = (long)B * nz;
  const float c1 = (float)(0.5 * step * step);  // float32(0.5 * s * s), the reference's scalar
  hipLaunchKernelGGL(z_update_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), z, g, n, nz, c1,
                     (float)step, with_noise, noise, seed, step_index, chain_base);
  return (int)hipGetLastError();
}

extern "C" int damc_philox_normal(float* out, int n_steps, int B, int nz, uint64_t seed, uint64_t step_offset,
                                  uint64_t chain_base, uint32_t stream_id, void* stream) {
  const long n = (long)n_steps * B * nz;
  if (!out || n <= 0) return DAMC_ERR_ARG;
  hipLaunchKernelGGL(philox_normal_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), out,
                     n_steps, B, nz, seed, step_offset, chain_base, stream_id);
  return (int)hipGetLastError();
}

// ---- packing: w1t = w1^T (nz, nh), w2t = w2^T (nh, nh)
__global__ void transpose_kernel(const float* in, int rows, int cols, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)rows * cols) return;
  const long r = i / cols, c = i - r * cols;
  out[c * rows + r] = in[i];
}

extern "C" int damc_pack_ebm(const damc_ebm_t* e, float* w1t, float* w2t, void* stream) {
  if (!e || !w1t || !w2t) return DAMC_ERR_ARG;
  hipStream_t s = as_stream(stream);
  long n1 = (long)e->nh * e->nz, n2 = (long)e->nh * e->nh;
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, s, e->w1, e->nh, e->nz, w1t);
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, s, e->w2, e->nh, e->nh, w2t);
  return (int)hipGetLastError();
}

// SURVEY.md §8b name of the EBM per-op hook
extern "C" int damc_ebm_grad(const damc_ebm_t* e, const float* z, int B, float* energy, float* grad, void* stream) {
  return damc_ebm_energy_grad(e, z, B, energy, grad, stream);
}

// ------------------------------------------------------------------------------------------------ E update
// The E update of a training iteration (round 5; workspace/train_gen_recon.py:233-241: e_pos, e_neg = E(zk_pos),
// E(zk_neg); (e_pos.mean() - e_neg.mean()).backward()) on the grouped small-GEMM kernel (gemm.hip
// small_gemm_group_kernel, exact fp32 products, fp32 sums): the forward keeps the two hidden activations, the backward
// is two elementwise kernels (LReLU' from the activations' signs, which are the pre-activations' signs for a positive
// slope) and two grouped launches holding every weight / bias gradient and the input gradient.
namespace {
struct EtWs {
  float *grow, *dh2, *dh2T, *dh1p, *dh1, *dh1T;
};
size_t et_carve(int nh, int B, char* base, EtWs* w) {
  size_t off = 0;
  auto take = [&](long n) {
    float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((size_t)n * sizeof(float) + 255) / 256 * 256;
    return p;
  };
  EtWs t;
  t.grow = take(B);
  t.dh2 = take((long)B * nh);
  t.dh2T = take((long)B * nh);
  t.dh1p = take((long)B * nh);
  t.dh1 = take((long)B * nh);
  t.dh1T = take((long)B * nh);
  if (w) *w = t;
  return off;
}
bool et_ok(const damc_ebm_t* e, int B) {
  return e && e->nz > 0 && e->nh > 0 && B > 0 && B % 4 == 0 && e->nz % 4 == 0 && e->nh % 4 == 0 && e->w1 && e->b1 &&
         e->w2 && e->b2 && e->w3 && e->b3;
}
// dh2 = (g w3) * lrelu'(h2), its transpose, and g as a contiguous row
__global__ void et_dh2_kernel(const float* __restrict__ g, long gs, const float* __restrict__ w3,
                              const float* __restrict__ h2, int B, int nh, float slope, float* __restrict__ grow,
                              float* __restrict__ dh2, float* __restrict__ dh2T) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * nh) return;
  const int b = (int)(i / nh), j = (int)(i - (long)b * nh);
  const float gb = g[b * gs];
  float v = mul_rn(gb, w3[j]);
  if (!(h2[i] > 0.f)) v = mul_rn(v, slope);
  dh2[i] = v;
  dh2T[(long)j * B + b] = v;
  if (j == 0) grow[b] = gb;
}
__global__ void et_mask_kernel(const float* __restrict__ d, const float* __restrict__ h, int B, int nh, float slope,
                               float* __restrict__ o, float* __restrict__ oT) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * nh) return;
  const int b = (int)(i / nh), j = (int)(i - (long)b * nh);
  const float v = h[i] > 0.f ? d[i] : mul_rn(d[i], slope);
  o[i] = v;
  oT[(long)j * B + b] = v;
}
damc::SmallGemm sg(const float* A, long lda, const float* Bm, long ldb, int bt, const float* bias, float* C, long ldc,
                   int M, int N, int K, int act, float slope) {
  damc::SmallGemm d;
  d.A = A;
  d.lda = lda;
  d.B = Bm;
  d.ldb = ldb;
  d.b_t = bt;
  d.bias = bias;
  d.C = C;
  d.ldc = ldc;
  d.M = M;
  d.N = N;
  d.K = K;
  d.act = act;
  d.slope = slope;
  return d;
}
damc::SmallGemm sg_colsum(const float* X, long R, int N, long ld, float* C) {
  damc::SmallGemm d;
  d.a_ones = 1;
  d.B = X;
  d.ldb = ld;
  d.C = C;
  d.ldc = N;
  d.M = 1;
  d.N = N;
  d.K = (int)R;
  return d;
}
}  // namespace

extern "C" size_t damc_ebm_train_workspace_bytes(const damc_ebm_t* e, int B) {
  if (!et_ok(e, B)) return 0;
  return et_carve(e->nh, B, nullptr, nullptr);
}

extern "C" int damc_ebm_train_forward(const damc_ebm_t* e, const float* z, int B, float* h1, float* h2, float* energy,
                                      void* stream) {
  if (!e || !z || !h1 || !h2 || !energy) return DAMC_ERR_ARG;
  if (!et_ok(e, B)) return DAMC_ERR_UNSUPPORTED;
  hipStream_t s = as_stream(stream);
  const int nz = e->nz, nh = e->nh;
  const damc::SmallGemm l1 = sg(z, nz, e->w1, nz, 1, e->b1, h1, nh, B, nh, nz, DAMC_ACT_LRELU, e->slope);
  const damc::SmallGemm l2 = sg(h1, nh, e->w2, nh, 1, e->b2, h2, nh, B, nh, nh, DAMC_ACT_LRELU, e->slope);
  const damc::SmallGemm l3 = sg(h2, nh, e->w3, nh, 1, e->b3, energy, 1, B, 1, nh, DAMC_ACT_NONE, 0.f);
  int rc = damc::launch_small_gemm_group(&l1, 1, s);
  if (!rc) rc = damc::launch_small_gemm_group(&l2, 1, s);
  if (!rc) rc = damc::launch_small_gemm_group(&l3, 1, s);
  return rc;
}

extern "C" int damc_ebm_train_backward(const damc_ebm_t* e, const float* z, const float* h1, const float* h2,
                                       const float* grad_energy, long grad_stride, int B, const damc_ebm_grads_t* gr,
                                       float* grad_z, void* workspace, size_t workspace_bytes, void* stream) {
  if (!e || !z || !h1 || !h2 || !grad_energy || !gr || grad_stride < 0) return DAMC_ERR_ARG;
  if (!et_ok(e, B)) return DAMC_ERR_UNSUPPORTED;
  const int nz = e->nz, nh = e->nh;
  if (!workspace || workspace_bytes < et_carve(nh, B, nullptr, nullptr)) return DAMC_ERR_WORKSPACE;
  EtWs w;
  et_carve(nh, B, static_cast<char*>(workspace), &w);
  hipStream_t s = as_stream(stream);
  const long n = (long)B * nh;
  hipLaunchKernelGGL(et_dh2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, grad_energy, grad_stride, e->w3,
                     h2, B, nh, e->slope, w.grow, w.dh2, w.dh2T);
  damc::SmallGemm g1[5];
  int k = 0;
  if (gr->w3) g1[k++] = sg(w.grow, B, h2, nh, 0, nullptr, gr->w3, nh, 1, nh, B, DAMC_ACT_NONE, 0.f);
  if (gr->b3) g1[k++] = sg_colsum(w.grow, B, 1, 1, gr->b3);
  if (gr->w2) g1[k++] = sg(w.dh2T, B, h1, nh, 0, nullptr, gr->w2, nh, nh, nh, B, DAMC_ACT_NONE, 0.f);
  if (gr->b2) g1[k++] = sg_colsum(w.dh2, B, nh, nh, gr->b2);
  const bool down = gr->w1 || gr->b1 || grad_z;
  if (down) g1[k++] = sg(w.dh2, nh, e->w2, nh, 0, nullptr, w.dh1p, nh, B, nh, nh, DAMC_ACT_NONE, 0.f);
  int rc = k ? damc::launch_small_gemm_group(g1, k, s) : 0;
  if (rc || !down) return rc ? rc : (int)hipGetLastError();
  hipLaunchKernelGGL(et_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float*)w.dh1p, h1, B, nh,
                     e->slope, w.dh1, w.dh1T);
  damc::SmallGemm g2[3];
  k = 0;
  if (gr->w1) g2[k++] = sg(w.dh1T, B, z, nz, 0, nullptr, gr->w1, nz, nh, nz, B, DAMC_ACT_NONE, 0.f);
  if (gr->b1) g2[k++] = sg_colsum(w.dh1, B, nh, nh, gr->b1);
  if (grad_z) g2[k++] = sg(w.dh1, nh, e->w1, nz, 0, nullptr, grad_z, nz, B, nz, nh, DAMC_ACT_NONE, 0.f);
  return k ? damc::launch_small_gemm_group(g2, k, s) : (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------ Q update: prior embedding
// Q.prior_emb = Linear(nz, nh) -> LeakyReLU(slope) -> Linear(nh, nout) (workspace/src/diffusion_net.py:577-581) as the
// Q update trains it through Q.calculate_loss (diffusion_net.py:624-641: the mask's prior rows, or every row with x
// None) on the grouped small-GEMM kernel, the E update's building blocks (exact fp32 products, fp32 sums): two launches
// forward keeping the hidden activation, backward a transpose, one grouped launch (W2, b2 and the hidden gradient), the
// LReLU' mask and one grouped launch (W1, b1).  The input is a fresh draw: no input gradient.
namespace {
struct PeWs {
  float *gT, *dhp, *dh, *dhT;
};
size_t pe_carve(const damc_prior_emb_t* e, int B, char* base, PeWs* w) {
  size_t off = 0;
  auto take = [&](long n) {
    float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((size_t)n * sizeof(float) + 255) / 256 * 256;
    return p;
  };
  PeWs t;
  t.gT = take((long)B * e->nout);
  t.dhp = take((long)B * e->nh);
  t.dh = take((long)B * e->nh);
  t.dhT = take((long)B * e->nh);
  if (w) *w = t;
  return off;
}
// the backward's LReLU' comes from the post-activation's sign: the pre-activation's only for slope >= 0
bool pe_ok(const damc_prior_emb_t* e, int B) {
  return e && e->nz > 0 && e->nh > 0 && e->nout > 0 && B > 0 && B % 4 == 0 && e->nz % 4 == 0 && e->nh % 4 == 0 &&
         e->nout % 4 == 0 && e->slope >= 0.f && e->w1 && e->b1 && e->w2 && e->b2;
}
}  // namespace

extern "C" size_t damc_prior_emb_train_workspace_bytes(const damc_prior_emb_t* e, int B) {
  if (!pe_ok(e, B)) return 0;
  return pe_carve(e, B, nullptr, nullptr);
}

extern "C" int damc_prior_emb_train_forward(const damc_prior_emb_t* e, const float* noise, int B, float* h, float* out,
                                            void* stream) {
  if (!e || !noise || !h || !out) return DAMC_ERR_ARG;
  if (!pe_ok(e, B)) return DAMC_ERR_UNSUPPORTED;
  hipStream_t s = as_stream(stream);
  const damc::SmallGemm l1 = sg(noise, e->nz, e->w1, e->nz, 1, e->b1, h, e->nh, B, e->nh, e->nz, DAMC_ACT_LRELU, e->slope);
  const damc::SmallGemm l2 = sg(h, e->nh, e->w2, e->nh, 1, e->b2, out, e->nout, B, e->nout, e->nh, DAMC_ACT_NONE, 0.f);
  int rc = damc::launch_small_gemm_group(&l1, 1, s);
  if (!rc) rc = damc::launch_small_gemm_group(&l2, 1, s);
  return rc;
}

extern "C" int damc_prior_emb_train_backward(const damc_prior_emb_t* e, const float* noise, const float* h,
                                             const float* grad_out, int B, const damc_prior_emb_grads_t* gr,
                                             void* workspace, size_t workspace_bytes, void* stream) {
  if (!e || !noise || !h || !grad_out || !gr) return DAMC_ERR_ARG;
  if (!pe_ok(e, B)) return DAMC_ERR_UNSUPPORTED;
  if (!workspace || workspace_bytes < pe_carve(e, B, nullptr, nullptr)) return DAMC_ERR_WORKSPACE;
  PeWs w;
  pe_carve(e, B, static_cast<char*>(workspace), &w);
  hipStream_t s = as_stream(stream);
  const int nz = e->nz, nh = e->nh, no = e->nout;
  const long ng = (long)B * no, nhb = (long)B * nh;
  const bool down = gr->w1 || gr->b1;
  damc::SmallGemm g1[3];
  int k = 0;
  if (gr->w2) {
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((ng + 255) / 256)), dim3(256), 0, s, grad_out, B, no, w.gT);
    g1[k++] = sg(w.gT, B, h, nh, 0, nullptr, gr->w2, nh, no, nh, B, DAMC_ACT_NONE, 0.f);
  }
  if (gr->b2) g1[k++] = sg_colsum(grad_out, B, no, no, gr->b2);
  if (down) g1[k++] = sg(grad_out, no, e->w2, nh, 0, nullptr, w.dhp, nh, B, nh, no, DAMC_ACT_NONE, 0.f);
  int rc = k ? damc::launch_small_gemm_group(g1, k, s) : 0;
  if (rc || !down) return rc ? rc : (int)hipGetLastError();
  hipLaunchKernelGGL(et_mask_kernel, dim3((unsigned)((nhb + 255) / 256)), dim3(256), 0, s, (const float*)w.dhp, h, B, nh,
                     e->slope, w.dh, w.dhT);
  damc::SmallGemm g2[2];
  k = 0;
  if (gr->w1) g2[k++] = sg(w.dhT, B, noise, nz, 0, nullptr, gr->w1, nz, nh, nz, B, DAMC_ACT_NONE, 0.f);
  if (gr->b1) g2[k++] = sg_colsum(w.dh, B, nh, nh, gr->b1);
  return damc::launch_small_gemm_group(g2, k, s);
}
