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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "gemm.h"

namespace {

#ifndef DAMC_CH_WAVES
#define DAMC_CH_WAVES 4
#endif
constexpr int CH_WAVES = DAMC_CH_WAVES;  // waves per chain workgroup, splitting K
constexpr int CH_THREADS = 64 * CH_WAVES;
constexpr int TM = 16;           // rows per workgroup
constexpr int TC = 8;            // output columns per workgroup (x 2 products)
constexpr int KG = 16 * CH_WAVES;  // K padding granule: one 16-deep k-group per wave
#ifndef DAMC_CH_CHUNK
#define DAMC_CH_CHUNK 4  // 8 until round 4: with the sentinel re-read paths the team kernel at 8 ran 3.92 ms per B=128
                         // sweep against 3.49 at 4 (same box, interleaved; profiles/r04/sweep_ab.txt)
#endif
constexpr int CH_CHUNK = DAMC_CH_CHUNK;  // k-groups whose loads a lane keeps in flight at once
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
  uint64_t* trace;  // tools only (DAMC_CHAIN_TRACE): [launch][512][2] 100 MHz stamps {block start, block end}
  int li;           // launch index in the sweep (trace row)
  int dbg;  // timing experiments only (DAMC_CHAIN_DBG, wrong results): 1 no x loads, 2 no weight loads, 4 no MFMA,
            // 8 no epilogue prefetch, 16 no output stores; in0: 32 no sin/cos, 64 no B loads, 128 no zB MFMA
};

__host__ __device__ inline int kpad(int din) { return (din + KG - 1) / KG * KG; }
__host__ __device__ inline int emb_ld(int kp) { return kp + 8; }  // in0 LDS image row stride (floats)

// in0's z B (16 rows x the wave's 16 columns, K = nz <= 128) as two independent MFMA chains over the even and the odd
// k-groups, then their sum: half the dependent-MFMA latency of one chain on the stage's critical path (chain_kernel, the team
// kernel and its rescue all use this function)
__device__ __forceinline__ f32x4 emb_zb(const f32x4 (&zv4)[EMB_G], const f32x4 (&bv)[EMB_G]) {
#ifdef DAMC_EMB_ONE_CHAIN  // A/B only (round 4 sweep attribution): round 2's single chain
  f32x4 a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < EMB_G; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(zv4[g][e], bv[g][e], a1, 0, 0, 0);
  return a1;
#endif
  f32x4 e0 = {0.f, 0.f, 0.f, 0.f}, e1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < EMB_G; g += 2)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      e0 = __builtin_amdgcn_mfma_f32_16x16x4f32(zv4[g][e], bv[g][e], e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f32_16x16x4f32(zv4[g + 1][e], bv[g + 1][e], e1, 0, 0, 0);
    }
  return e0 + e1;
}

// EMB: the in0 block (Fourier embedding, sin / cos with their large-argument path) is its own instantiation, so
// the six other blocks' kernels carry no scratch segment
template <bool EMB>
__global__ __launch_bounds__(CH_THREADS) void chain_kernel(ChainArgs a) {
  __shared__ __attribute__((aligned(16))) float red[CH_WAVES][TM][16];
  extern __shared__ __attribute__((aligned(16))) float embs[];  // in0: [TM][emb_ld(kp)]
  if (a.trace && threadIdx.x == 0) { a.trace[((long)a.li * 512 + blockIdx.x) * 8] = __builtin_amdgcn_s_memrealtime(); a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 2] = __builtin_amdgcn_s_memtime(); }
  if (a.trace && (threadIdx.x == 64 || threadIdx.x == 192)) a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 6 + (threadIdx.x >> 7)] = __builtin_amdgcn_s_memtime();
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
      // every per-call field in one round trip (not three dependent ones)
      const int with_noise = call->with_noise;
      const float* noise = call->noise;
      const uint64_t seed = call->seed, chain_base = call->chain_base, step_offset = call->step_offset;
      if (!a.last && with_noise) {
        if (noise) {
          xi = noise[((long)a.noisy_k * a.B + erow) * a.nz + ecol];
        } else {
          float n4[4];
          philox_normal4(seed, chain_base + erow, step_offset + a.noisy_k, (uint32_t)(ecol >> 2),
                         DAMC_STREAM_SWEEP, n4);
          xi = pick4(n4, ecol);
        }
      }
    }
  }

  // ---- this wave's K range and, for in0, its first weight chunk now: the embedding below is a dependent
  // load -> MFMA -> sin/cos phase, so the weights' memory round trip overlaps it instead of following it
  const int kq = a.kp / CH_WAVES;
  const int ng = kq >> 4;
  const int kbase = wave * kq;
  const float* wrow = a.w + ((long)tn * 16 + m) * a.kp + kbase + 4 * q;
  f32x4 wpre[CH_CHUNK];
  if (EMB) {
#pragma unroll
    for (int c = 0; c < CH_CHUNK; ++c)
      wpre[c] = (c < ng && !(a.dbg & 2)) ? *reinterpret_cast<const f32x4*>(wrow + 16 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
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
    for (int t = wave; t * 16 < half; t += CH_WAVES) {
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
      if (!(a.dbg & 128)) acc = emb_zb(zv4, bv);
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
  const int xrow = r0 + m;
  const bool xok = xrow < a.B;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int g0 = 0; g0 < ng; g0 += CH_CHUNK) {
    f32x4 xa[CH_CHUNK], wb[CH_CHUNK];
#pragma unroll
    for (int c = 0; c < CH_CHUNK; ++c) {
      const int g = g0 + c;
      const int k = kbase + 16 * g + 4 * q;
      f32x4 wv = {0.f, 0.f, 0.f, 0.f}, xv = {0.f, 0.f, 0.f, 0.f};
      if (g < ng) {
        if (EMB && g0 == 0) wv = wpre[c];
        else if (!(a.dbg & 2)) wv = *reinterpret_cast<const f32x4*>(wrow + 16 * g);
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
    if ((a.dbg & 1024) && g0 == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      if (a.trace && tid == 0) a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 3] = __builtin_amdgcn_s_memtime();
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
  if (a.trace && tid == 0) a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 4] = __builtin_amdgcn_s_memtime();

  if (!eok) return;
  float l = 0.f, sk = 0.f;
#pragma unroll
  for (int w = 0; w < CH_WAVES; ++w) {  // fixed order: deterministic
    l += red[w][er][ec];
    sk += red[w][er][8 + ec];
  }
  // ConcatSquashLinearSkipCtx.forward: ret = layer(x) * gate + bias; ret + skip(x)
  const float o = __builtin_fmaf(l + bl, gate, hb) + (sk + bs);  // the fma spelled out: every sweep form rounds alike
  if (!a.final_) {
    if (!(a.dbg & 16)) a.out[(long)erow * a.dout + ecol] = o;
    if (a.trace && tid == 0) { a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 1] = __builtin_amdgcn_s_memrealtime(); a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 5] = __builtin_amdgcn_s_memtime(); }
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
  if (a.trace && tid == 0) { a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 1] = __builtin_amdgcn_s_memrealtime(); a.trace[((long)a.li * 512 + blockIdx.x) * 8 + 5] = __builtin_amdgcn_s_memtime(); }
}

// sc1 (L1-bypassing) accesses of handed-off words (MI355X_MICROARCH.md, inter-workgroup visibility)
__device__ __forceinline__ f32x4 ld_sc1(const __amdgpu_buffer_rsrc_t& r, long byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 16));
}
__device__ __forceinline__ float ld_sc1_f(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a plain store to a global pointer the compiler cannot prove global (read from memory): as a global_store, since
// a FLAT store in flight makes every later vmcnt wait of the wave a full drain (the counter may run out of order)
__device__ __forceinline__ void st_global(float* p, float v) { *(__attribute__((address_space(1))) float*)p = v; }

// ------------------------------------------------------------------------------ team sweep (one launch, default)
// The whole dependent chain of a sweep as ONE launch of P = 8 T workgroups, one per CU, with every chain weight
// resident in LDS for the whole sweep.  Rows never mix, so the chain splits into independent row tiles; workgroup
// b belongs to team b % 8 (the dispatcher deals blocks round-robin over the 8 XCDs, so a team shares one XCD and
// one L2: speed only, never correctness) as slot b / 8, and team x owns row tiles x, x + 8, ...  Block j's
// column tile tn belongs to slot (tn + toff_j) mod T for every step, so its 16 packed weight rows (8 Wl + 8 Ws)
// are copied into that workgroup's LDS once, in MFMA fragment order (one ds_read_b128 per lane and k-group, no
// bank conflicts).  toff_j staggers the blocks' first tiles so the LDS load is even across slots (106.5 KB per
// workgroup at the CIFAR defaults, nf 4).
// Per stage (block j of step k, s = 7 k + j) a workgroup waits until every slot of its team has published stage
// s - 1, reads its row tile's block input, runs 16 x 16 v_mfma_f32_16x16x4_f32 tiles over K split in quarters by
// its 4 waves, and publishes its 16 x 8 outputs.  A block whose input is cat(prev, skip) takes the skip half
// (complete stages earlier) and its MFMAs BEFORE the wait, and only the prev half after it.
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 table): every handed-off value
// is stored sc1 and every storing wave drains vmcnt before the workgroup barrier, then ONE lane stores the
// slot's flag (= stages done) sc1; a consumer's wave 0 polls its team's T flags with sc1 loads, the other waves
// join it at a barrier, and every load of handed-off bytes is an sc1 load.  Outputs and z go to per-step ring
// slots, so no address is ever rewritten within a sweep.  Every wait is bounded: past the budget (or once any
// workgroup has failed) the workgroup records the failure in the error word and leaves, so the grid drains, and
// the copy-out writes NaN into zt.
// waves 0-3 compute (K in quarters), wave 4 polls, wave 5 stores the slot's flag: a poll issued behind the same
// wave's flag store would return only after that store's write-through ack (loads and stores share vmcnt, in order)
constexpr int TS_THREADS = 384;
constexpr int TS_PUB = 320;  // the publishing lane
constexpr int TS_MAXT = 64;     // slots per team (CUs per XCD)
constexpr int TS_TAB_STEPS = 256;  // steps whose schedule rows are kept in LDS

struct TsBlock {
  const float* w;    // packed [ntn][16][kp] (workspace)
  const float* bls;  // [ntn][16]
  int kp, dout, ntn;
  int wa, wb;        // widths of the input halves (in0: wa = din, the embedding; wb = 0: no skip half)
  int kpa, kpb;      // their K paddings (multiples of 64)
  int srcA, srcB;    // producing blocks of the halves (-1: none)
  long ooff;         // output (B, dout) within a step's ring slot, floats
  int ghoff;         // 2 * coloff: gate columns in a gh row
  int toff;          // column tile tn -> slot (tn + toff) % T
};

struct TsArgs {
  TsBlock b[7];
  const float* bmat;  // B^T (nz/2, nz)
  int nz, B, G, n, residual, T;
  const float* gh;    // (n, B, 2S)
  long ldgh;
  float* ring;        // (n, B*S): block outputs of step k at ring + k * ring_step
  long ring_step;
  float* zring;       // (n+1, B, nz): z before step k at zring + k * B * nz
  const float* tab;   // (n, 8): c0..c4, is_last, noisy_k
  const SweepCall* call;
  unsigned* flags;    // [8][TS_MAXT][TS_FS]: stages published by (team, slot)
  int* err;
  int* diag;          // [P][4]: a failed wait's {stage needed, flag of the first late slot, late-slot mask lo, hi}
  int sent;           // 1: sentinel hand-offs (TS_SENT): no drain before the flag, every handed-off load re-read until
                      // it holds no sentinel; 0: the drained-flag protocol (DAMC_SWEEP_SENT=0, read per call)
  long budget;        // wait budget in 100 MHz ticks
  int wlds;           // weight LDS floats per workgroup (host maximum over slots)
  int fast;           // 128 / 100: sweep_fast_kernel<fast, 128> (the shapes compiled in; DAMC_SWEEP_FAST=0: off)
  uint64_t* trace;    // tools only (DAMC_SWEEP_TRACE): [P][7n][4] 100 MHz stamps {wait begin (sent 2: task start),
                      // wait end, reduced, published}
  int dbg;            // timing experiments only (DAMC_SWEEP_DBG, wrong results): 1 no drain before the flag,
                      // 2 no payload loads, 4 no MFMA, 8 no epilogue operand loads, 16 no output stores,
                      // 32 no zB / sin / cos (in0), 64 no z loads (in0); tests: 4096 every workgroup reports a
                      // failed wait at once (exercises the rescue in team_finish_kernel)
};

// number of column tiles of block b that slot t owns, and the first one
__device__ __forceinline__ int ts_tiles(const TsBlock& b, int T, int t, int* tn0) {
  const int f = ((t - b.toff) % T + T) % T;
  *tn0 = f;
  return f < b.ntn ? (b.ntn - f + T - 1) / T : 0;
}

// wave 4 (which issues no other loads, so nothing queues in front of its poll) polls the T flags of the team (one
// 128-B line each: a shared line would serialise the producers' stores and the pollers' loads on one memory
// channel) until all have published `need` stages; every thread returns whether the wait succeeded (a barrier is
// inside).  One poll in flight: three staggered ones measured 4-5 % slower per sweep.
constexpr int TS_FS = 32;  // flag stride, unsigned
__device__ __forceinline__ bool ts_wait(const unsigned* fl, int T, unsigned need, int* err, long budget, int* sflag,
                                        int* diag) {
  if (threadIdx.x >= 256 && threadIdx.x < 320) {
    const int lane = threadIdx.x - 256;
    int ok = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 0;; ++it) {
      const unsigned v =
          lane < T ? __hip_atomic_load(fl + lane * TS_FS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : need;
      if (__all(v >= need)) break;
      __builtin_amdgcn_s_sleep(1);
      if ((it & 63) == 63) {
        const int e = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e || (long)(__builtin_amdgcn_s_memrealtime() - t0) > budget) {
          if (!e && lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // diagnostics: which slots of the team had not published `need` stages when this wait gave up
          const uint64_t late = __ballot(v < need);
          const int first = late ? __builtin_ctzll(late) : 0;
          const unsigned vf = __shfl(v, first);
          if (lane == 0) {
            int* dg = diag + blockIdx.x * 4;
            dg[0] = (int)need;
            dg[1] = e ? -1 : (int)vf;  // -1: gave up because another workgroup had failed
            dg[2] = (int)(unsigned)late;
            dg[3] = (int)(unsigned)(late >> 32);
          }
          ok = 0;
          break;
        }
      }
    }
    if (lane == 0) *sflag = ok;
  }
  __syncthreads();
  return *sflag != 0;
}

// Sentinel hand-offs.  Every ring slot (block outputs and z of every step) is written exactly once per sweep, and
// the setup kernel fills all of them with a NaN bit pattern no arithmetic produces (hardware NaNs are canonical,
// 0x7FC00000) before the launch.  A handed-off 4-B value is then either the sentinel or final (aligned 4-B stores
// do not tear), so the producer publishes its flag right behind its stores without draining them (one memory round
// trip less per stage), and a consumer that has seen the flag re-reads (sc1) any load group that still holds a
// sentinel.  The flag stays the cheap "probably ready" signal; the data itself proves readiness.
// The caller data that enters the ring unchanged is z; the setup kernel stores its NaNs canonical.  The other ring
// values are computed, and a VALU op may carry a (quieted) input NaN's payload through, so a weight or xemb holding
// exactly the TS_SENT pattern could still reach the ring.  Then the consumers' bounded wait expires (20 ms),
// team_finish_kernel recomputes the sweep bitwise and the process stays on the launch chain: slow, never wrong.
constexpr unsigned TS_SENT = 0x7FC0DEADu;
constexpr unsigned TS_OOB = 0xF0000000u;  // a buffer offset past any descriptor of the team kernel: the load reads 0
// a re-read loop gives up past the budget (setting the error word) or once another workgroup has failed
__device__ __forceinline__ bool ts_giveup(uint64_t t0, unsigned it, int* err, long budget) {
  if ((it & 15) != 15) return false;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
  if ((long)(__builtin_amdgcn_s_memrealtime() - t0) > budget) {
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}
__device__ __forceinline__ bool is_sent(float v) { return __builtin_bit_cast(unsigned, v) == TS_SENT; }
template <int N>
__device__ __forceinline__ bool any_sent(const f32x4 (&x)[N]) {
  bool b = false;
#pragma unroll
  for (int c = 0; c < N; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) b = b || is_sent(x[c][e]);
  return b;
}
// wave-uniform: re-issue ts_load<N> until its registers hold no sentinel; past the budget the error word is set
// (the team then drains and team_finish_kernel recomputes the sweep)
// acc += lrelu(x[rows][k0 .. k0 + kps)) . W^T over one input half: wave w takes k in [w kps/4, (w+1) kps/4);
// x rows come from src (width wsrc, zero past it) with sc1 loads, or from the in0 embedding image in LDS
template <bool EMB>
__device__ __forceinline__ void ts_half(f32x4& acc, const float* wl, int kps, const __amdgpu_buffer_rsrc_t& rs,
                                        long soff, int wsrc, int row, bool rok, const float* embs, int ld, int dbg,
                                        int sent = 0, int* err = nullptr, long budget = 0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, q = lane >> 4;
  const int kq = kps >> 2, ng = kq >> 4, kbase = wave * kq;
  const f32x4* wv = reinterpret_cast<const f32x4*>(wl) + (long)wave * ng * 64 + lane;
  for (int g0 = 0; g0 < ng; g0 += CH_CHUNK) {
    f32x4 xa[CH_CHUNK];
    auto load = [&]() {
#pragma unroll
      for (int c = 0; c < CH_CHUNK; ++c) {
        const int k = kbase + 16 * (g0 + c) + 4 * q;
        f32x4 xv = {0.f, 0.f, 0.f, 0.f};
        if (g0 + c < ng) {
          if (EMB) xv = *reinterpret_cast<const f32x4*>(embs + m * ld + k);
          else if (rok && k < wsrc && !(dbg & 2)) xv = ld_sc1(rs, (soff + (long)row * wsrc + k) * 4);
        }
        xa[c] = xv;
      }
    };
    load();
    if (!EMB && sent) {  // sentinel hand-off (see TS_SENT): re-read the chunk until it holds no sentinel
      bool bad = false;
#pragma unroll
      for (int c = 0; c < CH_CHUNK; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) bad = bad || (__builtin_bit_cast(unsigned, xa[c][e]) == 0x7FC0DEADu);
      if (__any(bad)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        unsigned it = 0;
        do {
          __builtin_amdgcn_s_sleep(1);
          if (ts_giveup(t0, ++it, err, budget)) break;
          load();
          bad = false;
#pragma unroll
          for (int c = 0; c < CH_CHUNK; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) bad = bad || (__builtin_bit_cast(unsigned, xa[c][e]) == 0x7FC0DEADu);
        } while (__any(bad));
      }
    }
#pragma unroll
    for (int c = 0; c < CH_CHUNK; ++c) {
      if (g0 + c >= ng) break;
      f32x4 x = xa[c];
      if (!EMB) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = x[e] > 0.f ? x[e] : 0.01f * x[e];
      }
      const f32x4 w = wv[(g0 + c) * 64];
      if (dbg & 4) {
        acc[0] += x[0] * w[0];
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[e], w[e], acc, 0, 0, 0);
    }
  }
}

// the two halves of ts_half for an input half of at most 64 N columns of K: this wave's x loads into registers
// (issued early), then its MFMAs
template <int N>
__device__ __forceinline__ void ts_load(f32x4 (&x)[N], int kps, const __amdgpu_buffer_rsrc_t& rs, long soff, int wsrc,
                                        int row, bool rok) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4;
  const int kq = kps >> 2, ng = kq >> 4, kbase = wave * kq;
  // every lane issues all N loads, out-of-range ones at an offset past the descriptor (they read 0): no branch per load
  // and a fixed count, so the waits for earlier loads count exactly (TS_OOB)
#pragma unroll
  for (int c = 0; c < N; ++c) {
    const int k = kbase + 16 * c + 4 * q;
    x[c] = ld_sc1(rs, (c < ng && rok && k < wsrc) ? (soff + (long)row * wsrc + k) * 4 : (long)TS_OOB);
  }
}
template <int N>
__device__ __forceinline__ void ts_mfma(f32x4& acc, const float* wl, int kps, const f32x4 (&x)[N], int dbg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ng = kps >> 6;
  const f32x4* wv = reinterpret_cast<const f32x4*>(wl) + (long)wave * ng * 64 + lane;
#pragma unroll
  for (int c = 0; c < N; ++c) {
    if (c >= ng) break;
    f32x4 xv = x[c];
#pragma unroll
    for (int e = 0; e < 4; ++e) xv[e] = xv[e] > 0.f ? xv[e] : 0.01f * xv[e];
    const f32x4 w = wv[c * 64];
    if (dbg & 4) {
      acc[0] += xv[0] * w[0];
      continue;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[e], w[e], acc, 0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void ts_ready(f32x4 (&x)[N], int kps, const __amdgpu_buffer_rsrc_t& rs, long soff, int wsrc,
                                         int row, bool rok, int* err, long budget) {
  if (!__any(any_sent(x))) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  unsigned it = 0;
  do {
    __builtin_amdgcn_s_sleep(1);
    if (ts_giveup(t0, ++it, err, budget)) return;
    ts_load<N>(x, kps, rs, soff, wsrc, row, rok);
  } while (__any(any_sent(x)));
}

// NT: threads per workgroup.  The flag protocols (sent 0 / 1) need the poll wave (threads 256..319) and the flag
// lane (TS_PUB): 384.  The data-driven hand-off (sent 2, the default) has neither, so it runs 4 waves, one per SIMD,
// which lifts the register cap from 256 to 512 per lane: at 384 threads the kernel spilled 38 VGPRs to scratch (152 B
// per lane) once the sentinel re-read paths were added, +17 % sweep time (round 4 A/B).
template <int NT>
__global__ __launch_bounds__(NT) void sweep_team_kernel(TsArgs a) {
  __shared__ __attribute__((aligned(16))) float red[4][TM][16];
  __shared__ int sflag;
  __shared__ uint64_t trs[3];                    // tools only: this stage's stamps
  __shared__ float tabs[8 * TS_TAB_STEPS];       // the step table (n <= TS_TAB_STEPS)
  __shared__ int lbase[7];                       // LDS float offset of block j's first owned tile
  __shared__ int tinfo[7][2];                    // block j: {column tiles this slot owns, the first one}
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [wlds weights][TM][emb_ld(kpa0)] in0 image
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, q = lane >> 4;
  const int er = tid >> 3, ec = tid & 7;
  const int T = a.T, team = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nz = a.nz, B = a.B, G = a.G;
  const int sent = NT == 256 ? 2 : a.sent;  // compile-time in the 4-wave (data-driven) instantiation
  if (team >= G || slot >= T) return;  // no row tile for this team (its flags are never waited on)
  if (a.dbg & 4096) {  // tests only: report a failed wait at once
    if (tid == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int nrt = (G - team + 7) / 8;  // row tiles of the team: team + 8 i
  unsigned* const myflag = a.flags + (team * TS_MAXT + slot) * TS_FS;
  const unsigned* const teamflags = a.flags + team * TS_MAXT * TS_FS;
  float* const embs = lds + a.wlds;
  const int ld0 = emb_ld(a.b[0].kpa);

  if (a.n <= TS_TAB_STEPS)
    for (int i = tid; i < 8 * a.n; i += NT) tabs[i] = a.tab[i];
  // ---- the owned weight tiles into LDS, fragment order: (half, wave, k-group, lane) -> f32x4
  if (tid == 0) {
    int off = 0;
    for (int j = 0; j < 7; ++j) {
      int tn0;
      const int c = ts_tiles(a.b[j], T, slot, &tn0);
      lbase[j] = off;
      tinfo[j][0] = c;
      tinfo[j][1] = tn0;
      off += c * 16 * (a.b[j].kpa + a.b[j].kpb);
    }
  }
  __syncthreads();
  for (int j = 0; j < 7; ++j) {
    const TsBlock& b = a.b[j];
    int tn0;
    const int c = ts_tiles(b, T, slot, &tn0);
    for (int i = 0; i < c; ++i) {
      const int tn = tn0 + i * T;
      float* dst = lds + lbase[j] + (long)i * 16 * (b.kpa + b.kpb);
      for (int h = 0; h < 2; ++h) {
        const int kps = h ? b.kpb : b.kpa, wsrc = h ? b.wb : b.wa, k0 = h ? b.wa : 0;
        const int ng = kps >> 6;  // k-groups per wave
        const int units = 4 * ng * 64;
        f32x4* d4 = reinterpret_cast<f32x4*>(dst + (h ? 16 * b.kpa : 0));
        for (int u = tid; u < units; u += NT) {
          const int l = u & 63, g = (u >> 6) % ng, w = (u >> 6) / ng;
          const int mm = l & 15, qq = l >> 4;
          const int k = w * (kps >> 2) + 16 * g + 4 * qq;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (k < wsrc) v = *reinterpret_cast<const f32x4*>(b.w + ((long)tn * 16 + mm) * b.kp + k0 + k);
          d4[u] = v;
        }
      }
    }
  }
  __syncthreads();

  const SweepCall* call = a.call;
  // the call's values are wave-uniform: in scalar registers, so branches and descriptors built on them stay scalar
  const int with_noise = __builtin_amdgcn_readfirstlane(call->with_noise);
  const float* noise = reinterpret_cast<const float*>(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)call->noise)) |
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)call->noise >> 32)) << 32));
  float* eps_log = call->eps_log;
  const int eps_log_steps = call->eps_log_steps;
  const uint64_t seed = call->seed, chain_base = call->chain_base, step_offset = call->step_offset;
  const long ring_bytes = a.ring_step * 4;
  unsigned known = 0;  // stages known complete team-wide (the last wait's target)
  const bool cw = wave < 4;  // compute wave
  // in0: wave w's B^T column tile (columns 16 w .. 16 w + 15 of zB), in registers for the whole sweep
  f32x4 bv[EMB_G];
  {
    const int half = nz >> 1, col = wave * 16 + m;
    int tn0;
    const bool own0 = ts_tiles(a.b[0], T, slot, &tn0) > 0;
#pragma unroll
    for (int g = 0; g < EMB_G; ++g) {
      const int kk = 16 * g + 4 * q;
      bv[g] = (own0 && cw && col < half && kk < nz) ? *reinterpret_cast<const f32x4*>(a.bmat + (long)col * nz + kk)
                                                    : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  for (int k = 0; k < a.n; ++k) {
    // the step's schedule row from LDS (a per-step scalar load from memory missed the scalar cache every step and
    // held the in0 stage's first LDS wait ~1 us)
    float tb[7];
    if (a.n <= TS_TAB_STEPS) {
#pragma unroll
      for (int i = 0; i < 7; ++i) tb[i] = tabs[8 * k + i];
    } else {
#pragma unroll
      for (int i = 0; i < 7; ++i) tb[i] = a.tab[8 * k + i];
    }
    const float c0 = tb[0], c1 = tb[1], c2 = tb[2], c3 = tb[3], c4 = tb[4];
    const bool last = tb[5] != 0.f;
    const int noisy_k = (int)tb[6];
    float* const rslot = a.ring + (long)k * a.ring_step;
    const float* const zk = a.zring + (long)k * B * nz;
    float* const zk1 = a.zring + (long)(k + 1) * B * nz;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)rslot, (short)0, (int)ring_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)zk, (short)0, B * nz * 4, 0x00020000);
#pragma unroll 1
    for (int j = 0; j < 7; ++j) {
      const TsBlock& b = a.b[j];
      const unsigned s = 7u * k + j;
      // the slot's tiles of block j from the prologue's table (two integer divisions per task otherwise)
      const int nt = __builtin_amdgcn_readfirstlane(tinfo[j][0]);
      const int tn0 = __builtin_amdgcn_readfirstlane(tinfo[j][1]);
      // tools only: the poll wave keeps its stamps in LDS (a global store in front of its poll would delay it);
      // the publishing lane writes them out after the flag
      const bool tr = a.trace != nullptr && tid == (NT > 256 ? 256 : 0);
      if (nt == 0) {  // nothing to compute: publish at once (this slot's earlier stores are drained)
        if (tid == TS_PUB && sent < 2) __hip_atomic_store(myflag, s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      // tools: with the data-driven hand-off there is no flag wait, so the first stamp marks the task's start instead
      if (tr && sent == 2) trs[0] = __builtin_amdgcn_s_memrealtime();
      const bool final_ = j == 6;
      const float* wbase = lds + lbase[j];
      // a skip half (produced at stage sb = 7 k + srcB, two or more stages back) always goes first, so every slot sums
      // in the same order (team_finish_kernel's rescue relies on it); it is normally known complete already (sb <
      // known); a slot that owned no tile of the stages since waits for it here
      const bool skip_early = b.kpb > 0;
      if (skip_early && sent < 2 && !(7u * k + b.srcB < known)) {
        if (!ts_wait(teamflags, T, 7u * k + b.srcB + 1, a.err, a.budget, &sflag, a.diag)) return;
        known = 7u * k + b.srcB + 1;
      }
      bool waited = false;
#pragma unroll 1
      for (int rt = 0; rt < nrt; ++rt) {
        const int tm = team + 8 * rt, r0 = tm * TM;
#pragma unroll 1
        for (int i = 0; i < nt; ++i) {
          const int tn = tn0 + i * T, n0 = tn * TC;
          const float* wl = wbase + (long)i * 16 * (b.kpa + b.kpb);
          const int erow = r0 + er, ecol = n0 + ec;
          const bool eok = tid < TM * TC && erow < B && ecol < b.dout;
          const int xrow = r0 + m;
          const bool xok = xrow < B;
          f32x4 xs[CH_CHUNK], xa[CH_CHUNK], zv4[EMB_G];
          auto load_z = [&]() {
#pragma unroll
            for (int g = 0; g < EMB_G; ++g) {
              const int kk = 16 * g + 4 * q;
              zv4[g] = ld_sc1(rz, (cw && xok && kk < nz && !(a.dbg & 64)) ? ((long)xrow * nz + kk) * 4 : (long)TS_OOB);
            }
          };
          // ---- independent of the previous stage: epilogue operands, the skip half
          float gate = 0.f, hb = 0.f, bl = 0.f, bs = 0.f, xi = 0.f;
          if (eok && !(a.dbg & 8)) {
            const float* ghr = a.gh + ((long)k * B + erow) * a.ldgh + b.ghoff;
            gate = ghr[ecol];
            hb = ghr[b.dout + ecol];
            bl = b.bls[tn * 16 + ec];
            bs = b.bls[tn * 16 + 8 + ec];
            if (final_ && !last && with_noise) {
              if (noise) {
                xi = noise[((long)noisy_k * B + erow) * nz + ecol];
              } else {
                float n4[4];
                philox_normal4(seed, chain_base + erow, step_offset + noisy_k, (uint32_t)(ecol >> 2),
                               DAMC_STREAM_SWEEP, n4);
                xi = pick4(n4, ecol);
              }
            }
          }
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          // a skip half that is complete already: its loads now (they land during the wait), its MFMAs while the
          // previous block's half is in flight
          const bool pre = skip_early && b.kpb <= 64 * CH_CHUNK && b.kpa <= 64 * CH_CHUNK;
          if (pre && cw) ts_load<CH_CHUNK>(xs, b.kpb, rr, a.b[b.srcB].ooff, b.wb, xrow, xok);
          if (skip_early && !pre && cw)
            ts_half<false>(acc, wl + 16 * b.kpa, b.kpb, rr, a.b[b.srcB].ooff, b.wb, xrow, xok, nullptr, 0, a.dbg,
                           sent, a.err, a.budget);
          const int half = nz >> 1;

          // ---- wait for stage s - 1 of the team (once per stage)
          if (!waited) {
            if (tr && sent < 2) trs[0] = __builtin_amdgcn_s_memrealtime();
            if (s > 0 && sent < 2 && !ts_wait(teamflags, T, s, a.err, a.budget, &sflag, a.diag)) return;
            if (tr) trs[1] = __builtin_amdgcn_s_memrealtime();
            known = s;
            waited = true;
          }

          if (j == 0) {  // in0: [sin 2pi zB, cos 2pi zB, z] of the 16 rows into LDS (as chain_kernel<true>)
            load_z();
            if (sent && cw && __any(any_sent(zv4))) {  // z of this step not landed yet: re-read (bounded)
              const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
              unsigned it = 0;
              do {
                __builtin_amdgcn_s_sleep(1);
                if (ts_giveup(t0, ++it, a.err, a.budget)) break;
                load_z();
              } while (__any(any_sent(zv4)));
            }
            if (cw && wave * 16 < half && !(a.dbg & 32)) {  // wave w: B^T columns 16 w .. 16 w + 15 (nz <= 128), in registers
              const int tt = wave;
              const int col = tt * 16 + m;
              const bool cok = col < half;
              const f32x4 e4 = emb_zb(zv4, bv);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int rrow = 4 * q + r;
                if (cok) {
                  const float t = e4[r] - rintf(e4[r]);
                  const bool ok = r0 + rrow < B;
                  embs[rrow * ld0 + col] = ok ? __builtin_amdgcn_sinf(t) : 0.f;
                  embs[rrow * ld0 + half + col] = ok ? __builtin_amdgcn_cosf(t) : 0.f;
                }
              }
            }
            if (wave == 0) {
#pragma unroll
              for (int g = 0; g < EMB_G; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const int kk = 16 * g + 4 * q + e;
                  if (kk < nz) embs[m * ld0 + 2 * half + kk] = zv4[g][e];
                }
            }
            for (int c = 2 * half + nz + tid; c < b.kpa; c += NT)
#pragma unroll
              for (int r = 0; r < TM; ++r) embs[r * ld0 + c] = 0.f;
            __syncthreads();
            if (cw) ts_half<true>(acc, wl, b.kpa, rr, 0, 0, xrow, xok, embs, ld0, a.dbg);
          } else if (cw && pre) {
            ts_load<CH_CHUNK>(xa, b.kpa, rr, a.b[b.srcA].ooff, b.wa, xrow, xok);
            if (sent) ts_ready<CH_CHUNK>(xs, b.kpb, rr, a.b[b.srcB].ooff, b.wb, xrow, xok, a.err, a.budget);
            ts_mfma<CH_CHUNK>(acc, wl + 16 * b.kpa, b.kpb, xs, a.dbg);
            if (sent) ts_ready<CH_CHUNK>(xa, b.kpa, rr, a.b[b.srcA].ooff, b.wa, xrow, xok, a.err, a.budget);
            ts_mfma<CH_CHUNK>(acc, wl, b.kpa, xa, a.dbg);
          } else if (cw) {
            ts_half<false>(acc, wl, b.kpa, rr, a.b[b.srcA].ooff, b.wa, xrow, xok, nullptr, 0, a.dbg, sent, a.err,
                           a.budget);
          }
          if (cw) {
#pragma unroll
            for (int r = 0; r < 4; ++r) red[wave][4 * q + r][m] = acc[r];
          }
          __syncthreads();
          if (tr && i == 0 && rt == 0) trs[2] = __builtin_amdgcn_s_memrealtime();
          if (eok) {
            float l = 0.f, sk = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {  // fixed order: deterministic
              l += red[w][er][ec];
              sk += red[w][er][8 + ec];
            }
            // ConcatSquashLinearSkipCtx.forward: ret = layer(x) * gate + bias; ret + skip(x)
            const float o = __builtin_fmaf(l + bl, gate, hb) + (sk + bs);  // the fma spelled out: every sweep form rounds alike
            if (!final_) {
              if (!(a.dbg & 16)) st_sc1_f(rslot + b.ooff + (long)erow * b.dout + ecol, o);
            } else {  // reverse step (diffusion_net.py:601-620): eps = z + out; pred = c0 (z - eps c1)
              const long zi = (long)erow * nz + ecol;
              float zv = ld_sc1_f(zk + zi);
              if (sent && is_sent(zv)) {  // this thread's own store of the previous step, not landed yet
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                unsigned it = 0;
                do {
                  __builtin_amdgcn_s_sleep(1);
                  if (ts_giveup(t0, ++it, a.err, a.budget)) break;
                  zv = ld_sc1_f(zk + zi);
                } while (is_sent(zv));
              }
              const float eps = a.residual ? zv + o : o;
              if (eps_log && k < eps_log_steps) st_global(eps_log + (long)k * B * nz + zi, eps);
              const float pred = mul_rn(c0, sub_rn(zv, mul_rn(eps, c1)));
              float zn;
              if (last) {
                zn = pred;
              } else {
                zn = add_rn(mul_rn(c2, zv), mul_rn(c3, pred));
                if (with_noise) zn = add_rn(zn, mul_rn(c4, xi));
              }
              st_sc1_f(zk1 + zi, zn);
            }
          }
          __syncthreads();  // red (and the in0 image) are reused by the next task
        }
      }
      // publish: (drained-flag protocol) every storing wave drains first; one lane then stores the slot's flag
      if (!sent && !(a.dbg & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == TS_PUB && sent < 2) __hip_atomic_store(myflag, s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.trace && tid == (NT > 256 ? TS_PUB : 0)) {
        uint64_t* tg = a.trace + ((long)blockIdx.x * 7 * a.n + s) * 4;
        tg[0] = trs[0];
        tg[1] = trs[1];
        tg[2] = trs[2];
        tg[3] = __builtin_amdgcn_s_memrealtime();
      }
    }
  }
}

// ---- the team sweep with the shapes compiled in (the default at the reference's denoiser, nf = 4: w = 128, and
// nz = 128 or 100).  sweep_team_kernel reads each block's widths, offsets and source blocks from the kernel
// arguments per task and keeps ~60 derived masks live across its block loop; at 100 SGPRs it spills them to VGPR
// lanes, and a task's setup ran ~1 us of v_readlane / v_writelane and scalar loads before its first MFMA
// (tools/sweep_timeline.py: 1.04-1.32 us from task start to wake, 2.8 us per task with every load and MFMA switched
// off).  Here the block loop is unrolled over compile-time blocks, so every width, K padding, column offset and
// source block is a constant, and each task:
//   * issues its handed-off loads first (the skip half, then the previous block's half; loads return in order), then
//     its epilogue operands as buffer loads that every lane issues (out-of-range offsets read 0), so their flight
//     covers the rest of the setup and every wait counts its loads exactly;
//   * double-buffers the wave-partial LDS tile, so one barrier per task goes (the next task writes the other buffer;
//     a wave reaches that task's barrier only after its epilogue reads of this one).
// Arithmetic, fragment order and MFMA order are sweep_team_kernel's (sent 2), so team_finish_kernel's rescue and the
// tests' bitwise gates hold unchanged.
constexpr int fs_dout(int j, int nz, int w) { return j == 0 ? w : (j <= 4 ? 2 * w : (j == 5 ? w : nz)); }
constexpr int fs_srcb(int j) { return j == 4 ? 2 : (j == 5 ? 1 : (j == 6 ? 0 : -1)); }
constexpr int fs_wa(int j, int nz, int w) { return j == 0 ? 2 * nz : fs_dout(j - 1, nz, w); }
constexpr int fs_wb(int j, int nz, int w) { return fs_srcb(j) >= 0 ? fs_dout(fs_srcb(j), nz, w) : 0; }
constexpr int fs_pad64(int x) { return (x + 63) / 64 * 64; }
constexpr int fs_coloff(int j, int nz, int w) { return j == 0 ? 0 : fs_coloff(j - 1, nz, w) + fs_dout(j - 1, nz, w); }
constexpr int fs_sumdout(int nz, int w) { return fs_coloff(7, nz, w); }

// per-thread and per-step state of the fast team kernel (force-inlined: it lives in registers)
struct FsCtx {
  const TsArgs* a;
  float (*red)[4][TM][16];  // [2] wave partials, double-buffered
  uint64_t* trs;
  float* lds;
  const int* lbase;
  const int (*tinfo)[2];
  float* embs;
  int tid, lane, wave, m, q, er, ec, team, slot, T, B, nrt;
  int par;  // which red buffer the next task writes
  // step
  int k, noisy_k;
  bool last;
  float c0, c1, c2, c3, c4;
  float* rslot;
  const float* zk;
  float* zk1;
  __amdgpu_buffer_rsrc_t rr, rz;
  // call
  const float* noise;
  float* eps_log;
  int with_noise, eps_log_steps;
  uint64_t seed, chain_base, step_offset;
};

template <int J, int NZ, int W>
__device__ __forceinline__ void fs_block(FsCtx& c, const f32x4 (&bv)[EMB_G]) {
  constexpr int DOUT = fs_dout(J, NZ, W), WA = fs_wa(J, NZ, W), WB = fs_wb(J, NZ, W);
  constexpr int KPA = fs_pad64(WA), KPB = fs_pad64(WB), SB = fs_srcb(J);
  constexpr int NTN = (DOUT + TC - 1) / TC, COL = fs_coloff(J, NZ, W), LDGH = 2 * fs_sumdout(NZ, W);
  constexpr bool FINAL = J == 6;
  static_assert(KPA <= 64 * CH_CHUNK && KPB <= 64 * CH_CHUNK, "one load chunk per half");
  // the halves' k-groups per wave, compile-time: only live loads are issued (ts_mfma sums c < kps / 64 either way)
  constexpr int NA = KPA / 64 > 0 ? KPA / 64 : 1, NB = KPB / 64 > 0 ? KPB / 64 : 1;
  const TsArgs& a = *c.a;
  const int B = c.B, tid = c.tid, wave = c.wave, m = c.m, q = c.q, er = c.er, ec = c.ec;
  const int nt = __builtin_amdgcn_readfirstlane(c.tinfo[J][0]);
  const int tn0 = __builtin_amdgcn_readfirstlane(c.tinfo[J][1]);
  if (nt == 0) return;
  const bool tr = a.trace != nullptr && tid == 0;
  if (tr) c.trs[0] = __builtin_amdgcn_s_memrealtime();
  const float* wbase = c.lds + c.lbase[J];
  const int ld0 = emb_ld(fs_pad64(2 * NZ));
  // this step's gate / hyper-bias rows, the block's biases, the injected noise (uniform descriptors)
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.gh + (long)c.k * B * LDGH), (short)0, B * LDGH * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.b[J].bls, (short)0, NTN * 16 * 4, 0x00020000);
  const bool nu = FINAL && !c.last && c.with_noise && c.noise;
  const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(nu ? c.noise + (long)c.noisy_k * B * NZ : a.b[J].bls), (short)0, nu ? B * NZ * 4 : 0, 0x00020000);
#pragma unroll 1
  for (int rt = 0; rt < c.nrt; ++rt) {
    const int r0 = (c.team + 8 * rt) * TM;
#pragma unroll 1
    for (int i = 0; i < nt; ++i) {
      const int tn = tn0 + i * c.T, n0 = tn * TC;
      const float* wl = wbase + i * 16 * (KPA + KPB);
      const int erow = r0 + er, ecol = n0 + ec;
      const bool eok = tid < TM * TC && erow < B && ecol < DOUT;
      const int xrow = r0 + m;
      const bool xok = xrow < B;
      // ---- handed-off loads first
      f32x4 xs[NB], xa[NA], zv4[EMB_G];
      auto load_z = [&]() {
#pragma unroll
        for (int g = 0; g < EMB_G; ++g) {
          const int kk = 16 * g + 4 * q;
          zv4[g] = ld_sc1(c.rz, (xok && kk < NZ) ? ((long)xrow * NZ + kk) * 4 : (long)TS_OOB);
        }
      };
      if constexpr (J == 0) {
        load_z();
      } else {
        if constexpr (SB >= 0) ts_load<NB>(xs, KPB, c.rr, (long)B * fs_coloff(SB, NZ, W), WB, xrow, xok);
        ts_load<NA>(xa, KPA, c.rr, (long)B * fs_coloff(J - 1, NZ, W), WA, xrow, xok);
      }
      // ---- epilogue operands (xi first: the last load, bs, is consumed by every block, so nothing is in flight at
      // the next task; the Philox draw has its own register)
      const int gofs = eok ? (erow * LDGH + 2 * COL + ecol) * 4 : (int)TS_OOB;
      const float xl = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rn, (eok && nu) ? (erow * NZ + ecol) * 4 : (int)TS_OOB, 0, 0));
      const float gate = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, gofs, 0, 0));
      const float hb = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rg, eok ? gofs + DOUT * 4 : (int)TS_OOB, 0, 0));
      const float bl = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rb, eok ? (tn * 16 + ec) * 4 : (int)TS_OOB, 0, 0));
      const float bs = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rb, eok ? (tn * 16 + 8 + ec) * 4 : (int)TS_OOB, 0, 0));
      float xp = 0.f;
      if constexpr (FINAL) {
        if (eok && !c.last && c.with_noise && !c.noise) {
          float n4[4];
          philox_normal4(c.seed, c.chain_base + erow, c.step_offset + c.noisy_k, (uint32_t)(ecol >> 2),
                         DAMC_STREAM_SWEEP, n4);
          xp = pick4(n4, ecol);
        }
      }
      if (tr && i == 0 && rt == 0) c.trs[1] = __builtin_amdgcn_s_memrealtime();
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (J == 0) {  // in0: [sin 2pi zB, cos 2pi zB, z] of the 16 rows into LDS (sweep_team_kernel's code)
        constexpr int HALF = NZ / 2;
        if (__any(any_sent(zv4))) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          unsigned it = 0;
          do {
            __builtin_amdgcn_s_sleep(1);
            if (ts_giveup(t0, ++it, a.err, a.budget)) break;
            load_z();
          } while (__any(any_sent(zv4)));
        }
        if (wave * 16 < HALF) {
          const int col = wave * 16 + m;
          const bool cok = col < HALF;
          const f32x4 e4 = emb_zb(zv4, bv);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rrow = 4 * q + r;
            if (cok) {
              const float t = e4[r] - rintf(e4[r]);
              const bool ok = r0 + rrow < B;
              c.embs[rrow * ld0 + col] = ok ? __builtin_amdgcn_sinf(t) : 0.f;
              c.embs[rrow * ld0 + HALF + col] = ok ? __builtin_amdgcn_cosf(t) : 0.f;
            }
          }
        }
        // z into the image: wave w writes k-groups 2w, 2w + 1 (every wave holds all of zv4); the pad columns past
        // 2 HALF + NZ were zeroed once in the prologue
#pragma unroll
        for (int g = 0; g < EMB_G; ++g) {
          if ((g >> 1) != wave) continue;  // wave-uniform; static register indices
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int kk = 16 * g + 4 * q + e;
            if (kk < NZ) c.embs[m * ld0 + 2 * HALF + kk] = zv4[g][e];
          }
        }
        __syncthreads();
        ts_half<true>(acc, wl, KPA, c.rr, 0, 0, xrow, xok, c.embs, ld0, 0);
      } else {
        if constexpr (SB >= 0) {
          ts_ready<NB>(xs, KPB, c.rr, (long)B * fs_coloff(SB, NZ, W), WB, xrow, xok, a.err, a.budget);
          ts_mfma<NB>(acc, wl + 16 * KPA, KPB, xs, 0);
        }
        ts_ready<NA>(xa, KPA, c.rr, (long)B * fs_coloff(J - 1, NZ, W), WA, xrow, xok, a.err, a.budget);
        ts_mfma<NA>(acc, wl, KPA, xa, 0);
      }
      float (*red)[TM][16] = c.red[c.par];
      c.par ^= 1;
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][4 * q + r][m] = acc[r];
      __syncthreads();
      if (tr && i == 0 && rt == 0) c.trs[2] = __builtin_amdgcn_s_memrealtime();
      if (eok) {
        float l = 0.f, sk = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // fixed order: deterministic
          l += red[w][er][ec];
          sk += red[w][er][8 + ec];
        }
        const float o = __builtin_fmaf(l + bl, gate, hb) + (sk + bs);  // the fma spelled out: every sweep form rounds alike
        if constexpr (!FINAL) {
          st_sc1_f(c.rslot + (long)B * COL + (long)erow * DOUT + ecol, o);
        } else {  // reverse step (diffusion_net.py:601-620): eps = z + out; pred = c0 (z - eps c1)
          const long zi = (long)erow * NZ + ecol;
          float zv = ld_sc1_f(c.zk + zi);
          if (is_sent(zv)) {  // this thread's own store of the previous step, not landed yet
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            unsigned it = 0;
            do {
              __builtin_amdgcn_s_sleep(1);
              if (ts_giveup(t0, ++it, a.err, a.budget)) break;
              zv = ld_sc1_f(c.zk + zi);
            } while (is_sent(zv));
          }
          const float eps = a.residual ? zv + o : o;
          if (c.eps_log && c.k < c.eps_log_steps) st_global(c.eps_log + (long)c.k * B * NZ + zi, eps);
          const float pred = mul_rn(c.c0, sub_rn(zv, mul_rn(eps, c.c1)));
          float zn;
          if (c.last) {
            zn = pred;
          } else {
            zn = add_rn(mul_rn(c.c2, zv), mul_rn(c.c3, pred));
            if (c.with_noise) zn = add_rn(zn, mul_rn(c.c4, c.noise ? xl : xp));
          }
          st_sc1_f(c.zk1 + zi, zn);
        }
      }
    }
  }
  if (tr) {
    const unsigned s = 7u * c.k + J;
    uint64_t* tg = a.trace + ((long)blockIdx.x * 7 * a.n + s) * 4;
    tg[0] = c.trs[0];
    tg[1] = c.trs[1];
    tg[2] = c.trs[2];
    tg[3] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int NZ, int W>
__global__ __launch_bounds__(256) void sweep_fast_kernel(TsArgs a) {
  __shared__ __attribute__((aligned(16))) float red[2][4][TM][16];
  __shared__ uint64_t trs[3];                    // tools only: this stage's stamps
  __shared__ float tabs[7 * TS_TAB_STEPS];       // the step table without its pad column (n <= TS_TAB_STEPS): the
                                                 // static LDS plus the largest weight set fits the CU's 160 KB
  __shared__ int lbase[7];
  __shared__ int tinfo[7][2];
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [wlds weights][TM][emb_ld(kpa0)] in0 image
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T, team = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int B = a.B, G = a.G;
  if (team >= G || slot >= T) return;
  if (a.dbg & 4096) {  // tests only: report a failed wait at once
    if (tid == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (a.n <= TS_TAB_STEPS)
    for (int i = tid; i < 7 * a.n; i += 256) tabs[i] = a.tab[8 * (i / 7) + i % 7];
  // ---- the owned weight tiles into LDS (sweep_team_kernel's layout)
  if (tid == 0) {
    int off = 0;
    for (int j = 0; j < 7; ++j) {
      int tn0;
      const int cnt = ts_tiles(a.b[j], T, slot, &tn0);
      lbase[j] = off;
      tinfo[j][0] = cnt;
      tinfo[j][1] = tn0;
      off += cnt * 16 * (a.b[j].kpa + a.b[j].kpb);
    }
  }
  __syncthreads();
  for (int j = 0; j < 7; ++j) {
    const TsBlock& b = a.b[j];
    int tn0;
    const int cnt = ts_tiles(b, T, slot, &tn0);
    for (int i = 0; i < cnt; ++i) {
      const int tn = tn0 + i * T;
      float* dst = lds + lbase[j] + (long)i * 16 * (b.kpa + b.kpb);
      for (int h = 0; h < 2; ++h) {
        const int kps = h ? b.kpb : b.kpa, wsrc = h ? b.wb : b.wa, k0 = h ? b.wa : 0;
        const int ng = kps >> 6;
        const int units = 4 * ng * 64;
        f32x4* d4 = reinterpret_cast<f32x4*>(dst + (h ? 16 * b.kpa : 0));
        for (int u = tid; u < units; u += 256) {
          const int l = u & 63, g = (u >> 6) % ng, w = (u >> 6) / ng;
          const int mm = l & 15, qq = l >> 4;
          const int kk = w * (kps >> 2) + 16 * g + 4 * qq;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (kk < wsrc) v = *reinterpret_cast<const f32x4*>(b.w + ((long)tn * 16 + mm) * b.kp + k0 + kk);
          d4[u] = v;
        }
      }
    }
  }
  __syncthreads();

  FsCtx c;
  c.a = &a;
  c.red = red;
  c.trs = trs;
  c.lds = lds;
  c.lbase = lbase;
  c.tinfo = tinfo;
  c.embs = lds + a.wlds;
  c.tid = tid;
  c.lane = lane;
  c.wave = wave;
  c.m = lane & 15;
  c.q = lane >> 4;
  c.er = tid >> 3;
  c.ec = tid & 7;
  c.team = team;
  c.slot = slot;
  c.T = T;
  c.B = B;
  c.nrt = (G - team + 7) / 8;
  c.par = 0;
  const SweepCall* call = a.call;
  c.with_noise = __builtin_amdgcn_readfirstlane(call->with_noise);
  c.noise = reinterpret_cast<const float*>(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)call->noise)) |
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)call->noise >> 32)) << 32));
  c.eps_log = call->eps_log;
  c.eps_log_steps = call->eps_log_steps;
  c.seed = call->seed;
  c.chain_base = call->chain_base;
  c.step_offset = call->step_offset;
  // in0: wave w's B^T column tile (columns 16 w .. 16 w + 15 of zB), in registers for the whole sweep
  f32x4 bv[EMB_G];
  {
    int tn0;
    const bool own0 = ts_tiles(a.b[0], T, slot, &tn0) > 0;
    const int col = wave * 16 + c.m;
#pragma unroll
    for (int g = 0; g < EMB_G; ++g) {
      const int kk = 16 * g + 4 * c.q;
      bv[g] = (own0 && col < NZ / 2 && kk < NZ) ? *reinterpret_cast<const f32x4*>(a.bmat + (long)col * NZ + kk)
                                                : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  {  // the in0 image's pad columns (past 2 (NZ / 2) + NZ), zero for the whole sweep
    const int ld0 = emb_ld(fs_pad64(2 * NZ));
    for (int cc = 2 * (NZ / 2) + NZ + tid; cc < fs_pad64(2 * NZ); cc += 256)
      for (int r = 0; r < TM; ++r) c.embs[r * ld0 + cc] = 0.f;
  }
  const long ring_bytes = a.ring_step * 4;
  for (int k = 0; k < a.n; ++k) {
    float tb[7];
    if (a.n <= TS_TAB_STEPS) {
#pragma unroll
      for (int i = 0; i < 7; ++i) tb[i] = tabs[7 * k + i];
    } else {
#pragma unroll
      for (int i = 0; i < 7; ++i) tb[i] = a.tab[8 * k + i];
    }
    c.k = k;
    c.c0 = tb[0];
    c.c1 = tb[1];
    c.c2 = tb[2];
    c.c3 = tb[3];
    c.c4 = tb[4];
    c.last = tb[5] != 0.f;
    c.noisy_k = (int)tb[6];
    c.rslot = a.ring + (long)k * a.ring_step;
    c.zk = a.zring + (long)k * B * NZ;
    c.zk1 = a.zring + (long)(k + 1) * B * NZ;
    c.rr = __builtin_amdgcn_make_buffer_rsrc((void*)c.rslot, (short)0, (int)ring_bytes, 0x00020000);
    c.rz = __builtin_amdgcn_make_buffer_rsrc((void*)c.zk, (short)0, B * NZ * 4, 0x00020000);
    fs_block<0, NZ, W>(c, bv);
    fs_block<1, NZ, W>(c, bv);
    fs_block<2, NZ, W>(c, bv);
    fs_block<3, NZ, W>(c, bv);
    fs_block<4, NZ, W>(c, bv);
    fs_block<5, NZ, W>(c, bv);
    fs_block<6, NZ, W>(c, bv);
  }
}

// ---- after the team launch: copy-out, or (a failed wait) the rescue
// acc += f(x) . W^T over one input half like ts_half, with the weight fragments read from the packed global array
// (the values and order the team's LDS copy holds): wrow = the lane's weight row at the half's first column
template <bool EMB>
__device__ __forceinline__ void rs_half(f32x4& acc, const float* wrow, int kps, int wsrc, const __amdgpu_buffer_rsrc_t& rs,
                                        long soff, int row, bool rok, const float* embs, int ld) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = lane & 15, q = lane >> 4;
  const int kq = kps >> 2, ng = kq >> 4, kbase = wave * kq;
  for (int c = 0; c < ng; ++c) {
    const int k = kbase + 16 * c + 4 * q;
    f32x4 x = {0.f, 0.f, 0.f, 0.f}, w = {0.f, 0.f, 0.f, 0.f};
    if (EMB) x = *reinterpret_cast<const f32x4*>(embs + m * ld + k);
    else if (rok && k < wsrc) x = ld_sc1(rs, (soff + (long)row * wsrc + k) * 4);
    if (k < wsrc) w = *reinterpret_cast<const f32x4*>(wrow + k);
    if (!EMB) {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = x[e] > 0.f ? x[e] : 0.01f * x[e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[e], w[e], acc, 0, 0, 0);
  }
}

// One workgroup (4 waves) per row tile.  err == 0: copy the sweep's result (zring[n]) to zt.  err != 0 (a team
// member's bounded wait gave up: a workgroup never became resident, e.g. another process or stream held CUs): the
// workgroup recomputes its row tile's whole sweep alone — every (step, block, column tile) with the team's
// arithmetic (same fragments and MFMA order, skip half first, the same fixed-order wave sum and epilogue), so the
// result is bitwise the team's — and marks the failure in host-visible memory (the library then runs the launch
// chain for the rest of the process).  A team failure costs time, never correctness, and never NaN.
__global__ __launch_bounds__(256) void team_finish_kernel(TsArgs a, float* zt, int* hostflag) {
  __shared__ __attribute__((aligned(16))) float red[4][TM][16];
  __shared__ __attribute__((aligned(16))) float embs[TM * (256 + 8)];  // in0 image (kpa of in0 <= 256: nz <= 128)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, q = lane >> 4;
  const int er = tid >> 3, ec = tid & 7;
  const int nz = a.nz, B = a.B;
  const int r0 = blockIdx.x * TM;
  const int rows = min(TM, B - r0);
  const int err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float* const zfin = a.zring + (long)a.n * B * nz;
  if (err) {
    if (blockIdx.x == 0 && tid == 0 && hostflag) __hip_atomic_store(hostflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const SweepCall* call = a.call;
    const int with_noise = call->with_noise;
    const float* noise = call->noise;
    float* eps_log = call->eps_log;
    const int eps_log_steps = call->eps_log_steps;
    const uint64_t seed = call->seed, chain_base = call->chain_base, step_offset = call->step_offset;
    const long ring_bytes = a.ring_step * 4;
    const int half = nz >> 1, ld0 = emb_ld(a.b[0].kpa);
    const int xrow = r0 + m;
    const bool xok = xrow < B;
    // B^T tile of in0's Fourier projection (wave w: columns 16 w .. 16 w + 15), as the team holds it
    f32x4 bv[EMB_G];
#pragma unroll
    for (int g = 0; g < EMB_G; ++g) {
      const int kk = 16 * g + 4 * q, col = wave * 16 + m;
      bv[g] = (col < half && kk < nz) ? *reinterpret_cast<const f32x4*>(a.bmat + (long)col * nz + kk)
                                      : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int k = 0; k < a.n; ++k) {
      const float* tb = a.tab + 8 * k;
      const float c0 = tb[0], c1 = tb[1], c2 = tb[2], c3 = tb[3], c4 = tb[4];
      const bool last = tb[5] != 0.f;
      const int noisy_k = (int)tb[6];
      float* const rslot = a.ring + (long)k * a.ring_step;
      const float* const zk = a.zring + (long)k * B * nz;
      float* const zk1 = a.zring + (long)(k + 1) * B * nz;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)rslot, (short)0, (int)ring_bytes, 0x00020000);
      const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)zk, (short)0, B * nz * 4, 0x00020000);
      // in0 image: [sin 2 pi zB, cos 2 pi zB, z] of the 16 rows (the team's in0 code)
      {
        f32x4 zv4[EMB_G];
#pragma unroll
        for (int g = 0; g < EMB_G; ++g) {
          const int kk = 16 * g + 4 * q;
          zv4[g] = (xok && kk < nz) ? ld_sc1(rz, ((long)xrow * nz + kk) * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if (wave * 16 < half) {
          const int col = wave * 16 + m;
          const f32x4 e4 = emb_zb(zv4, bv);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rrow = 4 * q + r;
            if (col < half) {
              const float t = e4[r] - rintf(e4[r]);
              const bool ok = r0 + rrow < B;
              embs[rrow * ld0 + col] = ok ? __builtin_amdgcn_sinf(t) : 0.f;
              embs[rrow * ld0 + half + col] = ok ? __builtin_amdgcn_cosf(t) : 0.f;
            }
          }
        }
        if (wave == 0) {
#pragma unroll
          for (int g = 0; g < EMB_G; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int kk = 16 * g + 4 * q + e;
              if (kk < nz) embs[m * ld0 + 2 * half + kk] = zv4[g][e];
            }
        }
        for (int c = 2 * half + nz + tid; c < a.b[0].kpa; c += 256)
#pragma unroll
          for (int r = 0; r < TM; ++r) embs[r * ld0 + c] = 0.f;
        __syncthreads();
      }
      for (int j = 0; j < 7; ++j) {
        const TsBlock& b = a.b[j];
        const bool final_ = j == 6;
        for (int tn = 0; tn < b.ntn; ++tn) {
          const int n0 = tn * TC, erow = r0 + er, ecol = n0 + ec;
          const bool eok = tid < TM * TC && erow < B && ecol < b.dout;
          float gate = 0.f, hb = 0.f, bl = 0.f, bs = 0.f, xi = 0.f;
          if (eok) {
            const float* ghr = a.gh + ((long)k * B + erow) * a.ldgh + b.ghoff;
            gate = ghr[ecol];
            hb = ghr[b.dout + ecol];
            bl = b.bls[tn * 16 + ec];
            bs = b.bls[tn * 16 + 8 + ec];
            if (final_ && !last && with_noise) {
              if (noise) {
                xi = noise[((long)noisy_k * B + erow) * nz + ecol];
              } else {
                float n4[4];
                philox_normal4(seed, chain_base + erow, step_offset + noisy_k, (uint32_t)(ecol >> 2), DAMC_STREAM_SWEEP, n4);
                xi = pick4(n4, ecol);
              }
            }
          }
          const float* wrow = b.w + ((long)tn * 16 + m) * b.kp;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          if (j == 0) {
            rs_half<true>(acc, wrow, b.kpa, b.wa, rr, 0, xrow, xok, embs, ld0);
          } else {
            if (b.kpb > 0) rs_half<false>(acc, wrow + b.wa, b.kpb, b.wb, rr, a.b[b.srcB].ooff, xrow, xok, nullptr, 0);
            rs_half<false>(acc, wrow, b.kpa, b.wa, rr, a.b[b.srcA].ooff, xrow, xok, nullptr, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) red[wave][4 * q + r][m] = acc[r];
          __syncthreads();
          if (eok) {
            float l = 0.f, sk = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              l += red[w][er][ec];
              sk += red[w][er][8 + ec];
            }
            const float o = __builtin_fmaf(l + bl, gate, hb) + (sk + bs);  // the fma spelled out: every sweep form rounds alike
            if (!final_) {
              rslot[b.ooff + (long)erow * b.dout + ecol] = o;
            } else {
              const long zi = (long)erow * nz + ecol;
              const float zv = ld_sc1_f(zk + zi);
              const float eps = a.residual ? zv + o : o;
              if (eps_log && k < eps_log_steps) eps_log[(long)k * B * nz + zi] = eps;
              const float pred = mul_rn(c0, sub_rn(zv, mul_rn(eps, c1)));
              float zn;
              if (last) {
                zn = pred;
              } else {
                zn = add_rn(mul_rn(c2, zv), mul_rn(c3, pred));
                if (with_noise) zn = add_rn(zn, mul_rn(c4, xi));
              }
              zk1[zi] = zn;
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this tile's outputs are in L2 before any wave reads them
          __syncthreads();
        }
      }
    }
  }
  // copy-out of the row tile (sc1: a rescue's own stores are read back past L1)
  for (int i = tid; i < rows * nz; i += 256) zt[(long)r0 * nz + i] = ld_sc1_f(zfin + (long)r0 * nz + i);
}

// ------------------------------------------------------------------------------ skinny GEMMs of the precompute
// Y[m][n] = act(sum_k f(A[m][k]) W[n][k] + bias[n]) for the sweep's short-M products (the time MLP and qt over
// n steps, px over B rows): the chain kernel's tile (16 rows x 16 columns, K split over 4 waves, every lane's
// f32x4 loads of a chunk in flight together) so a product of a few hundred rows fills the chip with one memory
// round trip per chunk, where 128 x 128 tiles would give it 9 workgroups walking K serially.  W is read in its
// PyTorch (out, in) layout; the N columns are up to 7 segments with their own weight rows and bias (the 7
// blocks' ctx Linears side by side).
struct SkSeg {
  const float* w;     // row n - n0 of the segment at w + (n - n0) * ldw
  const float* bias;  // or null
  long ldw;
  int n0;
};
struct SkArgs {
  const float* A;
  long lda;
  int M, N, K;
  SkSeg seg[7];
  int nseg;
  int silu_a, silu_y;
  float* Y;
  long ldy;
};

__global__ __launch_bounds__(256) void skinny_gemm_kernel(SkArgs a) {
  __shared__ __attribute__((aligned(16))) float red[4][16][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, q = lane >> 4;
  const int ntn = a.N >> 4;
  const int tn = blockIdx.x % ntn, tm = blockIdx.x / ntn;
  const int r0 = tm * 16, n0 = tn * 16;
  int sg = 0;
  while (sg + 1 < a.nseg && a.seg[sg + 1].n0 <= n0) ++sg;
  const SkSeg& S = a.seg[sg];
  const int kq = ((a.K + 63) >> 6) << 4;  // per-wave K span, whole 16-deep k-groups
  const int kbase = wave * kq;
  const int row = r0 + m, col = n0 + m;
  const bool rok = row < a.M;
  const float* arow = a.A + (long)row * a.lda;
  const float* wrow = S.w + (long)(col - S.n0) * S.ldw;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int g0 = 0; g0 < kq; g0 += 16 * CH_CHUNK) {
    f32x4 xa[CH_CHUNK], wb[CH_CHUNK];
#pragma unroll
    for (int c = 0; c < CH_CHUNK; ++c) {
      const int k = kbase + g0 + 16 * c + 4 * q;
      const bool ok = g0 + 16 * c < kq && k < a.K;
      xa[c] = (ok && rok) ? *reinterpret_cast<const f32x4*>(arow + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      wb[c] = ok ? *reinterpret_cast<const f32x4*>(wrow + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int c = 0; c < CH_CHUNK; ++c) {
      f32x4 x = xa[c];
      if (a.silu_a) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = x[e] / (1.f + expf(-x[e]));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[e], wb[c][e], acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][4 * q + r][m] = acc[r];
  __syncthreads();
  const int er = tid >> 4, ec = tid & 15;
  const int orow = r0 + er, ocol = n0 + ec;
  if (orow >= a.M) return;
  float v = ((red[0][er][ec] + red[1][er][ec]) + red[2][er][ec]) + red[3][er][ec];
  if (S.bias) v += S.bias[ocol - S.n0];
  if (a.silu_y) v = v / (1.f + expf(-v));
  a.Y[(long)orow * a.ldy + ocol] = v;
}

int launch_skinny(const SkArgs& a, const char* prof, hipStream_t s) {
  if (a.M <= 0 || (a.N & 15) || (a.K & 3) || (a.lda & 3) || a.nseg < 1 || a.nseg > 7) return DAMC_ERR_UNSUPPORTED;
  for (int i = 0; i < a.nseg; ++i)
    if ((a.seg[i].ldw & 3) || (a.seg[i].n0 & 15)) return DAMC_ERR_UNSUPPORTED;
  ProfScope ps(prof, 2.0 * a.M * a.N * a.K, s);
  const unsigned grid = (unsigned)(((a.M + 15) / 16) * (a.N / 16));
  hipLaunchKernelGGL(skinny_gemm_kernel, dim3(grid), dim3(256), 0, s, a);
  return (int)hipGetLastError();
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

// the same, 4 columns per thread (S % 4 == 0), grid.y = step: no 64-bit division per element, and SiLU on the
// transcendental unit (exp2 and reciprocal, ~1 ulp each) unless exact (DAMC_SWEEP_HYPER_SIGMOID=exact: ctx_kernel's
// expf and IEEE division); 16 M SiLUs per CIFAR sweep
__global__ __launch_bounds__(256) void ctx4_kernel(const float* __restrict__ px, const float* __restrict__ qt, int BS,
                                                   int S, int exact, float* __restrict__ c) {
  const int r4 = 4 * (blockIdx.x * 256 + threadIdx.x), k = blockIdx.y;
  if (r4 >= BS) return;
  const int s = r4 % S;
  const f32x4 a = *reinterpret_cast<const f32x4*>(px + r4), b = *reinterpret_cast<const f32x4*>(qt + (long)k * S + s);
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float u = a[e] + b[e];
    o[e] = exact ? u / (1.f + expf(-u)) : u * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-u * 1.4426950408889634f));
  }
  *reinterpret_cast<f32x4*>(c + (long)k * BS + r4) = o;
}

// the ctx launch of a sweep: ctx4_kernel where the rows allow float4 access
int launch_ctx(const float* px, const float* qt, int n, int B, int S, float* cx, hipStream_t s) {
  const char* hs = getenv("DAMC_SWEEP_HYPER_SIGMOID");  // (read per call)
  const int exact = hs && strcmp(hs, "exact") == 0;
  const long BS = (long)B * S;
  if (S % 4 == 0 && BS < (1L << 31) && (uintptr_t)px % 16 == 0 && (uintptr_t)qt % 16 == 0 && (uintptr_t)cx % 16 == 0) {
    hipLaunchKernelGGL(ctx4_kernel, dim3((unsigned)((BS / 4 + 255) / 256), (unsigned)n), dim3(256), 0, s, px, qt,
                       (int)BS, S, exact, cx);
  } else {
    const long tot = (long)n * BS;
    hipLaunchKernelGGL(ctx_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, px, qt, B, S, tot, cx);
  }
  return (int)hipGetLastError();
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

// the call's per-call record and z, and (team launch) the team flags, error word and diagnostics zeroed: a kernel in
// the stream, not a memset node, so a captured sweep orders it like every other kernel
__global__ void sweep_setup_kernel(SweepCall c, SweepCall* dst, const float* zt, float* zw, long n, unsigned* zero,
                                   long nzero, f32x4* s1, long ns1, f32x4* s2, long ns2) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *dst = c;
  // every range is grid-stride: the grid is capped (sweep_setup_grid), so B*nz may exceed the thread count
  const long st = (long)gridDim.x * blockDim.x;
  // a caller's NaN is stored canonical, so a NaN payload can never be the hand-off sentinel (TS_SENT) in the ring
  for (long j = i; j < n; j += st) {
    const float v = zt[j];
    zw[j] = (v != v) ? __builtin_bit_cast(float, 0x7FC00000u) : v;
  }
  for (long j = i; j < nzero; j += st) zero[j] = 0u;
  // sentinel hand-offs: every ring slot of the sweep (16 B per store)
  const float sv = __builtin_bit_cast(float, 0x7FC0DEADu);
  const f32x4 s4 = {sv, sv, sv, sv};
  for (long j = i; j < ns1; j += st) s1[j] = s4;
  for (long j = i; j < ns2; j += st) s2[j] = s4;
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
  // team sweep: per-step ring slots of the block outputs and of z, the step table, the team flags, the error word
  float *ring, *zring, *tab;
  unsigned* tflags;
  int* err;
  int* diag;
  size_t bytes;
};
constexpr long TS_CTL_WORDS = 8L * TS_MAXT * TS_FS + 64 + 8L * TS_MAXT * 4;

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
  t.ring = take((long)n * B * S);
  t.zring = take((long)(n + 1) * B * d->nz);
  t.tab = take(8L * n);
  // team flags, then the error word, then the failed waits' diagnostics
  t.tflags = reinterpret_cast<unsigned*>(take(TS_CTL_WORDS));
  t.err = reinterpret_cast<int*>(t.tflags + 8 * TS_MAXT * TS_FS);
  t.diag = reinterpret_cast<int*>(t.tflags + 8 * TS_MAXT * TS_FS + 64);
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

// tools only: DAMC_CHAIN_TRACE=<file> gives every chain launch a stamp row; chain_trace_dump writes them after the
// sweep (host sync) as {launches, then [launch][512][2] stamps}
uint64_t* g_trace = nullptr;
long g_trace_rows = 0;
uint64_t* chain_trace_buffer(long rows) {
  static const bool on = getenv("DAMC_CHAIN_TRACE") != nullptr;
  if (!on || rows > 4096) return nullptr;
  if (!g_trace) {
    if (hipMalloc(&g_trace, 4096L * 512 * 8 * sizeof(uint64_t)) != hipSuccess) g_trace = nullptr;
  }
  g_trace_rows = rows;
  return g_trace;
}
void chain_trace_dump(hipStream_t s) {
  if (!g_trace) return;
  std::vector<uint64_t> h((size_t)g_trace_rows * 512 * 8);
  if (hipStreamSynchronize(s) != hipSuccess) return;
  if (hipMemcpy(h.data(), g_trace, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return;
  if (FILE* f = fopen(getenv("DAMC_CHAIN_TRACE"), "wb")) {
    const long rows = g_trace_rows;
    fwrite(&rows, sizeof(rows), 1, f);
    fwrite(h.data(), sizeof(uint64_t), h.size(), f);
    fclose(f);
  }
  (void)hipMemsetAsync(g_trace, 0, h.size() * sizeof(uint64_t), s);
}

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
  uint64_t* trace = chain_trace_buffer(7L * n);
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
      a.trace = trace;
      a.li = 7 * k + j;
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

// ---- team sweep host side
// DAMC_SWEEP_TEAM=0 selects the launch chain (read per call, so one process can A/B the two)
bool team_enabled() {
  const char* e = getenv("DAMC_SWEEP_TEAM");
  return !(e && e[0] == '0');
}

constexpr size_t TS_LDS_MAX = 160 * 1024 - 16 * 1024;  // dynamic LDS a workgroup may take (static red, tabs etc. aside)
constexpr size_t TS_LDS_MIN = 84 * 1024;              // > half the CU's LDS: one workgroup per CU

// slots per team on this device: CUs / 8 (0 when the CUs do not split into 8 XCD groups)
int team_slots() {
  static std::mutex mu;
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> lk(mu);
  if (!cached[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev] = (cus % 8 == 0 && cus >= 8) ? std::min(cus / 8, TS_MAXT) : -1;
    (void)hipFuncSetAttribute((const void*)sweep_team_kernel<TS_THREADS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)TS_LDS_MAX);
    (void)hipFuncSetAttribute((const void*)sweep_team_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)TS_LDS_MAX);
    (void)hipFuncSetAttribute((const void*)sweep_fast_kernel<128, 128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)TS_LDS_MAX);
    (void)hipFuncSetAttribute((const void*)sweep_fast_kernel<100, 128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)TS_LDS_MAX);
  }
  return std::max(cached[dev], 0);
}

inline int pad64(int v) { return (v + 63) / 64 * 64; }

// the team launch of a sweep: 0, or DAMC_ERR_UNSUPPORTED when the weights do not fit the LDS of a team
int team_plan(const damc_denoiser_t* d, const SweepWs& w, int B, int n, TsArgs* a, int* P, size_t* smem) {
  const int T = team_slots();
  if (T < 1) return DAMC_ERR_UNSUPPORTED;
  if ((long)B * sum_dout(d) * 4 >= (1L << 31) || (long)B * d->nz * 4 >= (1L << 31)) return DAMC_ERR_UNSUPPORTED;
  memset(a, 0, sizeof(*a));
  const int srcA[7] = {-1, 0, 1, 2, 3, 4, 5}, srcB[7] = {-1, -1, -1, -1, 2, 1, 0};
  int coloff = 0, tiles = 0;
  for (int j = 0; j < 7; ++j) {
    const damc_csq_block_t& bk = d->blocks[j];
    TsBlock& p = a->b[j];
    p.w = w.w[j];
    p.bls = w.bls[j];
    p.kp = kpad(bk.din);
    p.dout = bk.dout;
    p.ntn = (bk.dout + TC - 1) / TC;
    p.srcA = srcA[j];
    p.srcB = srcB[j];
    p.wa = j ? d->blocks[j - 1].dout : bk.din;
    p.wb = srcB[j] >= 0 ? d->blocks[srcB[j]].dout : 0;
    if (p.wa + p.wb != bk.din) return DAMC_ERR_UNSUPPORTED;
    p.kpa = pad64(p.wa);
    p.kpb = pad64(p.wb);
    p.ooff = (long)B * coloff;
    p.ghoff = 2 * coloff;
    p.toff = tiles % T;
    tiles += p.ntn;
    coloff += bk.dout;
  }
  const char* lay = getenv("DAMC_SWEEP_LAYOUT");  // (read per call) 1: in0 placed after out2 (below); 0: in order
  if (!(lay && lay[0] == '0')) {
    for (int j = 1, t = 0; j < 7; ++j) {
      a->b[j].toff = t % T;
      t += a->b[j].ntn;
    }
  // block 0 (in0) right after out2's tiles: out2 -> in0 crosses the step, and a slot that has just published out2 would
  // otherwise start its in0 wait a publish + poll round trip late; with disjoint slots the in0 owners are already
  // polling when out2 completes (blocks 1..6 are placed in order from slot 0, which also keeps out1 / out2 disjoint)
    a->b[0].toff = (a->b[6].toff + a->b[6].ntn) % T;
  }
  long wl = 0;
  for (int t = 0; t < T; ++t) {
    long s = 0;
    for (int j = 0; j < 7; ++j) {
      const TsBlock& p = a->b[j];
      const int f = ((t - p.toff) % T + T) % T;
      const int c = f < p.ntn ? (p.ntn - f + T - 1) / T : 0;
      s += (long)c * 16 * (p.kpa + p.kpb);
    }
    wl = std::max(wl, s);
  }
  size_t sm = (size_t)(wl + (long)TM * emb_ld(a->b[0].kpa)) * sizeof(float);
  if (sm > TS_LDS_MAX) return DAMC_ERR_UNSUPPORTED;
  sm = std::max(sm, TS_LDS_MIN);
  {  // every workgroup must be resident (one per CU): otherwise the launch chain
    static std::mutex mu;
    static size_t ok_sm[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return DAMC_ERR_UNSUPPORTED;
    std::lock_guard<std::mutex> lk(mu);
    if (ok_sm[dev] != sm) {
      int per = 0;
      int per2 = 0;
      int per4 = 0, per5 = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, sweep_team_kernel<TS_THREADS>, TS_THREADS, sm) !=
              hipSuccess || per < 1 ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per2, sweep_team_kernel<256>, 256, sm) != hipSuccess ||
          per2 < 1 ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per4, sweep_fast_kernel<128, 128>, 256, sm) != hipSuccess ||
          per4 < 1 ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per5, sweep_fast_kernel<100, 128>, 256, sm) != hipSuccess ||
          per5 < 1)
        return DAMC_ERR_UNSUPPORTED;
      ok_sm[dev] = sm;
    }
  }
  a->bmat = w.bmat;
  a->nz = d->nz;
  a->B = B;
  a->G = (B + TM - 1) / TM;
  a->n = n;
  a->residual = d->residual;
  a->T = T;
  a->gh = w.gh;
  a->ldgh = 2L * sum_dout(d);
  a->ring = w.ring;
  a->ring_step = (long)B * sum_dout(d);
  a->zring = w.zring;
  a->tab = w.tab;
  a->call = w.call;
  a->flags = w.tflags;
  a->err = w.err;
  a->diag = w.diag;
  a->budget = 2000000;  // 20 ms at 100 MHz per wait: a stage takes microseconds
  a->wlds = (int)wl;
  // the shape-specialised kernel: only where every block matches the compiled-in table
  const char* fe = getenv("DAMC_SWEEP_FAST");  // (read per call) 0: the generic team kernel
  a->fast = 0;
  if (!(fe && fe[0] == '0') && (d->nz == 128 || d->nz == 100) && (long)B * a->ldgh * 4 < (1L << 31)) {
    const int nz = d->nz, w = 128;
    bool ok = a->ldgh == 2L * fs_sumdout(nz, w);
    for (int j = 0; j < 7 && ok; ++j) {
      const TsBlock& p = a->b[j];
      ok = p.dout == fs_dout(j, nz, w) && p.wa == fs_wa(j, nz, w) && p.wb == fs_wb(j, nz, w) &&
           p.kpa == fs_pad64(fs_wa(j, nz, w)) && p.kpb == fs_pad64(fs_wb(j, nz, w)) && p.srcB == fs_srcb(j) &&
           p.ooff == (long)B * fs_coloff(j, nz, w) && p.ghoff == 2 * fs_coloff(j, nz, w);
    }
    if (ok) {  // its static LDS differs from the generic kernel's: the launch must fit the CU
      hipFuncAttributes fa;
      const void* fn = nz == 128 ? (const void*)sweep_fast_kernel<128, 128> : (const void*)sweep_fast_kernel<100, 128>;
      if (hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.sharedSizeBytes + sm <= 160 * 1024) a->fast = nz;
    }
  }
  static const int dbg = [] {
    const char* e = getenv("DAMC_SWEEP_DBG");
    return e ? atoi(e) : 0;
  }();
  a->dbg = dbg;
  const char* ff = getenv("DAMC_SWEEP_FORCE_FAIL");  // tests (read per call): every wait fails, the rescue runs
  if (ff && ff[0] == '1') a->dbg |= 4096;
  *P = 8 * T;
  *smem = sm;
  return 0;
}


// the step table (c0..c4, is_last, noisy_k per step) of a schedule, uploaded once per (device, schedule) and kept:
// a sweep then copies nothing from the host, so it can be captured into a HIP graph (after one eager call with
// the same schedule, as torch.cuda.graphs' warm-up does)
struct TabEntry {
  int dev;
  std::vector<float> key;
  float* d;
};
std::mutex g_tab_mu;
std::vector<TabEntry> g_tabs;

int step_table(const float* coef, int n, hipStream_t s, const float** out) {
  int dev = 0;
  DAMC_CHECK(hipGetDevice(&dev));
  std::vector<float> key(coef, coef + 6 * (size_t)n);
  std::lock_guard<std::mutex> lk(g_tab_mu);
  for (const TabEntry& e : g_tabs)
    if (e.dev == dev && e.key == key) {
      *out = e.d;
      return 0;
    }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  DAMC_CHECK(hipStreamIsCapturing(s, &cs));
  if (cs != hipStreamCaptureStatusNone) return DAMC_ERR_UNSUPPORTED;  // first use of a schedule inside a capture
  std::vector<float> tab(8 * (size_t)n, 0.f);
  for (int k = 0, noisy = 0; k < n; ++k) {
    for (int i = 0; i < 6; ++i) tab[8 * k + i] = coef[6 * (size_t)k + i];
    tab[8 * k + 6] = (float)noisy;
    if (coef[6 * (size_t)k + 5] == 0.f) ++noisy;
  }
  float* d = nullptr;
  DAMC_CHECK(hipMalloc(&d, tab.size() * sizeof(float)));
  DAMC_CHECK(hipMemcpy(d, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice));
  if (g_tabs.size() >= 64) {  // a handful of schedules per process in practice
    (void)hipFree(g_tabs.front().d);
    g_tabs.erase(g_tabs.begin());
  }
  g_tabs.push_back(TabEntry{dev, std::move(key), d});
  *out = d;
  return 0;
}

int run_chain_team(TsArgs& a, int P, size_t smem, const float* coef, hipStream_t s) {
  const int n = a.n;
  int rc = step_table(coef, n, s, &a.tab);
  if (rc) return rc;
  static const bool trace = getenv("DAMC_SWEEP_TRACE") != nullptr;
  const size_t tbytes = (size_t)P * 7 * n * 4 * sizeof(uint64_t);
  if (trace) {
    DAMC_CHECK(hipMalloc(&a.trace, tbytes));
    DAMC_CHECK(hipMemsetAsync(a.trace, 0, tbytes, s));
  }
  if (a.sent == 2 && a.fast == 128)
    hipLaunchKernelGGL((sweep_fast_kernel<128, 128>), dim3(P), dim3(256), smem, s, a);
  else if (a.sent == 2 && a.fast == 100)
    hipLaunchKernelGGL((sweep_fast_kernel<100, 128>), dim3(P), dim3(256), smem, s, a);
  else if (a.sent == 2)
    hipLaunchKernelGGL((sweep_team_kernel<256>), dim3(P), dim3(256), smem, s, a);
  else
    hipLaunchKernelGGL((sweep_team_kernel<TS_THREADS>), dim3(P), dim3(TS_THREADS), smem, s, a);
  DAMC_LAUNCH_CHECK();
  if (trace) {  // tools/sweep_trace.py reads the dump: P, n, G, then the stamps
    std::vector<uint64_t> h((size_t)P * 7 * n * 4);
    DAMC_CHECK(hipStreamSynchronize(s));
    DAMC_CHECK(hipMemcpy(h.data(), a.trace, tbytes, hipMemcpyDeviceToHost));
    (void)hipFree(a.trace);
    a.trace = nullptr;
    if (FILE* f = fopen(getenv("DAMC_SWEEP_TRACE"), "wb")) {
      const int hdr[3] = {P, n, a.G};
      fwrite(hdr, sizeof(hdr), 1, f);
      fwrite(h.data(), sizeof(uint64_t), h.size(), f);
      fclose(f);
    }
  }
  return 0;
}

// A failed team launch (rescued on the device by team_finish_kernel) is reported through one host-visible word per
// device; the next sweep on that device reads it (no synchronisation: a failure still in flight is seen a call
// later) and the process keeps to the launch chain from then on.
struct TeamHealth {
  int* host = nullptr;  // pinned, mapped: host view
  int* dev = nullptr;   // its device address
  bool disabled = false;
  long failures = 0;
};
std::mutex g_health_mu;
TeamHealth g_health[64];

// the device's health word (allocated on first use outside a capture; null inside one: the rescue still runs)
int* team_health_word(int dev, bool capturing) {
  std::lock_guard<std::mutex> lk(g_health_mu);
  TeamHealth& h = g_health[dev];
  if (!h.host && !capturing) {
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
      h.host = static_cast<int*>(p);
      *reinterpret_cast<volatile int*>(h.host) = 0;
      void* d = nullptr;
      if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess) h.dev = static_cast<int*>(d);
    }
  }
  return h.dev;
}

// true when the team launch may be used on this device: no earlier team launch has needed the rescue
bool team_healthy(int dev) {
  std::lock_guard<std::mutex> lk(g_health_mu);
  TeamHealth& h = g_health[dev];
  if (h.disabled) return false;
  if (h.host && *reinterpret_cast<volatile int*>(h.host)) {
    *reinterpret_cast<volatile int*>(h.host) = 0;
    ++h.failures;
    static const bool keep = [] {
      const char* e = getenv("DAMC_SWEEP_TEAM_KEEP");  // tests: stay on the team launch after a rescue
      return e && e[0] == '1';
    }();
    if (!keep) {
      h.disabled = true;
      fprintf(stderr, "damc: a team reverse-sweep launch on device %d could not keep all its workgroups resident; "
                      "its result was recomputed on the device, and this process now uses the launch chain\n", dev);
      return false;
    }
  }
  return true;
}


// ---- the hyper GEMMs on the limb product (round 5): per block j, [gate | hyper bias] = [sigmoid(c Wg^T + bg) | c Wb^T]
// over all n * B (step, row) pairs, K = dout <= 512: one limb-engine sign block, so no sign alternation.  The weights
// are read as the PyTorch Linear rows themselves ([dout][dout], k contiguous; row n < dout of the [2 dout][dout] operand
// is Wg's, the rest Wb's) and split into limbs on their way into LDS, with c's rows; one workgroup = 128 rows x 64
// columns, 8 waves of 32 x 32, the limb engine's six-MFMA product (encoder.hip enc_head_x3_kernel has the same tile).
// The 7 blocks in one launch (tile table); the epilogue adds bg and applies the gate's sigmoid as gemm.hip's EPI_GATE.
typedef __bf16 hy8 __attribute__((ext_vector_type(8)));
typedef __bf16 hy4 __attribute__((ext_vector_type(4)));
constexpr int HY_BM = 128, HY_BN = 64, HY_KT = 32, HY_THREADS = 512, HY_ROWS = HY_BM + HY_BN, HY_NTMAX = 16;
constexpr size_t HY_LDS = 2 * 3 * HY_ROWS * 4 * sizeof(hy8);

struct HyperBlock {
  const float *a, *wg, *wb, *bg;
  float* c;
  long lda, ldc;
  int M, dout, ntn, tile0;
};
struct HyperGroup {
  HyperBlock b[7];
  int n, tiles;
  int exact_sig;  // 1: the gate's sigmoid as 1 / (1 + expf(-v)) with IEEE division (DAMC_SWEEP_HYPER_SIGMOID=exact)
};

__device__ __forceinline__ int hy_slot(int row, int q) {  // (encoder.hip hd_slot: conflict-free fragment reads)
  return row * 4 + (q ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3));
}
template <int N>
__device__ __forceinline__ void hy_split(const float* x, __bf16 (&h)[N], __bf16 (&m)[N], __bf16 (&l)[N]) {
#pragma unroll
  for (int e = 0; e < N; ++e) {
    const __bf16 b0 = (__bf16)x[e];
    const float r1 = sub_rn(x[e], (float)b0);
    const __bf16 b1 = (__bf16)r1;
    h[e] = b0;
    m[e] = b1;
    l[e] = (__bf16)sub_rn(r1, (float)b1);
  }
}

template <int PD>
__global__ __launch_bounds__(HY_THREADS) void hyper_x3_kernel(HyperGroup g) {
  extern __shared__ __attribute__((aligned(16))) hy8 hyl[];  // [2 K tiles][3 limbs][HY_ROWS][4 slots]
  int j = 0;
  while (j + 1 < g.n && (int)blockIdx.x >= g.b[j + 1].tile0) ++j;
  const HyperBlock& hb = g.b[j];
  const int u = blockIdx.x - hb.tile0, m0 = (u / hb.ntn) * HY_BM, n0 = (u % hb.ntn) * HY_BN;
  const int K = hb.dout, nt = K / HY_KT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // staging: A row fr octet fq (rows past M load row M - 1 again, never stored); B row br (of the [2 dout][dout]
  // operand) half octet bh -- every thread the same loads, no branch
  const int fr = tid >> 2, fq = tid & 3, br = tid >> 3, bh = tid & 7;
  const float* ap = hb.a + (long)min(m0 + fr, hb.M - 1) * hb.lda + 8 * fq;
  const int nrow = n0 + br;
  const float* bp = (nrow < hb.dout ? hb.wg + (long)nrow * K : hb.wb + (long)(nrow - hb.dout) * K) + 4 * bh;
  f32x4 pa[PD][2], pb[PD];
  auto gload = [&](int t, int st) {
    pa[st][0] = *reinterpret_cast<const f32x4*>(ap + t * HY_KT);
    pa[st][1] = *reinterpret_cast<const f32x4*>(ap + t * HY_KT + 4);
    pb[st] = *reinterpret_cast<const f32x4*>(bp + t * HY_KT);
  };
  auto lstore = [&](int buf, int st) {
    hy8* p = hyl + buf * 3 * HY_ROWS * 4;
    const float va[8] = {pa[st][0][0], pa[st][0][1], pa[st][0][2], pa[st][0][3],
                         pa[st][1][0], pa[st][1][1], pa[st][1][2], pa[st][1][3]};
    __bf16 h[8], m[8], l[8];
    hy_split<8>(va, h, m, l);
    const int s = hy_slot(fr, fq);
    p[s] = hy8{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]};
    p[HY_ROWS * 4 + s] = hy8{m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]};
    p[2 * HY_ROWS * 4 + s] = hy8{l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7]};
    const float vb[4] = {pb[st][0], pb[st][1], pb[st][2], pb[st][3]};
    __bf16 h4[4], m4[4], l4[4];
    hy_split<4>(vb, h4, m4, l4);
    hy4* p4 = reinterpret_cast<hy4*>(p);
    const int s4 = 2 * hy_slot(HY_BM + br, bh >> 1) + (bh & 1);
    p4[s4] = hy4{h4[0], h4[1], h4[2], h4[3]};
    p4[2 * HY_ROWS * 4 + s4] = hy4{m4[0], m4[1], m4[2], m4[3]};
    p4[4 * HY_ROWS * 4 + s4] = hy4{l4[0], l4[1], l4[2], l4[3]};
  };
  const int wr = wave & 3, wc = wave >> 2, m = lane & 15, q = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < PD; ++st)
    if (st < nt) gload(st, st);
  lstore(0, 0);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < HY_NTMAX; ++t) {
    if (t >= nt) break;  // (workgroup-uniform)
    if (t + PD < nt) gload(t + PD, t % PD);
    const hy8* p = hyl + (t & 1) * 3 * HY_ROWS * 4;
    hy8 fa[2][3], fb[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int l = 0; l < 3; ++l) {
        fa[i][l] = p[l * HY_ROWS * 4 + hy_slot(32 * wr + 16 * i + m, q)];
        fb[i][l] = p[l * HY_ROWS * 4 + hy_slot(HY_BM + 32 * wc + 16 * i + m, q)];
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        f32x4 c = acc[i][jj];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[jj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[jj][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[jj][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[jj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[jj][1], c, 0, 0, 0);
        acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[jj][0], c, 0, 0, 0);
      }
    if (t + 1 < nt) lstore((t + 1) & 1, (t + 1) % PD);
    __syncthreads();
  }
  // epilogue through LDS (free after the loop's last barrier): the tile's rows leave as 256-B runs of 16-B stores
  // instead of 64-B runs of 4-B stores (144 MB of gate / hyper-bias output per CIFAR sweep)
  constexpr int LD = HY_BN + 4;
  float* ot = reinterpret_cast<float*>(hyl);  // [HY_BM][LD]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = 32 * wr + 16 * i + 4 * q + r, lc = 32 * wc + 16 * jj + m, col = n0 + lc;
        float v = acc[i][jj][r];
        if (col < hb.dout) {  // the gate: sigmoid(v + bg)
          if (hb.bg) v += hb.bg[col];
          // exp2 and reciprocal on the transcendental unit (~1 ulp each, both saturate to 0 / 1 correctly): 16 M
          // sigmoids per CIFAR sweep, where expf plus the IEEE division took a sixth of this kernel
          v = g.exact_sig ? 1.f / (1.f + expf(-v))
                          : __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-v * 1.4426950408889634f));
        }
        ot[lr * LD + lc] = v;
      }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < HY_BM * HY_BN / 4 / HY_THREADS; ++k) {
    const int f = tid + k * HY_THREADS, lr = f / (HY_BN / 4), c4 = f % (HY_BN / 4), row = m0 + lr;
    if (row < hb.M)
      *reinterpret_cast<f32x4*>(hb.c + (long)row * hb.ldc + n0 + 4 * c4) =
          *reinterpret_cast<const f32x4*>(ot + lr * LD + 4 * c4);
  }
}

}  // namespace

extern "C" long damc_sweep_team_failures(int device) {
  if (device < 0 || device >= 64) return -1;
  (void)team_healthy(device);  // picks up a failure that has completed since the last sweep
  std::lock_guard<std::mutex> lk(g_health_mu);
  return g_health[device].failures;
}

extern "C" int damc_sweep_team_words(const damc_denoiser_t* d, int B, int n, const void* wsp, size_t wsb, int* out,
                                     int nwords) {
  if (validate(d) || B <= 0 || n <= 0 || !wsp || !out || nwords <= 0) return DAMC_ERR_ARG;
  if (wsb < carve(d, B, n, nullptr, nullptr)) return DAMC_ERR_WORKSPACE;
  SweepWs w;
  carve(d, B, n, reinterpret_cast<char*>(const_cast<void*>(wsp)), &w);
  const long cnt = std::min<long>(nwords, TS_CTL_WORDS);
  DAMC_CHECK(hipDeviceSynchronize());
  DAMC_CHECK(hipMemcpy(out, w.tflags, cnt * sizeof(int), hipMemcpyDeviceToHost));
  return 0;
}

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
    // the skinny precompute GEMMs read the time MLP and ctx Linears in their PyTorch layouts: no transposes
    bool sk = (nt & 15) == 0 && (nx & 3) == 0;
    for (int j = 0; j < 7; ++j) sk = sk && (d->blocks[j].dout & 15) == 0;
    hipLaunchKernelGGL(pack_denoiser_kernel, dim3((unsigned)((maxn + 255) / 256), 7, sk ? 2 : 3), dim3(256), 0, s, pa);
    const long ntt = (long)nt * nt;
    if (!sk) {
      hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((ntt + 255) / 256)), dim3(256), 0, s, d->tw1, nt, nt, w.tw1t);
      hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((ntt + 255) / 256)), dim3(256), 0, s, d->tw2, nt, nt, w.tw2t);
    }
    const long nb = (long)d->nz * (d->nz / 2);
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, d->bmat, d->nz, d->nz / 2,
                       w.bmat);
    DAMC_LAUNCH_CHECK();
  }

  // ---- 2. ctx: time MLP (n rows), xemb part (B rows), c for every (step, row)
  bool skinny = (nt & 15) == 0 && (nx & 3) == 0;
  for (int j = 0; j < 7; ++j) skinny = skinny && (d->blocks[j].dout & 15) == 0;
  if (skinny) {
    SkArgs g;
    memset(&g, 0, sizeof(g));
    g.M = n;
    g.N = nt;
    g.K = nt;
    g.A = temb_in;
    g.lda = nt;
    g.nseg = 1;
    g.seg[0] = SkSeg{d->tw1, d->tb1, nt, 0};
    g.silu_y = 1;
    g.Y = w.t1;
    g.ldy = nt;
    if ((rc = launch_skinny(g, "sweep_pre", s))) return rc;
    g.A = w.t1;
    g.seg[0] = SkSeg{d->tw2, d->tb2, nt, 0};
    g.Y = w.t2;  // the ctx Linear consumes SiLU(temb)
    if ((rc = launch_skinny(g, "sweep_pre", s))) return rc;
    g.A = w.t2;
    g.N = S;
    g.nseg = 7;
    for (int j = 0; j < 7; ++j) g.seg[j] = SkSeg{d->wctx[j], d->bctx[j], (long)nt + nx, coloff[j]};
    g.silu_y = 0;
    g.Y = w.qt;
    g.ldy = S;
    if ((rc = launch_skinny(g, "sweep_pre", s))) return rc;
    g.A = xemb;
    g.lda = nx;
    g.M = B;
    g.K = nx;
    for (int j = 0; j < 7; ++j) g.seg[j] = SkSeg{d->wctx[j] + nt, nullptr, (long)nt + nx, coloff[j]};
    g.silu_a = 1;
    g.Y = w.px;
    if ((rc = launch_skinny(g, "sweep_pre", s))) return rc;
    if ((rc = launch_ctx(w.px, w.qt, n, B, S, w.cx, s))) return rc;
  } else {
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
    if ((rc = launch_ctx(w.px, w.qt, n, B, S, w.cx, s))) return rc;
  }

  // ---- 3. every block's gate and hyper bias for every (step, row): [sigmoid(c Wg^T + bg) | c Wb^T]
  damc::GemmArgs hg[7];
  double hflops = 0.0;
  for (int j = 0; j < 7; ++j) {
    const int dout = d->blocks[j].dout;
    damc::GemmArgs& g = hg[j];
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
    hflops += 2.0 * n * B * dout * 2.0 * dout;
  }
  // round 5: on the limb product (hyper_x3_kernel) where every block fits it; DAMC_SWEEP_HYPER=fp32 (read per call)
  // keeps the fp32-MFMA engine below
  const char* hye = getenv("DAMC_SWEEP_HYPER");
  bool hy_ok = !(hye && strcmp(hye, "fp32") == 0) && (S % 4 == 0) && ((uintptr_t)w.cx % 16 == 0) &&
               ((uintptr_t)w.gh % 16 == 0);
  HyperGroup hgp{};
  hgp.n = 7;
  {
    const char* hs = getenv("DAMC_SWEEP_HYPER_SIGMOID");  // (read per call) exact: IEEE expf and division
    hgp.exact_sig = hs && strcmp(hs, "exact") == 0;
  }
  for (int j = 0; j < 7 && hy_ok; ++j) {
    const damc_csq_block_t& bk = d->blocks[j];
    const int dout = bk.dout;
    hy_ok = dout % 32 == 0 && dout <= HY_NTMAX * HY_KT && bk.wg && bk.wb && (uintptr_t)bk.wg % 16 == 0 &&
            (uintptr_t)bk.wb % 16 == 0 && coloff[j] % 4 == 0;
    HyperBlock& h = hgp.b[j];
    h.a = w.cx + coloff[j];
    h.lda = S;
    h.wg = bk.wg;
    h.wb = bk.wb;
    h.bg = bk.bg;
    h.c = w.gh + 2 * coloff[j];
    h.ldc = 2L * S;
    h.M = n * B;
    h.dout = dout;
    h.ntn = 2 * dout / HY_BN;
    h.tile0 = hgp.tiles;
    hgp.tiles += ((h.M + HY_BM - 1) / HY_BM) * h.ntn;
  }
  if (hy_ok) {
    static const bool lds_ok = [] {
      return hipFuncSetAttribute((const void*)hyper_x3_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)HY_LDS) == hipSuccess;
    }();
    hy_ok = lds_ok;
  }
  // one grouped launch (its tiles fill the chip; seven launches of 200-400 tiles each left half of it idle in their
  // last round); the general path when a block's rows are not float4-aligned
  // DAMC_SWEEP_HYPER_GROUP=0 (read per call): seven launches (tests/test_gpu_amortizer.py checks both are bitwise equal)
  const char* hge = getenv("DAMC_SWEEP_HYPER_GROUP");
  if (hy_ok) {
    ProfScope ps("sweep_hyper", hflops, s);
    hipLaunchKernelGGL(hyper_x3_kernel<4>, dim3(hgp.tiles), dim3(HY_THREADS), HY_LDS, s, hgp);
    rc = (int)hipGetLastError();
  } else {
    rc = (hge && atoi(hge) == 0) ? DAMC_ERR_UNSUPPORTED
                                 : damc::launch_gemm_group(hg, 7, damc::EPI_GATE, "sweep_hyper", hflops, s);
  }
  if (rc == DAMC_ERR_UNSUPPORTED) {
    for (int j = 0; j < 7; ++j) {
      const int dout = d->blocks[j].dout;
      if ((rc = damc::launch_gemm(hg[j], damc::A_DENSE, damc::EPI_GATE, damc::O_DENSE, 1, "sweep_hyper",
                                  2.0 * n * B * dout * 2.0 * dout, s)))
        return rc;
    }
  } else if (rc) {
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
  TsArgs ta;
  int tP = 0;
  size_t tsm = 0;
  // inside a caller's stream capture the launch chain (when it is used) records its kernels eagerly into the caller's
  // graph instead of replaying its own cached graph
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  DAMC_CHECK(hipStreamIsCapturing(s, &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  int dev = 0;
  DAMC_CHECK(hipGetDevice(&dev));
  // inside a caller's capture the team launch is recorded like any kernel (DAMC_SWEEP_CAPTURE_TEAM=0, read per
  // call: the launch chain instead).  Round 2 recorded the launch chain there because a replayed team launch timed
  // out: its flags were zeroed by a hipMemsetAsync node, which the replay did not order before the team kernel
  // (DAMC_SWEEP_MEMSET_FLAGS=1 restores that form for tools/diag_team_capture.py); the setup kernel zeroes them now.
  const char* tic = getenv("DAMC_SWEEP_CAPTURE_TEAM");
  const bool team_in_capture = !(tic && tic[0] == '0');
  const bool team = (!capturing || team_in_capture) && team_enabled() && dev < 64 && team_healthy(dev) &&
                    team_plan(d, w, B, n, &ta, &tP, &tsm) == 0;
  int* health = team ? team_health_word(dev, capturing) : nullptr;
  const char* mf = getenv("DAMC_SWEEP_MEMSET_FLAGS");  // diagnosis only: round 2's memset form (see above)
  const bool memset_flags = team && mf && mf[0] == '1';
  if (memset_flags) DAMC_CHECK(hipMemsetAsync(w.tflags, 0, TS_CTL_WORDS * sizeof(unsigned), s));
  const long nzero = (team && !memset_flags) ? TS_CTL_WORDS : 0;
  // hand-off protocol (read per call): 2 (default) data-driven sentinel hand-offs, no flags; 1 flags without drain +
  // sentinel checks; 0 drained flags.  Bitwise the same results; same-box A/B at B=128 (tools/sweep_ab.py): 2 is
  // 6-7 % faster than 0, 1 is 4-5 % slower than 0
  const char* se = getenv("DAMC_SWEEP_SENT");
  if (team) ta.sent = se ? atoi(se) : 2;
  const long ns1 = (team && ta.sent) ? (long)n * B * S / 4 : 0, ns2 = (team && ta.sent) ? (long)n * nzb / 4 : 0;
  const long sgrid = std::min<long>(std::max<long>(std::max(nzb, nzero), (ns1 + ns2) / 8), 1L << 16);
  hipLaunchKernelGGL(sweep_setup_kernel, dim3((unsigned)((sgrid + 255) / 256)), dim3(256), 0, s, call, w.call, zt,
                     team ? w.zring : w.z, nzb, w.tflags, nzero, reinterpret_cast<f32x4*>(w.ring), ns1,
                     reinterpret_cast<f32x4*>(w.zring + nzb), ns2);
  DAMC_LAUNCH_CHECK();
  double flops_step = 0;
  for (int j = 0; j < 7; ++j) flops_step += 2.0 * B * 2.0 * d->blocks[j].din * d->blocks[j].dout;
  {
    ProfScope ps("denoise_chain", flops_step * n, s);
    if (team) {
      if ((rc = run_chain_team(ta, tP, tsm, coef, s))) return rc;
    } else if (allow_graph && graphs_enabled() && !capturing) {
      if ((rc = run_chain_graph(d, w, wsp, wsb, B, n, coef, s))) return rc;
      chain_trace_dump(s);
    } else {
      std::vector<Launch> ls;
      chain_launches(d, w, B, n, coef, ls);
      if ((rc = launch_chain(ls, s))) return rc;
    }
  }
  if (team)
    hipLaunchKernelGGL(team_finish_kernel, dim3((unsigned)ta.G), dim3(256), 0, s, ta, zt, health);
  else
    hipLaunchKernelGGL(copy_kernel, dim3((unsigned)((nzb + 255) / 256)), dim3(256), 0, s,
                       w.z, zt, nzb);
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
