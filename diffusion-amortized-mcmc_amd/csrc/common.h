// common.h — shared device helpers for libdamc (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/damc.h"

#define DAMC_CHECK(expr)                        \
  do {                                          \
    hipError_t e_ = (expr);                     \
    if (e_ != hipSuccess) return (int)e_;       \
  } while (0)

#define DAMC_LAUNCH_CHECK()                     \
  do {                                          \
    hipError_t e_ = hipGetLastError();          \
    if (e_ != hipSuccess) return (int)e_;       \
  } while (0)

#define DAMC_REQUIRE(cond)                      \
  do {                                          \
    if (!(cond)) return DAMC_ERR_ARG;           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG + Box-Muller.  Counter = (dim/4, step, chain, stream_id),
// key = seed.  A chain's draw depends only on its global index -> shard-invariant noise.
// ------------------------------------------------------------------------------------------
struct Philox4 {
  uint32_t v[4];
};

__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += W0;
    k1 += W1;
  }
  Philox4 o;
  o.v[0] = c0;
  o.v[1] = c1;
  o.v[2] = c2;
  o.v[3] = c3;
  return o;
}

// uniform in (0, 1]: never 0, so log() is finite
__device__ __forceinline__ float u01_open(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }

// 4 N(0,1) values for (chain, step, quad) — element d of a chain uses quad d>>2, slot d&3
__device__ __forceinline__ void philox_normal4(uint64_t seed, uint64_t chain, uint64_t step, uint32_t quad,
                                               uint32_t stream_id, float out[4]) {
  Philox4 r = philox4x32_10(quad, (uint32_t)step, (uint32_t)chain, stream_id ^ (uint32_t)(chain >> 32) * 0x9E3779B9u,
                            (uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(step >> 32));
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    float u1 = u01_open(r.v[2 * p]);
    float u2 = u01_open(r.v[2 * p + 1]);
    float rad = sqrtf(-2.0f * logf(u1));
    // Box-Muller angle 2 pi u2 by the hardware sin / cos, whose argument is in revolutions (u2 in (0, 1]):
    // no argument reduction, hence no large-argument path whose private array would give every kernel that
    // draws noise a scratch segment
    const float s = __builtin_amdgcn_sinf(u2), c = __builtin_amdgcn_cosf(u2);
    out[2 * p] = rad * c;
    out[2 * p + 1] = rad * s;
  }
}

enum { DAMC_STREAM_POSTERIOR = 0x51, DAMC_STREAM_PRIOR = 0x52, DAMC_STREAM_SWEEP = 0x53 };

// element i & 3 of a 4-value draw without a runtime-indexed private array (which the compiler would place in
// scratch memory: a per-dispatch scratch setup and slow private loads for every kernel that draws noise)
__device__ __forceinline__ float pick4(const float (&v)[4], int i) {
  const int j = i & 3;
  return j == 0 ? v[0] : j == 1 ? v[1] : j == 2 ? v[2] : v[3];
}

// fp32 ops that must not be contracted into FMA (bit-level match with the reference's separately rounded
// PyTorch elementwise ops: z - (c*g), then + s*xi).  HIP's __fmul_rn & co. are plain operators, which
// -ffp-contract=fast fuses after inlining; the pragma (honoured under the Makefile's
// -ffp-contract=fast-honor-pragmas) leaves these operations without the contract flag.
__device__ __forceinline__ float mul_rn(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float add_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float sub_rn(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
  if (act == DAMC_ACT_LRELU) return v > 0.f ? v : v * slope;
  if (act == DAMC_ACT_TANH) return tanhf(v);
  if (act == DAMC_ACT_SILU) return v / (1.f + expf(-v));
  return v;
}
// derivative expressed through the post-activation value (sign(h) == sign(a) for LReLU)
__device__ __forceinline__ float act_grad_from_out(float h, int act, float slope) {
  if (act == DAMC_ACT_LRELU) return h > 0.f ? 1.f : slope;
  if (act == DAMC_ACT_TANH) return 1.f - h * h;
  return 1.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------- profiling hooks
namespace damc_prof {
bool enabled();
// returns an opaque slot; call end() after the launch
int begin(const char* name, double flops, hipStream_t s);
void end(int slot, hipStream_t s);
}  // namespace damc_prof

struct ProfScope {
  int slot;
  hipStream_t s;
  ProfScope(const char* name, double flops, hipStream_t st) : slot(-1), s(st) {
    if (damc_prof::enabled()) slot = damc_prof::begin(name, flops, st);
  }
  ~ProfScope() {
    if (slot >= 0) damc_prof::end(slot, s);
  }
};
