// optim.hip — clip_grad_norm_ + Adam/AdamW steps for the G, E and Q updates.
//
// The reference updates its three networks with stock PyTorch (train_gen_recon.py:155-157 builds
// optim.Adam(G), optim.AdamW(Q, weight_decay=1e-4), optim.Adam(E), all betas (0.5, 0.999); :219, :230, :240
// clip each gradient set with torch.nn.utils.clip_grad_norm_).  Stock PyTorch runs these as ~10
// multi-tensor passes over the parameters (foreach lerp, mul, addcmul, sqrt, div, add, addcdiv, plus
// the per-tensor norms and the scaling).  Here one pass reads p, g, m, v and writes p, m, v (and g
// when the clip is fused), with the per-element arithmetic in the same op order and the same
// roundings as torch's _multi_tensor_adam (torch/optim/adam.py):
//   g  = g * clip                                   (_foreach_mul_, clip_grad.py)
//   g  = g + wd * p          (Adam, L2)             (_foreach_add alpha=wd)
//   p  = p * (1 - lr wd)     (AdamW, decoupled)     (_foreach_mul_)
//   m  = lerp(m, g, 1 - b1)                         (_foreach_lerp_)
//   v  = v * b2;  v = v + (1 - b2) g g              (_foreach_mul_, _foreach_addcmul_)
//   s  = sqrt(v) / sqrt(1 - b2^t) + eps             (_foreach_sqrt, _foreach_div_, _foreach_add_)
//   p  = p + (-lr / (1 - b1^t)) * (m / s)           (_foreach_addcdiv_)
// The norm is a fixed-order two-level sum (per chunk, then over chunks): deterministic run to run.
// HBM-bound: 28 B per element per step (32 with the fused clip write-back).  Tensor pointers are kernel
// arguments, so a step costs no host-side table work when gradient buffers move.
#include <math.h>
#include <string.h>

#include "common.h"

namespace {

struct AdamChunk {  // 16 B: which tensor, where, how long
  long long off;
  int tensor;
  int n;
};
static_assert(sizeof(AdamChunk) == 16, "chunk layout");

// the tensors' device pointers travel in the kernel arguments (<= 4 KB): no table rebuild when autograd
// hands out new gradient buffers
struct GradPtrs {
  float* g[DAMC_ADAM_MAX_TENSORS];
};
struct AdamPtrs {
  float* p[DAMC_ADAM_MAX_TENSORS];
  float* g[DAMC_ADAM_MAX_TENSORS];
  float* m[DAMC_ADAM_MAX_TENSORS];
  float* v[DAMC_ADAM_MAX_TENSORS];
};
static_assert(sizeof(AdamPtrs) + sizeof(damc_adam_hparams_t) + 64 <= 4096, "kernel argument block");

constexpr int kThreads = 256;

__device__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

__device__ __forceinline__ float lerp_torch(float self, float end, float w) {
  // ATen's lerp (ATen/native/Lerp.h): two forms split at |w| < 0.5
  return (fabsf(w) < 0.5f) ? fmaf(w, end - self, self) : fmaf(-(end - self), 1.0f - w, end);
}

__device__ __forceinline__ void adam_elem(float& p, float& g, float& m, float& v, const damc_adam_hparams_t& h,
                                          float coef, bool clip) {
#pragma clang fp contract(off)
  if (clip) g = g * coef;
  float gg = g;
  if (!h.decoupled && h.weight_decay != 0.f) gg = fmaf(h.weight_decay, p, g);
  if (h.decoupled) p = p * h.decay_mul;
  m = lerp_torch(m, gg, h.one_minus_beta1);
  v = v * h.beta2;
  v = fmaf(h.one_minus_beta2 * gg, gg, v);
  float s = sqrtf(v);
  s = s / h.bc2_sqrt;
  s = s + h.eps;
  p = fmaf(h.neg_step_size, m / s, p);
}

template <bool CLIP>
__global__ __launch_bounds__(kThreads) void adam_kernel(const AdamChunk* __restrict__ chunks, AdamPtrs t,
                                                        damc_adam_hparams_t h, const float* __restrict__ clip) {
  const AdamChunk c = chunks[blockIdx.x];
  float* P = t.p[c.tensor] + c.off;
  float* G = t.g[c.tensor] + c.off;
  float* M = t.m[c.tensor] + c.off;
  float* V = t.v[c.tensor] + c.off;
  const float coef = CLIP ? clip[1] : 1.f;
  int i0 = 0;
  if (al16(P) && al16(G) && al16(M) && al16(V)) {
    const int n4 = c.n >> 2;
    for (int i = threadIdx.x; i < n4; i += kThreads) {
      f32x4 p = reinterpret_cast<const f32x4*>(P)[i];
      f32x4 g = reinterpret_cast<const f32x4*>(G)[i];
      f32x4 m = reinterpret_cast<const f32x4*>(M)[i];
      f32x4 v = reinterpret_cast<const f32x4*>(V)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = p[e], ge = g[e], me = m[e], ve = v[e];
        adam_elem(pe, ge, me, ve, h, coef, CLIP);
        p[e] = pe;
        g[e] = ge;
        m[e] = me;
        v[e] = ve;
      }
      reinterpret_cast<f32x4*>(P)[i] = p;
      reinterpret_cast<f32x4*>(M)[i] = m;
      reinterpret_cast<f32x4*>(V)[i] = v;
      if (CLIP) reinterpret_cast<f32x4*>(G)[i] = g;
    }
    i0 = n4 << 2;
  }
  for (int i = i0 + threadIdx.x; i < c.n; i += kThreads) {
    float p = P[i], g = G[i], m = M[i], v = V[i];
    adam_elem(p, g, m, v, h, coef, CLIP);
    P[i] = p;
    M[i] = m;
    V[i] = v;
    if (CLIP) G[i] = g;
  }
}

// fixed-order block sum of 256 per-thread values (wave butterflies in a fixed pattern, then 4 waves)
__device__ __forceinline__ float block_sum(float x, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(kThreads) void grad_sumsq_kernel(const AdamChunk* __restrict__ chunks, GradPtrs t,
                                                              float* __restrict__ partial) {
  __shared__ float red[4];
  const AdamChunk c = chunks[blockIdx.x];
  const float* G = t.g[c.tensor] + c.off;
  float acc = 0.f;
  int i0 = 0;
  if (al16(G)) {
    const int n4 = c.n >> 2;
    for (int i = threadIdx.x; i < n4; i += kThreads) {
      const f32x4 g = reinterpret_cast<const f32x4*>(G)[i];
      acc = fmaf(g[0], g[0], acc);
      acc = fmaf(g[1], g[1], acc);
      acc = fmaf(g[2], g[2], acc);
      acc = fmaf(g[3], g[3], acc);
    }
    i0 = n4 << 2;
  }
  for (int i = i0 + threadIdx.x; i < c.n; i += kThreads) acc = fmaf(G[i], G[i], acc);
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void grad_norm_finish_kernel(const float* __restrict__ partial, int n,
                                                                    float max_norm, float* __restrict__ out) {
  __shared__ double red[kThreads];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += kThreads) acc += (double)partial[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
#pragma clang fp contract(off)
    const float norm = (float)sqrt(red[0]);
    const float coef = max_norm / (norm + 1e-6f);  // clip_grad.py: max_norm / (total_norm + 1e-6), fp32
    out[0] = norm;
    // torch.clamp(coef, max=1.0) propagates a NaN (non-finite total norm); fminf would return 1 instead
    out[1] = (coef != coef) ? coef : fminf(coef, 1.0f);
  }
}

__global__ __launch_bounds__(kThreads) void grad_scale_kernel(const AdamChunk* __restrict__ chunks, GradPtrs t,
                                                              const float* __restrict__ clip) {
  const AdamChunk c = chunks[blockIdx.x];
  float* G = t.g[c.tensor] + c.off;
  const float coef = clip[1];
  int i0 = 0;
  if (al16(G)) {
    const int n4 = c.n >> 2;
    for (int i = threadIdx.x; i < n4; i += kThreads) {
      f32x4 g = reinterpret_cast<const f32x4*>(G)[i];
      g *= coef;
      reinterpret_cast<f32x4*>(G)[i] = g;
    }
    i0 = n4 << 2;
  }
  for (int i = i0 + threadIdx.x; i < c.n; i += kThreads) G[i] = G[i] * coef;
}

bool fill(float* const* src, int n, float** dst) {
  if (!src || n < 0 || n > DAMC_ADAM_MAX_TENSORS) return false;
  for (int i = 0; i < n; ++i) {
    if (!src[i]) return false;
    dst[i] = src[i];
  }
  for (int i = n; i < DAMC_ADAM_MAX_TENSORS; ++i) dst[i] = nullptr;
  return true;
}

}  // namespace

extern "C" {

size_t damc_adam_chunk_bytes(void) { return sizeof(AdamChunk); }

int damc_adam_chunk_count(const long long* numel, int n) {
  if (!numel || n < 0 || n > DAMC_ADAM_MAX_TENSORS) return -DAMC_ERR_ARG;
  long long c = 0;
  for (int i = 0; i < n; ++i) {
    if (numel[i] < 0) return -DAMC_ERR_ARG;
    c += (numel[i] + DAMC_ADAM_CHUNK - 1) / DAMC_ADAM_CHUNK;
  }
  return c > 0x7fffffffLL ? -DAMC_ERR_ARG : (int)c;
}

int damc_adam_build_chunks(const long long* numel, int n, void* host_chunks, int max_chunks) {
  const int need = damc_adam_chunk_count(numel, n);
  if (need < 0) return need;
  if (!host_chunks || need > max_chunks) return -DAMC_ERR_WORKSPACE;
  AdamChunk* out = static_cast<AdamChunk*>(host_chunks);
  int k = 0;
  for (int i = 0; i < n; ++i)
    for (long long s = 0; s < numel[i]; s += DAMC_ADAM_CHUNK) {
      AdamChunk c;
      c.off = s;
      c.tensor = i;
      c.n = (int)((numel[i] - s) < DAMC_ADAM_CHUNK ? (numel[i] - s) : DAMC_ADAM_CHUNK);
      out[k++] = c;
    }
  return k;
}

int damc_grad_norm(const void* dev_chunks, int nchunks, float* const* grads, int ntensors, float max_norm,
                   float* workspace, float* out, void* stream) {
  GradPtrs t;
  DAMC_REQUIRE(dev_chunks && workspace && out && nchunks >= 0 && fill(grads, ntensors, t.g));
  hipStream_t s = as_stream(stream);
  if (nchunks > 0) {
    grad_sumsq_kernel<<<nchunks, kThreads, 0, s>>>(static_cast<const AdamChunk*>(dev_chunks), t, workspace);
    DAMC_LAUNCH_CHECK();
  }
  grad_norm_finish_kernel<<<1, kThreads, 0, s>>>(workspace, nchunks, max_norm, out);
  DAMC_LAUNCH_CHECK();
  return 0;
}

int damc_grad_sumsq(const void* dev_chunks, int nchunks, float* const* grads, int ntensors, float* partial,
                    void* stream) {
  GradPtrs t;
  DAMC_REQUIRE(dev_chunks && partial && nchunks >= 0 && fill(grads, ntensors, t.g));
  if (nchunks == 0) return 0;
  grad_sumsq_kernel<<<nchunks, kThreads, 0, as_stream(stream)>>>(static_cast<const AdamChunk*>(dev_chunks), t,
                                                                  partial);
  DAMC_LAUNCH_CHECK();
  return 0;
}

int damc_grad_norm_finish(const float* partial, int n, float max_norm, float* out, void* stream) {
  DAMC_REQUIRE(out && n >= 0 && (partial || n == 0));
  grad_norm_finish_kernel<<<1, kThreads, 0, as_stream(stream)>>>(partial, n, max_norm, out);
  DAMC_LAUNCH_CHECK();
  return 0;
}

int damc_grad_scale(const void* dev_chunks, int nchunks, float* const* grads, int ntensors, const float* clip,
                    void* stream) {
  GradPtrs t;
  DAMC_REQUIRE(dev_chunks && clip && nchunks >= 0 && fill(grads, ntensors, t.g));
  if (nchunks == 0) return 0;
  grad_scale_kernel<<<nchunks, kThreads, 0, as_stream(stream)>>>(static_cast<const AdamChunk*>(dev_chunks), t,
                                                                  clip);
  DAMC_LAUNCH_CHECK();
  return 0;
}

int damc_adam_step(const void* dev_chunks, int nchunks, float* const* params, float* const* grads,
                   float* const* exp_avgs, float* const* exp_avg_sqs, int ntensors, const damc_adam_hparams_t* hp,
                   const float* clip, void* stream) {
  AdamPtrs t;
  DAMC_REQUIRE(dev_chunks && hp && nchunks >= 0 && fill(params, ntensors, t.p) && fill(grads, ntensors, t.g) &&
               fill(exp_avgs, ntensors, t.m) && fill(exp_avg_sqs, ntensors, t.v));
  if (nchunks == 0) return 0;
  const AdamChunk* ch = static_cast<const AdamChunk*>(dev_chunks);
  if (clip)
    adam_kernel<true><<<nchunks, kThreads, 0, as_stream(stream)>>>(ch, t, *hp, clip);
  else
    adam_kernel<false><<<nchunks, kThreads, 0, as_stream(stream)>>>(ch, t, *hp, nullptr);
  DAMC_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
