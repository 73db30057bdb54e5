/*
 * damc.h — C ABI of libdamc.so, the MI355X (gfx950) diffusion-amortized Langevin inner loop.
 *
 * The reference (yuPeiyu98/Diffusion-Amortized-MCMC) has no native/FFI layer: its hot path is
 * the Python call surface of workspace/src/MCMC.py and workspace/src/diffusion_net.py.  Each
 * entry point below replaces the device work behind one of those Python functions; the
 * Python mirror (diffusion-amortized-mcmc_amd/damc, bound with ctypes)
 * keeps the reference's names and signatures.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer to caller-owned fp32 memory unless noted;
 *   - images are NCHW exactly as the caller holds them; latents z are (B, nz) row-major;
 *   - weights are passed once per call to damc_pack_* in PyTorch layouts and re-laid out
 *     into caller-allocated packed buffers (no allocation inside the library);
 *   - `stream` is a hipStream_t passed as void*; no host synchronisation happens inside
 *     any call (everything is stream-ordered and graph-capturable);
 *   - return 0 on success, otherwise a hipError_t value or one of DAMC_ERR_* (the Python
 *     side raises RuntimeError with damc_error_string()).
 *   - step sizes / sigma are the reference's Python floats (double): the updates use float32(0.5 step^2) and
 *     float32(step) (and float32(1 / sigma^2)), the values PyTorch's fp32 scalar ops round them to;
 *   - noise: with_noise != 0 and noise == NULL draws xi ~ N(0,1) in-kernel from
 *     Philox4x32-10 keyed by (seed) with counter (dim/4, step + step_offset,
 *     chain_base + chain, stream_id): a chain's noise depends on its GLOBAL index only, so
 *     results are identical for any sharding of the batch over GPUs.  noise != NULL
 *     injects (n_steps, B, nz) values instead (parity tests).
 */
#ifndef DAMC_H
#define DAMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DAMC_ABI_VERSION 3
#define DAMC_MAX_LAYERS 10

enum {
  DAMC_OK = 0,
  DAMC_ERR_ARG = 1001,       /* invalid shape / argument */
  DAMC_ERR_WORKSPACE = 1002, /* workspace too small */
  DAMC_ERR_UNSUPPORTED = 1003
};

/* Generator layer kinds (workspace/src/diffusion_net.py:20-203, toy_example.py:22-47) */
enum {
  DAMC_LAYER_PROJ = 1,   /* ConvTranspose2d on a 1x1 input (first layer): a GEMM z·W        */
  DAMC_LAYER_UP2 = 2,    /* ConvTranspose2d k4 s2 p1 with Cout >= 8: phase-split implicit GEMM */
  DAMC_LAYER_SMALLC = 3, /* last ConvTranspose2d with Cout <= 4 (to RGB / gray)             */
  DAMC_LAYER_LINEAR = 4  /* nn.Linear (toy MLP generator)                                  */
};
enum { DAMC_ACT_NONE = 0, DAMC_ACT_LRELU = 1, DAMC_ACT_TANH = 2, DAMC_ACT_SILU = 3 };
/* Convolution engine of a generator layer (every layer of one generator must name the same one):
 *   DAMC_ENGINE_LIMB: layers whose gathered channel count is a multiple of 32 run on the limb engine —
 *     fp32 operands split into 3 bf16 limbs, 6 limb products per fp32 product on bf16 MFMA, fp32
 *     accumulation (error vs fp64 equal to fp32 MFMA's); the other layers on the fp32 MFMA engine;
 *   DAMC_ENGINE_FP32: every convolution on the fp32 MFMA engine (v_mfma_f32_32x32x2_f32).
 * Packed weights and workspaces are sized for either engine. */
enum { DAMC_ENGINE_LIMB = 0, DAMC_ENGINE_FP32 = 1 };

typedef struct {
  int kind;
  int cin, cout, k, stride, pad;
  int hin, win, hout, wout;  /* spatial sizes (1 for PROJ input / LINEAR)                 */
  int act;                   /* activation after this layer                               */
  float slope;               /* LeakyReLU slope (ReLU = 0)                                */
  const float* w_fwd;        /* packed forward weights  (damc_pack_generator_layer)       */
  const float* w_bwd;        /* packed dgrad weights                                      */
  const float* bias;         /* (cout) or NULL                                            */
  int engine;                /* DAMC_ENGINE_* (0 = limb engine, the default)              */
} damc_layer_t;

typedef struct {
  int n_layers;
  int nz;                     /* latent size                                               */
  int nc, h, w;               /* image shape (for LINEAR generators: nc = out features, h = w = 1) */
  damc_layer_t layers[DAMC_MAX_LAYERS];
} damc_generator_t;

/* Latent EBM _netE: Linear(nz,nh) LReLU Linear(nh,nh) LReLU Linear(nh,1) (diffusion_net.py:207-223) */
typedef struct {
  int nz, nh;
  float slope;
  const float *w1, *b1, *w2, *b2, *w3, *b3;  /* PyTorch layouts: w1 (nh,nz), w2 (nh,nh), w3 (1,nh) */
  const float *w1t, *w2t;                     /* packed transposes (damc_pack_ebm)                  */
} damc_ebm_t;

/* ---------------------------------------------------------------- library / packing */
int damc_abi_version(void);
const char* damc_error_string(int code);

/* floats needed by the packed forward / dgrad buffers of one generator layer */
int damc_generator_layer_packed_sizes(const damc_layer_t* layer, size_t* fwd_floats, size_t* bwd_floats);
/* re-lay PyTorch weight (ConvT: (Cin,Cout,k,k); Linear: (out,in)) into layer->w_fwd / w_bwd */
int damc_pack_generator_layer(const damc_layer_t* layer, const float* w_torch, float* w_fwd, float* w_bwd,
                              void* stream);
/* w1t (nz,nh) and w2t (nh,nh) from the PyTorch w1/w2 */
int damc_pack_ebm(const damc_ebm_t* ebm, float* w1t, float* w2t, void* stream);

/* ------------------------------------------------------------- posterior Langevin (a1) */
/* workspace bytes for damc_posterior_langevin / damc_likelihood_grad / damc_generator_forward */
size_t damc_posterior_workspace_bytes(const damc_generator_t* g, int batch);

/* sample_langevin_post_z_with_prior (workspace/src/MCMC.py:48-74):
 *   for i < n_steps:  z <- z - 0.5*step^2 * grad U(z) (+ step*xi),
 *   U = |G(z)-x|^2/(2 sigma^2) + sum E(z) + |z|^2/2     (E omitted when ebm == NULL)
 * z (B,nz) updated in place; x (B,nc,h,w) NCHW; diag (optional, n_steps*4 floats, zeroed by
 * the call): per step {sum E, |G(z)-x|^2/(2sigma^2), |z|^2/2, mean(grad)} before the update. */
int damc_posterior_langevin(const damc_generator_t* g, const damc_ebm_t* ebm, float* z, const float* x,
                            int batch, int n_steps, double sigma, double step, int with_noise,
                            const float* noise, uint64_t seed, uint64_t step_offset, uint64_t chain_base,
                            float* diag, void* workspace, size_t workspace_bytes, void* stream);

/* per-op hooks (parity tests): grad_z |G(z)-x|^2/(2 sigma^2) -> grad (B,nz) */
int damc_likelihood_grad(const damc_generator_t* g, const float* z, const float* x, int batch, double sigma,
                         float* grad, void* workspace, size_t workspace_bytes, void* stream);
/* x_hat = G(z) (B,nc,h,w) NCHW — gen_samples / gen_samples_with_diffusion_prior (MCMC.py:119-150) */
int damc_generator_forward(const damc_generator_t* g, const float* z, int batch, float* x_hat,
                           void* workspace, size_t workspace_bytes, void* stream);

/* per-op hooks for ONE k4 s2 p1 ConvTranspose2d (DAMC_LAYER_UP2) layer of a generator, NHWC
 * activations, the same kernels and engine choice as inside damc_posterior_langevin:
 *   damc_convT_fwd:   out (B, hout, wout, cout) = act(conv_transpose2d(in (B, hin, win, cin), W) + bias)
 *   damc_convT_dgrad: gin (B, hin, win, cin) = conv_transpose2d^T(gout (B, hout, wout, cout), W), multiplied by
 *                     act'(mask_pre) when mask_pre != NULL (the previous layer's activated output, act = mask_act)
 * layer: packed by damc_pack_generator_layer; workspace: damc_convT_workspace_bytes (limb copy of the input). */
size_t damc_convT_workspace_bytes(const damc_layer_t* layer, int batch);
int damc_convT_fwd(const damc_layer_t* layer, const float* in, int batch, float* out, void* workspace,
                   size_t workspace_bytes, void* stream);
int damc_convT_dgrad(const damc_layer_t* layer, const float* gout, int batch, const float* mask_pre, int mask_act,
                     float mask_slope, float* gin, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------- generator training step */
/* The G update of a training iteration (workspace/train_gen_recon.py:222-231):
 *   x_hat = G(z); g_loss = sum((x_hat - x)^2, [1,2,3]).mean(); g_loss.backward()
 * damc_generator_train_forward computes x_hat (NCHW) and keeps in the workspace what the backward reads;
 * damc_generator_train_backward then maps grad_xhat = dL/dx_hat (NCHW, from the caller's autograd) to the
 * weight and bias gradients of every layer (PyTorch layouts: ConvTranspose2d (Cin, Cout, k, k), Linear
 * (out, in); WRITTEN, not accumulated; NULL entries are skipped) and, if grad_z != NULL, dL/dz (B, nz).
 * The two calls must use the same descriptor, batch and workspace, with no other call on that workspace in
 * between: train_forward records (workspace, batch, engine) and train_backward returns DAMC_ERR_ARG for a
 * descriptor or batch that disagrees.  ConvT weight gradients run on the limb engine (fp32-accurate bf16
 * MFMA) whatever the layers' engine; layer inputs and gradients with a batch that is not a multiple of 32
 * are zero-padded to one. */
typedef struct {
  float* w[DAMC_MAX_LAYERS];
  float* b[DAMC_MAX_LAYERS];
} damc_generator_grads_t;
size_t damc_generator_train_workspace_bytes(const damc_generator_t* g, int batch);
int damc_generator_train_forward(const damc_generator_t* g, const float* z, int batch, float* x_hat, void* workspace,
                                 size_t workspace_bytes, void* stream);
int damc_generator_train_backward(const damc_generator_t* g, const float* z, const float* x_hat,
                                  const float* grad_xhat, int batch, const damc_generator_grads_t* grads,
                                  float* grad_z, void* workspace, size_t workspace_bytes, void* stream);

/* ----------------------------------------------------------------- prior Langevin (a2) */
/* sample_langevin_prior_z (MCMC.py:27-46): all n_steps in ONE persistent launch.
 * diag (optional, n_steps*2 floats): {sum E, |z|^2/2} per step before the update. */
int damc_prior_langevin(const damc_ebm_t* ebm, float* z, int batch, int n_steps, double step, int with_noise,
                        const float* noise, uint64_t seed, uint64_t step_offset, uint64_t chain_base,
                        float* diag, void* stream);
/* the same with the engine chosen per call: 0 = by batch size (the default above: the 16-chain MFMA tile kernel
 * from DAMC_EBM_MFMA_MIN_B = 2048 chains up, where the FC layers are real GEMMs), 1 = register-resident VALU
 * (one chain per workgroup), 2 = MFMA (nz % 16 == 0, nz and nh <= 256, else DAMC_ERR_UNSUPPORTED).
 * Engine 0 is keyed on THIS call's batch.  The two engines sum in different orders, so a sharded caller that needs
 * its shards' union bitwise equal to the unsharded block resolves the engine itself from the global chain count
 * (>= damc_ebm_mfma_min_chains() -> 2, else 1) and passes 1 or 2, as damc.langevin does. */
/* the threshold engine 0 uses: DAMC_EBM_MFMA_MIN_B, read once per process (default 2048) */
int damc_ebm_mfma_min_chains(void);
int damc_prior_langevin_engine(const damc_ebm_t* ebm, float* z, int batch, int n_steps, double step, int with_noise,
                               const float* noise, uint64_t seed, uint64_t step_offset, uint64_t chain_base,
                               float* diag, int engine, void* stream);
/* per-op hook: energy (B) and grad_z sum E (B,nz) */
int damc_ebm_energy_grad(const damc_ebm_t* ebm, const float* z, int batch, float* energy, float* grad,
                         void* stream);
/* the same under SURVEY.md §8b's name */
int damc_ebm_grad(const damc_ebm_t* ebm, const float* z, int batch, float* energy, float* grad, void* stream);
/* per-op hook: z <- z - 0.5 step^2 (g + z) (+ step xi) ; g (B,nz) */
int damc_z_update(float* z, const float* g, int batch, int nz, double step, int with_noise, const float* noise,
                  uint64_t seed, uint64_t step_index, uint64_t chain_base, void* stream);
/* Philox N(0,1) draw used by every Langevin kernel (statistical tests) -> out (n_steps,B,nz) */
int damc_philox_normal(float* out, int n_steps, int batch, int nz, uint64_t seed, uint64_t step_offset,
                       uint64_t chain_base, uint32_t stream_id, void* stream);

/* ---------------------------------------------------------------- Q amortizer (a8-a11) */
/* generic fp32 MFMA implicit-GEMM conv (NHWC) + bias: encoder building block.  workspace (floats, may be
 * NULL / 0): split-K slabs for convolutions whose output tiles would not fill the chip, sized by
 * damc_conv2d_workspace_floats (0 = no split for that shape) */
size_t damc_conv2d_workspace_floats(int batch, int hin, int win, int cin, int cout, int k, int stride, int pad);
int damc_conv2d_nhwc(const float* x, int batch, int hin, int win, int cin, const float* w_packed, const float* bias,
                     int cout, int k, int stride, int pad, float* y, float* workspace, size_t workspace_floats,
                     void* stream);
/* pack Conv2d weight (Cout,Cin,k,k) into the engine's layout (same element count; opaque to callers):
 * (Cout, k,k,Cin) for the K-major engine when Cin % 32 == 0, else (k,k,Cin,Cout) */
int damc_pack_conv2d(const float* w_torch, int cout, int cin, int k, float* w_packed, void* stream);
/* InstanceNorm2d(affine, eps) + LeakyReLU(slope), in place on NHWC (Welford partials merged with
 * Chan's formula); workspace: damc_instnorm_workspace_floats() floats */
size_t damc_instnorm_workspace_floats(int batch, int hw, int c);
int damc_instnorm_lrelu_nhwc(float* y, int batch, int hw, int c, const float* gamma, const float* beta, float eps,
                             float slope, float* workspace, void* stream);
/* Encoder training (the Q update's encoder backward; Encoder_* diffusion_net.py:227-413):
 * InstanceNorm2d(affine) + LeakyReLU keeping the conv output y: h = lrelu(IN(y)) into its own buffer and
 * stats (B, c, 2) = {mean, rstd}; workspace as damc_instnorm_workspace_floats */
int damc_instnorm_lrelu_train_nhwc(const float* y, int batch, int hw, int c, const float* gamma, const float* beta,
                                   float eps, float slope, float* h, float* stats, float* workspace, void* stream);
size_t damc_instnorm_bwd_workspace_floats(int batch, int hw, int c);
/* dh (grad of h) -> dy (grad of the conv output y), dgamma, dbeta (c) (either may be NULL) */
int damc_instnorm_lrelu_backward_nhwc(const float* y, const float* stats, const float* dh, int batch, int hw, int c,
                                      const float* gamma, const float* beta, float slope, float* dy, float* dgamma,
                                      float* dbeta, float* workspace, void* stream);
/* Conv2d backward on NHWC activations, weight in PyTorch (Cout, Cin, k, k): dx (NHWC, may be NULL), dw, db (may
 * be NULL).  Supported: k4 s2 p1 with H = 2 Ho (limb engine), the first k3 s1 p1 conv with Cin <= 4 (no dx), and
 * a last conv covering its whole input (p0, 1x1 output).  workspace bytes: 0 = shape not supported. */
size_t damc_conv2d_backward_workspace_bytes(int batch, int hin, int win, int cin, int cout, int k, int stride,
                                            int pad);
int damc_conv2d_backward_nhwc(const float* x, const float* dy, const float* w, int batch, int hin, int win, int cin,
                              int cout, int k, int stride, int pad, float* dx, float* dw, float* db, void* workspace,
                              size_t workspace_bytes, void* stream);

/* NCHW -> NHWC transpose (encoder input) */
int damc_nchw_to_nhwc(const float* x, int batch, int c, int hw, float* y, void* stream);

/* The whole Encoder_* forward of _netQ_U (SURVEY.md §8b damc_q_encoder_fwd; diffusion_net.py:227-372, a10):
 * [Conv2d -> InstanceNorm2d(affine) -> LeakyReLU]* -> Conv2d on the kernels above, x (B, nc, h, w) NCHW ->
 * xemb (B, nemb) with nemb = cout * ho * wo of the last conv (1 x 1 in every Encoder_*, where the NHWC and
 * the reference's NCHW flattening agree; other output sizes return DAMC_ERR_UNSUPPORTED).
 * engine DAMC_ENGINE_LIMB: the convolutions whose input channel count is a multiple of 32 (every one but the
 * first 3x3 at the reference's nif) run on the limb engine (fp32-accurate, bf16 MFMA; see DAMC_ENGINE_*), the
 * input activation split into limbs per call; w_x3 = damc_pack_conv2d_x3 of the layer's weight (then w_packed
 * may be NULL for that layer), or w_src = the weight itself (packed by the library per call, see below), or neither
 * (the library splits w_packed into the workspace per call). */
#define DAMC_MAX_ENC_LAYERS 8
typedef struct {
  int cin, cout, k, stride, pad;
  const float* w_packed;          /* damc_pack_conv2d layout (NULL allowed for a limb layer with w_x3) */
  const float* bias;              /* (cout) or NULL                                                   */
  const float *in_gamma, *in_beta; /* InstanceNorm2d affine (cout); NULL: no norm / activation after it */
  float in_eps, slope;
  const void* w_x3;               /* the limb B operand (damc_pack_conv2d_x3) or NULL                 */
  const float* w_src;             /* or the PyTorch Conv2d weight (cout, cin, k, k) of a limb layer, 16-B aligned:
                                     the library packs every such layer into the workspace per call, as extra
                                     workgroups of the first layer's launch (w_x3 and w_packed then unused)   */
} damc_enc_layer_t;
typedef struct {
  int n_layers, nc, h, w;
  damc_enc_layer_t layers[DAMC_MAX_ENC_LAYERS];
  int engine; /* DAMC_ENGINE_* */
} damc_encoder_t;
/* bytes of the limb copy of a packed conv weight (0: the layer does not run on the limb engine) */
size_t damc_conv2d_x3_bytes(int cout, int cin, int k);
/* k per sign block of the limb engine's weight operands (odd blocks stored negated; = its MFMA accumulation block
 * and its split-K granule) for the encoder's convs (damc_pack_conv2d_x3): the build's DAMC_X3_NEGK, 512 by default */
int damc_x3_sign_block(void);
/* 1 when a k x k Conv2d on cin channels has its limb weight operand (damc_pack_conv2d_x3) and its encoder GEMMs in the
 * 4 x 4 conv walk (k = 4, cin % 32 == 0: K index = (ci / 32) 512 + p 32 + ci % 32 with p the parity-grouped position of
 * tap (ky, kx): ((ky % 2) 2 + kx % 2) 4 + (ky / 2) 2 + kx / 2; sign blocks counted in that order), 0 when tap-major
 * [(ky, kx, ci)]; opt-in: DAMC_ENC_WALK=1 (read per call) selects the walk, tap-major otherwise */
int damc_x3_conv_walk(int k, int cin);
/* the sign block of a generator UP2 layer's limb weights (damc_pack_generator_layer), forward (input_grad = 0,
 * K = 4 Cin) or input gradient (1, K = 16 Cout): 512 or 1024 by the layer's shape alone (gemm.h x3_conv_negk);
 * 0 for a layer without limb weights */
int damc_x3_layer_sign_block(const damc_layer_t* L, int input_grad);
/* diagnostics: while buf (n_slots * 4 uint64, device memory) is set, every k4 s2 ConvT forward on the limb engine
 * stores, per workgroup w at buf[4 (w % n_slots)], {s_memtime, s_memrealtime} before and after its K loop: the
 * clock the chip holds in that loop is d(memtime) / d(realtime) x 100 MHz.  buf = NULL switches it off.  Not
 * thread-safe; keep it off in timed work (bench.py runs it on one extra block). */
int damc_clock_probe(unsigned long long* buf, int n_slots);
/* diagnostics: while buf (8 uint32, device memory, zeroed by the caller) is set, every split-K launch with the in-GEMM
 * fix-up (gemm.hip X3_FIXUP) adds to it: [0] workgroups, [1] waits that ran out, [2] bands the last arrivers took over,
 * [3] the longest wait (s_memrealtime ticks, 100 MHz), [4] the waits' total ticks, [5] last arrivers.  NULL: off */
int damc_x3_fixup_probe(unsigned* buf);
/* a Conv2d weight in its PyTorch layout (cout, cin, k, k), cin % 32 == 0 -> the limb engine's B operand of the
 * conv (damc_conv2d_x3_bytes bytes), in one pass */
int damc_pack_conv2d_x3(const float* w, int cout, int cin, int k, void* w_x3, void* stream);
/* one Conv2d (+ bias) on the limb engine, NHWC fp32 in and out (the Q update's encoder forward, which keeps every conv
 * output for its backward): w_x3 = damc_pack_conv2d_x3 of the weight; k4 s2 p1 convs stage x as fp32, other shapes
 * split it into limbs in the workspace (damc_conv2d_x3_workspace_bytes; 0 = the shape has no limb-engine form) */
size_t damc_conv2d_x3_workspace_bytes(int batch, int hin, int win, int cin, int cout, int k, int stride, int pad);
int damc_conv2d_x3_nhwc(const float* x, int batch, int hin, int win, int cin, const void* w_x3, const float* bias,
                        int cout, int k, int stride, int pad, float* y, void* workspace, size_t workspace_bytes,
                        void* stream);
size_t damc_q_encoder_workspace_bytes(const damc_encoder_t* enc, int batch);
int damc_q_encoder_fwd(const damc_encoder_t* enc, const float* x, int batch, float* xemb, void* workspace,
                       size_t workspace_bytes, void* stream);

/* The encoder of the Q update in two calls (round 5; Encoder_* forward and backward inside Q.calculate_loss,
 * diffusion_net.py:624-645, train_gen_recon.py:211-220): every layer's w_src = its PyTorch Conv2d weight, bias set,
 * in_gamma / in_beta on every layer but the last, whose output is 1 x 1 (xemb (B, cout)); engine as for
 * damc_q_encoder_fwd.  The forward keeps in `saved` (damc_encoder_train_saved_floats floats) the NHWC input, every
 * conv output, InstanceNorm statistics and activation; the backward maps grad_xemb (B, nemb) to the gradients
 * (written, not accumulated; NULL entries skipped).  One workspace size serves both calls; 0 = not supported. */
typedef struct {
  float *w[DAMC_MAX_ENC_LAYERS], *b[DAMC_MAX_ENC_LAYERS], *gamma[DAMC_MAX_ENC_LAYERS], *beta[DAMC_MAX_ENC_LAYERS];
} damc_encoder_grads_t;
size_t damc_encoder_train_saved_floats(const damc_encoder_t* enc, int batch);
size_t damc_encoder_train_workspace_bytes(const damc_encoder_t* enc, int batch);
int damc_encoder_train_forward(const damc_encoder_t* enc, const float* x, int batch, float* saved, float* xemb,
                               void* workspace, size_t workspace_bytes, void* stream);
int damc_encoder_train_backward(const damc_encoder_t* enc, const float* saved, const float* grad_xemb, int batch,
                                const damc_encoder_grads_t* grads, void* workspace, size_t workspace_bytes,
                                void* stream);

/* Dense fp32 MFMA GEMM: C(M,N) = act(A(M,K) · B(K,N) + bias) with B row-major (K,N) */
int damc_gemm(const float* a, int lda, const float* b, int ldb, const float* bias, float* c, int ldc, int m,
              int n, int k, int act, float slope, void* stream);

/* Denoiser Diffusion_UnetA (diffusion_net.py:417-533) and its reverse sweep (diffusion_net.py:595-622).
 * Seven ConcatSquashLinearSkipCtx blocks (in0 in1 in2 mid0 out0 out1 out2).  Every weight is the caller's
 * PyTorch tensor in its own layout (nn.Linear (out, in)); the library re-lays them out into its workspace per
 * call (the nets train between calls), so the caller does no per-call packing. */
typedef struct {
  int din, dout;
  /* PyTorch nn.Linear layout (out, in), k contiguous */
  const float *wl, *bl; /* _layer.0     (dout, din), (dout)  */
  const float *ws, *bs; /* _skip        (dout, din), (dout)  */
  const float *wg, *bg; /* _hyper_gate  (dout, dout), (dout) */
  const float* wb;      /* _hyper_bias  (dout, dout), no bias */
} damc_csq_block_t;

typedef struct {
  int nz, ntemb, nxemb, residual;
  const float* bmat;                  /* p.B (nz, nz/2)                                  */
  const float *tw1, *tb1, *tw2, *tb2; /* time_mlp[1], time_mlp[3]: (out, in), (out)      */
  damc_csq_block_t blocks[7];         /* in0 in1 in2 mid0 out0 out1 out2                 */
  const float* wctx[7];               /* _layer_ctx[1].weight (dout, ntemb + nxemb)       */
  const float* bctx[7];               /* _layer_ctx[1].bias (dout)                       */
} damc_denoiser_t;

/* workspace bytes for damc_reverse_sweep */
size_t damc_sweep_workspace_bytes(const damc_denoiser_t* d, int batch, int n_steps);
/* The reverse sweep (n_steps = n_interval denoiser evaluations, i = n_steps-1 .. 0, k = n_steps-1-i).
 * Per call the library packs the weights, then evaluates everything that does not depend on zt for all
 * steps at once: the time MLP (batch-invariant), the ctx Linear's xemb part (step-invariant), and for every
 * (step, row) a block's ctx c = SiLU(Lc(SiLU(cat(temb, xemb)))), its gate sigmoid(c Wg^T + bg) and hyper
 * bias c Wb^T (limb-product MFMA GEMMs over n*B rows).  The dependent chain — per step the 7 blocks'
 * x Wl^T / x Ws^T products plus the reverse-step update — then runs as ONE team launch (weights LDS-resident,
 * data-driven hand-offs between the workgroups of a team; at the reference's widths, nf = 4 with nz 128 or 100, a
 * kernel with those shapes compiled in, DAMC_SWEEP_FAST=0 the generic one, bitwise the same); DAMC_SWEEP_TEAM=0
 * runs it as 7 launches per step replayed from a HIP graph cached per (workspace, shapes, schedule).
 *   eps = p(zt, l_t, xemb); pred = c0 * (zt - eps * c1); zt <- last ? pred : c2*zt + c3*pred (+ c4*xi)
 * temb_in (n_steps, ntemb): SinusoidalPosEmb of the step's logsnr input (host, fp32, as the reference);
 * coef (n_steps, 6), a HOST pointer: {sqrt(1+e^-lt), rsqrt(1+e^lt), r*alpha_st, (1-r)*alpha_s, std,
 * is_last} (diffusion_helper_func.py:36-70, evaluated on the host in fp32 like the reference; the
 * scalars travel by value in each step's kernel arguments);
 * noise (n_steps-1, B, nz) injected or NULL for Philox; eps_log (optional) receives eps of the
 * first eps_log_steps steps. zt (B, nz) is updated in place; xemb (B, nxemb). */
int damc_reverse_sweep(const damc_denoiser_t* d, const float* xemb, float* zt, int batch, int n_steps,
                       const float* temb_in, const float* coef, int with_noise, const float* noise, uint64_t seed,
                       uint64_t chain_base, float* eps_log, int eps_log_steps, void* workspace,
                       size_t workspace_bytes, void* stream);
/* the same under SURVEY.md §8b's name */
int damc_q_reverse_sweep(const damc_denoiser_t* d, const float* xemb, float* zt, int batch, int n_steps,
                         const float* temb_in, const float* coef, int with_noise, const float* noise, uint64_t seed,
                         uint64_t chain_base, float* eps_log, int eps_log_steps, void* workspace,
                         size_t workspace_bytes, void* stream);
/* The team reverse sweep (default) needs all its workgroups resident at once.  If a member never starts (another
 * process or stream holding CUs), its bounded waits give up and the library recomputes the affected sweep on the
 * device (bitwise the team's arithmetic; never NaN), flags the device, and runs later sweeps on the launch chain.
 * damc_sweep_team_failures: how many such rescued launches this process has seen on a device (a rescue still in
 * flight is counted once it completes).  damc_sweep_team_words (tools; synchronises the device): the workspace's
 * team control words (flags [8][64][32], error word, then per workgroup {stage needed, first late flag, late-slot
 * mask lo, hi} of a failed wait). */
long damc_sweep_team_failures(int device);
int damc_sweep_team_words(const damc_denoiser_t* d, int batch, int n_steps, const void* workspace,
                          size_t workspace_bytes, int* out, int nwords);
/* per-op hook (SURVEY.md §8b damc_denoise_step): ONE reverse step = damc_reverse_sweep with n_steps = 1 on the
 * step's temb_row (ntemb) and coef_row (6, HOST); noise (B, nz) injected or NULL for Philox at step index
 * noise_step (the k-th noisy step of a sweep uses k); eps (B, nz) receives the denoiser output or NULL.
 * workspace: damc_sweep_workspace_bytes(d, batch, 1). */
int damc_denoise_step(const damc_denoiser_t* d, const float* xemb, float* zt, int batch, const float* temb_row,
                      const float* coef_row, int with_noise, const float* noise, uint64_t seed, uint64_t noise_step,
                      uint64_t chain_base, float* eps, void* workspace, size_t workspace_bytes, void* stream);

/* ----------------------------------------------- Q training: denoiser loss step */
/* The denoiser of Q.calculate_loss (workspace/src/diffusion_net.py:624-645, Diffusion_UnetA :463-533) as
 * trained by the Q update of every iteration (workspace/train_gen_recon.py:211-220): eps_pred =
 * p(zt, logsnr, xemb) with every intermediate kept, then the backward from dL/deps_pred to every parameter
 * of p, to zt and to xemb (which the caller's autograd carries into the encoder / prior_emb).  All weights
 * in PyTorch layouts (the damc_denoiser_t of the sweep).  temb_in (B, ntemb) is SinusoidalPosEmb of the
 * per-sample logsnr input, evaluated by the caller with the reference's op sequence (diffusion_net.py:447-461,
 * 490-491). */
typedef damc_denoiser_t damc_denoiser_train_t;
typedef struct { /* gradients, same layouts (written, not accumulated; NULL entries are skipped) */
  float* bmat;
  float *tw1, *tb1, *tw2, *tb2;
  float *wl[7], *bl[7], *ws[7], *bs[7], *wg[7], *bg[7], *wb[7], *wctx[7], *bctx[7];
} damc_denoiser_grads_t;
size_t damc_denoiser_train_workspace_bytes(const damc_denoiser_train_t* d, int batch);
int damc_denoiser_train_forward(const damc_denoiser_train_t* d, const float* zt, const float* temb_in,
                                const float* xemb, int batch, float* eps_pred, void* workspace, size_t workspace_bytes,
                                void* stream);
/* after damc_denoiser_train_forward on the same workspace: grad_eps (B, nz) -> grads, grad_zt (B, nz) and
 * grad_xemb (B, nxemb) (either may be NULL) */
int damc_denoiser_train_backward(const damc_denoiser_train_t* d, const float* grad_eps, int batch,
                                 const damc_denoiser_grads_t* grads, float* grad_zt, float* grad_xemb,
                                 void* workspace, size_t workspace_bytes, void* stream);

/* The rest of Q.calculate_loss around the denoiser (round 5; workspace/src/diffusion_net.py:633-642, no gradient
 * flows through any of it): from u (B) ~ U[0,1) (the caller's torch.rand, :633) and eps (B, nz) (torch.randn_like,
 * :636), logsnr (B) = logsnr_schedule_fn(u) (diffusion_helper_func.py:41-50; may be NULL), zt (B, nz) = the
 * diffusion_forward mean + std * eps (:72-78), temb_in (B, ntemb) = SinusoidalPosEmb of Diffusion_UnetA's logsnr input
 * (diffusion_net.py:447-461, 490-491) with freqs (ntemb / 2) the host's fp32 frequency table; one launch for what the
 * reference issues as ~25 elementwise ops, each op rounded as PyTorch's ROCm kernels round it. */
int damc_q_noise_glue(const float* u, const float* z, const float* eps, int batch, int nz, float logsnr_min,
                      float logsnr_max, const float* freqs, int ntemb, float* logsnr, float* zt, float* temb_in,
                      void* stream);
/* loss (B) = 0.5 * sum_j (eps - eps_pred)^2 (diffusion_net.py:642), and grad_eps_pred (B, nz) from grad_loss (B, element
 * stride grad_stride: 0 for the broadcast gradient of a .mean()) */
int damc_q_loss_forward(const float* eps, const float* eps_pred, int batch, int nz, float* loss, void* stream);
int damc_q_loss_backward(const float* eps, const float* eps_pred, const float* grad_loss, long grad_stride, int batch,
                         int nz, float* grad_eps_pred, void* stream);

/* ------------------------------------------------------- E update (round 5; SURVEY §8f, train_gen_recon.py:233-241)
 * E(z) of _netE (diffusion_net.py:207-223, e's PyTorch-layout w1..b3; w1t / w2t unused) keeping the hidden activations
 * h1, h2 (B, nh) for the backward; energy (B).  Batch and the layer widths multiples of 4, weights 16-B aligned
 * (DAMC_ERR_UNSUPPORTED otherwise: the caller keeps PyTorch). */
typedef struct { /* gradients, PyTorch layouts (written, not accumulated; NULL entries are skipped) */
  float *w1, *b1, *w2, *b2, *w3, *b3;
} damc_ebm_grads_t;
size_t damc_ebm_train_workspace_bytes(const damc_ebm_t* e, int batch);
int damc_ebm_train_forward(const damc_ebm_t* e, const float* z, int batch, float* h1, float* h2, float* energy,
                           void* stream);
/* grad_energy (B, element stride grad_stride: 0 for a .mean()'s broadcast) -> grads and grad_z (B, nz) or NULL */
int damc_ebm_train_backward(const damc_ebm_t* e, const float* z, const float* h1, const float* h2,
                            const float* grad_energy, long grad_stride, int batch, const damc_ebm_grads_t* grads,
                            float* grad_z, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------- Q update: prior embedding (round 6; SURVEY §8f, diffusion_net.py:624-641)
 * Q.prior_emb = Linear(nz, nh) -> LeakyReLU(slope >= 0) -> Linear(nh, nout) (diffusion_net.py:577-581), PyTorch-layout
 * weights; the forward keeps the hidden activation h (B, nh) for the backward.  Replaces the stock modules inside
 * Q.calculate_loss (the mask's prior rows / x None).  Batch and widths multiples of 4, weights 16-B aligned
 * (DAMC_ERR_UNSUPPORTED otherwise: the caller keeps PyTorch). */
typedef struct {
  int nz, nh, nout;
  float slope;
  const float *w1, *b1, *w2, *b2;
} damc_prior_emb_t;
typedef struct { /* gradients, PyTorch layouts (written, not accumulated; NULL entries are skipped) */
  float *w1, *b1, *w2, *b2;
} damc_prior_emb_grads_t;
size_t damc_prior_emb_train_workspace_bytes(const damc_prior_emb_t* e, int batch);
int damc_prior_emb_train_forward(const damc_prior_emb_t* e, const float* noise, int batch, float* h, float* out,
                                 void* stream);
/* grad_out (B, nout) contiguous -> the four parameter gradients (the input is a fresh draw: no input gradient) */
int damc_prior_emb_train_backward(const damc_prior_emb_t* e, const float* noise, const float* h, const float* grad_out,
                                  int batch, const damc_prior_emb_grads_t* grads, void* workspace,
                                  size_t workspace_bytes, void* stream);

/* --------------------------------------------------------------------------- optimiser steps
 * Replaces the G/E/Q updates' torch.nn.utils.clip_grad_norm_ + optim.Adam / optim.AdamW.step()
 * (train_gen_recon.py:155-157, 219-231, 240-241) by multi-tensor kernels.  A launch covers up to
 * DAMC_ADAM_MAX_TENSORS fp32 tensors whose device pointers travel in the kernel arguments (host arrays
 * here), so nothing is rebuilt when autograd hands out new gradient buffers.  The chunk table depends
 * only on the tensor sizes: entry = (tensor index, element offset, length <= DAMC_ADAM_CHUNK), built on
 * the host by damc_adam_build_chunks and copied to device memory by the caller (plain bytes). */
#define DAMC_ADAM_CHUNK 8192
#define DAMC_ADAM_MAX_TENSORS 96
typedef struct { /* per-step scalars, computed by the caller exactly as torch's _multi_tensor_adam does */
  float neg_step_size;   /* -(lr / (1 - beta1^t))                                           */
  float one_minus_beta1; /* lerp weight 1 - beta1                                            */
  float beta2, one_minus_beta2;
  float bc2_sqrt;        /* (1 - beta2^t) ** 0.5                                             */
  float eps;
  float weight_decay;    /* Adam (L2 into the gradient) when decoupled == 0                  */
  float decay_mul;       /* AdamW: 1 - lr * weight_decay                                     */
  int decoupled;
} damc_adam_hparams_t;
size_t damc_adam_chunk_bytes(void);
/* host only: number of chunks for tensors of these sizes */
int damc_adam_chunk_count(const long long* numel, int ntensors);
/* host only: writes the chunk table into host_chunks (max_chunks entries); returns the count or < 0 */
int damc_adam_build_chunks(const long long* numel, int ntensors, void* host_chunks, int max_chunks);
/* clip_grad_norm_(max_norm, norm_type=2), first half: out[0] = total norm, out[1] = min(max_norm /
 * (norm + 1e-6), 1).  grads: host array of ntensors (<= DAMC_ADAM_MAX_TENSORS) device pointers.
 * workspace: nchunks floats.  Gradients are not scaled here (damc_grad_scale, or damc_adam_step's clip). */
int damc_grad_norm(const void* dev_chunks, int nchunks, float* const* grads, int ntensors, float max_norm,
                   float* workspace, float* out, void* stream);
/* the two halves of damc_grad_norm, for gradient sets of more than DAMC_ADAM_MAX_TENSORS tensors: per-chunk
 * sums of squares into partial[0, nchunks) (call once per <= 96-tensor slice, each into its own range),
 * then the fixed-order total over all n partials */
int damc_grad_sumsq(const void* dev_chunks, int nchunks, float* const* grads, int ntensors, float* partial,
                    void* stream);
int damc_grad_norm_finish(const float* partial, int n, float max_norm, float* out, void* stream);
/* grads *= clip[1] (the second half of clip_grad_norm_) */
int damc_grad_scale(const void* dev_chunks, int nchunks, float* const* grads, int ntensors, const float* clip,
                    void* stream);
/* one Adam/AdamW step over every chunk (params, grads, exp_avgs, exp_avg_sqs: host arrays of device
 * pointers); clip (device, from damc_grad_norm) or NULL: when given, the gradient is scaled by clip[1]
 * first and written back, as clip_grad_norm_ would have left it */
int damc_adam_step(const void* dev_chunks, int nchunks, float* const* params, float* const* grads,
                   float* const* exp_avgs, float* const* exp_avg_sqs, int ntensors, const damc_adam_hparams_t* hp,
                   const float* clip, void* stream);

/* ------------------------------------------------------------ FID statistics */
/* calculate_fid* (workspace/src/MCMC.py:130-176) reduce Inception pool features to (mu, sigma) before the
 * Frechet distance (pytorch-fid's calculate_frechet_distance, via pfw.fid).  Here the statistics accumulate on
 * the device in fp64: s1 (d) += sum over the n rows of feats (n, d) fp32, s2 (d, d) += feats^T feats; across
 * GPUs the caller all-reduces (s1, s2, n) once (damc.fid over RCCL).  Deterministic (fixed summation order). */
int damc_fid_accumulate(const float* feats, int n, int d, double* s1, double* s2, void* stream);
/* mu = s1 / n, sigma = (s2 - n mu mu^T) / (n - 1) (np.cov's unbiased estimate); n > 1 */
int damc_fid_mean_cov(const double* s1, const double* s2, double n, int d, double* mu, double* sigma, void* stream);

/* --------------------------------------------------------------------------- profiling */
/* optional per-kernel HIP-event timing (bench.py roofline): records events around each
 * launch of the named kernel class on the launch stream; read back after a sync. */
int damc_prof_enable(int on);
/* record only the comma-separated kernel classes in `classes` (NULL: every class) */
int damc_prof_select(const char* classes);
int damc_prof_reset(void);
/* total ms and launch count for kernel class `name` ("upconv_fwd", "upconv_dgrad", ...) */
int damc_prof_query(const char* name, double* total_ms, long* launches, double* flops);

#ifdef __cplusplus
}
#endif
#endif /* DAMC_H */
