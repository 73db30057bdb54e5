// wgrad.h — kernels of the generator training backward (weight / bias gradients), wgrad.hip.
#pragma once
#include "common.h"

namespace damc {

// Pixel-major transpose of an NHWC map into the x3 limb layout the O_WGRAD GEMM reads:
//   dst[c][pq][n] (n fastest over Bp samples, zero for n >= B), pq = qy * Wq + qx over an Hq x Wq grid
//   sampling map pixel (sy * qy + oy, sx * qx + ox) of the H x W map.
// The source is fp32 (src32) or x3 limbs (src3, C % 8 == 0).  part (optional) receives per-(pq, 32-sample
// block) channel sums: part[(pq * (Bp / 32) + nb) * C + c] (bias gradients, reduced by launch_colsum).
int launch_transpose_x3(const float* src32, const unsigned short* src3, int B, int H, int W, int C, int Hq, int Wq,
                        int sy, int sx, int oy, int ox, int Bp, unsigned short* dst, float* part, hipStream_t s);
// the four output phases of a k4 s2 p1 layer's gradient (sy = sx = 2, offsets (ph >> 1, ph & 1)) in one launch: phase ph
// to dst + ph * dst_pstride (and part + ph * part_pstride when part is set)
int launch_transpose_x3_4ph(const float* src32, const unsigned short* src3, int B, int H, int W, int C, int Hq, int Wq,
                            int Bp, unsigned short* dst, long dst_pstride, float* part, long part_pstride,
                            hipStream_t s);

// dW (Cin, Cout, 4, 4) of a k4 s2 p1 ConvT from the O_WGRAD slabs [4 phases][S][4 * Cin][Cout]
int launch_up2_wgrad_reduce(const float* slabs, int S, int Cin, int Cout, float* dW, hipStream_t s);

// out[c] = sum over r < R of X[r * ld + c], fixed order (two passes through tmp when R is large)
size_t colsum_tmp_floats(long R, int C);
int launch_colsum(const float* X, long R, int C, long ld, float* out, float* tmp, hipStream_t s);
// column sums of X (R x C) with columns < split into out_lo and the rest into out_hi[c - split] (one launch when a single
// pass covers R; else two launch_colsum calls)
int launch_colsum2(const float* X, long R, int C, long ld, float* out_lo, float* out_hi, int split, float* tmp,
                   hipStream_t s);

// Output-layer (Cout <= 4) weight gradient, direct: h NHWC fp32, delta NHWC [pix][Cout]; part and tmp are
// scratch (per-block partials in the PyTorch order, reduced by launch_colsum)
size_t smallc_wgrad_part_floats(const damc_layer_t& L, int B);
size_t smallc_wgrad_tmp_floats(const damc_layer_t& L, int B);
int launch_smallc_wgrad(const damc_layer_t& L, const float* h, const float* delta, int B, float* part, float* tmp,
                        float* dW, hipStream_t s);

// delta[(n * HW + p) * NC + o] = g[n][o][p] * act'(x_hat) (tanh: 1 - x_hat^2; none: 1) from NCHW tensors
int launch_out_delta(const float* g, const float* xhat, int B, int NC, int HW, int act, float* delta, hipStream_t s);

// nn.Linear weight gradient dW[o][i] = sum_n d[n][o] * h[n][i]
int launch_linear_wgrad(const float* d, const float* h, int B, int nout, int nin, float* dW, hipStream_t s);

}  // namespace damc
