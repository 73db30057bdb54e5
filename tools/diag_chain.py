# stage-wise accuracy of the CelebA-HQ generator backward on REAL chain data: each k4 s2 layer's dgrad + LReLU mask
# applied to the fp64 chain's own pre-activation gradient (cast to fp32), through the damc_convT_dgrad hook and
# through CPU fp32 ATen, both against the fp64 stage; then the same stages chained on HIP values
import ctypes, os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import numpy as np
import torch
from conftest import rel_l2
from damc import _lib, plans
from damc._lib import ptr
from oracle import damc_oracle as orc
import test_gpu_configs as t
dev = torch.device("cuda:0")
nhwc = lambda a: a.permute(0, 2, 3, 1).contiguous()
nchw = lambda a: a.permute(0, 3, 1, 2).contiguous()
rows = lambda a, r: float(np.median([rel_l2(a[i], r[i]) for i in range(r.shape[0])]))
B = int(os.environ.get("DIAG_B", "8"))
G, E, x, z0 = t._case("celebaHQ", B, dev)
(L32, _), (L64, _) = t._oracles(G, E)
z64, x64 = z0.cpu().double(), x.cpu().double()
hs = orc.generator_forward(L64, z64)
r = hs[-1] - x64
d = r * orc._act_grad_from_out(hs[-1], L64[-1]["act"])
ds = {len(L64) - 1: d}  # fp64 pre-activation gradients per layer
for i in range(len(L64) - 1, 0, -1):
    L = L64[i]
    dh = torch.ops.aten.convolution_backward(d, hs[i - 1], L["W"], None, [L["stride"]] * 2, [L["pad"]] * 2, [1, 1],
                                             True, [0, 0], 1, [True, False, False])[0]
    d = orc._act_backward(dh, hs[i - 1], L64[i - 1]["act"])
    ds[i - 1] = d
gd = plans.generator_plan(G).refresh(dev, engine=0)
lib = _lib.lib(); stream = _lib.stream_ptr(dev)
chain = None
stage_z = {}
L0 = L64[0]
def proj64(d0):
    return torch.ops.aten.convolution_backward(d0, z64.reshape(B, -1, 1, 1), L0["W"], None, [1, 1], [0, 0], [1, 1],
                                               True, [0, 0], 1, [True, False, False])[0].reshape(B, -1)
def to_z(d, j):  # the pre-activation gradient of layer j through the exact fp64 chain to z
    for k in range(j, 0, -1):
        L = L64[k]
        dh = torch.ops.aten.convolution_backward(d, hs[k - 1], L["W"], None, [2, 2], [1, 1], [1, 1], True, [0, 0],
                                                 1, [True, False, False])[0]
        d = orc._act_backward(dh, hs[k - 1], L64[k - 1]["act"])
    return proj64(d)
for i in range(len(L64) - 2, 0, -1):  # UP2 layers: dgrad of layer i -> pre-activation gradient of layer i-1
    Ld = gd.layers[i]
    din = ds[i].float()
    mask = hs[i - 1].float()
    # CPU fp32 stage
    L = L32[i]
    dh32 = torch.ops.aten.convolution_backward(din, mask, L["W"], None, [2, 2], [1, 1], [1, 1], True, [0, 0], 1,
                                               [True, False, False])[0]
    c32 = orc._act_backward(dh32, mask, L32[i - 1]["act"]).double()
    nb = int(lib.damc_convT_workspace_bytes(ctypes.byref(Ld), B))
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    gin = torch.empty(B, Ld.hin, Ld.win, Ld.cin, device=dev)
    mk = nhwc(mask).to(dev)
    _lib.check(lib.damc_convT_dgrad(ctypes.byref(Ld), ptr(nhwc(din).to(dev)), B, ptr(mk), _lib.ACT_LRELU, 0.2,
                                    ptr(gin), ptr(ws), nb, stream))
    h = nchw(gin.cpu()).double()
    if chain is None:
        chain = din.to(dev)
    gin2 = torch.empty_like(gin)
    _lib.check(lib.damc_convT_dgrad(ctypes.byref(Ld), ptr(nhwc(chain)), B, ptr(mk), _lib.ACT_LRELU, 0.2, ptr(gin2),
                                    ptr(ws), nb, stream))
    chain = nchw(gin2).contiguous()
    ref = ds[i - 1]
    stage_z[i] = (to_z(h, i - 1), to_z(c32, i - 1))
    print("layer %d (%d->%d @%d): stage hip %.2e cpu32 %.2e | chained hip %.2e   |d| %.2e  cancellation %.1f" % (
        i, Ld.cout, Ld.cin, Ld.hout, rows(h.numpy(), ref.numpy()), rows(c32.numpy(), ref.numpy()),
        rows(chain.cpu().double().numpy(), ref.numpy()), float(ref.abs().mean()),
        float((torch.ops.aten.convolution_backward(ds[i].abs(), hs[i - 1], L64[i]["W"].abs(), None, [2, 2], [1, 1],
              [1, 1], True, [0, 0], 1, [True, False, False])[0].norm() / ref.norm()))), flush=True)

gz64 = proj64(ds[0])
for i in sorted(stage_z, reverse=True):
    print("stage %d error alone, carried exactly to z: hip %.2e cpu32 %.2e" % (
        i, rows(stage_z[i][0].numpy(), gz64.numpy()), rows(stage_z[i][1].numpy(), gz64.numpy())))
print("z-grad from the HIP-hook chain (fp64 proj): %.2e" % rows(proj64(chain.cpu().double()).numpy(), gz64.numpy()))
print("z-grad from the fp32-cast fp64 d0 (fp64 proj): %.2e" % rows(proj64(ds[0].float().double()).numpy(), gz64.numpy()))
from damc import langevin as lv
g = lv.likelihood_grad(z0, x, G, 1.0).cpu().double()
print("library z-grad: %.2e   (vs oracle likelihood_grad fp64 %.2e)" % (
    rows(g.numpy(), gz64.numpy()), rows(orc.likelihood_grad(L64, z64, x64, 1.0)[0].numpy(), gz64.numpy())))
g32 = orc.likelihood_grad(L32, z0.cpu(), x.cpu(), 1.0)[0].double()
print("cpu fp32 z-grad: %.2e" % rows(g32.numpy(), gz64.numpy()))
# HIP forward through the hooks: masks from HIP activations
hh = [None] * len(L64)
h = torch.nn.functional.leaky_relu(torch.nn.functional.conv_transpose2d(z0.cpu().reshape(B, -1, 1, 1), L32[0]["W"], L32[0]["b"]), 0.2)
hh[0] = h
cur = nhwc(h).to(dev)
for i in range(1, len(L64) - 1):
    Ld = gd.layers[i]
    nb = int(lib.damc_convT_workspace_bytes(ctypes.byref(Ld), B))
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    out = torch.empty(B, Ld.hout, Ld.wout, Ld.cout, device=dev)
    _lib.check(lib.damc_convT_fwd(ctypes.byref(Ld), ptr(cur), B, ptr(out), ptr(ws), nb, stream))
    cur = out
    hh[i] = nchw(out.cpu())
    print("fwd layer %d: hip %.2e  sign flips vs fp64: %d" % (i, rows(hh[i].double().numpy(), hs[i].numpy()),
          int(((hh[i] > 0) != (hs[i] > 0)).sum())))
