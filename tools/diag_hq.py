# per-layer accuracy of the HQ generator's k4 s2 p1 layers through the damc_convT hooks (fp64 references)
import ctypes, os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import torch, numpy as np
import torch.nn.functional as F
from conftest import rel_l2
from damc import _lib, plans, synth, langevin as lv
from damc._lib import ptr
from src import diffusion_net as dn
import test_gpu_configs as t
from oracle import damc_oracle as orc
dev = torch.device("cuda:0")
nhwc = lambda a: a.permute(0, 2, 3, 1).contiguous()
G = synth.load_into(dn._netG_celebaHQ(nz=128, ngf=128, nc=3), 0).to(dev).eval()
for eng in (0, 1):
    gd = plans.generator_plan(G).refresh(dev, engine=eng)
    L = _lib.lib(); stream = _lib.stream_ptr(dev)
    convs = [m for m in G.gen if isinstance(m, torch.nn.ConvTranspose2d)]
    for li in range(1, gd.n_layers - 1):
        Ld = gd.layers[li]; conv = convs[li]
        B = int(os.environ.get('DIAG_B', '8'))
        g = torch.Generator().manual_seed(li)
        h = torch.randn(B, Ld.cin, Ld.hin, Ld.win, generator=g, dtype=torch.float64)
        gout = torch.randn(B, Ld.cout, Ld.hout, Ld.wout, generator=g, dtype=torch.float64)
        w = conv.weight.detach().cpu().double(); b = conv.bias.detach().cpu().double()
        nb = int(L.damc_convT_workspace_bytes(ctypes.byref(Ld), B))
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        out = torch.empty(B, Ld.hout, Ld.wout, Ld.cout, device=dev)
        _lib.check(L.damc_convT_fwd(ctypes.byref(Ld), ptr(nhwc(h.float()).to(dev)), B, ptr(out), ptr(ws), nb, stream))
        ref = F.leaky_relu(F.conv_transpose2d(h.float().double(), w, b, stride=2, padding=1), 0.2)
        gin = torch.empty(B, Ld.hin, Ld.win, Ld.cin, device=dev)
        _lib.check(L.damc_convT_dgrad(ctypes.byref(Ld), ptr(nhwc(gout.float()).to(dev)), B, None, 0, 0.0, ptr(gin), ptr(ws), nb, stream))
        gref = F.conv2d(gout.float().double(), w, stride=2, padding=1)
        ref32 = F.leaky_relu(F.conv_transpose2d(h.float(), w.float(), b.float(), stride=2, padding=1), 0.2).double()
        gref32 = F.conv2d(gout.float(), w.float(), stride=2, padding=1).double()
        print("engine %d layer %d (%d->%d @%d): fwd %.2e (cpu32 %.2e) dgrad %.2e (cpu32 %.2e)" % (eng, li, Ld.cin, Ld.cout, Ld.hin,
              rel_l2(out.cpu().numpy(), nhwc(ref).numpy()), rel_l2(ref32.numpy(), ref.numpy()),
              rel_l2(gin.cpu().numpy(), nhwc(gref).numpy()), rel_l2(gref32.numpy(), gref.numpy())), flush=True)
        bias = lambda a, r: float(((a - r) * r).sum() / (r * r).sum())
        print("    scale bias: fwd hip %+.2e cpu %+.2e  dgrad hip %+.2e cpu %+.2e" % (
              bias(out.cpu().double(), nhwc(ref)), bias(ref32, ref), bias(gin.cpu().double(), nhwc(gref)),
              bias(gref32, gref)), flush=True)
G, E, x, z0 = t._case("celebaHQ", int(os.environ.get("DIAG_GB", "8")), dev)
(L32, _), (L64, _) = t._oracles(G, E)
for eng in (0, 1):
    with _lib.exact_fp32(eng == 1):
        gg = lv.likelihood_grad(z0, x, G, 1.0).cpu().numpy()
    g64 = orc.likelihood_grad(L64, z0.cpu().double(), x.cpu().double(), 1.0)[0].numpy()
    g32 = orc.likelihood_grad(L32, z0.cpu(), x.cpu(), 1.0)[0].numpy()
    print("engine %d HQ B=%d lik grad: %.2e (fp32 ref %.2e)" % (eng, z0.shape[0], rel_l2(gg, g64), rel_l2(g32, g64)))
    import numpy as np
    eh = np.array([rel_l2(gg[i], g64[i]) for i in range(len(gg))]); e3 = np.array([rel_l2(g32[i], g64[i]) for i in range(len(gg))])
    print("  per-row median hip %.2e cpu %.2e" % (np.median(eh), np.median(e3)), flush=True)
