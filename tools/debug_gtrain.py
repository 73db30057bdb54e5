"""Debug: per-parameter rel-L2 of the HIP G-update gradients vs the oracle at several batch sizes."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "diffusion-amortized-mcmc_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np, torch
from damc import synth
from src import diffusion_net as dn
from oracle import damc_oracle as orc
torch.set_num_threads(16)
ngf = int(sys.argv[1]) if len(sys.argv) > 1 else 128
for B in [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "32,40,64").split(",")]:
    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=ngf, nc=3), 0)
    z0 = torch.from_numpy(synth.normal_f32(2, 7, (B, 128)))
    x = torch.from_numpy(synth.uniform_f32(1, 7, (B, 3, 32, 32)))
    L = orc.generator_layers(G)
    xh = orc.generator_sample(L, z0)
    ref, gz_ref, _ = orc.generator_train_grads(L, z0, 2.0 * (xh - x) / B)
    Gd = G.cuda().train()
    zz = z0.cuda().requires_grad_(True)
    loss = torch.sum((Gd(zz) - x.cuda()) ** 2, dim=[1, 2, 3]).mean()
    loss.backward()
    flat = [t for gw, gb in ref for t in (gw, gb)]
    errs = []
    for p, r in zip(Gd.parameters(), flat):
        a = p.grad.detach().cpu().double().numpy(); b = r.double().numpy()
        errs.append(np.linalg.norm(a - b) / np.linalg.norm(b))
    e = zz.grad.cpu().double().numpy() - gz_ref.double().numpy()
    print("B=%d ngf=%d" % (B, ngf), " ".join("%.1e" % v for v in errs), "gz %.1e" % (np.linalg.norm(e) / np.linalg.norm(gz_ref.numpy())), flush=True)
    if errs[0] > 1e-4:
        a = Gd.gen[0].weight.grad.detach().cpu().numpy(); b = flat[0].numpy()
        d = np.abs(a - b).reshape(a.shape[0], -1)
        print("  w0 err per ci (first 8):", d.max(1)[:8], " per col block max:", d.reshape(128, 1024, 64).max(axis=(0, 2))[:8])
        print("  rows with err:", np.nonzero(d.max(1) > 1e-3 * np.abs(b).max())[0][:20])
        cols = np.nonzero(d.max(0) > 1e-3 * np.abs(b).max())[0]
        print("  cols with err:", cols[:20], len(cols))
