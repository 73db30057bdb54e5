"""Build-container only: time the reference posterior step against the oracle restatement
interleaved in one process (validates bench.py cpu_baseline). Reads /root/reference; never run on the GPU box."""
import sys, time, types, torch, importlib
torch.set_num_threads(8)
sys.path.insert(0,'/root/repo/diffusion-amortized-mcmc_amd'); sys.path.insert(0,'/root/repo')
from damc import synth
from src import diffusion_net as dn
from oracle import damc_oracle as orc
G = synth.load_into(dn._netG_cifar10(nz=128, ngf=128, nc=3), 0).eval()
E = synth.load_into(dn._netE(nz=128), 10).eval()
sdG, sdE = G.state_dict(), E.state_dict()
x = torch.from_numpy(synth.uniform_f32(1,0,(128,3,32,32))); z = torch.from_numpy(synth.normal_f32(2,0,(128,128)))
L, P = orc.generator_layers(G), orc.ebm_params(E)
for n in ('torchvision','torchvision.utils','pytorch_fid_wrapper'): sys.modules.setdefault(n, types.ModuleType(n))
sys.path.remove('/root/repo/diffusion-amortized-mcmc_amd')
for k in [k for k in sys.modules if k=='src' or k.startswith('src.')]: del sys.modules[k]
sys.path.insert(0,'/root/reference/workspace')
mc = importlib.import_module('src.MCMC'); rdn = importlib.import_module('src.diffusion_net')
Gr = rdn._netG_cifar10(nz=128, ngf=128, nc=3); Gr.load_state_dict(sdG); Er = rdn._netE(nz=128); Er.load_state_dict(sdE)
def ref(n):
    zz = z.clone().requires_grad_(True); mc.sample_langevin_post_z_with_prior(zz, x, Gr, Er, n, 0.1, False, 0.1)
def ora(n): orc.posterior_langevin(L,P,z,x,n,0.1,0.1)
ref(1); ora(1)
tr, to = [], []
for r in range(3):
    t=time.perf_counter(); ref(2); tr.append((time.perf_counter()-t)/2)
    t=time.perf_counter(); ora(2); to.append((time.perf_counter()-t)/2)
print('reference ms/step', [round(v*1e3) for v in tr], 'oracle', [round(v*1e3) for v in to], 'median ratio', sorted(to)[1]/sorted(tr)[1])
