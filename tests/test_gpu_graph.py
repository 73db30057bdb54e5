"""The HIP path is stream-ordered and neither allocates nor synchronises inside a call, so a
training loop can capture it in a torch.cuda.CUDAGraph (a HIP graph on ROCm) and replay it.  Captured here: the
bench's Langevin block body (posterior_langevin + prior_langevin, explicit Philox seeds) at full CIFAR width;
the replay must equal the eager calls bitwise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_langevin_block_replays_from_a_captured_graph(gpu_device):
    from damc import langevin as lv
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=128, nc=3), 0).to(gpu_device).eval()
    E = synth.load_into(dn._netE(nz=128), 10).to(gpu_device).eval()
    B = 32
    x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, 32, 32))).to(gpu_device)
    z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, 128))).to(gpu_device)
    p0 = torch.from_numpy(synth.normal_f32(3, 0, (2 * B, 128))).to(gpu_device)

    def body(z, p):
        lv.posterior_langevin(z, x, G, E, 3, 0.1, 0.1, True, seed=1234)
        lv.prior_langevin(p, E, 5, 0.4, True, seed=5678)

    # eager reference
    ze, pe = z0.clone(), p0.clone()
    body(ze, pe)
    torch.cuda.synchronize()
    # capture (after a warm-up on a side stream, as torch.cuda.graphs requires) and replay twice
    zg, pg = z0.clone(), p0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(zg.clone(), pg.clone())
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        body(zg, pg)
    for _ in range(2):
        zg.copy_(z0)
        pg.copy_(p0)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(zg, ze), "posterior chains differ between graph replay and eager"
        assert torch.equal(pg, pe), "prior chains differ between graph replay and eager"


def test_reverse_sweep_replays_from_a_captured_graph(gpu_device, monkeypatch):
    """Q's reverse sweep on the per-block launch chain (DAMC_SWEEP_TEAM=0) captured into a graph: the replay equals
    the eager launch chain bitwise (B=128, 20 steps, Philox noise)."""
    from damc import amortizer as am
    from damc import synth
    from src import diffusion_net as dn

    Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=20,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
    synth.load_into(Q, 20)
    Q.to(gpu_device).eval()
    xemb = torch.from_numpy(synth.normal_f32(7, 0, (128, 1024))).to(gpu_device)
    zt0 = torch.from_numpy(synth.normal_f32(8, 0, (128, 128))).to(gpu_device)
    ze = zt0.clone()
    monkeypatch.setenv("DAMC_SWEEP_TEAM", "0")
    am.reverse_sweep(Q, xemb, ze, seed=42)
    torch.cuda.synchronize()
    zg = zt0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        am.reverse_sweep(Q, xemb, zg.clone(), seed=42)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        am.reverse_sweep(Q, xemb, zg, seed=42)
    for _ in range(2):
        zg.copy_(zt0)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.isfinite(zg).all()
        assert torch.equal(zg, ze), "sweep differs between graph replay and the eager launch chain"


def test_team_sweep_replays_from_a_captured_graph(gpu_device, monkeypatch):
    """The default sweep (the TEAM launch) recorded into a graph and replayed: bitwise the eager team sweep, and no
    replay needed the device-side rescue (damc_sweep_team_failures unchanged), i.e. every replay kept all its
    workgroups resident and every hand-off completed."""
    from damc import _lib
    from damc import amortizer as am
    from damc import synth
    from src import diffusion_net as dn

    Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=20,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
    synth.load_into(Q, 20)
    Q.to(gpu_device).eval()
    xemb = torch.from_numpy(synth.normal_f32(7, 0, (128, 1024))).to(gpu_device)
    zt0 = torch.from_numpy(synth.normal_f32(8, 0, (128, 128))).to(gpu_device)
    L = _lib.lib()
    dev = gpu_device.index or 0
    ze = zt0.clone()
    am.reverse_sweep(Q, xemb, ze, seed=42)
    torch.cuda.synchronize()
    before = L.damc_sweep_team_failures(dev)
    monkeypatch.setenv("DAMC_SWEEP_TEAM_KEEP", "1")
    zg = zt0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        am.reverse_sweep(Q, xemb, zg.clone(), seed=42)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        am.reverse_sweep(Q, xemb, zg, seed=42)
    for _ in range(3):
        zg.copy_(zt0)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(zg, ze), "team sweep differs between graph replay and eager"
    assert L.damc_sweep_team_failures(dev) == before, "a replayed team launch needed the rescue"
