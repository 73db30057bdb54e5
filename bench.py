#!/usr/bin/env python
"""Benchmark: Langevin z-steps/sec, CIFAR-10 (B=128, z_dim=128, ngf=128) on 1..8 MI355X.

One bench "step" = the Langevin block of one reference training iteration
(workspace/train_gen_recon.py:203-209): 30 posterior steps on B=128 chains
(sample_langevin_post_z_with_prior, sigma=.1, s=.1, noise on) + 60 prior steps on 2B=256
chains (sample_langevin_prior_z, s=.4, noise on).  `value` counts POSTERIOR z-steps only
(30 per posterior chain and step) against the wall time of the whole block, i.e. the prior's time
is charged but its (cheap) z-steps are not — conservative against the CPU-reference's 130
posterior z-steps/s.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` with no launcher environment starts N ranks
itself (torch.distributed.run as a child process, before any GPU call); under torchrun it is one rank.
Chains never communicate, so there is no collective in the timed path (timing uses a barrier and a MAX
all-reduce of the elapsed time only); noise is keyed by the GLOBAL chain index (damc.dist.block_plan):
  --scaling strong (default): the global B=128 (and 2B prior) chains split over the ranks (BASELINE.md's
                    primary curve), "scaling": "strong"; the JSON records the per-rank batch.  For N > 1 a
                    weak-scaling pass (B=128 chains per rank) is timed after it and reported as "weak_scaling".
  --scaling weak:   B=128 chains per rank -> per-GPU work fixed, "scaling": "weak".

Data: synthetic (counter-hash weights / x ~ U[-1,1] / z0 ~ N(0,1); no datasets offline).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "diffusion-amortized-mcmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X dense fp32 (= f32 MFMA rate), MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (spec, no sparsity), MI355X_MICROARCH.md
PEAK_CLOCK_GHZ = 2.4  # the engine clock the dense peaks are quoted at (MI355X_MICROARCH.md)
LIMB_PRODUCTS = 6          # limb engine: 6 bf16 MFMA products per fp32 product (csrc/gemm.hip)
B, NZ, NGF = 128, 128, 128
POST_STEPS, PRIOR_STEPS = 30, 60
SIGMA, S_POST, S_PRIOR = 0.1, 0.1, 0.4


def build(device):
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=NZ, ngf=NGF, nc=3), 0).to(device).eval()
    E = synth.load_into(dn._netE(nz=NZ), 10).to(device).eval()
    for p in list(G.parameters()) + list(E.parameters()):
        p.requires_grad_(False)
    return G, E


def inputs(device, rank, plan, scaling):
    """This rank's posterior inputs (x, z0) and prior initial state p0 (its rows of cat(z0, N(0, I)))."""
    from damc import synth

    if scaling == "weak":  # a full batch per rank, seeded per rank
        x = synth.uniform_f32(1 + 1000 * rank, 0, (B, 3, 32, 32))
        z0 = synth.normal_f32(2 + 1000 * rank, 0, (B, NZ))
        p0 = np.concatenate([z0, synth.normal_f32(3 + 1000 * rank, 0, (B, NZ))])
    else:  # slices of the global batch
        s, c = plan["post_start"], plan["post_count"]
        qs, qc = plan["prior_start"], plan["prior_count"]
        zg = synth.normal_f32(2, 0, (B, NZ))
        x = synth.uniform_f32(1, 0, (B, 3, 32, 32))[s:s + c]
        z0 = zg[s:s + c]
        p0 = np.concatenate([zg, synth.normal_f32(3, 0, (B, NZ))])[qs:qs + qc]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    return t(x), t(z0), t(p0)


def one_block(lv, G, E, x, z0, p0, zbuf, pbuf, seed, plan):
    """30 posterior steps + 60 prior steps on this rank's chains (train_gen_recon.py:203-209)."""
    zbuf.copy_(z0)
    lv.posterior_langevin(zbuf, x, G, E, POST_STEPS, SIGMA, S_POST, True, seed=seed, chain_base=plan["post_start"])
    pbuf.copy_(p0)
    lv.prior_langevin(pbuf, E, PRIOR_STEPS, S_PRIOR, True, seed=seed + 1, chain_base=plan["prior_start"],
                      global_batch=plan["prior_global"])


def available_cores():
    """(cores, basis): the host cores this process may run on — the affinity mask, capped by a cgroup CPU quota
    (a GPU box's share of a large host), counted as physical cores when SMT siblings share the mask."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = list(range(os.cpu_count() or 1))
    phys = set()
    for c in cpus:
        try:
            with open("/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % c) as f:
                phys.add(f.read().strip())
        except OSError:
            phys.add(str(c))
    n, basis = len(phys), "%d physical cores in the affinity mask (%d logical)" % (len(phys), len(cpus))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
            if quota < n:
                n, basis = quota, "cgroup CPU quota %d (affinity: %s)" % (quota, basis)
    except (OSError, ValueError):
        pass
    return n, basis


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_baseline(budget_s=12.0, full=False):
    """Oracle (CPU restatement, fp32, op for op the reference algorithm) on the same CIFAR-10 inputs.

    Default (bounded, ~budget_s of CPU work): 1 warm-up call, then timed calls of 1 posterior step (B=128) +
    2 prior steps (2B=256) — the block's 30:60 step ratio — until the budget is spent; value = B / median
    per-call time.  full=True: BASELINE.md's protocol — 3 warm-up calls, then the median of 5 full-length
    calls (30 posterior + 60 prior steps each; several minutes of CPU)."""
    from damc import synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    threads, basis = available_cores()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    G = synth.load_into(dn._netG_cifar10(nz=NZ, ngf=NGF, nc=3), 0).eval()
    E = synth.load_into(dn._netE(nz=NZ), 10).eval()
    L, P = orc.generator_layers(G), orc.ebm_params(E)
    x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, 32, 32)))
    z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, NZ)))
    zp0 = torch.cat([z0, torch.from_numpy(synth.normal_f32(3, 0, (B, NZ)))])
    npost, nprior = (POST_STEPS, PRIOR_STEPS) if full else (1, 2)

    def call():
        orc.posterior_langevin(L, P, z0, x, npost, SIGMA, S_POST, noise=torch.randn(npost, B, NZ))
        orc.prior_langevin(P, zp0, nprior, S_PRIOR, noise=torch.randn(nprior, 2 * B, NZ))

    for i in range(3 if full else 1):
        call()
        if full:  # progress for a supervisor that reads silence as a hang
            print("cpu baseline: warm-up call %d done" % (i + 1), file=sys.stderr, flush=True)
    ts = []
    t0 = time.perf_counter()
    while True:
        t1 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t1)
        el = time.perf_counter() - t0
        if full:
            print("cpu baseline: timed call %d %.1f s" % (len(ts), ts[-1]), file=sys.stderr, flush=True)
        if (full and len(ts) >= 5) or (not full and ((el > budget_s and len(ts) >= 5) or len(ts) >= 200)):
            break
    torch.set_num_threads(prev_threads)
    med = sorted(ts)[len(ts) // 2]
    what = ("%d full-length calls (30 posterior steps on B=128 + 60 prior steps on 2B=256) after 3 warm-ups"
            % len(ts)) if full else ("%d timed calls of 1 posterior step (B=128) + 2 prior steps (2B=256) after 1 "
                                      "warm-up, %.1f s" % (len(ts), el))
    return dict(value=round(B * npost / med, 2), unit="z-steps/s", cores=threads, cores_basis=basis, kind="port",
                cpu_model=cpu_model(), statistic="median per call",
                sample="%s of the fp32 oracle restatement (CIFAR-10 _netG_cifar10 ngf=128 + _netE), torch %d threads"
                       % (what, threads))


def event_ms(fn, reps=5):
    """Median wall time of fn() in ms, HIP events on the current stream (the library launches there)."""
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def langevin_breakdown(lv, G, E, x, z0, p0, zbuf, pbuf, plan):
    """the posterior (a1) and prior (a2) legs of the block timed separately."""
    def post():
        zbuf.copy_(z0)
        lv.posterior_langevin(zbuf, x, G, E, POST_STEPS, SIGMA, S_POST, True, seed=7, chain_base=plan["post_start"])

    def prior():
        pbuf.copy_(p0)
        lv.prior_langevin(pbuf, E, PRIOR_STEPS, S_PRIOR, True, seed=8, chain_base=plan["prior_start"],
                          global_batch=plan["prior_global"])

    tp, tq = event_ms(post), event_ms(prior)
    nb, nq = zbuf.shape[0], pbuf.shape[0]
    return {"posterior_ms_per_langevin_step": round(tp / POST_STEPS, 4),
            "posterior_z_steps_per_s": round(nb * POST_STEPS / (tp / 1e3), 1),
            "prior_ms_per_langevin_step": round(tq / PRIOR_STEPS, 4),
            "prior_z_steps_per_s": round(nq * PRIOR_STEPS / (tq / 1e3), 1)}


# SURVEY.md §8(d) per-config posterior work (4 B MAC_G FLOP per batch-step) and BASELINE configs 2/4/5 at
# their per-rank sizes on one GPU: (name, generator ctor, nz, ngf, image, B, steps, sigma)
CONFIG_LEGS = (
    ("cifar10 B=16 (headline config, strong scaling per rank of 8)", "_netG_cifar10", 128, 128, 32, 16, 10, 0.1,
     1089.2e6),
    ("svhn B=64 (config 2)", "_netG_svhn", 100, 64, 32, 64, 30, 0.1, 69.5e6),
    ("celeba64 B=32 (config 4, per rank of 8)", "_netG_celeba64", 100, 128, 64, 32, 10, 0.1, 410.6e6),
    ("celeba64 B=256 (config 4, one GPU)", "_netG_celeba64", 100, 128, 64, 256, 5, 0.1, 410.6e6),
    ("celebaHQ B=8 (config 5, per rank of 8)", "_netG_celebaHQ", 128, 128, 256, 8, 5, 1.0, 6547.3e6),
    ("celebaHQ B=64 (config 5, one GPU)", "_netG_celebaHQ", 128, 128, 256, 64, 3, 1.0, 6547.3e6),
)


def config_legs(lv, device, peak):
    """ms per posterior Langevin step (G fwd + dgrad + E + update) and the fraction of the GEMM engine's
    peak for the other BASELINE configs' generators at full width (17.8 / 420.4 / 1,676
    GFLOP per batch-step at SVHN B=64 / CelebA-64 B=256 / CelebA-HQ B=64).  Each timed sample is three back-to-back
    calls of `steps` steps (median of 3 samples), so a call's host-side prologue overlaps the previous call's kernels
    as it does in a training loop."""
    from damc import synth
    from src import diffusion_net as dn

    out = {}
    for name, ctor, nz, ngf, hw, bsz, steps, sigma, mac in CONFIG_LEGS:
        G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(device).eval()
        E = synth.load_into(dn._netE(nz=nz), 10).to(device).eval()
        x = torch.from_numpy(synth.uniform_f32(61, 0, (bsz, 3, hw, hw))).to(device)
        z0 = torch.from_numpy(synth.normal_f32(62, 0, (bsz, nz))).to(device)
        z = torch.empty_like(z0)

        def run():
            z.copy_(z0)
            lv.posterior_langevin(z, x, G, E, steps, sigma, 0.1, True, seed=9)

        def run3():  # back-to-back calls: a call's host prologue overlaps the previous call's kernels (a training loop)
            for _ in range(3):
                run()

        ms = event_ms(run3, reps=3) / (3 * steps)
        flop = 4.0 * bsz * (mac + 65.8e3)
        out[name] = {"ms_per_step": round(ms, 3), "z_steps_per_s": round(bsz / (ms / 1e3), 1),
                     "gflop_per_step": round(flop / 1e9, 1), "tflops": round(flop / (ms / 1e3) / 1e12, 1),
                     "frac_of_peak": round(flop / (ms / 1e3) / 1e12 / peak, 3)}
        del G, E, x, z0, z
        torch.cuda.empty_cache()
    return out


def amortizer_bench(device):
    """Q(x) = encoder + 100-step reverse sweep, CIFAR-10 B=128 with the
    reference's training defaults (train_gen_recon.py:360-380: nif 64, nxemb 1024, ntemb 128,
    n_interval 100, logsnr [-5.1, 9.8], var 'large', residual, noise on)."""
    from damc import amortizer, synth
    from src import diffusion_net as dn

    n_int = 100
    Q = dn._netQ_U(nc=3, nz=NZ, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=n_int,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                   dataset="cifar10")
    synth.load_into(Q, 20)
    Q.to(device).eval()
    for p in Q.parameters():
        p.requires_grad_(False)
    x = torch.from_numpy(synth.uniform_f32(31, 0, (B, 3, 32, 32))).to(device)
    zt = torch.from_numpy(synth.normal_f32(32, 0, (B, NZ))).to(device)
    xemb = amortizer.encoder_forward(Q.encoder, x)
    zw = torch.empty_like(zt)

    def sweep():
        zw.copy_(zt)
        amortizer.reverse_sweep(Q, xemb, zw, seed=5)

    # three back-to-back calls per timed sample (a call's host-side prologue overlaps the previous call's kernels, as
    # in a training loop; one call per sample exposed ~0.1-0.2 ms of host time per call)
    t_enc = event_ms(lambda: [amortizer.encoder_forward(Q.encoder, x) for _ in range(3)]) / 3
    t_sw = event_ms(lambda: [sweep() for _ in range(3)]) / 3
    t_q = event_ms(lambda: [amortizer.q_forward(Q, x=x) for _ in range(3)]) / 3
    enc_flop = 2.0 * B * 110.8e6        # 110.8 M MAC / sample
    sweep_flop = 2.0 * B * 3.146e6 * n_int  # reference-algorithm FLOP (a9: 3.146 M MAC / sample / step)
    return {"config": "cifar10 Q(x) B=128, nif 64, nxemb 1024, ntemb 128, 100 steps",
            "q_forward_ms": round(t_q, 3), "encoder_ms": round(t_enc, 3), "sweep_ms": round(t_sw, 3),
            "us_per_denoise_step": round(1e3 * t_sw / n_int, 2),
            "encoder_tflops": round(enc_flop / (t_enc / 1e3) / 1e12, 2),
            "sweep_reference_equivalent_tflops": round(sweep_flop / (t_sw / 1e3) / 1e12, 2)}


def hq_q_legs(device):
    """BASELINE config 5's named workload: CelebA-HQ Q(x) = Encoder_celebaHQ(nif=64) + the 100-step 'large' reverse
    sweep (nxemb 1024, ntemb 128; train_gen_recon.py:360-380, diffusion_net.py:315-372,585-622), at the per-rank batch
    of 8 GPUs (B=8) and the whole batch on one GPU (B=64).  Encoder FLOP = 2 B x 6,362.8 M MAC."""
    from damc import amortizer, synth
    from src import diffusion_net as dn

    n_int = 100
    Q = dn._netQ_U(nc=3, nz=NZ, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=n_int,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                   dataset="celebaHQ")
    synth.load_into(Q, 20)
    Q.to(device).eval()
    for p in Q.parameters():
        p.requires_grad_(False)
    out = {}
    for bsz in (8, 64):
        x = torch.from_numpy(synth.uniform_f32(33, 0, (bsz, 3, 256, 256))).to(device)
        zt = torch.from_numpy(synth.normal_f32(34, 0, (bsz, NZ))).to(device)
        xemb = amortizer.encoder_forward(Q.encoder, x)
        zw = torch.empty_like(zt)

        def sweep():
            zw.copy_(zt)
            amortizer.reverse_sweep(Q, xemb, zw, seed=5)

        t_enc = event_ms(lambda: [amortizer.encoder_forward(Q.encoder, x) for _ in range(3)], reps=3) / 3
        t_sw = event_ms(lambda: [sweep() for _ in range(3)], reps=3) / 3
        t_q = event_ms(lambda: [amortizer.q_forward(Q, x=x) for _ in range(3)], reps=3) / 3
        enc_flop = 2.0 * bsz * 6362.8e6
        out["celebaHQ Q(x) B=%d" % bsz] = {
            "q_forward_ms": round(t_q, 3), "encoder_ms": round(t_enc, 3), "sweep_ms": round(t_sw, 3),
            "us_per_denoise_step": round(1e3 * t_sw / n_int, 2),
            "encoder_tflops": round(enc_flop / (t_enc / 1e3) / 1e12, 1)}
        del x, zt, xemb, zw
        torch.cuda.empty_cache()
    return out


def g_update_bench(device, with_torch=True):
    """SURVEY.md §8(f) row 1, the G update of a training iteration (train_gen_recon.py:222-231) at the bench
    config: x_hat = G(z); sum((x_hat - x)^2, [1,2,3]).mean().backward() with the drop-in _netG_cifar10
    (HIP forward + HIP training backward), and the same with the stock PyTorch modules (G.gen, MIOpen fp32:
    the reference's own GPU implementation of this step).  FLOP = 3 x 2 B MAC_G (forward, dgrad, wgrad)."""
    import ctypes

    from damc import _lib, synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=NZ, ngf=NGF, nc=3), 0).to(device).train()
    z = torch.from_numpy(synth.normal_f32(41, 0, (B, NZ))).to(device)
    x = torch.from_numpy(synth.uniform_f32(42, 0, (B, 3, 32, 32))).to(device)

    def step_hip():
        G.zero_grad(set_to_none=True)
        torch.sum((G(z) - x) ** 2, dim=[1, 2, 3]).mean().backward()

    def step_torch():
        G.zero_grad(set_to_none=True)
        torch.sum((G.gen(z.reshape(B, NZ, 1, 1)) - x) ** 2, dim=[1, 2, 3]).mean().backward()

    L = _lib.lib()
    t_hip = event_ms(step_hip)
    L.damc_prof_reset()
    L.damc_prof_select(b"wgrad_up2")
    L.damc_prof_enable(1)
    step_hip()
    torch.cuda.synchronize()
    L.damc_prof_enable(0)
    L.damc_prof_select(None)
    tot, n, fl = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
    L.damc_prof_query(b"wgrad_up2", ctypes.byref(tot), ctypes.byref(n), ctypes.byref(fl))
    flop = 3 * 2.0 * B * 1089.2e6
    out = {"config": "cifar10 _netG_cifar10 ngf=128, B=128: forward + loss + backward (weights and biases)",
           "hip_ms": round(t_hip, 3), "hip_tflops": round(flop / (t_hip / 1e3) / 1e12, 2)}
    if n.value:
        out["wgrad_up2_avg_ms"] = round(tot.value / n.value, 4)
        out["wgrad_up2_tflops"] = round(fl.value / (tot.value / 1e3) / 1e12, 2)
    # the update's clip_grad_norm_ + Adam (train_gen_recon.py:230-231) over G's 12.6 M parameters: damc.optim's
    # fused norm + step against torch's foreach clip_grad_norm_ + Adam
    from damc import optim as dopt

    step_hip()
    opt_t = torch.optim.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.999))
    opt_d = dopt.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.999))

    def adam_torch():
        torch.nn.utils.clip_grad_norm_(G.parameters(), max_norm=100)
        opt_t.step()

    out["clip_adam_hip_ms"] = round(event_ms(lambda: opt_d.clip_and_step(100)), 4)
    out["clip_adam_torch_ms"] = round(event_ms(adam_torch), 4)
    if with_torch:
        print("bench: timing the stock PyTorch G update (MIOpen may tune on first use)", file=sys.stderr, flush=True)
        t_torch = event_ms(step_torch, reps=3)
        out["torch_miopen_ms"] = round(t_torch, 3)
        out["speedup_vs_torch"] = round(t_torch / t_hip, 2)
    return out


def q_update_bench(device, with_torch=True):
    """SURVEY.md §8(f) row 2, one Q update (train_gen_recon.py:211-220; 6 per iteration) at the bench config
    (Q: nif 64, nxemb 1024, ntemb 128, B=128): Q.calculate_loss(x, z, mask).mean().backward() + clip + AdamW,
    the denoiser's forward/backward on libdamc (drop-in), and the same on the stock PyTorch modules."""
    import torch.optim as optim

    from damc import synth, training
    from src import diffusion_net as dn

    Q = dn._netQ_U(nc=3, nz=NZ, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                   dataset="cifar10")
    synth.load_into(Q, 20)
    Q.to(device).train()
    from damc import optim as dopt

    opt = optim.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
    opt_d = dopt.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
    x = torch.from_numpy(synth.uniform_f32(51, 0, (B, 3, 32, 32))).to(device)
    z = torch.from_numpy(synth.normal_f32(52, 0, (B, NZ))).to(device)
    mask = (torch.from_numpy(synth.uniform_f32(53, 0, (B, 1), 0.0, 1.0)) >= 0.2).float().to(device)

    def step():  # the reference's sequence on stock PyTorch
        opt.zero_grad(set_to_none=True)
        Q.calculate_loss(x=x, z=z, mask=mask).mean().backward()
        torch.nn.utils.clip_grad_norm_(Q.parameters(), max_norm=100)
        opt.step()

    def step_hip():  # drop-in modules + damc.optim's fused clip + AdamW
        opt_d.zero_grad(set_to_none=True)
        Q.calculate_loss(x=x, z=z, mask=mask).mean().backward()
        opt_d.clip_and_step(100)

    def six(fn):  # the reference's six consecutive Q updates per iteration (train_gen_recon.py:211-220): an update's
        return lambda: [fn() for _ in range(6)]  # host half overlaps the previous update's kernels, as in training

    out = {"config": "cifar10 Q update B=128 (nif 64, nxemb 1024, ntemb 128): loss fwd+bwd, clip, AdamW",
           "hip_ms": round(event_ms(six(step_hip)) / 6, 3), "hip_ms_isolated": round(event_ms(step_hip), 3),
           "timing": "hip_ms / torch_ms: six back-to-back updates per sample / 6 (the training loop's form); "
                     "hip_ms_isolated: one update per sample (its host time not overlapped)"}
    if with_torch:
        with training.stock_pytorch():
            out["torch_ms"] = round(event_ms(six(step)) / 6, 3)
        out["speedup_vs_torch"] = round(out["torch_ms"] / out["hip_ms"], 2)
    return out


def traffic_from_profiles(kernel_class):
    """(HBM bytes per launch, the FETCH_SIZE read part as counted before the gfx950 x2) of a kernel class from
    profiles/pmc_traffic.json (tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE passes; the stored read bytes
    already carry MI355X_MICROARCH.md's x2 for 16-B streaming and LDS-DMA reads)."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f).get(kernel_class, {})
        rd = d.get("fetch_bytes_per_launch")
        return d.get("hbm_bytes_per_launch"), (rd / 2 if rd is not None else None)
    except (OSError, ValueError):
        return None, None


# the two ConvT k4 s2 forwards of _netG_cifar10 ngf=128 (diffusion_net.py:33,38): (cin, hin, cout, fused projection)
UPCONV_FWD_LAYERS = ((1024, 8, 512, False), (512, 16, 256, True))


def upconv_fwd_algorithmic_bytes(bsz):
    """Algorithmic HBM bytes of one upconv_fwd launch, averaged over the class's two layers:
    the fp32 NHWC input read once (F32A stages fp32), the 4-phase weight's limb copy read once (6 B per weight), and
    the epilogue's writes -- the fp32 activation plus its sign bits (layer 2), or, where the output layer's projection
    runs in the epilogue (layer 3, proj_nostore), the sign bits plus the 2 x 32 per-pixel projection partials."""
    tot = 0.0
    for cin, hin, cout, proj in UPCONV_FWD_LAYERS:
        npix_in, npix_out = bsz * hin * hin, bsz * 4 * hin * hin
        a = 4.0 * npix_in * cin
        w = 6.0 * 16 * cin * cout
        out = npix_out * cout / 8.0 + (4.0 * npix_out * 32 * (cout // 128) if proj else 4.0 * npix_out * cout)
        tot += a + w + out
    return tot / len(UPCONV_FWD_LAYERS)


def upconv_dgrad_algorithmic_bytes(bsz):
    """Algorithmic HBM bytes of one upconv_dgrad launch (the input gradient through the same two ConvT layers), averaged
    over the class's two layers: the fp32 output gradient read once (F32A stages fp32), the weight's limb copy read once,
    the previous layer's sign bits read once (the epilogue's LReLU' mask), and the fp32 input gradient written once."""
    tot = 0.0
    for cin, hin, cout, _ in UPCONV_FWD_LAYERS:
        npix_in, npix_out = bsz * hin * hin, bsz * 4 * hin * hin
        tot += 4.0 * npix_out * cout + 6.0 * 16 * cin * cout + npix_in * cin / 8.0 + 4.0 * npix_in * cin
    return tot / len(UPCONV_FWD_LAYERS)


def launch_ranks(n, argv):
    """`bench.py --gpus N` outside a launcher: run N ranks under torch.distributed.run as a CHILD process (this
    process has not touched the GPU, and is never replaced by exec) and return its exit code.  Rank 0 prints the
    JSON line to the inherited stdout."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=dict(os.environ, DAMC_BENCH_LAUNCHED="1"))


def dry_run(args, rank, world):
    from damc import dist as ddist

    if world > 1:
        import torch.distributed as tdist

        tdist.init_process_group("gloo")
        if tdist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: process group has %d ranks, --gpus %d" % (tdist.get_world_size(), args.gpus))
        plans = [None] * world
        tdist.all_gather_object(plans, ddist.block_plan(B, rank, world, args.scaling))
        tdist.destroy_process_group()
    else:
        plans = [ddist.block_plan(B, 0, 1, args.scaling)]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "scaling": args.scaling, "plans": plans}))
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default): the global B=128 split over the ranks; weak: B=128 chains per rank")
    ap.add_argument("--no-weak-extra", action="store_true", help="N > 1: skip the weak-scaling pass after the timed one")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--cpu-full", action="store_true",
                    help="CPU baseline by BASELINE.md's full protocol (median of 5 full-length calls; minutes)")
    ap.add_argument("--no-config-legs", action="store_true", help="skip the SVHN / CelebA-64 / CelebA-HQ legs")
    ap.add_argument("--no-extras", action="store_true", help="skip the per-leg, amortizer and G-update timings")
    ap.add_argument("--no-torch-g", action="store_true", help="skip the stock-PyTorch G/Q-update comparisons")
    ap.add_argument("--no-live-prof", action="store_true", help="no per-launch HIP events in the timed region")
    ap.add_argument("--exact-fp32", action="store_true",
                    help="run the generator convolutions on the fp32-MFMA engine instead of the limb engine")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: the ranks rendezvous over gloo, check the world size and "
                         "print their block plans")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if os.environ.get("DAMC_BENCH_LAUNCHED"):
            raise SystemExit("bench.py: the rank launcher did not set WORLD_SIZE")
        return launch_ranks(args.gpus, sys.argv[1:])
    if args.exact_fp32:
        os.environ["DAMC_EXACT_FP32"] = "1"
    limb = os.environ.get("DAMC_EXACT_FP32", "0") != "1"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d ranks" % (args.gpus, world))
    # DAMC_BENCH_PG=1 (tests only): the process group and its barrier / MAX all-reduce even for one rank, so a 1-GPU box
    # exercises RCCL (backend nccl) on the bench's own code path
    dist = world > 1 or os.environ.get("DAMC_BENCH_PG") == "1"
    if args.dry_run:
        return dry_run(args, rank, world)
    # DAMC_DIST_BACKEND=gloo (tests only): several ranks sharing one GPU (RCCL needs one GPU per rank); the
    # driver's multi-GPU runs use the default, nccl = RCCL over xGMI
    backend = os.environ.get("DAMC_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
        if tdist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: process group has %d ranks, --gpus %d" % (tdist.get_world_size(), args.gpus))
    device = torch.device("cuda", local)

    from damc import _lib
    from damc import dist as ddist
    from damc import langevin as lv

    plan = ddist.block_plan(B, rank, world, args.scaling)
    G, E = build(device)
    x, z0, p0 = inputs(device, rank, plan, args.scaling)
    zbuf = torch.empty_like(z0)
    pbuf = torch.empty_like(p0)

    def barrier():
        torch.cuda.synchronize(device)
        if dist:
            tdist.barrier()
        torch.cuda.synchronize(device)

    def max_over_ranks(v):
        if not dist:
            return v
        t = torch.tensor([float(v)], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        return float(t.item())

    for i in range(args.warmup):
        one_block(lv, G, E, x, z0, p0, zbuf, pbuf, 1000 + i, plan)
    L = _lib.lib()
    L.damc_prof_reset()
    # live HIP events only around the dominant kernel classes (every event pair costs the stream a gap)
    L.damc_prof_select(b"upconv_fwd,upconv_dgrad")
    L.damc_prof_enable(0 if args.no_live_prof else 1)
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_block(lv, G, E, x, z0, p0, zbuf, pbuf, 2000 + i, plan)
    barrier()
    elapsed = time.perf_counter() - t0
    L.damc_prof_enable(0)
    if not torch.isfinite(zbuf).all() or not torch.isfinite(pbuf).all():
        raise RuntimeError("non-finite chains after the timed region")
    dump = os.environ.get("DAMC_BENCH_DUMP")
    if dump:  # tests only: this rank's chains after its last block, with its slice of the global batch
        torch.save({"z": zbuf.cpu(), "p": pbuf.cpu(), "plan": dict(plan)}, os.path.join(dump, "rank%d.pt" % rank))

    # per-class kernel time from the live HIP events
    import ctypes

    def query():
        out = {}
        for name in ("upconv_fwd", "upconv_dgrad", "proj_fwd", "proj_dgrad", "smallc_fwd", "smallc_dgrad",
                     "posterior_update", "slab_sum", "prior_chain", "split_x3"):
            ms, n, fl = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
            _lib.check(L.damc_prof_query(name.encode(), ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)))
            if n.value:
                out[name] = dict(total_ms=ms.value, launches=n.value, flops=fl.value)
        return out

    classes = query()
    # every kernel class, from one more (untimed) block with events around every launch
    L.damc_prof_reset()
    L.damc_prof_select(None)
    L.damc_prof_enable(1)
    one_block(lv, G, E, x, z0, p0, zbuf, pbuf, 3000, plan)
    torch.cuda.synchronize(device)
    L.damc_prof_enable(0)
    breakdown = query()
    # the clock the dominant kernel's K loops hold, from in-kernel stamps (damc_clock_probe) over one more untimed
    # block right behind the timed ones (MI355X_MICROARCH.md, DVFS give-back item 6)
    clk = torch.zeros(4096 * 4, dtype=torch.int64, device=device)
    L.damc_clock_probe(clk.data_ptr(), 4096)
    one_block(lv, G, E, x, z0, p0, zbuf, pbuf, 3001, plan)
    torch.cuda.synchronize(device)
    L.damc_clock_probe(None, 0)
    cs = clk.view(-1, 4).cpu().double()
    ok = cs[:, 3] > cs[:, 1]
    clock_ghz = float(((cs[ok, 2] - cs[ok, 0]) / (cs[ok, 3] - cs[ok, 1])).median()) * 0.1 if ok.any() else None

    t_max = max_over_ranks(elapsed)
    # the dominant class's mean launch time, max over ranks (a strong-scaling rank's per-rank batch)
    dom = max(("upconv_fwd", "upconv_dgrad"), key=lambda k: classes.get(k, {}).get("total_ms", 0.0))
    dom_c = classes.get(dom)
    dom_avg_ms = dom_c["total_ms"] / dom_c["launches"] if dom_c else float("nan")
    dom_avg_ms_max = max_over_ranks(dom_avg_ms)

    weak = None
    if dist and args.scaling == "strong" and not args.no_weak_extra:
        # secondary curve: B=128 chains per rank, its own timed pass after the headline one
        wplan = ddist.block_plan(B, rank, world, "weak")
        wx, wz0, wp0 = inputs(device, rank, wplan, "weak")
        wz, wp = torch.empty_like(wz0), torch.empty_like(wp0)
        for i in range(args.warmup):
            one_block(lv, G, E, wx, wz0, wp0, wz, wp, 4000 + i, wplan)
        barrier()
        tw = time.perf_counter()
        for i in range(args.steps):
            one_block(lv, G, E, wx, wz0, wp0, wz, wp, 5000 + i, wplan)
        barrier()
        tw_max = max_over_ranks(time.perf_counter() - tw)
        weak = {"value": round(world * B * POST_STEPS * args.steps / tw_max, 2), "unit": "z-steps/s",
                "ms_per_step": round(1e3 * tw_max / args.steps, 3), "global_batch": world * B,
                "per_rank_batch": B, "scaling": "weak"}
        del wx, wz0, wp0, wz, wp

    extras = None
    if not args.no_extras and rank == 0:
        # outside the timed region (after the max-over-ranks reduction): does not enter `value`; rank 0 only
        extras = langevin_breakdown(lv, G, E, x, z0, p0, zbuf, pbuf, plan)
        extras["amortizer"] = amortizer_bench(device)
        extras["amortizer"]["celebaHQ"] = hq_q_legs(device)
        extras["g_update"] = g_update_bench(device, with_torch=not args.no_torch_g)
        extras["q_update"] = q_update_bench(device, with_torch=not args.no_torch_g)

    limb_peak = PEAK_BF16_TFLOPS / LIMB_PRODUCTS if limb else PEAK_FP32_TFLOPS
    legs = None
    if not args.no_extras and not args.no_config_legs and rank == 0:
        legs = config_legs(lv, device, limb_peak)

    if rank == 0:
        chains = world * B if args.scaling == "weak" else B
        zsteps = chains * POST_STEPS * args.steps
        value = zsteps / t_max
        c = classes.get(dom, dict(total_ms=float("nan"), launches=1, flops=float("nan")))
        avg_s = c["total_ms"] / c["launches"] / 1e3
        flops_per_launch = c["flops"] / c["launches"]
        achieved = flops_per_launch / avg_s / 1e12
        peak = limb_peak
        traffic, fetch_raw = traffic_from_profiles(dom)
        algo_bytes = (upconv_fwd_algorithmic_bytes if dom == "upconv_fwd" else upconv_dgrad_algorithmic_bytes)(
            plan["post_count"])
        gemm_ms = sum(breakdown[k]["total_ms"] for k in breakdown if k.startswith(("upconv", "proj"))) or None
        gemm_fl = sum(breakdown[k]["flops"] for k in breakdown if k.startswith(("upconv", "proj")))
        post_flops_step = 4.0 * B * 1089.2e6  # 4 * B * MAC_G per posterior step
        out = {
            "metric": "Langevin z-steps/sec (B=128, z_dim=128, CIFAR-10)",
            "value": round(value, 2),
            "unit": "z-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * t_max / args.steps, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-hash weights, x~U[-1,1], z0~N(0,1); CIFAR-10 _netG_cifar10 ngf=128 + _netE)",
            "config": {
                "workload": "cifar10 train-iteration Langevin block: 30 posterior steps on B=128 + 60 prior "
                            "steps on 2B=256 %s (value counts posterior z-steps only)"
                            % ("per rank" if args.scaling == "weak" else "split over the ranks"),
                "global_batch": chains, "per_rank_batch": plan["post_count"],
                "per_rank_prior_chains": plan["prior_count"], "z_dim": NZ, "ngf": NGF, "posterior_steps": POST_STEPS,
                "prior_steps": PRIOR_STEPS, "sigma": SIGMA, "step_size": S_POST, "prior_step_size": S_PRIOR,
                "parallelism": "dp%d (chains sharded, no collective)" % world,
            },
            "roofline": {
                "bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": round(peak, 1),
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "flops_per_launch": flops_per_launch, "avg_launch_ms": round(avg_s * 1e3, 4),
                "traffic": traffic,
                "traffic_basis": "HBM bytes per launch = 2 x FETCH_SIZE (the gfx950 half-count correction, "
                                 "MI355X_MICROARCH.md HBM) + WRITE_SIZE, separate PMC passes of the same bench "
                                 "(profiles/pmc_traffic.json)",
                "traffic_fetch_size_uncorrected": fetch_raw,
                "algorithmic_bytes": algo_bytes,
                "traffic_over_algorithmic": round(traffic / algo_bytes, 2) if traffic and algo_bytes else None,
                "clock_ghz": round(clock_ghz, 3) if clock_ghz else None,
                "frac_at_clock": round(achieved / (peak * clock_ghz / PEAK_CLOCK_GHZ), 4) if clock_ghz else None,
                "clock_basis": "median over the workgroups of one upconv_fwd launch of d(s_memtime) / "
                               "d(s_memrealtime) x 100 MHz around the K loop, one untimed block after the timed ones; "
                               "peak is quoted at %.1f GHz" % PEAK_CLOCK_GHZ,
                "peak_basis": ("limb engine: fp32 FLOP at the bf16 dense MFMA peak %.0f / %d limb products "
                               "(executed bf16 MFMA %.0f TFLOP/s)" % (PEAK_BF16_TFLOPS, LIMB_PRODUCTS,
                                                                       achieved * LIMB_PRODUCTS)) if limb
                              else "fp32 MFMA dense peak",
            },
            "gemm_arith": ("fp32 operands as 3 bf16 limbs, 6 limb products per fp32 product on "
                           "v_mfma_f32_16x16x32_bf16, fp32 accumulation; error vs fp64 equal to the fp32-MFMA "
                           "engine's (profiles/r01/gemm_bench.txt)") if limb
                          else "fp32 v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chains)",
            "posterior_tflops_effective": round(post_flops_step * POST_STEPS * args.steps / t_max / 1e12, 2),
            "gemm_classes_tflops": round(gemm_fl / (gemm_ms / 1e3) / 1e12, 2) if gemm_ms else None,
            "kernel_classes": {k: dict(avg_ms=round(v["total_ms"] / v["launches"], 4), launches=v["launches"])
                               for k, v in breakdown.items()},
            "prior_us_per_step": round(1e3 * breakdown["prior_chain"]["total_ms"]
                                       / breakdown["prior_chain"]["launches"] / PRIOR_STEPS, 2)
            if "prior_chain" in breakdown else None,
            "batch_iterations_per_s": round(args.steps / t_max, 3),
            "cpu_baseline": None,
        }
        if dist:
            out["per_rank"] = {"dominant_class": dom, "avg_launch_ms_max_over_ranks": round(dom_avg_ms_max, 4),
                               "backend": backend}
        if weak:
            out["weak_scaling"] = weak
        if extras:
            out["langevin_legs"] = {k: v for k, v in extras.items() if k not in ("amortizer", "g_update", "q_update")}
            out["amortizer"] = extras["amortizer"]
            out["g_update"] = extras["g_update"]
            out["q_update"] = extras["q_update"]
        if legs:
            out["config_legs"] = legs
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args.cpu_budget, full=args.cpu_full)
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu"] = round(value / cb["value"], 1)
        print(json.dumps(out))
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
