"""CPU: libdamc.so loads and exports every entry point include/damc.h declares (no compute calls)."""
import ctypes
import os
import re

from conftest import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "damc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(damc_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = _declared()
    for required in ("damc_posterior_langevin", "damc_prior_langevin", "damc_reverse_sweep",
                     "damc_generator_forward", "damc_likelihood_grad", "damc_ebm_energy_grad", "damc_z_update"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from damc import _lib

    assert os.path.exists(_lib.LIB_PATH), "build libdamc.so first (__graft_entry__.build())"
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(so, n)]
    assert not missing, missing
    # the Python binding covers the whole header
    assert sorted(_lib.EXPORTED_SYMBOLS) == _declared()


def test_host_only_calls():
    from damc import _lib

    L = _lib.lib()
    assert L.damc_abi_version() == _lib.ABI_VERSION == 3
    assert b"invalid" in L.damc_error_string(1001)
    # descriptor validation runs on the host: an empty generator has no workspace
    g = _lib.Generator()
    assert L.damc_posterior_workspace_bytes(ctypes.byref(g), 8) == 0


def _cifar_desc(ngf=16):
    """_netG_cifar10 topology (diffusion_net.py:20-51) as a host-side descriptor (no device pointers)."""
    from damc import _lib

    g = _lib.Generator()
    g.n_layers, g.nz, g.nc, g.h, g.w = 4, 128, 3, 32, 32
    spec = [(_lib.LAYER_PROJ, 128, ngf * 8, 8, 1, 0, 1, 8), (_lib.LAYER_UP2, ngf * 8, ngf * 4, 4, 2, 1, 8, 16),
            (_lib.LAYER_UP2, ngf * 4, ngf * 2, 4, 2, 1, 16, 32), (_lib.LAYER_SMALLC, ngf * 2, 3, 3, 1, 1, 32, 32)]
    for i, (kind, cin, cout, k, s, p, hin, hout) in enumerate(spec):
        d = g.layers[i]
        d.kind, d.cin, d.cout, d.k, d.stride, d.pad = kind, cin, cout, k, s, p
        d.hin = d.win = hin
        d.hout = d.wout = hout
        d.act, d.slope = (_lib.ACT_TANH, 0.0) if i == 3 else (_lib.ACT_LRELU, 0.2)
    return g


def test_engine_field_is_validated_host_only():
    """The convolution engine is a per-descriptor field (ABI 2): limb (default) and fp32 descriptors are
    valid and size the same workspace; a generator mixing engines, or naming an unknown one, is refused."""
    from damc import _lib

    L = _lib.lib()
    g = _cifar_desc()
    n_limb = L.damc_posterior_workspace_bytes(ctypes.byref(g), 8)
    assert n_limb > 0
    for i in range(4):
        g.layers[i].engine = _lib.ENGINE_FP32
    assert L.damc_posterior_workspace_bytes(ctypes.byref(g), 8) == n_limb
    g.layers[2].engine = _lib.ENGINE_LIMB
    assert L.damc_posterior_workspace_bytes(ctypes.byref(g), 8) == 0
    g.layers[2].engine = 7
    assert L.damc_posterior_workspace_bytes(ctypes.byref(g), 8) == 0
    # the Python default engine is per thread
    assert _lib.current_engine() == _lib.ENGINE_LIMB
    with _lib.exact_fp32():
        assert _lib.current_engine() == _lib.ENGINE_FP32
    assert _lib.current_engine() == _lib.ENGINE_LIMB


def test_training_shape_support_host_only():
    """Host-side shape logic of the training entry points (no device work): which Conv2d backward shapes the
    library covers (workspace 0 = unsupported), and descriptor validation of the denoiser training path."""
    from damc import _lib

    L = _lib.lib()
    ws = L.damc_conv2d_backward_workspace_bytes
    assert ws(128, 16, 16, 64, 128, 4, 2, 1) > 0       # k4 s2 p1, H = 2 Ho: limb-engine path
    assert ws(128, 32, 32, 3, 64, 3, 1, 1) > 0         # first conv (Cin <= 4)
    assert ws(128, 4, 4, 512, 1024, 4, 1, 0) > 0       # last conv covering its input
    assert ws(128, 7, 7, 64, 128, 4, 2, 1) > 0         # mnist 7 -> 3 (H = 2 Ho + 1): the zero-padded path
    assert ws(128, 7, 7, 4, 128, 4, 2, 1) == 0         # ... whose transposed view needs Cin % 8 == 0
    assert ws(128, 32, 32, 64, 64, 3, 1, 1) == 0       # a k3 conv that is not the first
    assert L.damc_conv2d_workspace_floats(128, 8, 8, 256, 512, 4, 2, 1) > 0  # under-filled: split-K slabs
    d = _lib.DenoiserTrain()
    assert L.damc_denoiser_train_workspace_bytes(ctypes.byref(d), 128) == 0  # empty descriptor rejected
    g = _lib.Generator()
    assert L.damc_generator_train_workspace_bytes(ctypes.byref(g), 128) == 0


def test_encoder_training_dispatch_host_only():
    """encoder_train_supported: the CIFAR / CelebA / mnist topologies take the HIP path (host logic)."""
    import torch

    from damc import training
    from src import diffusion_net as dn

    x32 = torch.empty(4, 3, 32, 32)
    assert training.encoder_train_supported(dn.Encoder_cifar10(nc=3, nemb=64, nif=8), x32)
    assert training.encoder_train_supported(dn.Encoder_celeba64(nc=3, nemb=64, nif=8), torch.empty(2, 3, 64, 64))
    assert training.encoder_train_supported(dn.Encoder_mnist(nc=1, nemb=64, nif=8), torch.empty(2, 1, 28, 28))


def test_adam_chunk_table_host_only():
    """damc_adam_build_chunks (host-only, no GPU): 8192-element chunks per tensor, empty tensors skipped, at
    most 96 tensors per table; damc.optim refuses CPU tensors (no fallback)."""
    import ctypes as C

    import pytest
    import torch

    from damc import _lib, optim

    L = _lib.lib()
    assert L.damc_adam_chunk_bytes() == 16
    sizes = [20000, 0, 5, 8192]
    arr = (C.c_longlong * len(sizes))(*sizes)
    assert L.damc_adam_chunk_count(arr, len(sizes)) == 3 + 0 + 1 + 1
    buf = (C.c_ubyte * (16 * 5))()
    assert L.damc_adam_build_chunks(arr, len(sizes), buf, 4) < 0  # too small
    assert L.damc_adam_build_chunks(arr, len(sizes), buf, 5) == 5
    raw = bytes(buf)
    rows = [(int.from_bytes(raw[16 * i:16 * i + 8], "little"), int.from_bytes(raw[16 * i + 8:16 * i + 12], "little"),
             int.from_bytes(raw[16 * i + 12:16 * i + 16], "little")) for i in range(5)]
    assert rows == [(0, 0, 8192), (8192, 0, 8192), (16384, 0, 20000 - 16384), (0, 2, 5), (0, 3, 8192)]
    many = (C.c_longlong * 97)(*([1] * 97))
    assert L.damc_adam_chunk_count(many, 97) < 0  # > DAMC_ADAM_MAX_TENSORS per table
    p = torch.nn.Parameter(torch.zeros(4))
    p.grad = torch.ones(4)
    with pytest.raises(_lib.DamcError):
        optim.Adam([p]).step()
    with pytest.raises(_lib.DamcError):
        optim.clip_grad_norm_([p], 1.0)
    with pytest.raises(NotImplementedError):
        optim.Adam([p], amsgrad=True)
    assert sorted(optim.AdamW([p]).defaults) == sorted(torch.optim.AdamW([p]).defaults)


def test_layer_sign_block_rule(monkeypatch):
    """gemm.h x3_conv_negk, through damc_x3_layer_sign_block (host only): the generator's UP2 limb weights take 1024-k
    sign blocks where 16 samples would already split 512-k blocks two per workgroup (every UP2 GEMM of the headline
    _netG_cifar10 ngf=128 and of _netG_celebaHQ), 512 for _netG_celeba64 ngf=128 and 256 for _netG_svhn ngf=64,
    whose batches fill the chip only with the finer split; by shape only; DAMC_X3_NEGK_RULE pins it."""
    from damc import _lib

    L = _lib.lib()

    def up2(cin, cout, hin):
        d = _lib.Layer()
        d.kind, d.cin, d.cout, d.k, d.stride, d.pad = _lib.LAYER_UP2, cin, cout, 4, 2, 1
        d.hin = d.win = hin
        d.hout = d.wout = 2 * hin
        return d

    def blocks(layers):
        return [(L.damc_x3_layer_sign_block(ctypes.byref(d), 0), L.damc_x3_layer_sign_block(ctypes.byref(d), 1))
                for d in layers]

    cifar = [up2(1024, 512, 8), up2(512, 256, 16)]
    svhn = [up2(512, 256, 4), up2(256, 128, 8)]
    celeba64 = [up2(1024, 512, 4), up2(512, 256, 8), up2(256, 128, 16)]
    hq = [up2(2048, 1024, 4), up2(1024, 512, 8), up2(512, 512, 16), up2(512, 256, 32), up2(256, 128, 64)]
    assert blocks(cifar) == [(1024, 1024)] * 2
    assert blocks(svhn) == [(256, 256)] * 2
    assert blocks(celeba64) == [(512, 512)] * 3
    assert blocks(hq) == [(1024, 1024)] * 5
    monkeypatch.setenv("DAMC_X3_NEGK_RULE", "512")
    assert blocks(cifar) == [(512, 512)] * 2
    monkeypatch.setenv("DAMC_X3_NEGK_RULE", "1024")
    assert blocks(svhn) == [(1024, 1024)] * 2
    monkeypatch.setenv("DAMC_X3_NEGK_RULE", "256")
    assert blocks(cifar) == [(256, 256)] * 2
    d = _lib.Layer()
    d.kind = _lib.LAYER_SMALLC
    assert L.damc_x3_layer_sign_block(ctypes.byref(d), 0) == 0


def test_round5_host_only_entry_points():
    """Host-side argument checks of the round-5 entry points (no kernel is launched): the E-update workspace is 0 for
    shapes the C side does not take (batch or widths not a multiple of 4), the glue / loss calls refuse NULL
    pointers and odd embedding widths."""
    from damc import _lib

    L = _lib.lib()
    e = _lib.Ebm()
    e.nz, e.nh, e.slope = 128, 200, 0.2
    assert L.damc_ebm_train_workspace_bytes(ctypes.byref(e), 128) == 0  # no weight pointers
    e.w1 = e.b1 = e.w2 = e.b2 = e.w3 = e.b3 = 256  # host-only size query: any non-null address
    assert L.damc_ebm_train_workspace_bytes(ctypes.byref(e), 128) > 0
    assert L.damc_ebm_train_workspace_bytes(ctypes.byref(e), 130) == 0
    e.nh = 202
    assert L.damc_ebm_train_workspace_bytes(ctypes.byref(e), 128) == 0
    assert L.damc_q_noise_glue(None, None, None, 128, 128, -5.1, 9.8, None, 128, None, None, None, None) == 1001
    assert L.damc_q_noise_glue(8, 8, 8, 128, 128, -5.1, 9.8, 8, 127, None, 8, 8, None) == 1001
    assert L.damc_q_loss_forward(None, None, 128, 128, None, None) == 1001
    assert L.damc_q_loss_backward(8, 8, 8, -1, 128, 128, 8, None) == 1001
    pe = _lib.PriorEmb()
    pe.nz, pe.nh, pe.nout, pe.slope = 128, 128, 1024, 0.01
    assert L.damc_prior_emb_train_workspace_bytes(ctypes.byref(pe), 128) == 0  # no weight pointers
    pe.w1 = pe.b1 = pe.w2 = pe.b2 = 256
    assert L.damc_prior_emb_train_workspace_bytes(ctypes.byref(pe), 128) > 0
    assert L.damc_prior_emb_train_workspace_bytes(ctypes.byref(pe), 130) == 0
    pe.slope = -0.1  # LReLU' is read from the activation's sign: negative slopes stay on the stock modules
    assert L.damc_prior_emb_train_workspace_bytes(ctypes.byref(pe), 128) == 0
    assert L.damc_prior_emb_train_forward(None, None, 128, None, None, None) == 1001


def test_optim_step_counters_with_a_fixed_subset_host_only():
    """damc.optim's step counters on CPU scalars (no kernel): when the same subset of a group's parameters has
    gradients every step, each parameter's count is the number of steps it took part in (torch's semantics), and
    the updated subset ends up sharing ONE counter private to it (the fast path of later steps)."""
    import torch

    from damc import optim

    ps = [torch.nn.Parameter(torch.zeros(2)) for _ in range(4)]
    opt = optim.AdamW(ps)
    group = opt.param_groups[0]

    def advance(active):
        for i, p in enumerate(ps):
            p.grad = torch.ones(2) if i in active else None
        steps = []
        for p in ps:
            if p.grad is None:
                continue
            st = opt.state[p]
            if not st:
                st["step"] = torch.tensor(0.0)
            steps.append(st["step"])
        return opt._advance_steps(group, steps)

    assert advance({0, 1, 2, 3}) == 1.0
    assert advance({0, 1, 2}) == 2.0
    assert advance({0, 1, 2}) == 3.0
    assert advance({0, 1, 2}) == 4.0
    assert [float(opt.state[p]["step"]) for p in ps] == [4.0, 4.0, 4.0, 1.0]
    shared = opt.state[ps[0]]["step"]
    assert opt.state[ps[1]]["step"] is shared and opt.state[ps[2]]["step"] is shared
    assert opt.state[ps[3]]["step"] is not shared
    assert advance({3}) == 2.0  # the left-out parameter keeps its own count
    assert [float(opt.state[p]["step"]) for p in ps] == [4.0, 4.0, 4.0, 2.0]
    assert advance({0, 1, 2, 3}) is None  # counts differ: one launch per value (the caller's slow path)


def test_grad_buffers_and_ebm_eligibility_host_only():
    """training._grad_buffers: one fp32 allocation, a view per needed parameter with its shape, 16-B aligned starts,
    None where no gradient is needed; training._ebm_layers accepts _netE's default topology only."""
    import torch

    from damc import training
    from src import diffusion_net as dn

    params = [torch.zeros(3, 5), torch.zeros(7), torch.zeros(2, 2), torch.zeros(6)]
    out = training._grad_buffers(params, [True, False, True, True])
    assert out[1] is None
    assert [tuple(t.shape) for t in out if t is not None] == [(3, 5), (2, 2), (6,)]
    base = out[0].untyped_storage().data_ptr()
    assert all(t.untyped_storage().data_ptr() == base and (t.data_ptr() - base) % 16 == 0 for t in out if t is not None)
    assert all(t.is_contiguous() for t in out if t is not None)
    assert training._grad_buffers(params, [False] * 4) == [None] * 4
    assert training._ebm_layers(dn._netE(nz=128)) is not None
    assert training._ebm_layers(dn._netE(nz=128, nez=2)) is None
    assert training._ebm_layers(dn._netE(nz=128, e_sn=True)) is None
