"""Drop-in for workspace/src/diffusion_helper_func.py: the latent-diffusion schedule algebra.

These tensor helpers are used by the training loss (``_netQ_U.calculate_loss``).  The reverse
sweep on the HIP path evaluates the same formulas once per step on the host
(``damc.amortizer.step_coefficients``) and fuses them into the denoiser's epilogue.
"""
import math

import torch
import torch.nn.functional as F

_LOG2 = math.log(2.0)


class log1mexp(torch.autograd.Function):
    """log(1 - exp(-x)) for x > 0, numerically stable branch at log 2 (diffusion_helper_func.py:9-32)."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.where(x > _LOG2, torch.log1p(-torch.exp(-x)), torch.log(-torch.expm1(-x)))

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g / torch.expm1(x)


mylog1mexp = log1mexp.apply


def pred_x_from_eps(z, eps, logsnr):
    """x0 = sqrt(1 + e^-l) (z - eps / sqrt(1 + e^l))  (:36-39)."""
    return torch.sqrt(1.0 + torch.exp(-logsnr)) * (z - eps * torch.rsqrt(1.0 + torch.exp(logsnr)))


def logsnr_schedule_fn(t, logsnr_min=-20, logsnr_max=20):
    """Cosine-style schedule l(t) = -2 log tan(a t + b), l(0) = logsnr_max, l(1) = logsnr_min (:41-50)."""
    lmin = logsnr_min * torch.ones_like(t)
    lmax = logsnr_max * torch.ones_like(t)
    b = torch.arctan(torch.exp(-0.5 * lmax))
    a = torch.arctan(torch.exp(-0.5 * lmin)) - b
    return -2.0 * torch.log(torch.tan(a * t + b))


def diffusion_reverse(x, z_t, logsnr_s, logsnr_t, pred_var_type="small"):
    """Posterior q(z_s | z_t, x) for s < t (:52-70)."""
    alpha_st = torch.sqrt((1.0 + torch.exp(-logsnr_t)) / (1.0 + torch.exp(-logsnr_s)))
    alpha_s = torch.sqrt(torch.sigmoid(logsnr_s))
    r = torch.exp(logsnr_t - logsnr_s)
    one_minus_r = -torch.expm1(logsnr_t - logsnr_s)
    log_one_minus_r = mylog1mexp(logsnr_s - logsnr_t)
    mean = r * alpha_st * z_t + one_minus_r * alpha_s * x
    if pred_var_type == "large":
        var = one_minus_r * torch.sigmoid(-logsnr_t)
        logvar = log_one_minus_r + torch.log(torch.sigmoid(-logsnr_t))
    elif pred_var_type == "small":
        a_t, a_s = torch.sigmoid(logsnr_t), torch.sigmoid(logsnr_s)
        var = (1.0 - a_s) / (1.0 - a_t) * (1 - a_t / a_s)
        logvar = torch.log(var)
    else:
        raise NotImplementedError(pred_var_type)
    return {"mean": mean, "std": torch.sqrt(var), "var": var, "logvar": logvar}


def diffusion_forward(x, logsnr):
    """q(z_t | x) (:72-78)."""
    var = torch.sigmoid(-logsnr)
    return {"mean": x * torch.sqrt(torch.sigmoid(logsnr)), "std": torch.sqrt(var), "var": var, "logvar": torch.log(var)}


def denoise_true(z, x0, logsnr_t, logsnr_tminus1):
    """Ancestral step with the 'small' variance (:80-87, unused by the drivers)."""
    n = len(z)
    dist = diffusion_reverse(x=x0, z_t=z, logsnr_s=logsnr_tminus1.reshape(n, 1), logsnr_t=logsnr_t.reshape(n, 1))
    a_t, a_s = F.sigmoid(logsnr_t), F.sigmoid(logsnr_tminus1)
    std = torch.sqrt((1.0 - a_s) / (1.0 - a_t) * (1 - a_t / a_s)).reshape(n, 1)
    return dist["mean"] + std * torch.randn_like(z)
