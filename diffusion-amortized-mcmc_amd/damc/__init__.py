"""damc — MI355X-native diffusion-amortized Langevin inner loop (HIP/gfx950 via libdamc.so).

Public API (tensor level); the reference-compatible call surface lives in the sibling
``src`` package (src/MCMC.py, src/diffusion_net.py) and forwards here.
"""
from . import synth  # noqa: F401  (pure numpy, importable without a GPU)
from ._lib import DamcError, EXPORTED_SYMBOLS, LIB_PATH, lib  # noqa: F401

__all__ = ["DamcError", "lib", "LIB_PATH", "EXPORTED_SYMBOLS", "synth"]


def __getattr__(name):
    # lazy: torch-dependent modules load on first use
    if name in ("langevin", "plans", "amortizer", "dist"):
        import importlib

        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
