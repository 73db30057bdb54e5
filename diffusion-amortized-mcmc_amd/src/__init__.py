"""Drop-in replacement for the reference package ``workspace/src`` (MI355X HIP path).

``MCMC``, ``diffusion_net`` and ``diffusion_helper_func`` come from this directory.  The
reference's ``src`` is a namespace package (no __init__.py), so with this directory on
PYTHONPATH ``import src`` resolves here even when the reference workspace is the current
directory; extending ``__path__`` lets the reference's other modules (``src.utils``,
``src.stylegan``, ``src.diffusion_net_stylegan`` — outside the hot path) still import from any
other ``src`` directory on sys.path.  See INTEGRATION.md.
"""
import pkgutil

__path__ = pkgutil.extend_path(__path__, __name__)
