"""CPU: libdamc.so loads and exports every entry point include/damc.h declares (no compute calls)."""
import ctypes
import os
import re

from conftest import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "damc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(damc_[a-z0-9_]+)\s*\(", src)))


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
    assert L.damc_abi_version() == 1
    assert b"invalid" in L.damc_error_string(1001)
    # descriptor validation runs on the host: an empty generator has no workspace
    g = _lib.Generator()
    assert L.damc_posterior_workspace_bytes(ctypes.byref(g), 8) == 0
