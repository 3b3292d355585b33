"""CPU-side checks of the C ABI: the in-tree library loads and exports every symbol
include/heist.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os

import pytest

from heist_amd import _build, _native


def test_library_built_and_loads():
    if _build.needs_build():
        _build.build()
    lib = _native.lib()
    assert lib.heist_abi_version() == 5


def test_every_header_symbol_is_exported():
    names = _native.header_functions()
    assert len(names) >= 15
    lib = ctypes.CDLL(_build.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and every binding signature refers to a declared function
    assert set(_native.SIGNATURES) == set(names)


def test_argument_validation_without_device():
    """Bad sizes fail with HEIST_EINVAL before any device work."""
    lib = _native.lib()
    h = ctypes.c_void_p()
    consts = (ctypes.c_double * 3)(-0.01, -1.0, 10.0)
    rc = lib.heist_create(2, 2, 200, 0, 0, 1, 1, consts, 4, 2, 2, 8, ctypes.byref(h))
    assert rc == 100000 and b"rows" in lib.heist_last_error()
    rc = lib.heist_ppo_loss(None, None, None, None, None, None, 0, 5, 0.2, 0.5, 0.05, None, None, None, None, None)
    assert rc == 100000


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from heist_amd import HeistEnv
    with pytest.raises(_native.HeistError):
        HeistEnv(4)


def test_env_build_keeps_slp_workaround():
    """heist_env.hip builds with -fno-slp-vectorize: ROCm 7.2 clang's packed-fp32 forms of the
    fast raycast were miscompiled (tools/forensic/slp_check.sh runs the parity tests on a
    build without the flag and records what it finds, profiles/r04*_slp_*)."""
    import os
    from heist_amd import _build
    if "HEIST_ENV_FLAGS" in os.environ:
        return  # an explicit A/B build
    assert "-fno-slp-vectorize" in _build.FILE_FLAGS["heist_env.hip"]
