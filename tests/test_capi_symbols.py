"""CPU-side checks of the C-ABI boundary (no GPU, no compute calls).

- libplantos_hip.so loads and exports every function include/*.h declares;
- the ctypes layer (plantos_amd._capi) binds exactly that set;
- struct layout of pe_config agrees between C and ctypes;
- without a usable device, the product path fails loudly (no CPU fallback).
"""
import ctypes
import glob
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(glob.glob(os.path.join(REPO, "include", "*.h")))
DECL = re.compile(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(pe_[a-z0-9_]+)\s*\(", re.M)


def declared():
    names = []
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += DECL.findall(src)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib_path():
    from plantos_amd import _capi
    if not os.path.exists(_capi.LIB_PATH):
        subprocess.run(["python", os.path.join(REPO, "rl-env_amd", "build.py")], check=True)
    return _capi.LIB_PATH


def test_headers_declare_the_boundary():
    names = declared()
    for must in ("pe_create", "pe_reset", "pe_step", "pe_get_state", "pe_set_state", "pe_destroy",
                 "pe_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    L = ctypes.CDLL(lib_path)
    for n in declared():
        assert hasattr(L, n), n


def test_ctypes_binding_matches_header(lib_path):
    from plantos_amd import _capi
    assert sorted(_capi.EXPORTS) == declared()
    L = _capi.lib()
    for n in _capi.EXPORTS:
        assert getattr(L, n).restype is not None or n == "pe_default_config"


def test_config_struct_layout(lib_path):
    """pe_default_config writes the reference defaults (plantos_env.py:25-27,76-83,120)
    through the C struct; pe_obs_dim = 5C+27 (plantos_env.py:55-57)."""
    from plantos_amd import _capi
    c = _capi.default_config(20, 10, 12, 6, 16)
    assert (c.abi_version, c.grid_size, c.num_plants, c.num_obstacles, c.lidar_range,
            c.lidar_channels) == (_capi.PE_ABI_VERSION, 20, 10, 12, 6, 16)
    assert c.max_steps == 1000 and c.autoreset == 1
    assert c.thirsty_plant_prob == 0.7
    assert (c.r_goal, c.r_mistake, c.r_invalid, c.r_water_empty) == (20, -10, -5, -5)
    assert (c.r_step, c.r_exploration, c.r_revisit, c.r_complete) == (-0.1, 10, -1, 50)
    assert _capi.lib().pe_obs_dim(ctypes.byref(c)) == 107


def test_config_struct_matches_c_compiler(tmp_path):
    """sizeof/offsetof of pe_config from gcc on include/plantos_batch.h == ctypes."""
    from plantos_amd import _capi
    fields = [f[0] for f in _capi.PEConfig._fields_]
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "plantos_batch.h"', "int main(void){",
           'printf("%zu\\n", sizeof(pe_config));']
    src += [f'printf("%zu\\n", offsetof(pe_config, {f}));' for f in fields]
    src += ["return 0;}"]
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(c)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(_capi.PEConfig)
    for f, off in zip(fields, vals[1:]):
        assert getattr(_capi.PEConfig, f).offset == off, f


def test_no_cpu_fallback_without_device(lib_path):
    """pe_create must fail with PE_ERR_DEVICE (or ARG) rather than run on the host."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from plantos_amd import _capi
    c = _capi.default_config(20, 10, 12, 6, 16)
    h = ctypes.c_void_p()
    rc = _capi.lib().pe_create(ctypes.byref(c), 0, 64, ctypes.byref(h))
    assert rc == _capi.PE_ERR_DEVICE
    assert b"no HIP device" in _capi.lib().pe_last_error()
    from plantos_amd import PlantOSBatch
    with pytest.raises(Exception):
        PlantOSBatch(64, device="cpu")
