"""The C-ABI library loads and exports every symbol include/psim.h declares.

CPU-only: no compute call is made without a GPU; psim_create must fail
loudly (PSIM_ENODEV) when no device is visible.
"""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "psim.h")
LIB = os.path.join(ROOT, "partisan_amd", "libpsim.so")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(psim_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("psim_create", "psim_destroy", "psim_load_csr", "psim_plumtree_broadcast", "psim_run",
              "psim_step", "psim_get_plumtree", "psim_strerror"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "libpsim.so not built (run __graft_entry__.build())"
    L = C.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_library_has_no_undefined_internal_symbols():
    """Every psim:: function the library calls is defined in it (a declaration
    matching a definition hidden in an anonymous namespace links as a shared
    object and only fails at load or first call)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", LIB], capture_output=True, text=True, check=True).stdout
    assert not [l for l in out.splitlines() if "psim" in l.lower()], out


def test_python_binding_covers_header():
    from partisan_amd._lib import SIGNATURES
    assert sorted(SIGNATURES) == declared_symbols()


def test_strerror_names_codes():
    from partisan_amd._lib import lib
    assert lib().psim_strerror(0) == b"ok"
    assert lib().psim_strerror(-8) == b"no usable HIP device"
    assert lib().psim_strerror(-7) == b"previous broadcast not quiescent"


def test_create_rejects_bad_abi_version():
    from partisan_amd._lib import Config, lib
    cfg = Config(abi_version=999, device=-1, lazy_tick_rounds=1)
    h = C.c_void_p()
    assert lib().psim_create(C.byref(cfg), C.byref(h)) != 0


def _gpu_visible():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-device path")
def test_no_device_fails_loudly():
    from partisan_amd import PsimError, Simulator
    with pytest.raises(PsimError) as ei:
        Simulator()
    assert ei.value.name == "PSIM_ENODEV"


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "partisan_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert "pyoracle" not in src and "liboracle" not in src and "oracle.h" not in src, f


def test_nif_shim_typechecks():
    """erl/c_src/partisan_gpu_sim_nif.c against include/psim.h (erl_nif.h is a
    declarations-only stand-in: this image has no erts)."""
    import subprocess
    src = os.path.join(ROOT, "erl", "c_src", "partisan_gpu_sim_nif.c")
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-std=c11",
                        "-I" + os.path.join(ROOT, "tests", "nif_mock"), "-I" + os.path.join(ROOT, "include"), src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_nif_calls_only_declared_symbols():
    import re
    hdr = open(os.path.join(ROOT, "include", "psim.h")).read()
    declared = set(re.findall(r"\b(psim_\w+)\s*\(", hdr))
    nif = open(os.path.join(ROOT, "erl", "c_src", "partisan_gpu_sim_nif.c")).read()
    used = set(re.findall(r"\b(psim_\w+)\s*\(", nif))
    assert used and used <= declared, used - declared


def test_erlang_stubs_cover_the_nif_table():
    """Every entry of the shim's ErlNifFunc table has an exported stub of the
    same arity in erl/src/partisan_gpu_sim.erl (what erlang:load_nif/2
    requires), and the behaviour adapters export every callback of the
    reference behaviours (src/partisan_membership_strategy.erl:55-77,
    src/partisan_plumtree_broadcast_handler.erl:47-78)."""
    nif = open(os.path.join(ROOT, "erl", "c_src", "partisan_gpu_sim_nif.c")).read()
    table = set(re.findall(r'\{"(\w+)", (\d+), nif_\w+,', nif))
    erl = open(os.path.join(ROOT, "erl", "src", "partisan_gpu_sim.erl")).read()
    exports = set()
    for block in re.findall(r"-export\(\[(.*?)\]\)\.", erl, re.S):
        exports |= {tuple(x.strip().split("/")) for x in block.split(",") if "/" in x}
    assert table, "no NIF table parsed"
    missing = {(f, a) for f, a in table if (f, a) not in exports}
    assert not missing, missing
    for f, _a in table:
        assert re.search(rf"^{f}\(" + r"[^)]*\) ->\s*erlang:nif_error", erl, re.M), f
    def exported(path):
        src = open(os.path.join(ROOT, "erl", "src", path)).read()
        out = set()
        for block in re.findall(r"-export\(\[(.*?)\]\)\.", src, re.S):
            out |= {x.strip() for x in block.split(",")}
        return src, out
    src, ex = exported("partisan_gpu_sim_membership_strategy.erl")
    assert "-behaviour(partisan_membership_strategy)." in src
    assert {"init/1", "join/3", "leave/2", "compare/2", "periodic/1", "prune/2", "handle_message/2"} <= ex
    src, ex = exported("partisan_gpu_sim_plumtree_handler.erl")
    assert "-behaviour(partisan_plumtree_broadcast_handler)." in src
    assert {"broadcast_data/1", "broadcast_channel/0", "merge/2", "is_stale/1", "graft/1", "exchange/1"} <= ex
