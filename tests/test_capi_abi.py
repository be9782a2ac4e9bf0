"""The C-ABI library loads and exports every entry point include/swarmrl_amd.h
declares (no device calls: runs without a GPU)."""

import ctypes
import re

from conftest import ROOT


def _declared_functions():
    text = (ROOT / "include" / "swarmrl_amd.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(swarm_[a-z_]+)\s*\(", text)))


def test_header_declares_expected_api():
    names = _declared_functions()
    for must in ["swarm_engine_create", "swarm_engine_integrate", "swarm_vision_cone",
                 "swarm_field_distance", "swarm_engine_remove_overlap"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    import __graft_entry__ as g

    if not g.HIP_LIB.exists():
        g.build()
    lib = ctypes.CDLL(str(g.HIP_LIB))
    missing = [n for n in _declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from swarmrl_amd import _capi

    assert set(_declared_functions()) == set(_capi.exported_symbols())


def test_params_struct_layout_matches_oracle():
    from oracle import oracle
    from swarmrl_amd import _capi

    assert ctypes.sizeof(_capi.SwarmParams) == ctypes.sizeof(oracle.Params)
    for (n1, t1), (n2, t2) in zip(_capi.SwarmParams._fields_, oracle.Params._fields_):
        assert n1 == n2 and ctypes.sizeof(t1) == ctypes.sizeof(t2)
