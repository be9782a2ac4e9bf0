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


def _header_struct_fields(name):
    """Member names of `typedef struct ... } name;` in include/swarmrl_amd.h."""
    text = (ROOT / "include" / "swarmrl_amd.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    body = re.search(r"typedef struct[^{]*\{([^}]*)\}\s*" + name + r"\s*;", text).group(1)
    return re.findall(r"\b([A-Za-z_0-9]+)\s*(?:\[[^\]]*\])?\s*;", body)


def test_params_struct_matches_header():
    from swarmrl_amd import _capi

    assert [n for n, _ in _capi.SwarmParams._fields_] == _header_struct_fields("swarm_params_t")


def test_integration_sketch_matches_binding():
    """INTEGRATION.md's maintainer sketch (the reference-side ctypes stub)
    declares swarm_params_t exactly as the binding does, and creates the
    engine with reuse_forces = 1 -- the reference's
    integrator.run(k, reuse_forces=True) (espresso.py:1304-1306)."""
    from swarmrl_amd import _capi

    text = (ROOT / "INTEGRATION.md").read_text()
    block = next(b for b in re.findall(r"```python\n(.*?)```", text, flags=re.S)
                 if "class SwarmParams" in b)
    cls = re.search(r"class SwarmParams\(ctypes\.Structure\):.*?\n\n", block, flags=re.S).group(0)
    ns = {"ctypes": ctypes}
    exec(cls, ns)  # the sketch's struct definition only (no library calls)
    sketch = ns["SwarmParams"]
    assert [n for n, _ in sketch._fields_] == [n for n, _ in _capi.SwarmParams._fields_]
    for (n, t1), (_, t2) in zip(sketch._fields_, _capi.SwarmParams._fields_):
        assert ctypes.sizeof(t1) == ctypes.sizeof(t2), n
    assert ctypes.sizeof(sketch) == ctypes.sizeof(_capi.SwarmParams)
    create = re.search(r"p = SwarmParams\((.*?)\)\n", block, flags=re.S).group(1)
    assert re.search(r"\breuse_forces\s*=\s*1\b", create)


def test_lib_env_selects_the_library(tmp_path):
    """SWARMRL_AMD_LIB points the binding at another build of the same
    library (read once, when swarmrl_amd._capi is imported)."""
    import subprocess
    import sys

    code = ("import swarmrl_amd._capi as c, sys; "
            "sys.stdout.write(str(c._LIB_PATH))")
    alt = tmp_path / "libswarmrl_amd_alt.so"
    env = dict(__import__("os").environ, SWARMRL_AMD_LIB=str(alt))
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=str(ROOT),
                         capture_output=True, text=True, check=True).stdout
    assert out == str(alt)


def test_library_build_id_matches_the_sources():
    """swarm_build_id: the library was compiled from the checkout's HIP
    sources and header (the hash __graft_entry__.build compiles in)."""
    import __graft_entry__ as g

    if not g.HIP_LIB.exists():
        g.build()
    lib = ctypes.CDLL(str(g.HIP_LIB))
    lib.swarm_build_id.restype = ctypes.c_char_p
    from swarmrl_amd import _capi

    assert lib.swarm_build_id().decode() == _capi.source_hash() == g._source_hash()
