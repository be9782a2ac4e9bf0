"""
Driver entry points.

build(): compile the HIP engine for gfx950 into swarmrl_amd/libswarmrl_amd.so
         (in-tree, travels with the repo snapshot), build the CPU oracle
         (test infrastructure) and import the package.
smoke(): one small rollout on cuda:0 through the product API, checked bit for
         bit against the CPU oracle.
"""

import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent
HIP_SRC = ROOT / "swarmrl_amd" / "csrc" / "swarm_engine.hip"
HIP_LIB = ROOT / "swarmrl_amd" / "libswarmrl_amd.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-ffp-contract=off",  # fixed fp32 operation order (number formats)
    "-Wall",
]


def build() -> None:
    cmd = [HIPCC, *HIP_FLAGS, "-o", str(HIP_LIB), str(HIP_SRC)]
    subprocess.run(cmd, check=True, cwd=ROOT)
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    # test-only device-math probe (tests/csrc), same compiler flags
    selftest = ROOT / "tests" / "csrc" / "devmath_selftest.hip"
    subprocess.run([HIPCC, *HIP_FLAGS, "-o", str(ROOT / "tests" / "csrc" / "libdevmath.so"),
                    str(selftest)], check=True, cwd=ROOT)
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    import swarmrl_amd  # noqa: F401
    from swarmrl_amd import _capi

    _capi.lib()  # the library loads and resolves every declared symbol


def smoke() -> None:
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    import numpy as np
    import torch

    from oracle import oracle
    from swarmrl_amd import _capi
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.engine import MDParams, SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    _capi.require_gpu()
    torch.cuda.set_device(0)
    ureg = UnitRegistry()
    params = MDParams(
        ureg=ureg,
        box_length=ureg.Quantity([40.0, 40.0, 40.0], "micrometer"),
        time_step=ureg.Quantity(1e-3, "second"),
        time_slice=ureg.Quantity(1e-2, "second"),
        write_interval=ureg.Quantity(1e-2, "second"),
    )
    eng = SwarmEngine(params, n_dims=2, seed=7, out_folder="/tmp/swarm_smoke")
    eng.add_colloids(48, ureg.Quantity(1.0, "micrometer"),
                     ureg.Quantity(np.array([20.0, 20.0, 0.0]), "micrometer"),
                     ureg.Quantity(12.0, "micrometer"))
    pos0 = np.stack(eng._pos[0])
    dir0 = np.stack(eng._dir[0])
    eng.integrate(2, ForceFunction({"0": dummy_models.ConstForce(5.0)}))
    got = eng.get_raw_state()

    key = eng._species_keys[0]
    p = oracle.make_params(eng._box, eng._time_step, eng._kT(),
                           params.WCA_epsilon.m_as("sim_energy"), 7, [key])
    st = oracle.state_from_positions(pos0, dir0, eng._box)
    sp = np.zeros(48, np.uint8)
    st, _ = oracle.sd_run(p, st, sp, 1000)
    # reuse_forces (the engine's default, espresso.py:1304-1306): the first
    # sub-step swims with the forces of the last force calculation -- the
    # overlap removal's, with no swim force yet
    st, _, _ = oracle.bd_run(p, st, sp, np.full(48, 5.0, np.float32), np.zeros(48, np.float32),
                             eng.params.steps_per_slice * 2,
                             prev={"f": np.zeros(48), "t": np.zeros(48), "ang": st["ang"]})
    for k in ("q", "img", "ang"):
        if not np.array_equal(got[k], st[k]):
            raise AssertionError(f"smoke: HIP engine and CPU oracle differ in {k}")
    print("smoke: HIP engine == CPU oracle (bit-exact), 48 colloids, 20 BD steps")


if __name__ == "__main__":
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "smoke":
        smoke()
