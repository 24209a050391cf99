import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; calls the HIP library")
    config.addinivalue_line("markers", "spawns_gpu_procs: starts GPU processes; runs before this process "
                                       "touches the GPU")


def pytest_collection_modifyitems(config, items):
    """Tests that start GPU processes run first: no process is ever started from a
    pytest process that has already initialised the GPU."""
    first = [i for i in items if i.get_closest_marker("spawns_gpu_procs")]
    items[:] = first + [i for i in items if not i.get_closest_marker("spawns_gpu_procs")]


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    """One HIP context for the GPU tests (fails loudly if the extension or the GPU
    is missing — there is no fallback)."""
    from rbe550_final_project_amd import build, model
    from rbe550_final_project_amd.native import Context
    build.build(verbose=False)
    ctx = Context(device=0, robot=model.robot_desc())
    yield ctx
    ctx.close()
