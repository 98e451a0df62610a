import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"
SCENES = ROOT / "scenes"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")


@pytest.fixture(scope="session")
def golden():
    import json
    return json.loads((GOLDEN / "reference_components.json").read_text())


@pytest.fixture(scope="session")
def pa():
    import pbrt_amd
    return pbrt_amd


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(autouse=True)
def _oracle_math_mode():
    """Every test -- GPU parity included -- sees the oracle in its libm mode: glibc's float
    transcendentals, as pbrt's CPU build calls them, in which the component tests pin it to the
    reference's goldens.  The device kernels' core/detmath.h restates those functions bit for bit
    (tools/detmath_exhaustive.cpp), so no separate device-math mode exists any more."""
    import pyoracle
    pyoracle.set_math_mode(pyoracle.MATH_LIBM)
    yield
    pyoracle.set_math_mode(pyoracle.MATH_LIBM)


def fl(v):
    """golden JSON floats ('inf'/'nan' strings) -> float"""
    if isinstance(v, list):
        return [fl(x) for x in v]
    return float(v)


def cornell_with_sampler(pa, sampler_line, **overrides):
    """The Cornell scene with its Sampler directive replaced (e.g. a zsobol configuration)."""
    text = (SCENES / "cornell-box.pbrt").read_text()
    lines = [sampler_line if ln.startswith("Sampler ") else ln for ln in text.splitlines()]
    return pa.Scene.from_string("\n".join(lines) + "\n", SCENES, **overrides)
