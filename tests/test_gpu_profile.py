"""Per-stage kernel profile (ReportKernelStats analogue, gpu/util.cpp:128-246)."""
import io

import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu


def test_kernel_profile_reports_every_stage(pa):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=64, yresolution=48, spp=4)
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 20)
    integ.set_kernel_profiling(True)
    integ.render()
    integ.synchronize()
    ks = {k["description"]: k for k in integ.kernel_stats()}
    depth = sc.info.max_depth
    assert ks["Generate camera rays (k_camera)"]["launches"] == 1
    assert ks["Tracing closest hit rays (k_closest)"]["launches"] == depth + 1
    assert ks["Tracing shadow rays (k_shadow)"]["launches"] == depth
    assert ks["Evaluate materials/BSDFs for DiffuseMaterial (k_shade_diffuse)"]["launches"] == depth
    assert ks["Update film (k_film)"]["launches"] == 1
    for k in ks.values():
        assert 0 < k["min_ms"] <= k["total_ms"] / k["launches"] <= k["max_ms"]
    buf = io.StringIO()
    integ.report_kernel_stats(buf)
    assert "Wavefront Kernel Profile:" in buf.getvalue() and "Total rendering time" in buf.getvalue()
    # a second render accumulates; reset clears
    integ.render()
    integ.synchronize()
    assert {k["description"]: k for k in integ.kernel_stats()}["Update film (k_film)"]["launches"] == 2
    integ.reset_stats()
    assert integ.kernel_stats() == []

