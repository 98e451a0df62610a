"""C ABI surface: the library loads without a GPU, exports every entry point declared in
include/pbrt_amd.h (the renderer API) and include/pbrt_amd_debug.h (component entry points for
tests and tools), and the loader fails loudly on unsupported input (pbrt's ErrorExit)."""
import ctypes
import re

import pytest

from conftest import ROOT, SCENES


def header_symbols(names=("pbrt_amd.h", "pbrt_amd_debug.h")):
    text = "".join((ROOT / "include" / n).read_text() for n in names)
    return sorted(set(re.findall(r"\b(pbrt_[a-z0-9_]+)\s*\(", text)))


def test_renderer_header_has_no_debug_entry_points():
    assert not [s for s in header_symbols(("pbrt_amd.h",)) if s.startswith("pbrt_debug_")]


def test_header_declares_python_symbol_list(pa):
    assert header_symbols() == sorted(pa.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(pa):
    lib = pa._lib()
    for name in header_symbols():
        assert hasattr(lib, name), name


def test_scene_info_cornell(pa):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")
    i = sc.info
    assert (i.xres, i.yres, i.spp, i.max_depth, i.seed) == (256, 256, 16, 5, 0)
    assert i.n_triangles == 32 and i.n_area_lights == 2 and i.n_light_nodes == 3
    assert i.uniform_light_sampler == 0
    assert (i.filter_radius_x, i.filter_radius_y) == (0.5, 0.5)


def test_overrides(pa):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=64, seed=3,
                       pixelbounds="10,20,30,40")
    i = sc.info
    assert (i.xres, i.yres, i.spp, i.seed) == (1280, 720, 64, 3)
    assert (i.px0, i.px1, i.py0, i.py1) == (10, 20, 30, 40)


@pytest.mark.parametrize("text,msg", [
    ('WorldBegin\nShape "hyperboloid"\n', "not supported"),
    ('WorldBegin\nFoo 1 2 3\n', "unknown directive"),
    ('Sampler "pmj02bn"\nWorldBegin\nAttributeBegin\nAreaLightSource "diffuse"\nShape "trianglemesh" "point3 P" [0 0 0 1 0 0 0 1 0]\nAttributeEnd\n', "not supported"),
    ('Sampler "halton"\nWorldBegin\nShape "trianglemesh" "point3 P" [0 0 0 1 0 0 0 1 0]\n', "No light sources"),
    ('WorldBegin\nMaterial "diffuse" "rgb reflectance" [2 0 0]\n', "[0,1]"),
])
def test_loader_fails_loudly(pa, text, msg):
    with pytest.raises(pa.PbrtError, match=re.escape(msg)):
        pa.Scene.from_string(text)


def test_single_light_uses_uniform_sampler(pa):
    text = ('Sampler "halton"\nWorldBegin\nAttributeBegin\nAreaLightSource "diffuse" "rgb L" [1 1 1]\n'
            'Shape "trianglemesh" "point3 P" [0 0 0 1 0 0 0 1 0]\nAttributeEnd\n')
    sc = pa.Scene.from_string(text)
    assert sc.info.uniform_light_sampler == 1


def test_missing_library_is_an_error(pa, monkeypatch, tmp_path):
    monkeypatch.setattr(pa, "_LIB", None)
    monkeypatch.setattr(pa, "LIB_PATH", tmp_path / "nope.so")
    with pytest.raises(pa.PbrtError, match="no CPU fallback"):
        pa._lib()
