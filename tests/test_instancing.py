"""Object instancing (ObjectBegin / ObjectEnd / ObjectInstance, scene.cpp:309-395): instances
are flattened into render-space triangles.  An instanced scene must load to exactly the
triangles of the same geometry written out explicitly (same transforms composed), and render
identically on the oracle (GPU parity: test_gpu_parity.py)."""
import numpy as np
import pytest

from conftest import SCENES

HEAD = """LookAt 0 0 -6  0 0 0  0 1 0
Camera "perspective" "float fov" [ 40 ]
Film "rgb" "integer xresolution" [ 32 ] "integer yresolution" [ 32 ]
Sampler "halton" "integer pixelsamples" [ 4 ]
WorldBegin
LightSource "infinite" "rgb L" [ 0.5 0.5 0.5 ]
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [ 4 4 4 ]
  Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ] "point3 P" [ -1 3 -1  1 3 -1  1 3 1  -1 3 1 ]
AttributeEnd
"""
TRI = 'Shape "trianglemesh" "integer indices" [ 0 1 2 ] "point3 P" [ 0 0 0  1 0 0  0 1 0.5 ]'


def tris(sc):
    f = sc.flat()
    v = np.ctypeslib.as_array(f.vertices, shape=(f.n_vertices, 3))
    t = np.ctypeslib.as_array(f.triangles, shape=(f.n_triangles, 3))
    return v[t]


def test_instances_equal_explicit_geometry(pa):
    inst = HEAD + f"""
ObjectBegin "thing"
  Material "diffuse" "rgb reflectance" [ 0.2 0.5 0.8 ]
  Translate 0.25 0 0
  {TRI}
ObjectEnd
AttributeBegin Translate -1 0 0  Rotate 30 0 0 1  ObjectInstance "thing" AttributeEnd
AttributeBegin Translate 1 -0.5 0.5  Scale 1 -1 1  ObjectInstance "thing" AttributeEnd
"""
    expl = HEAD + f"""
AttributeBegin
  Material "diffuse" "rgb reflectance" [ 0.2 0.5 0.8 ]
  AttributeBegin Translate -1 0 0  Rotate 30 0 0 1  Translate 0.25 0 0  {TRI} AttributeEnd
  AttributeBegin Translate 1 -0.5 0.5  Scale 1 -1 1  Translate 0.25 0 0  {TRI} AttributeEnd
AttributeEnd
"""
    a = pa.Scene.from_string(inst, SCENES)
    b = pa.Scene.from_string(expl, SCENES)
    np.testing.assert_array_equal(tris(a), tris(b))
    fa, fb = a.flat(), b.flat()
    n = fa.n_triangles
    np.testing.assert_array_equal(np.ctypeslib.as_array(fa.tri_flip, shape=(n,)),
                                  np.ctypeslib.as_array(fb.tri_flip, shape=(n,)))  # Scale -1: handedness


def test_instance_use_before_definition(pa):
    text = HEAD + f'ObjectInstance "later"\nObjectBegin "later"\n  {TRI}\nObjectEnd\n'
    assert pa.Scene.from_string(text, SCENES).info.n_triangles == 3


@pytest.mark.parametrize("bad,msg", [
    ('ObjectInstance "nope"', "not defined"),
    ('ObjectBegin "a"\nObjectBegin "b"\nObjectEnd\nObjectEnd', "inside of instance definition"),
    ('ObjectEnd', "outside of instance definition"),
    ('ObjectBegin "a"\nObjectEnd\nObjectBegin "a"\nObjectEnd', "redefine"),
])
def test_instancing_errors(pa, bad, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(HEAD + bad + "\n", SCENES)


def test_instanced_render_equals_explicit_on_oracle(pa, oracle):
    inst = HEAD + f"""
ObjectBegin "thing"
  Material "diffuse" "rgb reflectance" [ 0.7 0.5 0.3 ]
  {TRI}
ObjectEnd
AttributeBegin Translate -0.5 -0.5 0  ObjectInstance "thing" AttributeEnd
AttributeBegin Translate 0.2 0 -0.3  Rotate 60 0 1 0  ObjectInstance "thing" AttributeEnd
"""
    expl = HEAD + f"""
Material "diffuse" "rgb reflectance" [ 0.7 0.5 0.3 ]
AttributeBegin Translate -0.5 -0.5 0  {TRI} AttributeEnd
AttributeBegin Translate 0.2 0 -0.3  Rotate 60 0 1 0  {TRI} AttributeEnd
"""
    a = oracle.render(pa.Scene.from_string(inst, SCENES), threads=8)
    b = oracle.render(pa.Scene.from_string(expl, SCENES), threads=8)
    np.testing.assert_array_equal(a, b)
