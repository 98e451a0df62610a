"""BVHLightSampler construction (lightsamplers.cpp:109-238) pinned to the reference's own code:
tests/golden/reference_components.json["light_bvh"] holds the trees that the unmodified
lightsamplers.cpp buildBVH produced (oracle/ref/refgold.cpp) over synthetic LightBounds --
degenerate boxes, identical centroids, planar and point-only sets, zero-power lights.  The
loader's builder (csrc/host/build.cpp) and the oracle's independent restatement (oracle.cpp
lbvh) must reproduce every node (decoded CompactLightBounds, child / light index, leaf flag)
and every bit trail bit for bit; on real scenes the two must agree node for node, so the
oracle no longer consumes the product's light tree."""
import numpy as np
import pytest

from conftest import SCENES, fl


def _golden_cases(golden):
    for c in golden["light_bvh"]:
        lights = np.array([fl(r) for r in c["lights"]], np.float32)
        nodes = np.array([fl(n["decoded"]) for n in c["nodes"]], np.float32).reshape(-1, 12)
        info = np.array([[n["child"], n["leaf"], n["q"][8]] for n in c["nodes"]], np.int32).reshape(-1, 3)
        trails = np.array([t if t >= 0 else 0xFFFFFFFF for t in c["bit_trails"]], np.uint32)
        yield lights, nodes, info, trails


def _same(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_product_light_bvh_matches_reference(pa, golden):
    n = 0
    for lights, nodes, info, trails in _golden_cases(golden):
        pn, pi, pt = pa.debug_light_bvh(lights)
        assert _same(pn, nodes) and np.array_equal(pi, info) and np.array_equal(pt, trails)
        n += 1
    assert n >= 10


def test_oracle_light_bvh_matches_reference(oracle, golden):
    for lights, nodes, info, trails in _golden_cases(golden):
        on, oi, ot = oracle.light_bvh(lights13=lights)
        assert _same(on, nodes) and np.array_equal(oi, info) and np.array_equal(ot, trails)


def many_emitters_text(seed=4, n=70):
    """Emissive triangles at random places and orientations (one- and two-sided, reversed,
    RGB / blackbody / scaled), with point and spot lights among them."""
    rng = np.random.default_rng(seed)
    out = ['LookAt 0 0 -30  0 0 0  0 1 0', 'Camera "perspective" "float fov" [ 50 ]',
           'Film "rgb" "integer xresolution" [ 32 ] "integer yresolution" [ 24 ]',
           'Sampler "halton" "integer pixelsamples" [ 4 ]', 'Integrator "volpath" "integer maxdepth" [ 3 ]',
           'WorldBegin', 'Material "diffuse"']
    for i in range(n):
        c = rng.uniform(-10, 10, 3)
        P = c + rng.normal(size=(3, 3)) * rng.uniform(0.1, 2)
        L = (f'"blackbody L" [ {rng.uniform(2000, 9000):.1f} ]' if i % 4 == 0
             else f'"rgb L" [ {rng.uniform(0.1, 5):.3f} {rng.uniform(0.1, 5):.3f} {rng.uniform(0.1, 5):.3f} ]')
        two = '"bool twosided" true' if i % 5 == 0 else ''
        scale = f'"float scale" [ {rng.uniform(0.5, 3):.3f} ]' if i % 3 == 0 else ''
        rev = 'ReverseOrientation' if i % 7 == 3 else ''
        out.append(f'AttributeBegin {rev} AreaLightSource "diffuse" {L} {two} {scale} '
                   f'Shape "trianglemesh" "integer indices" [ 0 1 2 ] "point3 P" [ {" ".join(f"{v:.5f}" for v in P.ravel())} ] '
                   'AttributeEnd')
        if i % 10 == 4:
            f = rng.uniform(-8, 8, 3)
            out.append(f'LightSource "point" "rgb I" [ 1 0.8 0.6 ] "float scale" [ {rng.uniform(1, 20):.2f} ] '
                       f'"point3 from" [ {f[0]:.4f} {f[1]:.4f} {f[2]:.4f} ]')
        if i % 10 == 9:
            f, t = rng.uniform(-8, 8, 3), rng.uniform(-8, 8, 3)
            out.append(f'LightSource "spot" "rgb I" [ 0.7 0.9 1 ] "point3 from" [ {f[0]:.4f} {f[1]:.4f} {f[2]:.4f} ] '
                       f'"point3 to" [ {t[0]:.4f} {t[1]:.4f} {t[2]:.4f} ] "float coneangle" [ {rng.uniform(10, 60):.2f} ] '
                       f'"float conedeltaangle" [ {rng.uniform(1, 10):.2f} ]')
    return "\n".join(out) + "\n"


def _scenes(pa):
    from test_delta_lights import cornell_with_delta
    yield "cornell", pa.load_scene(SCENES / "cornell-box.pbrt")
    yield "cornell+delta", pa.Scene.from_string(cornell_with_delta(), SCENES, xresolution=32, yresolution=32, spp=4)
    for seed in (4, 5):
        yield f"emitters{seed}", pa.Scene.from_string(many_emitters_text(seed), SCENES)


def test_scene_light_bvh_oracle_matches_loader(pa, oracle):
    """Real scenes: the oracle builds its tree from the flat light list (triangle vertices,
    scales, spectra, point / spot parameters); it must equal the loader's node for node."""
    import ctypes
    for name, sc in _scenes(pa):
        f = sc.flat()
        m = f.n_light_nodes
        pn = np.ctypeslib.as_array(f.light_node_bounds, shape=(m * 12,)).reshape(m, 12) if m else np.zeros((0, 12), np.float32)
        pi = np.ctypeslib.as_array(f.light_node_info, shape=(m * 3,)).reshape(m, 3) if m else np.zeros((0, 3), np.int32)
        nb = f.n_area_lights + f.n_point_spot
        on, oi, ot = oracle.light_bvh(sc)
        assert on.shape[0] == m, name
        assert _same(on, pn.astype(np.float32)), name
        assert np.array_equal(oi[:, :2], pi[:, :2]) and np.array_equal(oi[:, 2], pi[:, 2]), name
        leaves = pi[:, 1] == 1
        pt = np.ctypeslib.as_array(f.light_bit_trail, shape=(nb,)) if nb else np.zeros(0, np.uint32)
        members = pi[leaves, 0]
        np.testing.assert_array_equal(ot[members], pt[members], err_msg=name)
