#!/usr/bin/env python3
"""Extract the standard CIE tables the renderer needs into a JSON data file.

The data are the public CIE 1931 2-degree colour matching functions (1 nm, 360-830 nm),
the CIE D65 relative SPD, and the 5 nm CIE/D65 tables plus sRGB<->XYZ matrices that
pbrt's RGB->spectrum optimiser (cmd/rgb2spec_opt.cpp) integrates against.  They are
measurement data, not code: this script only parses the numeric literals out of the
reference's sources

    src/pbrt/util/spectrum.cpp   CIE_X / CIE_Y / CIE_Z / CIE_lambda (:273-567),
                                 CIE_Illum_D6500 (:770)
    src/pbrt/cmd/rgb2spec_opt.cpp cie_x / cie_y / cie_z / cie_d65 (:46-128),
                                 xyz_to_srgb / srgb_to_xyz (:191-197)
    src/pbrt/util/color.cpp      SRGBToLinearLUT (:286-330), the 8-bit sRGB decode table
                                 every sRGB-encoded image texel goes through
    src/pbrt/util/mipmap.cpp     MIPFilterLUT (:59-191), the EWA filter weight table
    src/pbrt/util/spectrum.cpp   the interleaved (lambda, value) tables behind the named
                                 metal and glass spectra (:1128-1440), keyed by the names
                                 Spectra::Init registers them under (:2666-2690), the camera
                                 sensor curves (<camera>_r/_g/_b) and the CIE daylight basis
                                 S0 / S1 / S2 (Spectra::D)
    src/pbrt/film.cpp            the 24 ColorChecker swatch reflectances of PixelSensor
    src/pbrt/util/noise.cpp      NoisePerm (:17-46), Perlin's gradient-noise permutation table
                                 (the CloudMedium density)

and writes pbrt-v4_amd/data/spectral_data.json, which is committed.  Run it only in a
container that has /root/reference; the GPU box uses the committed JSON.
"""
import json
import re
import sys
from pathlib import Path

REF = Path("/root/reference/src/pbrt")
OUT = Path(__file__).resolve().parents[1] / "pbrt-v4_amd" / "data" / "spectral_data.json"

NUM = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?"


# name -> array as registered in Spectra::Init's namedSpectra map (util/spectrum.cpp:2666-2690)
NAMED = {
    "glass-BK7": "GlassBK7_eta", "glass-BAF10": "GlassBAF10_eta", "glass-FK51A": "GlassFK51A_eta",
    "glass-LASF9": "GlassLASF9_eta", "glass-F5": "GlassSF5_eta", "glass-F10": "GlassSF10_eta",
    "glass-F11": "GlassSF11_eta",
    "metal-Ag-eta": "Ag_eta", "metal-Ag-k": "Ag_k", "metal-Al-eta": "Al_eta", "metal-Al-k": "Al_k",
    "metal-Au-eta": "Au_eta", "metal-Au-k": "Au_k", "metal-Cu-eta": "Cu_eta", "metal-Cu-k": "Cu_k",
    "metal-CuZn-eta": "CuZn_eta", "metal-CuZn-k": "CuZn_k", "metal-MgO-eta": "MgO_eta",
    "metal-MgO-k": "MgO_k", "metal-TiO2-eta": "TiO2_eta", "metal-TiO2-k": "TiO2_k",
}


def array_body(text, name):
    m = re.search(r"(?:const\s+(?:Float|double)\s+)" + re.escape(name) + r"\s*(?:\[[^\]]*\]\s*)+=\s*\{", text)
    if not m:
        raise SystemExit(f"array {name} not found")
    depth, i = 1, m.end()
    while depth:
        c = text[i]
        depth += c == "{"
        depth -= c == "}"
        i += 1
    return text[m.end():i - 1]


def numbers(body):
    body = re.sub(r"//[^\n]*", "", body)
    return [float(x) for x in re.findall(NUM, body)]


def main():
    spec = (REF / "util" / "spectrum.cpp").read_text()
    opt = (REF / "cmd" / "rgb2spec_opt.cpp").read_text()
    data = {}
    for name in ("CIE_X", "CIE_Y", "CIE_Z", "CIE_lambda"):
        data[name] = numbers(array_body(spec, name))
        assert len(data[name]) == 471, (name, len(data[name]))
    d65 = numbers(array_body(spec, "CIE_Illum_D6500"))
    data["CIE_Illum_D6500_interleaved"] = d65
    # rgb2spec_opt tables: the N(x) macro divides by a constant; keep raw and the divisor
    for name in ("cie_x", "cie_y", "cie_z"):
        data["opt_" + name] = numbers(array_body(opt, name))
        assert len(data["opt_" + name]) == 95
    body = array_body(opt, "cie_d65")
    raw = [float(x) for x in re.findall(r"N\((" + NUM + r")\)", body)]
    assert len(raw) == 95
    div = float(re.search(r"#define N\(x\) \(x / (" + NUM + r")\)", opt[:opt.find("cie_d65")][-400:]).group(1))
    data["opt_cie_d65_raw"] = raw
    data["opt_cie_d65_divisor"] = div
    for name in ("xyz_to_srgb", "srgb_to_xyz"):
        data["opt_" + name] = numbers(array_body(opt, name))
        assert len(data["opt_" + name]) == 9
    # the other gamuts rgb2spec_opt builds tables for (init_tables, :408-486): ACES2065-1 under its
    # D60 illuminant, Rec.2020 and DCI-P3 under D65
    body = array_body(opt, "cie_d60")
    raw = [float(x) for x in re.findall(r"N\((" + NUM + r")\)", body)]
    # cie_d60[CIE_SAMPLES] has 94 initialisers: C++ zero-fills the 95th (830 nm) entry
    assert len(raw) == 94
    raw.append(0.0)
    div = float(re.search(r"#define N\(x\) \(x / (" + NUM + r")\)", opt[:opt.find("cie_d60[")][-200:]).group(1))
    data["opt_cie_d60_raw"] = raw
    data["opt_cie_d60_divisor"] = div
    for g in ("aces2065_1", "rec2020", "dcip3"):
        for name in ("xyz_to_" + g, g + "_to_xyz"):
            data["opt_" + name] = numbers(array_body(opt, name))
            assert len(data["opt_" + name]) == 9
    # the normalised standard illuminants Spectra::Init registers (util/spectrum.cpp:2604-2650,
    # 2689-2707: FromInterleaved(..., normalize = true)): "stdillum-*" and "illum-acesD60"
    illums = {"stdillum-A": "CIE_Illum_A", "stdillum-D50": "CIE_Illum_D5000", "stdillum-D65": "CIE_Illum_D6500",
              "illum-acesD60": "ACES_Illum_D60"}
    for k in range(1, 13):
        illums[f"stdillum-F{k}"] = f"CIE_Illum_F{k}"
    for name, arr in illums.items():
        vals = numbers(array_body(spec, arr))
        assert len(vals) % 2 == 0 and len(vals) >= 4, (name, len(vals))
        data["illum:" + name] = vals
    color = (REF / "util" / "color.cpp").read_text()
    m = re.search(r"Float\s+SRGBToLinearLUT\s*\[256\]\s*=\s*\{", color)
    body = color[m.end():color.index("}", m.end())]
    data["SRGBToLinearLUT"] = numbers(body)
    assert len(data["SRGBToLinearLUT"]) == 256
    mip = (REF / "util" / "mipmap.cpp").read_text()
    m = re.search(r"Float\s+MIPFilterLUT\s*\[MIPFilterLUTSize\]\s*=\s*\{", mip)
    body = mip[m.end():mip.index("};", m.end())]
    data["MIPFilterLUT"] = numbers(body)
    assert len(data["MIPFilterLUT"]) == 128, len(data["MIPFilterLUT"])
    for name, arr in NAMED.items():
        vals = numbers(array_body(spec, arr))
        assert len(vals) % 2 == 0 and len(vals) >= 4, (name, len(vals))
        data["named:" + name] = vals
    # camera sensor response curves, registered in Spectra::Init as
    # {"<camera>_r|g|b", PiecewiseLinearSpectrum::FromInterleaved(<array>, false, alloc)}
    # (util/spectrum.cpp:2707-...), looked up by PixelSensor::Create (film.cpp:222-262)
    for name, arr in re.findall(r'\{"(\w+_[rgb])",\s*PiecewiseLinearSpectrum::FromInterleaved\((\w+),\s*false,\s*alloc\)\}',
                                spec):
        vals = numbers(array_body(spec, arr))
        assert len(vals) % 2 == 0 and len(vals) >= 4, (name, len(vals))
        data["sensor:" + name] = vals
    assert sum(k.startswith("sensor:") for k in data) >= 30
    # CIE daylight basis S0, S1, S2 over CIE_S_lambda (Spectra::D, util/spectrum.cpp:632-690, 2537-2570)
    for name in ("CIE_S_lambda", "CIE_S0", "CIE_S1", "CIE_S2"):
        data[name] = numbers(array_body(spec, name))
        assert len(data[name]) == 107, (name, len(data[name]))
    # the 24 ColorChecker swatch reflectances PixelSensor fits XYZFromSensorRGB on
    # (PixelSensor::swatchReflectances, film.cpp:268-...: BabelColor measurements)
    film = (REF / "film.cpp").read_text()
    m = re.search(r"Spectrum PixelSensor::swatchReflectances\[nSwatchReflectances\]\{", film)
    body = film[m.end():film.index("};", m.end())]
    sw = re.findall(r"FromInterleaved\(\s*\{([^}]*)\}", body)
    assert len(sw) == 24, len(sw)
    for i, b in enumerate(sw):
        data[f"swatch:{i}"] = numbers(b)
    # Perlin noise permutation (util/noise.cpp NoisePerm[2 * NoisePermSize])
    noise = (REF / "util" / "noise.cpp").read_text()
    m = re.search(r"NoisePerm\s*\[2 \* NoisePermSize\]\s*=\s*\{", noise)
    body = noise[m.end():noise.index("};", m.end())]
    body = re.sub(r"//[^\n]*", "", body)
    data["NoisePerm"] = numbers(body)
    assert len(data["NoisePerm"]) == 512, len(data["NoisePerm"])
    # medium scattering presets (GetMediumScatteringProperties' SubsurfaceParameterTable,
    # media.cpp:74-151): name -> sigma_prime_s RGB, sigma_a RGB in mm^-1 (spaces in names as "_")
    media = (REF / "media.cpp").read_text()
    m = re.search(r"static MeasuredSS SubsurfaceParameterTable\[\] = \{", media)
    body = media[m.end():media.index("};", m.end())]
    presets = re.findall(r'\{"([^"]+)",\s*RGB\(([^)]*)\),\s*RGB\(([^)]*)\)\}', body)
    assert len(presets) == 47, len(presets)
    for name, sps, sa in presets:
        data["mediumpreset:" + name.replace(" ", "_")] = numbers(sps) + numbers(sa)
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text(json.dumps(data))
    print("wrote", OUT, {k: len(v) if isinstance(v, list) else v for k, v in data.items()})




def write_text(data, path):
    """Plain 'name count v0 v1 ...' lines for the C++ loader (no JSON parser needed)."""
    with open(path, "w") as f:
        for k, v in data.items():
            vals = v if isinstance(v, list) else [v]
            f.write(k + " " + str(len(vals)) + " " + " ".join(repr(float(x)) for x in vals) + "\n")


if __name__ == "__main__":
    main()
    write_text(json.loads(OUT.read_text()), OUT.with_suffix(".txt"))
