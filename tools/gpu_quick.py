"""Quick GPU check: render the Cornell box at C1 and C2 settings, print timing + stats."""
import sys, time
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
import pbrt_amd as pa

out = ROOT / "gpurun_out"
out.mkdir(exist_ok=True)
for name, ov in [("c1", dict(xresolution=256, yresolution=256, spp=16)),
                 ("c2", dict(xresolution=1280, yresolution=720, spp=64))]:
    sc = pa.load_scene(ROOT / "scenes/cornell-box.pbrt", **ov)
    integ = pa.WavefrontPathIntegrator(sc)
    integ.render(first_sample=0, n_samples=1)  # warm-up
    integ.synchronize()
    integ.film_clear()
    integ.reset_stats()
    t = time.time()
    integ.render(time_closest=True)
    integ.synchronize()
    dt = time.time() - t
    img = integ.film_rgb()
    st = integ.stats()
    i = sc.info
    ms = i.xres * i.yres * i.spp / dt / 1e6
    print(name, f"{dt*1e3:.1f} ms  {ms:.1f} Msamples/s  mean {img.mean(axis=(0,1))}  finite {np.isfinite(img).all()}"
          f"  passes {st.passes} closest {st.closest_launches} launches {st.closest_ms:.2f} ms", flush=True)
    pa.write_pfm(out / f"cornell_{name}.pfm", img)
