#!/usr/bin/env python3
"""Regenerate tests/golden/reference_components.json from the reference sources.

Runs only where /root/reference exists: builds oracle/_ref/refgold with oracle/ref/Makefile
(reference sources compiled unmodified) and runs it.  The JSON holds inputs and the
reference's outputs for the hot-path components (see oracle/ref/refgold.cpp)."""
import json
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
OUT = ROOT / "tests" / "golden" / "reference_components.json"
# util/sobolmatrices.cpp's tables as the product's data file (constant data the SobolSampler
# needs bit for bit; written by the reference's own compiled table)
SOBOL = ROOT / "pbrt-v4_amd" / "data" / "sobol_tables.bin"


def main():
    subprocess.check_call(["make", "-s", "-j8"], cwd=HERE)
    OUT.parent.mkdir(parents=True, exist_ok=True)
    tmp = OUT.with_suffix(".tmp")
    subprocess.check_call([str(ROOT / "oracle" / "_ref" / "refgold"), str(tmp)])
    data = json.loads(tmp.read_text())
    OUT.write_text(json.dumps(data, separators=(",", ":")))
    tmp.unlink()
    subprocess.check_call([str(ROOT / "oracle" / "_ref" / "refgold"), "--sobol-tables", str(SOBOL)])
    print("wrote", SOBOL, SOBOL.stat().st_size, "bytes")
    print("wrote", OUT, OUT.stat().st_size, "bytes", sorted(data))


if __name__ == "__main__":
    sys.exit(main())
