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


def main():
    subprocess.check_call(["make", "-s", "-j8"], cwd=HERE)
    OUT.parent.mkdir(parents=True, exist_ok=True)
    tmp = OUT.with_suffix(".tmp")
    subprocess.check_call([str(ROOT / "oracle" / "_ref" / "refgold"), str(tmp)])
    data = json.loads(tmp.read_text())
    OUT.write_text(json.dumps(data, separators=(",", ":")))
    tmp.unlink()
    print("wrote", OUT, OUT.stat().st_size, "bytes", sorted(data))


if __name__ == "__main__":
    sys.exit(main())
