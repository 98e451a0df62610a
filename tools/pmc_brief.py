#!/usr/bin/env python3
"""Per-kernel digest of tools/pmc_summary.py output: instructions per wave, VALU issue share."""
import json
import sys

d = json.load(open(sys.argv[1]))
print(f"{'kernel':34s} {'waves':>7s} {'VALU/w':>8s} {'SALU/w':>7s} {'LDS/w':>6s} {'VMEM/w':>7s} "
      f"{'TRANS/w':>7s} {'cyc/w':>8s} {'valu%':>6s} {'waitany%':>8s} {'waitinst%':>9s}")
for k, c in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    w = c.get("SQ_WAVES", 0)
    if not w or k.startswith("__"):
        continue
    cyc = c.get("SQ_WAVE_CYCLES", 0)
    vm = c.get("SQ_INSTS_VMEM_RD", 0) + c.get("SQ_INSTS_VMEM_WR", 0)
    print(f"{k[:34]:34s} {w:7.0f} {c.get('SQ_INSTS_VALU', 0)/w:8.0f} {c.get('SQ_INSTS_SALU', 0)/w:7.0f} "
          f"{c.get('SQ_INSTS_LDS', 0)/w:6.0f} {vm/w:7.0f} {c.get('SQ_INSTS_VALU_TRANS_F32', 0)/w:7.0f} "
          f"{cyc/w:8.0f} {100*c.get('SQ_ACTIVE_INST_VALU', 0)/max(cyc,1):6.1f} "
          f"{100*c.get('SQ_WAIT_ANY', 0)/max(cyc,1):8.1f} {100*c.get('SQ_WAIT_INST_ANY', 0)/max(cyc,1):9.1f}")
