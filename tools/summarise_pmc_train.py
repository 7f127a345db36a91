"""Per-kernel SQ counter summary of a tools/pmc_train.sh run (rocprofv3 --pmc passes).
Per wave: instruction counts; cycles per wave: WAVE / WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY /
WAIT_INST_LDS (SQ cycle counters, as the r3h summary); per dispatch: LDS bank conflicts, MFMA busy.
usage: python tools/summarise_pmc_train.py gpurun_out/pmc_train_TAG > profiles/TAG_train_pmc.txt"""
import collections
import csv
import sys
from pathlib import Path

src = Path(sys.argv[1])
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(src.rglob("*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        tot[short][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(short, r["Counter_Name"])].add(r["Dispatch_Id"])
for k in sorted(tot):
    c = tot[k]
    nd = max(len(disp[(k, n)]) for n in c)
    waves = c.get("SQ_WAVES", 0.0)
    if not waves:
        continue
    pw = lambda n: c.get(n, 0.0) / waves
    pd = lambda n: c.get(n, 0.0) / max(1, len(disp[(k, n)]))
    print(f"{k}: dispatches {nd}, waves/dispatch {waves / max(1, len(disp[(k, 'SQ_WAVES')])):.0f}")
    print("   per wave: " + ", ".join(f"{n[9:] if n.startswith('SQ_INSTS_') else n} {pw(n):.0f}" for n in
                                      ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM",
                                       "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")))
    w = pw("SQ_WAVE_CYCLES")
    print(f"   cycles per wave: WAVE {w:.0f}, WAIT_ANY {pw('SQ_WAIT_ANY'):.0f} ({pw('SQ_WAIT_ANY') / max(w, 1):.0%}), "
          f"WAIT_INST_ANY {pw('SQ_WAIT_INST_ANY'):.0f}, ACTIVE_INST_ANY {pw('SQ_ACTIVE_INST_ANY'):.0f} "
          f"({pw('SQ_ACTIVE_INST_ANY') / max(w, 1):.0%}), WAIT_INST_LDS {pw('SQ_WAIT_INST_LDS'):.0f}; per dispatch: "
          f"LDS_BANK_CONFLICT {pd('SQ_LDS_BANK_CONFLICT'):.0f}, MFMA_BUSY {pd('SQ_VALU_MFMA_BUSY_CYCLES'):.0f}, "
          f"BUSY {pd('SQ_BUSY_CYCLES'):.0f}")
