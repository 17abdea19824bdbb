"""Summarize the PMC passes written by scripts/pmc_session.sh: mean counter value per dispatch
for every grr kernel, plus derived busy fractions.

    python scripts/pmc_summary.py gpurun_out/pmc_<kernel>
"""
import collections
import csv
import glob
import os
import sys


def main(base):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in glob.glob(os.path.join(base, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "grr" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("(")[0]
            per[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, cs in per.items():
        m = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        print(k)
        for c in sorted(m):
            print(f"   {c:32s} {m[c]:.4g}")
        gui = m.get("GRBM_GUI_ACTIVE")
        if gui:
            simd_cycles = gui / 8 * 1024       # GRBM summed over 8 XCDs; 1024 SIMDs
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                print(f"   -> MFMA busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.1%}")
            if "SQ_BUSY_CYCLES" in m:
                print(f"   -> SQ busy per SE {m['SQ_BUSY_CYCLES'] / (gui / 8 * 32):.1%}")
        if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_INST_ANY" in m:
            print(f"   -> wait_inst/wave_cycles {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.1%}, "
                  f"active_inst/wave_cycles {m['SQ_ACTIVE_INST_ANY'] / m['SQ_WAVE_CYCLES']:.1%}")
        if "FETCH_SIZE" in m:
            print(f"   -> HBM read (2xFETCH) {2 * m['FETCH_SIZE'] * 1024 / 1e9:.3f} GB, "
                  f"write {m.get('WRITE_SIZE', 0) * 1024 / 1e9:.3f} GB")


if __name__ == "__main__":
    main(sys.argv[1])
