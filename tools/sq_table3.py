"""Summarise tools/gpu_sq3.sh passes: per kernel, the mean per-dispatch value of each counter and the
derived shares (SQ_WAVE_CYCLES / WAIT_* / ACTIVE_* count quad-cycles per wave, summed over waves;
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE count cycles; MI355X_MICROARCH.md 'rocprofv3 PMC slots').
    python tools/sq_table3.py gpurun_out/sq3_<tag>_1 gpurun_out/sq3_<tag>_2
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    acc, cnt = defaultdict(float), defaultdict(int)
    for d in sys.argv[1:]:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(fn)):
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[r["Counter_Name"]] += 1
    m = {k: acc[k] / cnt[k] for k in acc}
    for k in sorted(m):
        print(f"{k:36s} {m[k]:16.0f}")
    w = m.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_INST_CYCLES_VMEM_RD", "SQ_WAIT_INST_LDS"):
            if k in m:
                print(f"  {k} / WAVE_CYCLES = {m[k] / w:.3f}")
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
        # MFMA busy per SIMD: busy cycles summed over all SIMDs / (GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
        print(f"  MFMA busy / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs) = {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")


if __name__ == "__main__":
    main()
