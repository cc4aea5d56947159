"""Summarise rocprofv3 --pmc CSV output per kernel (mean over dispatches).

    python scripts/pmc_summary.py gpurun_out/pmc/*_counter_collection.csv [--match SUBSTR]

Derived columns (MI355X_MICROARCH.md, DVFS + PMC units):
  clk_GHz   = GRBM_GUI_ACTIVE / 8 / kernel wall time (GRBM is summed over the 8 XCDs)
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 · 1024 SIMDs)   (busy cycles sum over SIMDs)
  wait_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (fraction of wave time waiting on an s_waitcnt)
  lds_conf  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""

import argparse
import collections
import csv
import glob
import os


def load(paths, match=None):
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # (file, kernel) -> ctr -> [v]
    wall = collections.defaultdict(dict)
    for p in paths:
        tag = os.path.basename(p).replace("_counter_collection.csv", "")
        with open(p) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "?")
                if match and match not in k:
                    continue
                key = (tag, k[:70])
                disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
                per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                try:
                    wall[key][disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                except (KeyError, ValueError):
                    pass
    return per, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match")
    a = ap.parse_args()
    paths = [q for p in a.paths for q in (glob.glob(p) or [p])]
    per, wall = load(paths, a.match)
    for key in sorted(per):
        c = {n: sum(v) / len(v) for n, v in per[key].items()}
        w = wall[key]
        t = sum(w.values()) / len(w) if w else 0.0
        out = [f"{key[0]:<28} {key[1]:<70}", f"us={t * 1e6:9.1f}"]
        if "GRBM_GUI_ACTIVE" in c and t > 0:
            out.append(f"clk_GHz={c['GRBM_GUI_ACTIVE'] / 8 / t / 1e9:5.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            out.append(f"mfma_util={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):5.3f}")
        if "SQ_WAIT_INST_ANY" in c and c.get("SQ_WAVE_CYCLES"):
            out.append(f"wait_frac={c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:5.3f}")
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"lds_conf={c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:5.3f}")
        out += [f"{n}={v:.4g}" for n, v in sorted(c.items())]
        print("  ".join(out))


if __name__ == "__main__":
    main()
