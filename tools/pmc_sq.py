"""Per-kernel occupancy and VALU activity from rocprofv3 SQ/GRBM counter passes.

usage: python tools/pmc_sq.py out.json <pass1 run_counter_collection.csv> [<pass2 csv> ...]

Each pass is its own `rocprofv3 --pmc ...` run of the same command (counters do not split over
passes on gfx950). Counters are summed per kernel name over its dispatches, then:

  waves                    SQ_WAVES / dispatches
  valu_insts_per_wave      SQ_INSTS_VALU / SQ_WAVES
  salu_insts_per_wave      SQ_INSTS_SALU / SQ_WAVES, lds_insts_per_wave likewise
  wait_any / wait_inst     SQ_WAIT_ANY, SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES (parked / issue-stalled
                           fractions of a resident wave's life)
  clock_ghz                GRBM_GUI_ACTIVE / summed dispatch duration / 8 (rocprofv3 sums GRBM over the
                           8 XCDs): 2.1-2.45 GHz on every busy kernel
  waves_per_simd           SQ_WAVE_CYCLES * U / (kernel cycles * 1024 SIMDs): achieved occupancy (mean
                           resident waves per SIMD); kernel cycles = summed duration x clock_ghz
  cyc_per_valu_wave        SQ_WAVE_CYCLES * U / SQ_INSTS_VALU: cycles between two VALU issues of ONE
                           wave (the issue interval tools/issuebench.hip measures: 5.1-6.1 at 1
                           wave/SIMD, 4.15-4.3 at 8)
  cyc_per_valu_simd        kernel cycles * 1024 / SQ_INSTS_VALU: cycles between VALU issues of a SIMD
  valu_busy                SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES as rocprofv3 reports it (on gfx950
                           SQ_ACTIVE_INST_VALU == SQ_INSTS_VALU: one count per instruction)
U = 4: SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md). Cross-checks: k_miller_f, which its
512 VGPR+AGPR budget pins at exactly 1 wave/SIMD, reads 0.99, and its 1-wave issue interval reads
5.5 cycles, as tools/issuebench.hip measures. A counter collected in several passes is averaged.
"""
import csv
import json
import sys
from collections import defaultdict

N_SIMD = 1024
GRBM_UNITS = 8
U = 4.0


def short(name):
    base = name.split("(")[0]
    for pre in ("void ", "blsk::"):
        base = base.replace(pre, "")
    return base.strip()


def main():
    out_path, paths = sys.argv[1], sys.argv[2:]
    val = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(dict)  # per pass: kernel -> summed ns
    disp = defaultdict(set)
    npass = defaultdict(lambda: defaultdict(set))  # kernel -> counter -> passes that collected it
    for pi, p in enumerate(paths):
        seen = set()
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            if not k.startswith("k_") and "k_" not in k:
                continue
            val[k][r["Counter_Name"]] += float(r["Counter_Value"])
            npass[k][r["Counter_Name"]].add(pi)
            key = (pi, r["Dispatch_Id"])
            disp[k].add(r["Dispatch_Id"]) if pi == 0 else None
            if (k, key) not in seen:
                seen.add((k, key))
                dur[pi][k] = dur[pi].get(k, 0.0) + float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    res = {"source": "rocprofv3 --pmc passes: " + ", ".join(paths),
           "formulas": __doc__.split("then:")[1].strip(), "kernels": {}}
    for k, c in sorted(val.items()):
        c = {n: v / len(npass[k][n]) for n, v in c.items()}
        ns = [d[k] for d in dur.values() if k in d]
        t_ns = sum(ns) / len(ns) if ns else 0.0
        w = c.get("SQ_WAVES", 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        e = {"dispatches": len(disp[k]) or None, "kernel_ms_total": round(t_ns / 1e6, 3),
             "raw": {n: v for n, v in sorted(c.items())}}
        if w:
            e["waves"] = round(w / max(1, len(disp[k])))
            for cn, nm in (("SQ_INSTS_VALU", "valu_insts_per_wave"), ("SQ_INSTS_SALU", "salu_insts_per_wave"),
                           ("SQ_INSTS_LDS", "lds_insts_per_wave")):
                if cn in c:
                    e[nm] = round(c[cn] / w)
        if wc:
            if "SQ_INSTS_VALU" in c and c["SQ_INSTS_VALU"]:
                e["cyc_per_valu_wave"] = round(wc * U / c["SQ_INSTS_VALU"], 2)
            for cn, nm in (("SQ_ACTIVE_INST_VALU", "valu_busy"), ("SQ_WAIT_ANY", "wait_any"),
                           ("SQ_WAIT_INST_ANY", "wait_inst"), ("SQ_ACTIVE_INST_ANY", "active_any")):
                if cn in c:
                    e[nm] = round(c[cn] / wc, 3)
        clk = None
        if "GRBM_GUI_ACTIVE" in c and t_ns:
            clk = c["GRBM_GUI_ACTIVE"] / t_ns / GRBM_UNITS
            e["clock_ghz"] = round(clk, 3)
        cyc = t_ns * (clk or 2.4)
        if wc and cyc:
            e["waves_per_simd"] = round(wc * U / (cyc * N_SIMD), 2)
        if c.get("SQ_INSTS_VALU") and cyc:
            e["cyc_per_valu_simd"] = round(cyc * N_SIMD / c["SQ_INSTS_VALU"], 2)
        res["kernels"][k] = e
    txt = json.dumps(res, indent=1)
    open(out_path, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
