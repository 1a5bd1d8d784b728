"""Per-stage HBM traffic per beacon from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; each in its
own run), corrected as /opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]" prescribes: FETCH_SIZE
is in KiB and reports 1/2 of the bytes of coalesced streaming reads on gfx950 (doubled here);
WRITE_SIZE (KiB) is taken as is. Our accesses are dword-per-lane, a width the guide lists as
uncalibrated, so tools/pmccal.hip measured them on a known 576 bytes per item (profiles/r05k_pmccal.json):
  one lane per item (256 contiguous bytes per wave instruction): FETCH_SIZE = 288 B/item -> x2 exact,
                                                                 WRITE_SIZE exact;
  three lanes per item (tri.h, 21 items = 84 bytes per wave instruction): FETCH_SIZE = 713 B/item
                                                                 -> x0.808, WRITE_SIZE x0.900.
"bytes_per_beacon" keeps the guide's x2 for every kernel (comparable with earlier rounds);
"calibrated_bytes_per_beacon" applies the 3-lane factors to the 3-lane kernels (k_fexp_tri,
k_miller_f_tri), whose staging reads are that pattern (their park and scratch reads are
one-lane-per-word, so the calibrated figure is a lower estimate for them and the x2 one an upper).

usage: python tools/pmc_traffic.py <fetch_run_counter_collection.csv> <write_...csv> <beacons> [out.json]
"""
import csv
import json
import sys
from collections import defaultdict

STAGES = (("k_hash", "hash"), ("k_decompress_g2", "decompress"), ("k_subgroup_g2", "decompress"), ("k_miller", "miller"), ("k_fexp", "final_exp"),
          ("k_finish", "finish"))


def stage_of(name):
    base = name.split("(")[0].replace("void ", "").replace("blsk::", "")
    for pre, st in STAGES:
        if base.startswith(pre):
            return st
    return None


TRI_READ, TRI_WRITE = 576.0 / 713.16, 12.0 / 13.33  # tools/pmccal.hip, profiles/r05k_pmccal.json


def is_tri(name):
    return "_tri" in name.split("(")[0]


def kernel_of(name):
    return name.split("(")[0].replace("void ", "").replace("blsk::", "")


def totals(path, counter, tri_factor=None, per_kernel=False):
    out = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        st = stage_of(r["Kernel_Name"])
        if st and per_kernel:
            st = kernel_of(r["Kernel_Name"])
        if st:
            v = float(r["Counter_Value"]) * 1024.0
            if tri_factor is not None:
                v *= tri_factor[1] if is_tri(r["Kernel_Name"]) else tri_factor[0]
            out[st] += v
    return out


def main():
    fetch = totals(sys.argv[1], "FETCH_SIZE")
    write = totals(sys.argv[2], "WRITE_SIZE")
    n = float(sys.argv[3])
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs), %d beacons verified" % n,
           "correction": "read bytes = 2 x FETCH_SIZE KiB (gfx950), write bytes = WRITE_SIZE KiB",
           "bytes_per_beacon": {}}
    for st in sorted(set(fetch) | set(write)):
        rd, wr = 2 * fetch.get(st, 0.0) / n, write.get(st, 0.0) / n
        res["bytes_per_beacon"][st] = {"read": round(rd, 1), "write": round(wr, 1), "total": round(rd + wr, 1)}
    cf = totals(sys.argv[1], "FETCH_SIZE", (2.0, TRI_READ))
    cw = totals(sys.argv[2], "WRITE_SIZE", (1.0, TRI_WRITE))
    res["calibrated_bytes_per_beacon"] = {}
    for st in sorted(set(cf) | set(cw)):
        rd, wr = cf.get(st, 0.0) / n, cw.get(st, 0.0) / n
        res["calibrated_bytes_per_beacon"][st] = {"read": round(rd, 1), "write": round(wr, 1), "total": round(rd + wr, 1)}
    # per kernel, guide's x2 (the Miller targets are per kernel: k_miller_f reads / writes)
    kf = totals(sys.argv[1], "FETCH_SIZE", per_kernel=True)
    kw = totals(sys.argv[2], "WRITE_SIZE", per_kernel=True)
    res["kernel_bytes_per_beacon"] = {}
    for k in sorted(set(kf) | set(kw)):
        rd, wr = 2 * kf.get(k, 0.0) / n, kw.get(k, 0.0) / n
        res["kernel_bytes_per_beacon"][k] = {"read": round(rd, 1), "write": round(wr, 1)}
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
