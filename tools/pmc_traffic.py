"""Per-stage HBM traffic per beacon from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; each in its
own run), corrected as /opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]" prescribes: FETCH_SIZE
is in KiB and reports 1/2 of the bytes of coalesced streaming reads on gfx950 (doubled here);
WRITE_SIZE (KiB) is taken as is. Our accesses are dword-per-lane coalesced (256 B per wave
instruction), a width the guide lists as uncalibrated -- ratios between kernels are reliable.

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


def totals(path, counter):
    out = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        st = stage_of(r["Kernel_Name"])
        if st:
            out[st] += float(r["Counter_Value"]) * 1024.0
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
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
