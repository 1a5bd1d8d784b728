"""Regenerate profiles/opcount.json (algorithmic Fp multiplications per beacon, per stage) from the
host build of the engine's device headers (tools/opcount). Run after changing any algorithm."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
subprocess.run(["make", "-C", os.path.join(ROOT, "tools"), "opcount"], check=True, capture_output=True)
g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["chained"]
b = g["beacons"][5]
out = json.loads(subprocess.run([os.path.join(ROOT, "tools", "opcount"), g["pk"], str(b["round"]), b["prev"], b["sig"]],
                                capture_output=True, text=True, check=True).stdout)
out["source"] = ("tools/opcount (drand_amd/csrc headers compiled for the host, -DBLS_HOST), golden chained beacon "
                 "round %d" % b["round"])
out["total_fp_mul"] = sum(out["fp_mul"].values())
with open(os.path.join(ROOT, "profiles", "opcount.json"), "w") as f:
    json.dump(out, f, indent=1)
print(out)
