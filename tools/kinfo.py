#!/usr/bin/env python3
"""Kernel resource summary of built objects (no GPU): registers, scratch and instruction counts.

    python3 tools/kinfo.py drand_amd/csrc/build/k_miller.o [more.o ...]
    python3 tools/kinfo.py --funcs drand_amd/csrc/build/k_miller.o   # also per-function VALU counts

Extracts the gfx950 code object from each object's .hip_fatbin bundle (clang-offload-bundler), reads
the AMDGPU metadata notes (vgpr/agpr counts, private segment = scratch bytes per lane) and counts the
instructions of each function symbol in the disassembly. Faster than `make resource-usage`, which
recompiles every unit.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"


def code_object(path, tmp):
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, "k.co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def kernels(co):
    out = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    ks, cur = [], {}
    for line in out.splitlines():
        m = re.match(r"\s*(-?)\s*\.(\w+):\s+(.*)$", line)
        if not m:
            continue
        dash, k, v = m.group(1), m.group(2), m.group(3).strip()
        if dash and cur:  # a new list entry (each kernel's metadata map starts with "- ")
            ks.append(cur)
            cur = {}
        if k in ("agpr_count", "name", "private_segment_fixed_size", "vgpr_count", "sgpr_count"):
            cur[k] = v
    if cur:
        ks.append(cur)
    return [k for k in ks if "name" in k and "vgpr_count" in k]


def func_sizes(co):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True, text=True,
                         check=True).stdout
    sizes, cur, n = {}, None, {}
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1)
            n = sizes.setdefault(cur, {"all": 0, "valu": 0, "mad": 0})
            continue
        if cur and line.startswith("\t") and line.strip():
            ins = line.strip().split()[0]
            n["all"] += 1
            if ins.startswith("v_"):
                n["valu"] += 1
            if ins.startswith("v_mad_u64_u32") or ins.startswith("v_mad_i64_i32"):
                n["mad"] += 1
    return sizes


def main():
    args = sys.argv[1:]
    funcs = "--funcs" in args
    args = [a for a in args if a != "--funcs"]
    for path in args:
        with tempfile.TemporaryDirectory() as tmp:
            co = code_object(path, tmp)
            print(f"== {path}")
            for k in kernels(co):
                print(f"  {k['name'][:70]:70s} vgpr {k['vgpr_count']:>4} agpr {k.get('agpr_count', '0'):>4} "
                      f"scratch {k['private_segment_fixed_size']:>5}")
            if funcs:
                for f, n in sorted(func_sizes(co).items(), key=lambda kv: -kv[1]["all"]):
                    if n["all"] > 200:
                        print(f"    {f[:80]:80s} insts {n['all']:>7} valu {n['valu']:>7} mad {n['mad']:>6}")


if __name__ == "__main__":
    main()
