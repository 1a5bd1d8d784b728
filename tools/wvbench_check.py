"""Check tools/wvbench's chain results against Python integers and summarise its timings.
usage: python tools/wvbench_check.py wvbench.json [out.json]"""
import json
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RINV = pow(1 << 400, P - 2, P)


def val(words, half):
    return sum(words[32 * half + k] << (25 * k) for k in range(16))


def m2(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def main():
    d = json.load(open(sys.argv[1]))
    inp, n = d["inputs"], d["iters"]
    a0 = (val(inp, 0), val(inp, 1))
    b = (val(inp[64:], 0), val(inp[64:], 1))
    rinv = (RINV, 0)
    ok = {}
    for mode, rec in d["modes"].items():
        a = a0
        for _ in range(n):
            if mode == "mul2":
                a = m2(m2(a, b), rinv)
            elif mode == "sqr2":
                a = m2(m2(a, a), rinv)
            elif mode == "mulp":
                a = (a[0] * b[0] * RINV % P, a[1] * b[1] * RINV % P)
            elif mode == "dot6":
                a = m2(m2(m2(a, b), rinv), (6, 0))
            else:
                a = (a[0] * (P + 1) // 2 % P, a[1] * (P + 1) // 2 % P)
        out = rec["out"]
        got = (val(out, 0) % P, val(out, 1) % P)
        ok[mode] = got == a
    summary = {"chain_correct": ok,
               "latency_us_per_op": {m: r["grid1"]["us_per_op"] for m, r in d["modes"].items()},
               "cycles_per_op_one_wave": {m: r["grid1"]["cycles_per_op_wave0"] for m, r in d["modes"].items()},
               "throughput_ops_per_s": {m: {g: r[g]["ops_per_s"] for g in r if g.startswith("grid")}
                                        for m, r in d["modes"].items()}}
    txt = json.dumps(summary, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)
    sys.exit(0 if all(ok.values()) else 1)


if __name__ == "__main__":
    main()
