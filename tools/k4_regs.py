#!/usr/bin/env python3
"""Register / spill report of the K4 kernels from a device-only assembly listing.

    hipcc <Makefile flags> -x hip csrc/vct_trace.hip --cuda-device-only -S -o trace.s
    python tools/k4_regs.py trace.s [trace_b.s]

Prints, per k4_trace instantiation: VGPRs, SGPRs, SGPR / VGPR spills, scratch bytes per
lane and the count of scalar dword loads in its body (the D3 brick test is one).
With two listings, prints both side by side.
"""
import re
import sys


def parse(path):
    s = open(path).read()
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S*k4_trace\S*)\n((?:\s{4}\..*\n)+)", s):
        body = m.group(2)

        def f(k):
            x = re.search(r"\." + k + r":\s+(\d+)", body)
            return int(x.group(1)) if x else None
        meta[m.group(1)] = dict(vgpr=f("vgpr_count"), sgpr=f("sgpr_count"), sspill=f("sgpr_spill_count"),
                                vspill=f("vgpr_spill_count"), scratch=f("private_segment_fixed_size"))
    for name in meta:
        a = s.find("\n" + name + ":")
        b = s.find(".Lfunc_end", a)
        text = s[a:b] if a >= 0 else ""
        meta[name]["s_load"] = len(re.findall(r"\ts_load_dword(?:x\d)?\b", text))
        meta[name]["lines"] = text.count("\n")
    return meta


def short(name):
    m = re.search(r"k4_traceIL(b\d)ELi(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)E", name)
    if not m:
        return name[:60]
    brick, minw, union, o32, split, cnt = m.groups()
    return f"brick={brick[-1]} minw={minw} union={union} o32={o32} split={split} cnt={cnt}"


def main():
    ms = [parse(p) for p in sys.argv[1:]]
    for name in ms[0]:
        row = [short(name)]
        for m in ms:
            d = m.get(name)
            row.append("-" if d is None else
                       f"v{d['vgpr']} s{d['sgpr']} ssp{d['sspill']} vsp{d['vspill']} scr{d['scratch']} sld{d['s_load']}")
        print(" | ".join(row))


if __name__ == "__main__":
    main()
