#!/usr/bin/env python3
"""Per-kernel instruction and register statistics of a gfx950 device .s file.

usage: isa_stats.py FILE.s [name-substring ...]

Prints, for every kernel whose demangled name contains one of the
substrings: VGPR/SGPR counts, spills, LDS bytes, and static instruction
counts by class (VALU, packed VALU, SALU, LDS, global/buffer memory).
Static counts only: loops are not unrolled here, so a count is per body.
"""
import re
import subprocess
import sys


def demangle(name: str) -> str:
    return subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()


def main() -> None:
    path = sys.argv[1]
    keys = sys.argv[2:] or [""]
    text = open(path).read()
    # kernel descriptors: .amdhsa_kernel NAME ... .end_amdhsa_kernel
    meta = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", text, re.S):
        d = {}
        for key in ("next_free_vgpr", "next_free_sgpr", "accum_offset", "group_segment_fixed_size",
                    "private_segment_fixed_size"):
            mm = re.search(r"\.amdhsa_" + key + r"\s+(\d+)", m.group(2))
            d[key] = int(mm.group(1)) if mm else None
        meta[m.group(1)] = d
    # bodies
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\s*\.Lfunc_end", text, re.S | re.M):
        name = m.group(1)
        dem = demangle(name)
        if not any(k in dem for k in keys):
            continue
        lines = [l.strip() for l in m.group(2).split("\n")]
        ins = [l for l in lines if l and not l.startswith((".", ";")) and not l.endswith(":")]
        cnt = lambda pred: sum(1 for l in ins if pred(l))
        v = cnt(lambda l: l.startswith("v_"))
        pk = cnt(lambda l: l.startswith("v_pk_"))
        s = cnt(lambda l: l.startswith("s_") and not l.startswith(("s_waitcnt", "s_nop", "s_barrier")))
        ds = cnt(lambda l: l.startswith("ds_"))
        gm = cnt(lambda l: l.startswith(("global_", "buffer_", "flat_")))
        md = meta.get(name, {})
        print(f"{dem[:110]}\n    vgpr {md.get('next_free_vgpr')} sgpr {md.get('next_free_sgpr')} "
              f"scratch {md.get('private_segment_fixed_size')} "
              f"static-lds {md.get('group_segment_fixed_size')} | VALU {v} (pk {pk}) SALU {s} DS {ds} VMEM {gm}")


if __name__ == "__main__":
    main()
