#!/usr/bin/env python3
"""Instruction-mix summary per kernel of a hipcc `-S` listing (developer tool).

usage: python tools/asm_stats.py file.s [substring-filter]
"""
import re
import sys
from collections import Counter


def stats(path, filt=""):
    cur = None
    out = {}
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            out[cur] = Counter()
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
        if cur and line.startswith("\t") and not line.strip().startswith((".", ";")):
            out[cur][line.split()[0]] += 1
    for name, c in out.items():
        if filt not in name:
            continue
        tot = sum(c.values())
        grp = lambda p: sum(v for k, v in c.items() if k.startswith(p))
        print(f"{name[:70]:70s} tot={tot:6d} pk_fma={c['v_pk_fma_f32']:5d} fma={c['v_fma_f32']+c['v_fmac_f32_e32']:5d} "
              f"s_load={grp('s_load'):4d} ds_read={grp('ds_read'):4d} ds_write={grp('ds_write'):4d} "
              f"gload={grp('global_load'):4d} gstore={grp('global_store'):4d} wait={c['s_waitcnt']:4d} "
              f"mfma={grp('v_mfma'):4d}")


if __name__ == "__main__":
    stats(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
