#!/usr/bin/env python3
"""Instruction classes per MARK region of one kernel in a -DSFS2D_MARK build (static counts: a region's
instructions once, whatever its trip count).  usage: python tools/mark_count.py <asm> <mangled-name-prefix>"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"\n(%s\w*):" % re.escape(sys.argv[2]), s)
i = m.start()
j = s.index("s_endpgm", i)
cur, cnt, order = "pro", {}, ["pro"]
for line in s[i:j].split("\n"):
    mm = re.search(r"; MARK (\d+)", line)
    if mm:
        cur = int(mm.group(1))
        if cur not in order:
            order.append(cur)
        continue
    t = line.strip()
    if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op.startswith("v_"):
        c = "fp64" if re.search(r"_f64|_F64", op) else "valu"
    elif op.startswith("s_"):
        c = "salu" if not op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_barrier", "s_nop")) else "ctl"
    elif op.startswith("ds_"):
        c = "lds"
    elif op.startswith(("buffer_", "global_", "flat_")):
        c = "vmem"
    elif op.startswith("scratch_"):
        c = "scratch"
    else:
        c = "other"
    d = cnt.setdefault(cur, {})
    d[c] = d.get(c, 0) + 1
for k in order:
    print(k, cnt.get(k, {}))
