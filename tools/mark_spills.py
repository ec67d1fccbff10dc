#!/usr/bin/env python3
"""Scratch (spill) instructions per MARK region of the k_scan_w variants in a -DSFS2D_MARK build.

usage: python tools/mark_spills.py [asm file]   (default: builds /tmp/sfs2d_mark.s first)
The hot window loop is MARK 19-26; the batched finish (flush) is MARK 30-31.
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "2dsfs-scan_amd", "csrc")
if len(sys.argv) > 1:
    path = sys.argv[1]
else:
    path = "/tmp/sfs2d_mark.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-Wno-unused-result", "-Wno-unused-value", "-mllvm",
                           "-amdgpu-atomic-optimizer-strategy=None", "-DSFS2D_MARK", "-I../../include", "-S",
                           "--cuda-device-only", "sfs2d.hip", "-o", path], cwd=CSRC)
s = open(path).read()
for k in ["1ELb1ELb1", "1ELb1ELb0", "1ELb0ELb1", "1ELb0ELb0", "0ELb1ELb1", "0ELb0ELb0"]:
    m = re.search(r"\n(_ZN6sfs2dk8k_scan_wILb%sEE\w*):" % k, s)
    if not m:
        continue
    i = m.start()
    j = s.index("s_endpgm", i)
    cur, cnt = None, {}
    for line in s[i:j].split("\n"):
        mm = re.search(r"; MARK (\d+)", line)
        if mm:
            cur = int(mm.group(1))
            continue
        if "scratch_" in line:
            cnt[cur] = cnt.get(cur, 0) + 1
    md = s[s.index(".name:           _ZN6sfs2dk8k_scan_wILb%sEE" % k):][:3000]
    regs = dict(re.findall(r"\.(vgpr_count|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", md))
    print("k_scan_w<%s>" % k.replace("ELb", ","), "scratch ops by region (None = prologue):", cnt, regs)
