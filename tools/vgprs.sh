#!/bin/bash
# per-kernel VGPR / scratch / occupancy of the gfx950 build
cd "$(dirname "$0")/../2dsfs-scan_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -c --cuda-device-only sfs2d.hip \
  -o /tmp/sfs2d_dev.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        n = m.group(1); k = re.search(r"sfs2dk\d+([a-z_0-9]+?)(I.*?E)?E?v?N", n)
        cur = re.sub(r"^_ZN6sfs2dk\d+", "", n)[:24]; continue
    for key in ("VGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"):
        m = re.search(re.escape(key) + r": (\d+)", line)
        if m and cur: print(f"{cur:26s} {key.split()[0]:12s} {m.group(1)}")
'
