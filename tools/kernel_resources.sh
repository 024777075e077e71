#!/bin/bash
# VGPR / SGPR / occupancy / LDS / scratch per kernel of one HIP source, from
# the compiler's resource-usage remarks (gfx950):
#   tools/kernel_resources.sh stereovisionarray_amd/csrc/wta_h.hip [name-filter]
set -eu
src=$1 filt=${2:-}
cd "$(dirname "$0")/../stereovisionarray_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -I../../include \
  -Rpass-analysis=kernel-resource-usage -c "$(basename "$src")" -o /dev/null 2>&1 |
python3 -c '
import sys, re
flt = sys.argv[1]
cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}
        continue
    m = re.search(r"remark: .*?(VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = m.group(2)
for n, r in rows.items():
    if flt and flt not in n: continue
    print("%-80s vgpr=%s sgpr=%s occ=%s lds=%s scratch=%s" % (n[:80], r.get("VGPRs"), r.get("SGPRs"), r.get("Occupancy"), r.get("LDS"), r.get("ScratchSize")))
' "$filt"
