"""Per-kernel resource usage from hipcc -Rpass-analysis=kernel-resource-usage
(stdin): name, VGPRs, AGPRs, scratch bytes/lane, occupancy, VGPR / SGPR spills."""
import re
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" ")[0] + ("_spill" if "Spill" in k else "")] = v
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat in r["name"]:
        print("%-70s vgpr %4s agpr %4s scratch %5s occ %2s spillv %4s spills %4s" % (
            r["name"][:70], r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize"),
            r.get("Occupancy"), r.get("VGPRs_spill"), r.get("SGPRs_spill")))
