"""Print one LM outer iteration of a rocprofv3 kernel trace (gaps, durations)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_jacobian' in r['Kernel_Name']]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
a, b = idx[k], idx[k + 1]
seg = rows[a - 3:b - 2]
t0 = int(seg[0]['Start_Timestamp']); prev = None; busy = 0
for r in seg:
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    busy += (e - s)
    print(f"{(s-t0)/1e3:8.2f} gap {gap:6.2f} dur {(e-s)/1e3:6.2f} grid {int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']):6d} {r['Kernel_Name'][:50]}")
    prev = e
print("span %.1f us, busy %.1f us, %d launches" % ((prev - t0) / 1e3, busy / 1e3, len(seg)))
