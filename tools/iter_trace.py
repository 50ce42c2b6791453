"""Print one LM outer iteration of a rocprofv3 kernel trace (gaps, durations).

usage: iter_trace.py TRACE.csv [ITERATION] [MARKER]
MARKER: substring of the kernel that starts an iteration (default: the first
of k_jac_ne_u / k_jacobian / k_batch_lm present in the trace)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'] for r in rows]
marker = sys.argv[3] if len(sys.argv) > 3 else next(
    (m for m in ('k_jac_ne_u', 'k_jacobian', 'k_batch_lm') if any(m in n for n in names)), None)
idx = [i for i, n in enumerate(names) if marker and marker in n]
if len(idx) < 2:
    print("no two iterations marked by %r" % marker)
    sys.exit(0)
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
k = min(k, len(idx) - 2)
a, b = idx[k], idx[k + 1]
seg = rows[max(a - 3, 0):max(b - 2, a + 1)]
t0 = int(seg[0]['Start_Timestamp']); prev = None; busy = 0
for r in seg:
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    busy += (e - s)
    print(f"{(s-t0)/1e3:8.2f} gap {gap:6.2f} dur {(e-s)/1e3:6.2f} grid {int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']):6d} {r['Kernel_Name'][:50]}")
    prev = e
print("marker %s: span %.1f us, busy %.1f us, %d launches" % (marker, (prev - t0) / 1e3, busy / 1e3, len(seg)))
