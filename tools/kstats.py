"""Print the top kernels of a rocprofv3 kernel_stats.csv (name, calls, avg us, %)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel total %.2f ms" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print("  %-44s calls=%7s avg=%10.1f us  %5.1f%%" % (
        r["Name"].split("(")[0][:44], r["Calls"], float(r["AverageNs"]) / 1e3,
        100 * float(r["TotalDurationNs"]) / tot))
