"""Per-kernel averages of SQ counters (rocprofv3 --pmc counter_collection.csv
under DIR): wave cycles split into active / issue-stall / parked
(MI355X_MICROARCH.md, rocprofv3 PMC slots: the three are disjoint and sum to
SQ_WAVE_CYCLES), VALU instructions per wave."""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
if not any("SQ_WAVES" in c for c in acc.values()):
    # other counters (FETCH_SIZE / WRITE_SIZE, KB per launch): per-kernel means
    for k, c in sorted(acc.items(), key=lambda kc: -sum(sum(v) for v in kc[1].values())):
        print("%-42s " % k[:42] + "  ".join("%s=%.1f (n=%d)" % (n, sum(v) / len(v), len(v))
                                              for n, v in sorted(c.items())))
    sys.exit(0)
rows = []
for k, c in acc.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    n = len(c.get("SQ_WAVES", [0]))
    rows.append((m.get("SQ_WAVE_CYCLES", 0) * n, k, m, n))
for _, k, m, n in sorted(rows, reverse=True)[:14]:
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    w = m.get("SQ_WAVES", 0) or 1
    print("%-42s n=%4d waves=%7.0f cyc/wave=%8.0f active=%4.0f%% install=%4.0f%% parked=%4.0f%% "
          "valu_act=%4.0f%% valu_inst/wave=%6.0f busy=%.0f" % (
              k[:42], n, w, wc / w, 100 * m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
              100 * m.get("SQ_WAIT_INST_ANY", 0) / wc, 100 * m.get("SQ_WAIT_ANY", 0) / wc,
              100 * m.get("SQ_ACTIVE_INST_VALU", 0) / wc, m.get("SQ_INSTS_VALU", 0) / w,
              m.get("SQ_BUSY_CYCLES", 0)))
