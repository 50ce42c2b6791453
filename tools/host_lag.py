"""Host lag in the C4 iteration (round 6): for the last iterations, the
host API calls between the end of the trial's reduction (k_reduce_multi,
whose result the host waits for) and the launch call of the first kernel
the host enqueues after its decision (argv[2], default k_schur_obs), with
times relative to that reduction's end, and the GPU idle gap before that
kernel.  Input: a rocprofv3 --kernel-trace --hip-runtime-trace directory.
usage: python tools/host_lag.py TRACE_DIR [KERNEL]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_schur_obs"


def rows(pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


kt = sorted(rows("*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
ht = sorted(rows("*hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
corr = {r.get("Correlation_Id"): r for r in ht}
tgt = [k for k in kt if name in k["Kernel_Name"]]
print("kernels %d, api calls %d, %s %d" % (len(kt), len(ht), name, len(tgt)))
for r in tgt[-6:]:
    s = int(r["Start_Timestamp"])
    prev = [k for k in kt if int(k["End_Timestamp"]) <= s]
    red = [k for k in prev if "k_reduce_multi" in k["Kernel_Name"]]
    if not red:
        continue
    t0 = int(red[-1]["End_Timestamp"])
    gap = (s - int(prev[-1]["End_Timestamp"])) / 1e3
    call = corr.get(r.get("Correlation_Id"))
    cs = int(call["Start_Timestamp"]) if call else s
    between = [h for h in ht if t0 <= int(h["Start_Timestamp"]) <= cs]
    print("%s: gap %.1f us before it; launch call at +%.1f us after the reduction's end; "
          "GPU start +%.1f" % (name, gap, (cs - t0) / 1e3, (s - t0) / 1e3))
    print("    " + ", ".join("%s@%.1f(%.1f)" % (h["Function"], (int(h["Start_Timestamp"]) - t0) / 1e3,
                                          (int(h["End_Timestamp"]) - int(h["Start_Timestamp"])) / 1e3)
                          for h in between if h["Function"] != "hipStreamQuery"))
    print("    hipStreamQuery x%d, last at +%.1f" % (
        sum(1 for h in between if h["Function"] == "hipStreamQuery"),
        max([(int(h["Start_Timestamp"]) - t0) / 1e3 for h in between
             if h["Function"] == "hipStreamQuery"] or [0])))
