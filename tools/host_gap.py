"""Where the host launches k_ne_bnd_jb relative to the GPU timeline
(tools/gpu_hosttrace.sh): for each of the last iterations, the launch call's
start/end against the end of the k_jac_ne_u before it and the start of the
k_ne_bnd_jb it launched, plus the host calls between the previous trial
reduction's end and that launch.  usage: python tools/host_gap.py TRACE_DIR"""
import csv
import glob
import os
import sys

d = sys.argv[1]


def rows(pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


kt = rows("*kernel_trace.csv")
ht = rows("*hip_api_trace.csv")
kt.sort(key=lambda r: int(r["Start_Timestamp"]))
ht.sort(key=lambda r: int(r["Start_Timestamp"]))
corr = {r.get("Correlation_Id"): r for r in ht}
jb = [r for r in kt if "k_ne_bnd_jb" in r["Kernel_Name"]]
print("kernels %d, api calls %d, k_ne_bnd_jb %d" % (len(kt), len(ht), len(jb)))
for r in jb[-6:]:
    s = int(r["Start_Timestamp"])
    prev = [k for k in kt if int(k["End_Timestamp"]) <= s]
    pj = prev[-1]
    red = [k for k in prev if "k_reduce_multi" in k["Kernel_Name"]]
    red_end = int(red[-2]["End_Timestamp"]) if len(red) >= 2 else int(pj["Start_Timestamp"])
    call = corr.get(r.get("Correlation_Id"))
    line = "jb start %.1f us after %s ends" % ((s - int(pj["End_Timestamp"])) / 1e3,
                                            pj["Kernel_Name"][:28])
    if call:
        cs, ce = int(call["Start_Timestamp"]), int(call["End_Timestamp"])
        line += "; launch call %.1f..%.1f us rel. to that end; trial reduction ended %.1f us before it" % (
            (cs - int(pj["End_Timestamp"])) / 1e3, (ce - int(pj["End_Timestamp"])) / 1e3,
            (int(pj["End_Timestamp"]) - red_end) / 1e3)
        between = [h for h in ht if red_end <= int(h["Start_Timestamp"]) <= cs]
        line += "\n    host calls since the trial reduction ended: " + ", ".join(
            "%s@%.1f" % (h["Function"], (int(h["Start_Timestamp"]) - red_end) / 1e3) for h in between[:14])
    print(line)
