"""Summarise tools/ab_prof.sh output: ms/step, iterations, top kernels per variant."""
import csv, glob, json, os, sys
d = sys.argv[1]
for p in sorted(glob.glob(d + "/p*")):
    i = p[len(d) + 2:]
    env = open(p + "/env.txt").read().strip()
    j = json.load(open(d + "/b%s.json" % i))
    rows = list(csv.DictReader(open(glob.glob(p + "/*kernel_stats.csv")[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    it = j["lm_iterations_per_solve"] * 3
    print("== %s: ms/step %.2f iters/solve %d kernel ms/iter %.3f" % (
        env, j["ms_per_step"], j["lm_iterations_per_solve"], tot / 1e6 / it))
    for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 8]:
        print("   %-34s calls=%5s avg=%8.1fus" % (r["Name"].split("(")[0][:34], r["Calls"], float(r["AverageNs"]) / 1e3))
