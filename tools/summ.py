"""Summarise gpurun_out/cycle bench lines and kernel stats."""
import csv, json, sys, glob
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cycle"
for f in sorted(glob.glob(d + "/bench_*.json")):
    try:
        j = json.load(open(f))
    except Exception as e:
        print(f, "unreadable", e); continue
    print("%-38s val=%.4g %s lm/s=%.1f ms/step=%.2f it=%d rms=%.4f frac=%.4f chol_ms=%.3f split=%s" % (
        j["config"]["workload"], j["value"], j["unit"], j.get("lm_iterations_per_s", 0),
        j["ms_per_step"], j["lm_iterations_per_solve"],
        j["final_rms_px"], j["roofline"]["frac"], j["reduced_cholesky"]["avg_ms"],
        {k: round(v * 1e3, 2) for k, v in j["time_split_s"].items()}))
for f in glob.glob(d + "/prof/*kernel_stats.csv"):
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("kernel total %.1f ms" % (tot / 1e6))
    for r in rows[:14]:
        print("  %-28s calls=%6s avg=%9.1fus  %5.1f%%" % (r["Name"].split("(")[0][:28], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
