import csv, glob, statistics as st, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_vcache<double, 3" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-int(sys.argv[2]):]
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last]
g = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(last, last[1:])]
print(f"timed launches: duration median {st.median(d)/1e3:.2f} us, gap median {st.median(g)/1e3:.2f} us, max {max(g)/1e3:.2f} us")
