"""Start-to-start interval and duration statistics of consecutive stage-kernel
dispatches in a rocprofv3 kernel trace, split into runs at gaps > 50 us."""
import csv, statistics, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "stage_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
runs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["Start_Timestamp"]) > 50000:
        runs.append(cur); cur = []
    cur.append(b)
runs.append(cur)
for i, r in enumerate(runs):
    if len(r) < 30:
        continue
    st = [int(x["Start_Timestamp"]) for x in r]
    du = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in r]
    iv = [b - a for a, b in zip(st, st[1:])]
    print(f"run {i}: n={len(r)} interval median {statistics.median(iv)/1e3:.2f} us  mean {statistics.mean(iv)/1e3:.2f}  "
          f"duration median {statistics.median(du)/1e3:.2f} us  queue {r[0]['Queue_Id']} stream {r[0]['Stream_Id']}")
