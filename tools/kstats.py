"""Print the top kernels of a rocprofv3 --stats CSV."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{r['Name'][:64]:64s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:9.2f}ms "
          f"{float(r['AverageNs'])/1e3:9.1f}us {float(r['Percentage']):6.2f}%")
