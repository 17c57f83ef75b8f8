import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print(f"{r['Name'][:48]:48s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.1f} per_step_us={float(r['TotalDurationNs'])/1e3/calls:9.1f} pct={float(r['Percentage']):5.1f}")
