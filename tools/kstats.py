"""Top kernels of rocprofv3 kernel_stats.csv files: tools/kstats.py FILE... [--top N]"""
import csv
import sys

top = 14
args = sys.argv[1:]
if "--top" in args:
    i = args.index("--top")
    top = int(args[i + 1])
    del args[i:i + 2]
for f in args:
    print("==", f)
    for x in list(csv.DictReader(open(f)))[:top]:
        print(f"{x['Name'][:70]:70s} n={x['Calls']:>5} avg_us={float(x['AverageNs']) / 1000:9.1f} "
              f"{float(x['Percentage']):6.2f}%")
